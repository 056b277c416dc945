// lbk8s_tpe.h — the thread-per-env path for E <= 8 endpoints (the default 8-endpoint
// scenario and run_baselines' 6-endpoint one).
//
// One lane = one env: the per-env scalar work (Philox draws, the float64 log of the
// exponential draws, reward, accumulators) runs once per env instead of once per
// endpoint lane, and every state load/store is a fully coalesced 64-lane access of the
// endpoint-major SoA layout (endpoint arrays are [E][B]: es = B, ee = 1).
//
// Observations: each lane writes a compact image of its env (29 words: per endpoint
// {zone|cap, cpu f32, lat f32}, plus req zone/threshold, dt, topology) into LDS; the
// wave then copies its 64 envs' (R x 8) float32 rows out as contiguous float4 runs
// (tpe_copy_out), so the 288-byte-per-env obs stream leaves the CU as full cache lines
// instead of 64 scattered 16-byte pieces per store instruction.
#pragma once

#include "lbk8s_common.h"
#include "lbk8s_slice.h"

namespace lbk {

// image words: [0] rz | thr_idx<<2 | flag<<5   [1] f32 dt   [2],[3] topology lo/hi
//              [4+3e] zone | cap<<2   [5+3e] f32 cpu   [6+3e] f32 latency
constexpr int TPE_CW = 4 + 3 * TPE_E + 1;  // 29: odd stride -> conflict-free per-lane writes
constexpr int TPE_FLAG = 1 << 5;

struct TEnv {
    double t, dt, total, last_r;
    uint64_t sum_lat, sum_cpu;  // exact fixed-point episode sums (xsum_add)
    uint64_t topo, zcap, acc2, acc3, nz0, nz1;
    uint32_t sum_hi;
    Scal s;
};

template <bool TRACE>
__device__ __forceinline__ void tpe_request_draws(const Params& p, int64_t env, uint32_t episode,
                                                  uint32_t slot, bool from_reset, double& x1, double& x2,
                                                  int& r, int& n) {
    if constexpr (TRACE) {
        if (from_reset) {
            x1 = p.tr.reset_x1[env]; x2 = p.tr.reset_x2[env]; r = p.tr.reset_r[env]; n = p.tr.reset_n[env];
        } else {
            x1 = p.tr.step_x1[env]; x2 = p.tr.step_x2[env]; r = p.tr.step_r[env]; n = p.tr.step_n[env];
        }
    } else {  // draw map: (D_REQ_X) -> x1 words 0,1 / x2 words 2,3; (D_REQ_I) -> r word 0 / n word 1
        U4 a = draw(p, env, episode, slot, D_REQ_X);
        U4 b = draw(p, env, episode, slot, D_REQ_I);
        x1 = p.inv_rate * std_exp(a.x, a.y);
        x2 = p.call * std_exp(a.z, a.w);
        r = (int)bounded(b.x, 7);
        n = (int)bounded(b.y, (uint32_t)p.N);
    }
}

// Philox mode: an episode's scenario (endpoint latencies and hosts, node types / zones /
// cpu, topology) is a pure function of (seed, global env id, episode), so the step
// recomputes what it needs instead of loading it: 19 Philox blocks replace 112 of the
// ~220 bytes per env-step it reads (lat0 f64 + emeta per endpoint, topology, node zones).
// Measured (A/B builds, profiles/r01_ablation.jsonl, default scenario): 2^20 envs 0.111 -> 0.107 ms, 2^22 envs
// 0.678 -> 0.591 ms; but below 2^18 envs, where a step is latency bound rather than
// bandwidth bound, the serial Philox work lengthens each wave (4096 envs 12.6 -> 15.0 us),
// so lb_step recomputes only from SCEN_RECOMPUTE_MIN_B envs.  reset() still stores the
// scenario (lb_get_field / lb_policy read it); trace mode keeps the stored scenario (its
// values come from the reference's generator).
constexpr int64_t SCEN_RECOMPUTE_MIN_B = 1 << 18;

// endpoint latencies / packed metadata of the episode (reset() :328, :379-386)
__device__ __forceinline__ void tpe_scenario(const Params& p, int64_t env, uint32_t episode,
                                             double (&lat0)[TPE_E], uint32_t (&em)[TPE_E]) {
    int node[TPE_E];
#pragma unroll
    for (int e = 0; e < TPE_E; ++e) {
        lat0[e] = 0.0;
        node[e] = 0;
        if (e < p.E) {
            U4 w = draw(p, env, episode, (uint32_t)e, D_EP);
            lat0[e] = 1.0 + 99.0 * u53(w.x, w.y);
            node[e] = (int)bounded(w.z, 24);
        }
    }
#pragma unroll
    for (int e = 0; e < TPE_E; ++e) {
        em[e] = 0u;
        if (e < p.E) {
            int owner = e;  // first endpoint hosted on the same node (shares its cpu)
#pragma unroll
            for (int e2 = TPE_E - 1; e2 >= 0; --e2)
                if (e2 < e && node[e2] == node[e]) owner = e2;
            int ty, zo, cpu;
            node_draw<false>(p, env, episode, node[e], ty, zo, cpu);
            em[e] = em_pack(zo, owner, ty, cpu, node[e]);
        }
    }
}

__device__ __forceinline__ void tpe_image_env(uint32_t* me, const TEnv& v, int flag) {
    me[0] = (uint32_t)v.s.rz | ((uint32_t)v.s.thr_idx << 2) | (uint32_t)flag;
    me[1] = __float_as_uint((float)v.dt);
    me[2] = (uint32_t)v.topo;
    me[3] = (uint32_t)(v.topo >> 32);
}

// get_state() (:688-758) for the wave's envs: rows [zone, cap, cpu, topo, lat, rz, thr, dt],
// plus the reject row [-1 x 5, rz, thr, dt].  which: COPY_ALL, or only the envs whose
// image flag is set (COPY_FLAGGED) / clear (COPY_UNFLAGGED).
enum { COPY_ALL = 0, COPY_FLAGGED = 1, COPY_UNFLAGGED = 2 };
__device__ __forceinline__ void tpe_copy_out(const Params& p, float* out, const uint32_t* img,
                                             int64_t env0, int which) {
    const int lane = threadIdx.x & 63;
    const int P = 2 * p.R;  // float4 pieces per env (<= 18)
    const int G = 64 / P;   // envs per store instruction
    const int eo = lane / P, piece = lane - eo * P;
    if (eo >= G) return;
    const int row = piece >> 1, half = piece & 1;
    const int64_t left = p.B - env0;
    const int nenv = left < 64 ? (int)left : 64;
    for (int el = eo; el < nenv; el += G) {
        const uint32_t* c = img + el * TPE_CW;
        const uint32_t w0 = c[0];
        if (which != COPY_ALL && (which == COPY_FLAGGED) != ((w0 & TPE_FLAG) != 0)) continue;
        const int rz = (int)(w0 & 3);
        const float thr = (float)threshold((int)((w0 >> 2) & 7));
        const float dt = __uint_as_float(c[1]);
        float4 v;
        if (row < p.E) {
            if (half == 0) {
                const uint32_t q = c[4 + 3 * row];
                const int z = (int)(q & 3);
                const uint64_t topo = (uint64_t)c[2] | ((uint64_t)c[3] << 32);
                v = make_float4((float)z, (float)(q >> 2), __uint_as_float(c[5 + 3 * row]),
                                (float)topo_val(topo, z, rz));
            } else {
                v = make_float4(__uint_as_float(c[6 + 3 * row]), (float)rz, thr, dt);
            }
        } else {
            v = half == 0 ? make_float4(-1.f, -1.f, -1.f, -1.f) : make_float4(-1.f, (float)rz, thr, dt);
        }
        st_stream(reinterpret_cast<float4*>(out + (env0 + el) * (int64_t)p.R * 8) + piece, v);
    }
}

// reset() (:290-400) for this lane's env: draws, per-episode state stores, image.
template <bool TRACE>
__device__ void tpe_reset(const Params& p, int64_t env, TEnv& v, uint32_t* me) {
    const int E = p.E;
    const uint32_t episode = (uint32_t)(v.acc3 >> 32) + 1;
    // next_request() closing reset() (:397), drawn first: its node's zone is captured
    // while the node words are built (Philox is counter-based; trace values are given)
    double x1, x2;
    int r, n;
    tpe_request_draws<TRACE>(p, env, episode, 0, true, x1, x2, r, n);
    // nodes (:349-373): zone capacity + 2-bit zone words
    uint64_t zc = 0, nzq = 0;
    v.nz0 = 0;
    v.nz1 = 0;
    for (int w = 0; w < p.NZW; ++w) {
        uint64_t word = 0;
        const int nend = 32 * (w + 1) < p.N ? 32 * (w + 1) : p.N;
        for (int k = 32 * w; k < nend; ++k) {
            int ty, zo, cpu;
            node_draw<TRACE>(p, env, episode, k, ty, zo, cpu);
            zc += (uint64_t)node_cpu_int(ty) << (16 * zo);
            word |= (uint64_t)zo << (2 * (k & 31));
        }
        if (w == 0) v.nz0 = word;
        if (w == 1) v.nz1 = word;
        if (w == (n >> 5)) nzq = word;
        p.nzone[w * p.B + env] = word;
    }
    // endpoints (:328, :379-386)
    double lat0[TPE_E];
    int node[TPE_E];
#pragma unroll
    for (int e = 0; e < TPE_E; ++e) {
        lat0[e] = 0.0;
        node[e] = 0;
        if (e < E) {
            if constexpr (TRACE) {
                lat0[e] = p.tr.reset_lat0[env * E + e];
                node[e] = p.tr.reset_enode[env * E + e];
            } else {
                U4 w = draw(p, env, episode, (uint32_t)e, D_EP);
                lat0[e] = 1.0 + 99.0 * u53(w.x, w.y);
                node[e] = (int)bounded(w.z, 24);
            }
        }
    }
#pragma unroll
    for (int e = 0; e < TPE_E; ++e) {
        if (e < E) {
            int owner = e;  // first endpoint hosted on the same node (shares its cpu)
#pragma unroll
            for (int e2 = TPE_E - 1; e2 >= 0; --e2)
                if (e2 < e && node[e2] == node[e]) owner = e2;
            int ty, zo, cpu;
            node_draw<TRACE>(p, env, episode, node[e], ty, zo, cpu);
            const int64_t i = (int64_t)e * p.B + env;
            p.lat0[i] = lat0[e];
            p.emeta[i] = em_pack(zo, owner, ty, cpu, node[e]);
            p.edyn[i] = 0;
            me[4 + 3 * e] = (uint32_t)zo | ((uint32_t)zcap_val(zc, zo) << 2);
            me[5 + 3 * e] = __float_as_uint((float)cpu);
            me[6 + 3 * e] = __float_as_uint((float)lat0[e]);
        }
    }
    // topology (:331-338): symmetric, diag 1; the 4x4 zone block is all that is observable
    uint64_t topo = 0;
    if constexpr (TRACE) {
        const int32_t* d = p.tr.reset_topo + env * (int64_t)p.Z * (p.Z - 1);
        int q = 0;
        for (int i = 0; i < 4; ++i)
            for (int j = i + 1; j < 4; ++j, ++q)  // last writer: (z1=j, z2=i)
                topo |= (uint64_t)(d[j * (p.Z - 1) + i] & 0x1FF) << (9 * q);
    } else {
        U4 a = draw(p, env, episode, 0, D_TOPO), b = draw(p, env, episode, 1, D_TOPO);
        topo = (uint64_t)(1 + bounded(a.x, 499)) | ((uint64_t)(1 + bounded(a.y, 499)) << 9) |
               ((uint64_t)(1 + bounded(a.z, 499)) << 18) | ((uint64_t)(1 + bounded(a.w, 499)) << 27) |
               ((uint64_t)(1 + bounded(b.x, 499)) << 36) | ((uint64_t)(1 + bounded(b.y, 499)) << 45);
    }
    v.topo = topo;
    v.zcap = zc;
    v.acc2 = 0;
    v.acc3 = (uint64_t)episode << 32;
    v.sum_lat = 0;
    v.sum_cpu = 0;
    v.sum_hi = 0;
    v.total = 0.0;
    v.last_r = p.init_last_r;
    v.s.step = 0; v.s.acc = 0; v.s.intra = 0; v.s.penalty = 0; v.s.reset_done = 1;
    const double arrival = v.t + x1;
    const double departure = arrival + x2;
    v.dt = departure - arrival;
    v.t = arrival;
    v.s.thr_idx = (r + 6) % 7;
    v.s.rz = (int)((nzq >> (2 * (n & 31))) & 3);
    p.topo[env] = topo;
    p.zcap[env] = zc;
}

__device__ __forceinline__ void tpe_store_scalars(const Params& p, int64_t env, const TEnv& v) {
    *(p.t + env) = (v.t);
    *(p.sc + env) = (sc_pack(v.s));
    *(p.acc2 + env) = (v.acc2);
    *(p.acc3 + env) = (v.acc3);
    *(p.sum_lat + env) = (v.sum_lat);
    *(p.sum_cpu + env) = (v.sum_cpu);
    *(p.sum_hi + env) = (v.sum_hi);
    *(p.total + env) = (v.total);
    if (p.reward_fn != LB_REWARD_NAIVE) *(p.last_r + env) = (v.last_r);
}

// NB: threads per block.  Everything here is per wave (LDS image, copy-out), so small
// batches launch 64-thread blocks: one wave per CU instead of four on a quarter of the CUs.
template <bool TRACE, int NB = BLOCK>
__global__ __launch_bounds__(NB) void k_reset_tpe(Params p) {
    __shared__ uint32_t lds[NB * TPE_CW];
    const int lane = threadIdx.x & 63;
    uint32_t* img = lds + (threadIdx.x & ~63) * TPE_CW;
    uint32_t* me = img + lane * TPE_CW;
    const int64_t env0 = (int64_t)blockIdx.x * NB + (threadIdx.x & ~63);
    const int64_t env = env0 + lane;
    const bool doit = env < p.B && (!p.reset_mask || p.reset_mask[env]);
    me[0] = 0;
    if (doit) {
        TEnv v;
        v.t = p.t[env];
        v.acc3 = p.acc3[env];
        v.s = sc_unpack(p.sc[env]);
        tpe_reset<TRACE>(p, env, v, me);
        tpe_image_env(me, v, TPE_FLAG);
        tpe_store_scalars(p, env, v);
    }
    __syncthreads();
    if (p.obs) tpe_copy_out(p, p.obs, img, env0, COPY_FLAGGED);
}

constexpr int RO_STRIDE = 19;  // float4 per lane in the rollout's obs image (2R <= 18, + 1 pad)
constexpr int RO_REC_OFF = 512;  // words: a wave region's reset records, past its list (<= 449 words)
// lanes per reset in the rollout: a whole wave per finishing env (the 24 node draws, 8
// endpoint draws and the request in parallel, a chain about 3 Philox blocks deep), each of
// the block's waves takes one listed env per round.  With staggered episodes a 256-env
// block has ~2.6 finishing envs per step: 8-lane groups left three waves parked at the
// barrier behind one wave's 5-block-deep reset chain (2^20 envs: 111 us per step vs 78
// lockstep).
constexpr int RO_RW = 64;

// get_state() (:688-758) rows of this lane's env from registers, into its LDS image
__device__ __forceinline__ void tpe_obs_rows(const Params& p, float4* row, const TEnv& v,
                                             const uint32_t (&em)[TPE_E], const float (&olat)[TPE_E],
                                             const float (&ocpu)[TPE_E]) {
    const float rz = (float)v.s.rz, thr = (float)threshold(v.s.thr_idx), dt = (float)v.dt;
#pragma unroll
    for (int e = 0; e < TPE_E; ++e) {
        if (e < p.E) {
            const int z = em_zone(em[e]);
            row[2 * e] = make_float4((float)z, (float)zcap_val(v.zcap, z), ocpu[e], (float)topo_val(v.topo, z, v.s.rz));
            row[2 * e + 1] = make_float4(olat[e], rz, thr, dt);
        }
    }
    if (p.R > p.E) {  // the reject row
        row[2 * p.E] = make_float4(-1.f, -1.f, -1.f, -1.f);
        row[2 * p.E + 1] = make_float4(-1.f, rz, thr, dt);
    }
}

// envs el0 .. el0 + nstage - 1 of the wave from its image (lane el - el0 holds env el's rows)
// as contiguous float4 runs (G envs per store instruction); m = the wave's finishing envs,
// which = COPY_ALL / FLAGGED / UNFLAGGED
__device__ __forceinline__ void tpe_copy_rows(const Params& p, float* out, const float4* wimg, int64_t env0,
                                              uint64_t m, int which, int el0, int nstage) {
    const int lane = threadIdx.x & 63;
    const int P = 2 * p.R;
    const int G = 64 / P;
    const int eo = lane / P, piece = lane - eo * P;
    if (eo >= G) return;
    const int64_t left = p.B - env0;
    const int nenv = left < el0 + nstage ? (int)left : el0 + nstage;
    float4* base = reinterpret_cast<float4*>(out + env0 * (int64_t)p.R * 8) + piece;
    for (int el = el0 + eo; el < nenv; el += G) {
        if (which != COPY_ALL && (which == COPY_FLAGGED) != (((m >> el) & 1) != 0)) continue;
        st_stream(base + el * P, wimg[(el - el0) * RO_STRIDE + piece]);
    }
}

// The LDS image and the copy-out are wave-local: a wave orders its own LDS accesses, so it
// needs no block barrier (which would also wait for every global store the wave has in
// flight); the compiler is kept from moving LDS accesses across the point.
__device__ __forceinline__ void wave_lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
// LDS-only block barrier: the waves' global stores stay in flight.
__device__ __forceinline__ void block_lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// step() (:403-513) of this lane's env held in registers, in two parts.  tpe_prep: the
// action's decode, the selected endpoint and the 4 table values take_action needs (they
// depend only on the action and the counters, so a multi-step kernel issues them for the
// next step while the current step's rows are being stored).
struct TPrep {
    int a, ai, oA, jA, Mn, jn;
    bool accept, reject;
    uint32_t emA, edA, edO;
    double lat0A, lut_selA, sel_cpu, next_lat, next_cpu;
    double x1, x2;  // the step's next_request() draws (tpe_prep_request; Philox mode)
    int r, n;
};
// the draws of the next_request() that closes the coming step (slot = its step count)
__device__ __forceinline__ void tpe_prep_request(const Params& p, int64_t ev, const TEnv& v, TPrep& pr) {
    const int slot = v.s.step < 0xFFFF ? v.s.step + 1 : 0xFFFF;
    tpe_request_draws<false>(p, ev, (uint32_t)(v.acc3 >> 32), (uint32_t)slot, false, pr.x1, pr.x2, pr.r, pr.n);
}
__device__ __forceinline__ TPrep tpe_prep(const Params& p, const double (&lat0)[TPE_E], const uint32_t (&em)[TPE_E],
                                          const uint32_t (&ed)[TPE_E], int a) {
    TPrep r;
    const int E = p.E;
    r.a = a;
    r.accept = a >= -E && a < E;
    r.reject = a == E;
    r.ai = r.accept ? (a < 0 ? a + E : a) : 0;
    r.emA = em[0];
    r.edA = ed[0];
    r.lat0A = lat0[0];
#pragma unroll
    for (int e = 1; e < TPE_E; ++e)
        if (r.ai == e) { r.emA = em[e]; r.edA = ed[e]; r.lat0A = lat0[e]; }
    r.oA = em_owner(r.emA);
    r.edO = ed[0];
#pragma unroll
    for (int e = 1; e < TPE_E; ++e)
        if (r.oA == e) r.edO = ed[e];
    r.jA = ed_j(r.edA);
    r.Mn = ed_M(r.edO) < CMAX ? ed_M(r.edO) + 1 : CMAX;
    r.jn = r.jA < CMAX ? r.jA + 1 : CMAX;
    const int k0A = (int)r.lat0A, c0A = em_c0(r.emA);
    r.lut_selA = p.lat_lut[(r.jA) * LAT_ROWS + k0A];
    r.sel_cpu = p.cpu_lut[(ed_m(r.edA)) * CPU_ROWS + c0A];
    r.next_lat = p.lat_lut[(r.jn) * LAT_ROWS + k0A];
    r.next_cpu = p.cpu_lut[(r.Mn) * CPU_ROWS + c0A];
    return r;
}

// tpe_apply (after the step counter advanced): take_action (:578-686), reward (:516-567),
// next_request() (:1131-1163).  Writes the endpoint words of the env's obs image (me) and
// returns the reward.  ED_REGS: the history counters advance in ed[] (the multi-step
// rollout keeps them in registers); otherwise the changed words are stored at once when
// keep is set.  ED_REGS also keeps the observed latency / cpu of every endpoint in olat /
// ocpu (float32, the obs columns): only the selected endpoint's change in a step, so the
// rollout gathers 4 table values per step instead of up to 2E + 4.  STORED: the request
// node's zone comes from the node-zone words (nodes >= 64 from HBM) instead of a redraw.
template <bool TRACE, bool STORED, bool ED_REGS, bool OBS_REGS = ED_REGS, bool REQ_PREP = false>
__device__ __forceinline__ double tpe_apply(const Params& p, const TPrep& pr, int64_t ev, int64_t env, bool keep,
                                            TEnv& v, const double (&lat0)[TPE_E], const uint32_t (&em)[TPE_E],
                                            uint32_t (&ed)[TPE_E], float (&olat)[TPE_E], float (&ocpu)[TPE_E],
                                            uint32_t* me) {
    constexpr bool stored = STORED;
    const int E = p.E;
    const int a = pr.a, ai = pr.ai, oA = pr.oA, jA = pr.jA, Mn = pr.Mn, jn = pr.jn;
    const bool accept = pr.accept, reject = pr.reject;
    const uint32_t emA = pr.emA, edA = pr.edA, edO = pr.edO;
    const double lat0A = pr.lat0A, lut_selA = pr.lut_selA, sel_cpu = pr.sel_cpu, next_lat = pr.next_lat,
                 next_cpu = pr.next_cpu;
    if (a < -E) v.s.bad = 1;  // reference: IndexError; here: treated as unrecognised
    if (!v.s.reset_done) v.s.bad = 1;
    int cnt = 0;  // #{e != ai : loads[e] <= loads[ai]} for the O(E) Gini update
#pragma unroll
    for (int e = 0; e < TPE_E; ++e) {
        if (e < E) {
            const int j = ed_j(ed[e]);
            // table rows 0 are the initial values: only endpoints selected (j > 0) /
            // refreshed (m > 0) this episode gather from the LUTs
            float ol, oc;
            if constexpr (ED_REGS) {
                ol = olat[e];
                oc = ocpu[e];
            } else {  // (the single step gathers the observed values of every endpoint)
                const int m = ed_m(ed[e]);
                double l = lat0[e], c = (double)em_c0(em[e]);
                if (j) l = p.lat_lut[j * LAT_ROWS + (int)lat0[e]];
                if (m) c = p.cpu_lut[m * CPU_ROWS + em_c0(em[e])];
                ol = (float)l;
                oc = (float)c;
            }
            if (accept && e == ai) { ol = (float)next_lat; oc = (float)next_cpu; }
            if constexpr (OBS_REGS) {  // (the caller writes the obs rows from olat / ocpu)
                olat[e] = ol;
                ocpu[e] = oc;
            } else {
                const int z = em_zone(em[e]);
                me[4 + 3 * e] = (uint32_t)z | ((uint32_t)zcap_val(v.zcap, z) << 2);
                me[5 + 3 * e] = __float_as_uint(oc);
                me[6 + 3 * e] = __float_as_uint(ol);
            }
            if (e != ai && j <= jA) ++cnt;
        }
    }

    // ---- take_action (:578-686)
    double reward;
    if (accept) {
        const int zA = em_zone(emA);
        const double sel_lat = jA == 0 ? lat0A : lut_selA;
        const int tl = topo_val(v.topo, v.s.rz, zA);
        const uint32_t gnum = (uint32_t)(v.acc2 >> 32) + (uint32_t)(2 * (2 * cnt - (E - 1)));
        const uint32_t sum_topo = (uint32_t)v.acc2 + (uint32_t)tl;
        v.acc2 = ((uint64_t)gnum << 32) | sum_topo;
        v.acc3 += (uint64_t)node_cost(em_type(emA));
        v.s.acc = v.s.acc < 0xFFFF ? v.s.acc + 1 : 0xFFFF;
        if (v.s.rz == zA) v.s.intra = v.s.intra < 0xFFFF ? v.s.intra + 1 : 0xFFFF;
        xsum_add(v.sum_lat, v.sum_cpu, v.sum_hi, sel_lat, sel_cpu, tl, v.s.rz != zA);
        // increase_resources / increase_endpoint_latency (:674-677) and the same step's
        // decrease in next_request() (:1137-1143) -> the history counters advance
        const uint32_t edA_new = ((oA == ai ? (uint32_t)Mn : (uint32_t)ed_M(edA)) << 20) |
                                 ((uint32_t)Mn << 10) | (uint32_t)jn;
        if constexpr (ED_REGS) {
            // select-stores over constant indices (a runtime-indexed store would move ed[]
            // out of registers)
#pragma unroll
            for (int e = 0; e < TPE_E; ++e) {
                const uint32_t edo = e == oA ? (ed[e] & ~(0x3FFu << 20)) | ((uint32_t)Mn << 20) : ed[e];
                ed[e] = e == ai ? edA_new : edo;
            }
        } else if (keep) {
            if (oA != ai) *(p.edyn + (int64_t)oA * p.B + env) = ((edO & ~(0x3FFu << 20)) | ((uint32_t)Mn << 20));
            *(p.edyn + (int64_t)ai * p.B + env) = (edA_new);
        }
        v.s.penalty = 0;
        reward = accept_reward(p, sel_lat, tl, sel_cpu, v.acc2, v.s.acc);
        v.last_r = reward;
    } else if (reject) {
        v.s.penalty = 1;
        reward = p.reward_fn == LB_REWARD_LATENCY ? -1000.0 : -1.0;
        v.last_r = reward;
    } else {  // unrecognised action (:685-686): penalty and selected_* stay stale
        reward = p.reward_fn == LB_REWARD_NAIVE ? (v.s.penalty ? -1.0 : 1.0) : v.last_r;
    }
    v.total += reward;

    // ---- next_request (:1131-1163)
    {
        double x1, x2;
        int r, n;
        if constexpr (REQ_PREP) {
            x1 = pr.x1; x2 = pr.x2; r = pr.r; n = pr.n;
        } else {
            tpe_request_draws<TRACE>(p, ev, (uint32_t)(v.acc3 >> 32), (uint32_t)v.s.step, false, x1, x2, r, n);
        }
        const double arrival = v.t + x1;
        const double departure = arrival + x2;
        v.dt = departure - arrival;
        v.t = arrival;
        v.s.thr_idx = (r + 6) % 7;  // endpoint_list[r - 1] (:1117)
        if constexpr (stored) {
            const uint64_t word = n < 32 ? v.nz0 : (n < 64 ? v.nz1 : p.nzone[(int64_t)(n >> 5) * p.B + ev]);
            v.s.rz = (int)((word >> (2 * (n & 31))) & 3);
        } else {  // the zone of the request's node (:1120-1121), drawn again
            int ty, zo, cpu;
            node_draw<false>(p, ev, (uint32_t)(v.acc3 >> 32), n, ty, zo, cpu);
            v.s.rz = zo;
        }
    }
    return reward;
}


// step() (:403-513) fused with next_request(), get_state(), reward and done.  RECOMPUTE
// (Philox mode, many envs): the scenario is redrawn instead of loaded.
// VecEnv auto-reset: an env whose episode ends gets its terminal obs and episode-stats row,
// then its reset() in this kernel with RS_W = 8 lanes (the node draws spread over the
// lanes instead of one lane's ~36 serial Philox blocks): each wave lists its finishing envs
// (id, t, acc3, sc) in its own LDS image once the copy-out has read it, and after one
// LDS-only block barrier the block's waves take the block's list 8 envs per wave-round.
// The step skips the state stores the reset rewrites (scalars, history counters).
// Measured against a separate reset kernel over per-wave lists (round 2, bench workload,
// profiles/r01_ablation.jsonl): 131,072 envs 25.4 -> 23.9 us per step, 2^19 67 -> 64.5,
// 2^20 equal (112 us): the second launch's ramp, not the reset work, was the cost.
constexpr int RS_LIST_W = 7;  // words per list item: env, t (2), acc3 (2), sc (2)
constexpr int STEP_STAGE = 32;  // k_step_tpe: envs per obs staging pass (half a wave)
template <bool TRACE, bool RECOMPUTE, int NB = BLOCK>
__global__ __launch_bounds__(NB) void k_step_tpe(Params p) {
    constexpr int NW = NB / 64;
    // per wave: half the wave's finished (R x 8) rows at a time (the list of finishing envs
    // reuses the region); 39 KB per 256-thread block keeps 4 blocks per CU
    __shared__ float4 oimg[NW][STEP_STAGE * RO_STRIDE];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    float4* wimg = oimg[wv];
    uint32_t* img = reinterpret_cast<uint32_t*>(wimg);
    float4* mine = wimg + (lane % STEP_STAGE) * RO_STRIDE;
    const int64_t env0 = (int64_t)blockIdx.x * NB + (threadIdx.x & ~63);
    const int64_t env = env0 + lane;
    const bool live = env < p.B;
    const int64_t ev = live ? env : 0;  // dead lanes read env 0 (harmless) and store nothing
    const int E = p.E;

    // ---- phase 0: every independent load, coalesced across the wave
    TEnv v;
    double lat0[TPE_E];
    uint32_t em[TPE_E], ed[TPE_E];
    constexpr bool stored = TRACE || !RECOMPUTE;
#pragma unroll
    for (int e = 0; e < TPE_E; ++e) {
        const int64_t i = (int64_t)e * p.B + ev;
        if constexpr (stored) {
            lat0[e] = e < E ? *(p.lat0 + i) : 0.0;
            em[e] = e < E ? *(p.emeta + i) : 0u;
        }
        ed[e] = e < E ? *(p.edyn + i) : 0u;
    }
    int a = p.actions ? *(p.actions + ev) : 0;
    v.t = *(p.t + ev);
    v.s = sc_unpack(*(p.sc + ev));
    v.zcap = *(p.zcap + ev);
    v.acc2 = *(p.acc2 + ev);
    v.acc3 = *(p.acc3 + ev);
    if (!p.actions) a = random_action(p, ev, v.acc3, v.s.step);  // fused random policy
    if constexpr (stored) {
        v.topo = *(p.topo + ev);
        v.nz0 = *(p.nzone + ev);
        v.nz1 = p.NZW > 1 ? *(p.nzone + p.B + ev) : 0;
    } else {
        const uint32_t episode = (uint32_t)(v.acc3 >> 32);
        tpe_scenario(p, ev, episode, lat0, em);
        v.topo = scen_topo(p, ev, episode);
        v.nz0 = 0;
        v.nz1 = 0;
    }
    v.sum_lat = *(p.sum_lat + ev);
    v.sum_cpu = *(p.sum_cpu + ev);
    v.sum_hi = *(p.sum_hi + ev);
    v.total = *(p.total + ev);
    v.last_r = p.reward_fn != LB_REWARD_NAIVE ? *(p.last_r + ev) : 0.0;

    // ---- phase 1: decode the action, pick the selected endpoint, table lookups
    v.s.step = v.s.step < 0xFFFF ? v.s.step + 1 : 0xFFFF;
    const bool done = live && v.s.step == p.L;  // (:472)
    const bool do_reset = done && p.auto_reset;
    const bool keep = live && !do_reset;  // the state stores reset() below does not redo
    float olat[TPE_E], ocpu[TPE_E];  // observed endpoint latency / cpu after the step
    const TPrep pr = tpe_prep(p, lat0, em, ed, a);
    const double reward = tpe_apply<TRACE, stored, false, true>(p, pr, ev, env, keep, v, lat0, em, ed, olat, ocpu,
                                                                nullptr);
    if (live) {
        if (p.reward) *(p.reward + env) = ((float)reward);
        if (p.rew64) p.rew64[env] = reward;
        if (p.done) p.done[env] = (uint8_t)done;
    }

    // ---- VecEnv auto-reset: terminal obs + episode stats, then reset() below
    const uint64_t m = __ballot(do_reset);
    if (do_reset && p.ep_stats)
        write_stats_row(p, p.ep_stats + env * LB_ST_K, v.s, v.acc2, v.acc3, v.total, v.sum_lat, v.sum_cpu, v.sum_hi);
    if (keep) tpe_store_scalars(p, env, v);
    // get_state() rows built once per env, staged half a wave at a time; the finished envs'
    // post-reset obs come from their reset()
    for (int el0 = 0; el0 < 64; el0 += STEP_STAGE) {
        if (lane / STEP_STAGE == el0 / STEP_STAGE) tpe_obs_rows(p, mine, v, em, olat, ocpu);
        wave_lds_sync();
        if (p.term_obs && m) tpe_copy_rows(p, p.term_obs, wimg, env0, m, COPY_FLAGGED, el0, STEP_STAGE);
        if (p.obs) tpe_copy_rows(p, p.obs, wimg, env0, m, p.auto_reset ? COPY_UNFLAGGED : COPY_ALL, el0, STEP_STAGE);
        wave_lds_sync();
    }
    if (p.auto_reset) {  // uniform over the grid: every wave reaches the barrier
        if (do_reset) {  // the wave's list replaces its (copied-out) image
            uint32_t* it = img + 1 + RS_LIST_W * __popcll(m & ((1ull << lane) - 1));
            const uint64_t tb = (uint64_t)__double_as_longlong(v.t), sc = sc_pack(v.s);
            it[0] = (uint32_t)env;
            it[1] = (uint32_t)tb; it[2] = (uint32_t)(tb >> 32);
            it[3] = (uint32_t)v.acc3; it[4] = (uint32_t)(v.acc3 >> 32);
            it[5] = (uint32_t)sc; it[6] = (uint32_t)(sc >> 32);
        }
        if (lane == 0) img[0] = (uint32_t)__popcll(m);
        if (NW > 1) block_lds_sync();
        else wave_lds_sync();
        int pre[NW + 1];
        pre[0] = 0;
#pragma unroll
        for (int w = 0; w < NW; ++w) pre[w + 1] = pre[w] + (int)reinterpret_cast<const uint32_t*>(oimg[w])[0];
        const int g = lane / RS_W, gl = lane % RS_W;
        for (int i = wv * (64 / RS_W) + g; i < pre[NW]; i += NW * (64 / RS_W)) {
            int q = 0;
#pragma unroll
            for (int w = 1; w < NW; ++w) q += i >= pre[w];
            int base = 0;
#pragma unroll
            for (int w = 1; w < NW; ++w) base = q == w ? pre[w] : base;
            const uint32_t* it = reinterpret_cast<const uint32_t*>(oimg[q]) + 1 + RS_LIST_W * (i - base);
            const int64_t renv = (int64_t)it[0];
            SEnv<1> sv;
            sv.t = __longlong_as_double((long long)((uint64_t)it[1] | ((uint64_t)it[2] << 32)));
            sv.acc3 = (uint64_t)it[3] | ((uint64_t)it[4] << 32);
            sv.s = sc_unpack((uint64_t)it[5] | ((uint64_t)it[6] << 32));
            slice_reset<RS_W, 1, TRACE>(p, renv, gl, sv);
            if (p.obs) slice_write_obs<RS_W, 1>(p, p.obs, renv, gl, sv);
            if (gl == 0) slice_store_scalars<1>(p, renv, sv);
        }
    }
}

// envs/baselines.py (:6-35) on one lane's registers (k_policy's values): argmin topology
// latency / argmax zone cpu capacity / argmin endpoint cpu over feasible = mask[:-1]
// (masks are all True, :808-821), first index on ties; or the uniform random action.
// (The kind is a template parameter: the endpoint-cpu gathers would otherwise hold
// registers in every instantiation of the rollout.)
template <int KIND>
__device__ __forceinline__ int tpe_policy(const Params& p, int64_t ev, const TEnv& v, const uint32_t (&em)[TPE_E],
                                          const uint32_t (&ed)[TPE_E]) {
    if constexpr (KIND == LB_POLICY_RANDOM) return random_action(p, ev, v.acc3, v.s.step);
    const int nf = p.A - 1;
    if (nf <= 0) return p.A - 1;
    double best = 0.0;
    int bi = 0;
#pragma unroll
    for (int e = 0; e < TPE_E; ++e) {
        if (e >= nf) continue;
        const int z = em_zone(em[e]);
        double val;
        if constexpr (KIND == LB_POLICY_TOPOLOGY_GREEDY) val = (double)topo_val(v.topo, z, v.s.rz);
        else if constexpr (KIND == LB_POLICY_ZONE_CPU_GREEDY) val = -(double)zcap_val(v.zcap, z);
        else val = cpu_of(p, em[e], ed[e]);
        if (e == 0 || val < best) { best = val; bi = e; }
    }
    return bi;
}

// lb_rollout on the thread-per-env layout: K vector steps under an on-device policy in ONE
// launch, each lane's env held in registers from the first step to the last (including the
// observed latency / cpu of every endpoint, so a step gathers 4 table values); step k's
// obs / reward / done / action go to slot k.  The state is read once and written once per
// launch instead of once per step, and there is one launch ramp per K steps.
// Observations: each lane writes its env's finished (R x 8) float32 rows into the wave's LDS
// image (a 76-word stride per lane: 16-byte writes of 8 consecutive lanes cover all 32
// banks), and the wave copies its 64 envs' rows out as contiguous float4 runs; building
// the rows once per env instead of decoding a compact image per stored piece took the
// copy-out from about half of the step's VALU instructions to a load and a store.
// Auto-reset, PRE (episode_length >= K, so an env ends at most once per launch; the bench's
// L = K = 100): before the first step each wave draws the next episode of its envs that end
// inside the launch into their records (tpe_write_record, 8 lanes per env); the step that
// ends an episode loads the record at its start and starts the new episode from it
// (tpe_start_episode) -- no barrier and no reset chain inside the step loop.  Otherwise
// (L < K): each wave lists its finishing envs in its image region (as k_step_tpe), and after
// an LDS-only block barrier the block's waves run the listed resets RO_RW = 64 lanes per env,
// one env per wave per round; a reset writes the env's post-reset obs into slot k and its new
// episode into an LDS record (RS_REC_W words), from which the owning lane reloads its
// registers after a second barrier.  Nothing but the outputs leaves the CU between steps, so
// no barrier waits on global stores.  Needs N <= 64 (the node-zone words stay in registers).
// Bit for bit K x (lb_policy + lb_step) and the C oracle (tests/test_gpu_api.py,
// tests/test_gpu_parity.py).
constexpr int RS_REC_W = 40;   // LDS record of an in-loop reset: lat0 (16), emeta (8), topo, zcap, nz0, nz1, t, acc3, sc
// The next episode of an env, as reset() (:290-400) draws it in Philox mode, into its
// RO_REC_BYTES record (p.rec): W lanes per env, lane e < E its endpoint (the same draws and
// owner rule as slice_reset).  Words: lat0 [0,16), emeta [16,24), topo, zcap, nz0, nz1, the
// first request's x1, x2 (f64) [24,36), thr_idx | rz << 8 [36].  The clock is not in it:
// arrival = t + x1 is applied when the episode starts.
template <int W>
__device__ __forceinline__ void tpe_write_record(const Params& p, int64_t env, uint32_t episode, int lane) {
    uint64_t zc = 0, nz0 = 0, nz1 = 0;
    for (int w = 0; w < p.NZW; ++w) {  // nodes (:349-373)
        uint64_t word = 0;
        for (int n = 32 * w + lane; n < 32 * (w + 1) && n < p.N; n += W) {
            int ty, zo, cpu;
            node_draw<false>(p, env, episode, n, ty, zo, cpu);
            zc += (uint64_t)node_cpu_int(ty) << (16 * zo);
            word |= (uint64_t)zo << (2 * (n & 31));
        }
        word = slice_or64<W>(word);
        if (w == 0) nz0 = word;
        if (w == 1) nz1 = word;
    }
    zc = slice_sum64<W>(zc);
    double lat0 = 0.0;  // endpoints (:328, :379-386)
    int node = 0;
    if (lane < p.E) {
        const U4 d = draw(p, env, episode, (uint32_t)lane, D_EP);
        lat0 = 1.0 + 99.0 * u53(d.x, d.y);
        node = (int)bounded(d.z, 24);
    }
    int owner = lane;  // first endpoint hosted on the same node
    for (int e2 = 0; e2 < p.E; ++e2) {
        const int nd2 = (int)shfl_u32<W>((uint32_t)node, e2);
        if (nd2 == node && e2 < owner) owner = e2;
    }
    uint32_t* out = reinterpret_cast<uint32_t*>(p.rec + env * (RO_REC_BYTES / 16));
    if (lane < p.E) {
        int ty, zo, cpu;
        node_draw<false>(p, env, episode, node, ty, zo, cpu);
        const uint64_t lb = (uint64_t)__double_as_longlong(lat0);
        *reinterpret_cast<uint2*>(out + 2 * lane) = make_uint2((uint32_t)lb, (uint32_t)(lb >> 32));
        out[16 + lane] = em_pack(zo, owner, ty, cpu, node);
    }
    const uint64_t topo = scen_topo(p, env, episode);  // (:331-338)
    double x1, x2;  // next_request() closing reset() (:397)
    int r, n;
    slice_request_draws<W, false>(p, env, episode, 0, lane, true, x1, x2, r, n);
    if (lane == 0) {
        const int rz = (int)(((n < 32 ? nz0 : nz1) >> (2 * (n & 31))) & 3);
        const uint64_t w[6] = {topo, zc, nz0, nz1, (uint64_t)__double_as_longlong(x1),
                               (uint64_t)__double_as_longlong(x2)};
#pragma unroll
        for (int j = 0; j < 6; ++j)
            *reinterpret_cast<uint2*>(out + 24 + 2 * j) = make_uint2((uint32_t)w[j], (uint32_t)(w[j] >> 32));
        out[36] = (uint32_t)((r + 6) % 7) | ((uint32_t)rz << 8);
    }
}

// reset() from the env's record: the episode counter advances, the clock runs on (t is
// never reset, :1135), the first request arrives at t + x1
// (q: the record's first 38 words; loaded where the episode starts: loading them at the
// start of the step held 40 more registers across it, 2^20: 67.5 -> 66.2 us per step)
__device__ __forceinline__ void tpe_start_episode(const Params& p, const uint4 (&q)[10], TEnv& v,
                                                  double (&lat0)[TPE_E], uint32_t (&em)[TPE_E],
                                                  uint32_t (&ed)[TPE_E], float (&olat)[TPE_E],
                                                  float (&ocpu)[TPE_E]) {
    uint32_t w[40];
#pragma unroll
    for (int j = 0; j < 10; ++j) {
        w[4 * j] = q[j].x; w[4 * j + 1] = q[j].y; w[4 * j + 2] = q[j].z; w[4 * j + 3] = q[j].w;
    }
    auto u64 = [&](int i) { return (uint64_t)w[i] | ((uint64_t)w[i + 1] << 32); };
#pragma unroll
    for (int e = 0; e < TPE_E; ++e) {
        lat0[e] = e < p.E ? __longlong_as_double((long long)u64(2 * e)) : 0.0;
        em[e] = e < p.E ? w[16 + e] : 0u;
        ed[e] = 0u;
        olat[e] = (float)lat0[e];  // table rows 0: the initial values
        ocpu[e] = (float)em_c0(em[e]);
    }
    v.topo = u64(24);
    v.zcap = u64(26);
    v.nz0 = u64(28);
    v.nz1 = u64(30);
    const uint32_t episode = (uint32_t)(v.acc3 >> 32) + 1;
    v.acc3 = (uint64_t)episode << 32;
    v.acc2 = 0;
    v.sum_lat = 0;
    v.sum_cpu = 0;
    v.sum_hi = 0;
    v.total = 0.0;
    v.last_r = p.init_last_r;
    v.s.step = 0; v.s.acc = 0; v.s.intra = 0; v.s.penalty = 0; v.s.reset_done = 1;
    v.s.thr_idx = (int)(w[36] & 7);
    v.s.rz = (int)((w[36] >> 8) & 3);
    const double arrival = v.t + __longlong_as_double((long long)u64(32));
    const double departure = arrival + __longlong_as_double((long long)u64(34));
    v.dt = departure - arrival;
    v.t = arrival;
}

template <int NB, int KIND, bool PRE>
__global__ __launch_bounds__(NB) void k_rollout_tpe(Params p, int K, int32_t* act_out) {
    constexpr int NW = NB / 64, RS_ROUND = NW * (64 / RO_RW);
    __shared__ float4 oimg[NW][64 * RO_STRIDE];
    __shared__ uint32_t cnt[2][NW];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    float4* wimg = oimg[wv];
    uint32_t* wreg = reinterpret_cast<uint32_t*>(wimg);  // the region as words (list, records)
    float4* mine = wimg + lane * RO_STRIDE;
    const int64_t env0 = (int64_t)blockIdx.x * NB + (threadIdx.x & ~63);
    const int64_t env = env0 + lane;
    const bool live = env < p.B;
    const int64_t ev = live ? env : 0;  // dead lanes step env 0's copy in registers and store nothing
    const int E = p.E;

    TEnv v;
    double lat0[TPE_E];
    uint32_t em[TPE_E], ed[TPE_E];
#pragma unroll
    for (int e = 0; e < TPE_E; ++e) {
        const int64_t i = (int64_t)e * p.B + ev;
        lat0[e] = e < E ? p.lat0[i] : 0.0;
        em[e] = e < E ? p.emeta[i] : 0u;
        ed[e] = e < E ? p.edyn[i] : 0u;
    }
    v.t = p.t[ev];
    v.s = sc_unpack(p.sc[ev]);
    v.zcap = p.zcap[ev];
    v.acc2 = p.acc2[ev];
    v.acc3 = p.acc3[ev];
    v.topo = p.topo[ev];
    v.nz0 = p.nzone[ev];
    v.nz1 = p.NZW > 1 ? p.nzone[p.B + ev] : 0;
    v.sum_lat = p.sum_lat[ev];
    v.sum_cpu = p.sum_cpu[ev];
    v.sum_hi = p.sum_hi[ev];
    v.total = p.total[ev];
    v.last_r = p.reward_fn != LB_REWARD_NAIVE ? p.last_r[ev] : 0.0;
    float olat[TPE_E], ocpu[TPE_E];  // observed endpoint latency / cpu (obs columns 4, 2)
#pragma unroll
    for (int e = 0; e < TPE_E; ++e) {
        olat[e] = e < E ? (float)lat_of(p, lat0[e], ed[e]) : 0.f;
        ocpu[e] = e < E ? (float)cpu_of(p, em[e], ed[e]) : 0.f;
    }
    bool new_episode = false;  // the scenario arrays need writing back
    const int64_t obs_slot = p.B * (int64_t)p.R * 8;
    // episodes at least as long as the launch end at most once per env in it: their next episode is
    // drawn here, before the first step, into the env's record (RS_W lanes per env, every
    // finishing env of the wave in rounds of 8), and the step that ends one only reloads
    // the registers from it -- no barrier and no serial reset chain inside the step loop.
    // Shorter episodes take the in-loop block-list path below.
    constexpr bool pre = PRE;  // (host: auto_reset && L >= K: an env ending at step k ends next at k + L >= K)
    if (pre) {
        const int to_done = p.L - v.s.step;
        const bool fin = live && to_done >= 1 && to_done <= K;  // ends at step to_done - 1 of this launch
        const uint64_t fm = __ballot(fin);
        if (fin) {
            uint32_t* it = wreg + 2 * __popcll(fm & ((1ull << lane) - 1));
            it[0] = (uint32_t)lane;
            it[1] = (uint32_t)(v.acc3 >> 32) + 1;
        }
        wave_lds_sync();
        const int nf = __popcll(fm), g = lane / RS_W, gl = lane % RS_W;
        for (int r0 = 0; r0 < nf; r0 += 64 / RS_W) {
            const int i = r0 + g;
            if (i < nf) tpe_write_record<RS_W>(p, env0 + (int64_t)wreg[2 * i], wreg[2 * i + 1], gl);
        }
        // the records are read back by other lanes of this wave; the list region becomes the
        // first step's obs image
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    }

    // step 0's action and table values; each later step's are issued at the end of the step
    // before it, so their gathers are in flight while that step's rows are stored
    // (PRE only: the in-loop block-list resets hold too many registers for it)
    TPrep pr;
    if constexpr (PRE) {
        pr = tpe_prep(p, lat0, em, ed, tpe_policy<KIND>(p, ev, v, em, ed));
        tpe_prep_request(p, ev, v, pr);
    }
    for (int k = 0; k < K; ++k) {
        if constexpr (!PRE) pr = tpe_prep(p, lat0, em, ed, tpe_policy<KIND>(p, ev, v, em, ed));
        if (act_out && live) act_out[k * p.B + env] = pr.a;
        v.s.step = v.s.step < 0xFFFF ? v.s.step + 1 : 0xFFFF;
        const bool done = live && v.s.step == p.L;  // (:472)
        const bool do_reset = done && p.auto_reset;
        const double reward =
            tpe_apply<false, true, true, true, PRE>(p, pr, ev, env, false, v, lat0, em, ed, olat, ocpu, nullptr);
        if (live) {
            if (p.reward) p.reward[k * p.B + env] = (float)reward;
            if (p.done) p.done[k * p.B + env] = (uint8_t)done;
        }
        const uint64_t m = __ballot(do_reset);
        if (do_reset && p.ep_stats)
            write_stats_row(p, p.ep_stats + env * LB_ST_K, v.s, v.acc2, v.acc3, v.total, v.sum_lat, v.sum_cpu, v.sum_hi);
        float* obs_k = p.obs ? p.obs + k * obs_slot : nullptr;
        if constexpr (PRE) {
            if (p.term_obs && m) {  // the finishing envs' terminal rows first
                if (do_reset) tpe_obs_rows(p, mine, v, em, olat, ocpu);
                wave_lds_sync();
                tpe_copy_rows(p, p.term_obs, wimg, env0, m, COPY_FLAGGED, 0, 64);
                wave_lds_sync();
            }
            if (do_reset) {
                uint4 q[10];  // the next episode's record
                const uint4* rp = p.rec + env * (RO_REC_BYTES / 16);
#pragma unroll
                for (int j = 0; j < 10; ++j) q[j] = rp[j];
                tpe_start_episode(p, q, v, lat0, em, ed, olat, ocpu);
                new_episode = true;
            }
            if (k + 1 < K) {
                pr = tpe_prep(p, lat0, em, ed, tpe_policy<KIND>(p, ev, v, em, ed));
                tpe_prep_request(p, ev, v, pr);
            }
            tpe_obs_rows(p, mine, v, em, olat, ocpu);
            wave_lds_sync();
            if (obs_k) tpe_copy_rows(p, obs_k, wimg, env0, m, COPY_ALL, 0, 64);
            continue;
        }
        tpe_obs_rows(p, mine, v, em, olat, ocpu);
        wave_lds_sync();
        if (p.term_obs && m) tpe_copy_rows(p, p.term_obs, wimg, env0, m, COPY_FLAGGED, 0, 64);
        if (obs_k) tpe_copy_rows(p, obs_k, wimg, env0, m, p.auto_reset ? COPY_UNFLAGGED : COPY_ALL, 0, 64);
        if (!p.auto_reset) continue;  // uniform over the grid
        wave_lds_sync();
        if (do_reset) {  // the wave's list replaces its (copied-out) image
            uint32_t* it = wreg + 1 + RS_LIST_W * __popcll(m & ((1ull << lane) - 1));
            const uint64_t tb = (uint64_t)__double_as_longlong(v.t), sc = sc_pack(v.s);
            it[0] = (uint32_t)env;
            it[1] = (uint32_t)tb; it[2] = (uint32_t)(tb >> 32);
            it[3] = (uint32_t)v.acc3; it[4] = (uint32_t)(v.acc3 >> 32);
            it[5] = (uint32_t)sc; it[6] = (uint32_t)(sc >> 32);
        }
        // per-wave counts, double-buffered by step parity: a wave can be one barrier ahead
        if (lane == 0) cnt[k & 1][wv] = (uint32_t)__popcll(m);
        if (NW > 1) block_lds_sync();
        else wave_lds_sync();
        int pre[NW + 1];
        pre[0] = 0;
#pragma unroll
        for (int w = 0; w < NW; ++w) pre[w + 1] = pre[w] + (int)cnt[k & 1][w];
        const int mine_i = do_reset ? pre[wv] + __popcll(m & ((1ull << lane) - 1)) : -1;
        const int g = lane / RO_RW, gl = lane % RO_RW;
        for (int r0 = 0; r0 < pre[NW]; r0 += RS_ROUND) {  // uniform over the block
            const int i = r0 + wv * (64 / RO_RW) + g;
            if (i < pre[NW]) {
                int q = 0;
#pragma unroll
                for (int w = 1; w < NW; ++w) q += i >= pre[w];
                int base = 0;
#pragma unroll
                for (int w = 1; w < NW; ++w) base = q == w ? pre[w] : base;
                const uint32_t* it = reinterpret_cast<const uint32_t*>(oimg[q]) + 1 + RS_LIST_W * (i - base);
                const int64_t renv = (int64_t)it[0];
                SEnv<1> sv;
                sv.t = __longlong_as_double((long long)((uint64_t)it[1] | ((uint64_t)it[2] << 32)));
                sv.acc3 = (uint64_t)it[3] | ((uint64_t)it[4] << 32);
                sv.s = sc_unpack((uint64_t)it[5] | ((uint64_t)it[6] << 32));
                slice_reset<RO_RW, 1, false, false>(p, renv, gl, sv);
                if (obs_k) slice_write_obs<RO_RW, 1>(p, obs_k, renv, gl, sv);
                // record (i - r0) lives in wave (i - r0) / 8's region, past its list: this group's
                uint32_t* rc = wreg + RO_REC_OFF + g * RS_REC_W;
                if (gl < E) {
                    const uint64_t lb = (uint64_t)__double_as_longlong(sv.lat0[0]);
                    rc[2 * gl] = (uint32_t)lb;
                    rc[2 * gl + 1] = (uint32_t)(lb >> 32);
                    rc[16 + gl] = sv.em[0];
                }
                if (gl == 0) {
                    const uint64_t tb = (uint64_t)__double_as_longlong(sv.t), sc = sc_pack(sv.s);
                    const uint64_t w8[7] = {sv.topo, sv.zcap, sv.nz0, sv.nz1, tb, sv.acc3, sc};
#pragma unroll
                    for (int j = 0; j < 7; ++j) {
                        rc[24 + 2 * j] = (uint32_t)w8[j];
                        rc[25 + 2 * j] = (uint32_t)(w8[j] >> 32);
                    }
                }
            }
            block_lds_sync();
            if (mine_i >= r0 && mine_i < r0 + RS_ROUND) {  // the owner reloads its new episode
                const int j = mine_i - r0;
                const uint32_t* rc =
                    reinterpret_cast<const uint32_t*>(oimg[j / (64 / RO_RW)]) + RO_REC_OFF + (j % (64 / RO_RW)) * RS_REC_W;
                auto u64 = [&](int w) { return (uint64_t)rc[w] | ((uint64_t)rc[w + 1] << 32); };
#pragma unroll
                for (int e = 0; e < TPE_E; ++e) {
                    lat0[e] = e < E ? __longlong_as_double((long long)u64(2 * e)) : 0.0;
                    em[e] = e < E ? rc[16 + e] : 0u;
                    ed[e] = 0u;
                    olat[e] = (float)lat0[e];  // table rows 0: the initial values
                    ocpu[e] = (float)em_c0(em[e]);
                }
                v.topo = u64(24);
                v.zcap = u64(26);
                v.nz0 = u64(28);
                v.nz1 = u64(30);
                v.t = __longlong_as_double((long long)u64(32));
                v.acc3 = u64(34);
                v.s = sc_unpack(u64(36));
                v.acc2 = 0;
                v.sum_lat = 0;
                v.sum_cpu = 0;
                v.sum_hi = 0;
                v.total = 0.0;
                v.last_r = p.init_last_r;
                new_episode = true;
            }
            block_lds_sync();  // the records and lists are free for the next round / step
        }
    }
    if (!live) return;
#pragma unroll
    for (int e = 0; e < TPE_E; ++e) {
        if (e >= E) continue;
        const int64_t i = (int64_t)e * p.B + env;
        p.edyn[i] = ed[e];
        if (new_episode) {
            p.lat0[i] = lat0[e];
            p.emeta[i] = em[e];
        }
    }
    if (new_episode) {
        p.topo[env] = v.topo;
        p.zcap[env] = v.zcap;
        p.nzone[env] = v.nz0;
        if (p.NZW > 1) p.nzone[p.B + env] = v.nz1;
    }
    tpe_store_scalars(p, env, v);
}
}  // namespace lbk
