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
    double t, dt, sum_lat, sum_cpu, total, last_r;
    uint64_t topo, zcap, acc2, acc3, nz0, nz1;
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
    v.sum_lat = 0.0;
    v.sum_cpu = 0.0;
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

// The LDS image and the copy-out are wave-local: a wave orders its own LDS accesses, so it
// needs no block barrier (which would also wait for every global store the wave has in
// flight); the compiler is kept from moving LDS accesses across the point.
__device__ __forceinline__ void wave_lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
// LDS-only block barrier: the waves' global stores stay in flight.
__device__ __forceinline__ void block_lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

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
template <bool TRACE, bool RECOMPUTE, int NB = BLOCK>
__global__ __launch_bounds__(NB) void k_step_tpe(Params p) {
    __shared__ uint32_t lds[NB * TPE_CW];
    const int lane = threadIdx.x & 63;
    uint32_t* img = lds + (threadIdx.x & ~63) * TPE_CW;
    uint32_t* me = img + lane * TPE_CW;
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
    v.total = *(p.total + ev);
    v.last_r = p.reward_fn != LB_REWARD_NAIVE ? *(p.last_r + ev) : 0.0;

    // ---- phase 1: decode the action, pick the selected endpoint, table lookups
    v.s.step = v.s.step < 0xFFFF ? v.s.step + 1 : 0xFFFF;
    const bool done = live && v.s.step == p.L;  // (:472)
    const bool do_reset = done && p.auto_reset;
    const bool keep = live && !do_reset;  // the state stores reset() below does not redo
    const bool accept = a >= -E && a < E;
    const bool reject = a == E;
    if (a < -E) v.s.bad = 1;  // reference: IndexError; here: treated as unrecognised
    if (!v.s.reset_done) v.s.bad = 1;
    const int ai = accept ? (a < 0 ? a + E : a) : 0;
    uint32_t emA = em[0], edA = ed[0];
    double lat0A = lat0[0];
#pragma unroll
    for (int e = 1; e < TPE_E; ++e)
        if (ai == e) { emA = em[e]; edA = ed[e]; lat0A = lat0[e]; }
    const int oA = em_owner(emA);
    uint32_t edO = ed[0];
#pragma unroll
    for (int e = 1; e < TPE_E; ++e)
        if (oA == e) edO = ed[e];
    const int jA = ed_j(edA);
    const int Mn = ed_M(edO) < CMAX ? ed_M(edO) + 1 : CMAX;
    const int jn = jA < CMAX ? jA + 1 : CMAX;
    const int k0A = (int)lat0A, c0A = em_c0(emA);
    const double lut_selA = p.lat_lut[(jA) * LAT_ROWS + k0A];
    const double sel_cpu = p.cpu_lut[(ed_m(edA)) * CPU_ROWS + c0A];
    const double next_lat = p.lat_lut[(jn) * LAT_ROWS + k0A];
    const double next_cpu = p.cpu_lut[(Mn) * CPU_ROWS + c0A];
    int cnt = 0;  // #{e != ai : loads[e] <= loads[ai]} for the O(E) Gini update
#pragma unroll
    for (int e = 0; e < TPE_E; ++e) {
        if (e < E) {
            const int j = ed_j(ed[e]);
            // table rows 0 are the initial values: only endpoints selected (j > 0) /
            // refreshed (m > 0) this episode gather from the LUTs
            const int m = ed_m(ed[e]);
            double l = lat0[e], c = (double)em_c0(em[e]);
            if (j) l = p.lat_lut[j * LAT_ROWS + (int)lat0[e]];
            if (m) c = p.cpu_lut[m * CPU_ROWS + em_c0(em[e])];
            float ol = (float)l;
            float oc = (float)c;
            if (accept && e == ai) { ol = (float)next_lat; oc = (float)next_cpu; }
            const int z = em_zone(em[e]);
            me[4 + 3 * e] = (uint32_t)z | ((uint32_t)zcap_val(v.zcap, z) << 2);
            me[5 + 3 * e] = __float_as_uint(oc);
            me[6 + 3 * e] = __float_as_uint(ol);
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
        v.sum_lat += sel_lat;
        v.sum_cpu += sel_cpu;
        // increase_resources / increase_endpoint_latency (:674-677) and the same step's
        // decrease in next_request() (:1137-1143) -> the history counters advance
        const uint32_t edA_new = ((oA == ai ? (uint32_t)Mn : (uint32_t)ed_M(edA)) << 20) |
                                 ((uint32_t)Mn << 10) | (uint32_t)jn;
        if (keep) {
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
        tpe_request_draws<TRACE>(p, ev, (uint32_t)(v.acc3 >> 32), (uint32_t)v.s.step, false, x1, x2, r, n);
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
    if (live) {
        if (p.reward) *(p.reward + env) = ((float)reward);
        if (p.done) p.done[env] = (uint8_t)done;
    }
    tpe_image_env(me, v, do_reset ? TPE_FLAG : 0);

    // ---- VecEnv auto-reset: terminal obs + episode stats, then reset() below
    const uint64_t m = __ballot(do_reset);
    if (do_reset && p.ep_stats)
        write_stats_row(p, p.ep_stats + env * LB_ST_K, v.s, v.acc2, v.acc3, v.total, v.sum_lat, v.sum_cpu);
    if (keep) tpe_store_scalars(p, env, v);
    wave_lds_sync();
    if (p.term_obs && m) tpe_copy_out(p, p.term_obs, img, env0, COPY_FLAGGED);
    // finished envs' post-reset obs come from their reset()
    if (p.obs) tpe_copy_out(p, p.obs, img, env0, p.auto_reset ? COPY_UNFLAGGED : COPY_ALL);
    if (p.auto_reset) {  // uniform over the grid: every wave reaches the barrier
        constexpr int NW = NB / 64;
        wave_lds_sync();
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
        for (int w = 0; w < NW; ++w) pre[w + 1] = pre[w] + (int)lds[w * 64 * TPE_CW];
        const int wv = threadIdx.x >> 6, g = lane / RS_W, gl = lane % RS_W;
        for (int i = wv * (64 / RS_W) + g; i < pre[NW]; i += NW * (64 / RS_W)) {
            int q = 0;
#pragma unroll
            for (int w = 1; w < NW; ++w) q += i >= pre[w];
            int base = 0;
#pragma unroll
            for (int w = 1; w < NW; ++w) base = q == w ? pre[w] : base;
            const uint32_t* it = lds + q * 64 * TPE_CW + 1 + RS_LIST_W * (i - base);
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

}  // namespace lbk
