// lbk8s_slice.h — the "slice" path for E > 8 endpoints (e.g. the 64-endpoint
// deep-sets scenario): one env = one W-lane slice of a wave (W = 16, 32 or 64), a lane
// owns endpoint(s) e = lane + k*W, k < EPL.  Each lane writes its own 32-byte obs rows,
// so a slice's stores cover the env's contiguous R x 32-byte block.  Per-env scalars are
// loaded by every lane (same-address loads coalesce) and stored by lane 0; the three
// Philox blocks of a request are computed by lanes 0/1/2 in one instruction stream.
// Endpoint arrays are [env][EP] (es = 1, ee = EP).
#pragma once

#include "lbk8s_common.h"

namespace lbk {


template <int W>
__device__ __forceinline__ int slice_sum(int v) {
#pragma unroll
    for (int m = W / 2; m >= 1; m >>= 1) v += __shfl_xor(v, m, W);
    return v;
}
template <int W>
__device__ __forceinline__ uint64_t slice_sum64(uint64_t v) {
#pragma unroll
    for (int m = W / 2; m >= 1; m >>= 1) {
        uint32_t lo = __shfl_xor((uint32_t)v, m, W), hi = __shfl_xor((uint32_t)(v >> 32), m, W);
        v += ((uint64_t)hi << 32) | lo;
    }
    return v;
}
template <int W>
__device__ __forceinline__ uint64_t slice_or64(uint64_t v) {
#pragma unroll
    for (int m = W / 2; m >= 1; m >>= 1) {
        uint32_t lo = __shfl_xor((uint32_t)v, m, W), hi = __shfl_xor((uint32_t)(v >> 32), m, W);
        v |= ((uint64_t)hi << 32) | lo;
    }
    return v;
}
template <int W>
__device__ __forceinline__ uint32_t shfl_u32(uint32_t v, int src) { return (uint32_t)__shfl((int)v, src, W); }
template <int W>
__device__ __forceinline__ double shfl_f64(double v, int src) { return __shfl(v, src, W); }

// a[k] for a runtime k, as a chain of selects over constant indices (a runtime-indexed
// private array would be placed in scratch memory)
template <int EPL, int I = EPL - 1, typename T>
__device__ __forceinline__ T sel(const T (&a)[EPL], int k) {
    if constexpr (I == 0) return a[0];
    else return k == I ? a[I] : sel<EPL, I - 1>(a, k);
}

// next_request()'s draws (:1132-1133, :1116, :1120).  Draw map: block (D_REQ_X) ->
// x1 from words (0,1), x2 from (2,3); block (D_REQ_I) -> r from word 0, n from word 1.
// Lanes 0 and 1 compute the X block, lane 2 the I block; lanes 0/1 each take one log.
template <int W, bool TRACE>
__device__ __forceinline__ void slice_request_draws(const Params& p, int64_t env, uint32_t episode,
                                                    uint32_t slot, int lane, bool from_reset, double& x1,
                                                    double& x2, int& r, int& n) {
    if constexpr (TRACE) {
        if (from_reset) {
            x1 = p.tr.reset_x1[env]; x2 = p.tr.reset_x2[env]; r = p.tr.reset_r[env]; n = p.tr.reset_n[env];
        } else {
            x1 = p.tr.step_x1[env]; x2 = p.tr.step_x2[env]; r = p.tr.step_r[env]; n = p.tr.step_n[env];
        }
    } else {
        const int role = lane & 3;
        U4 w = draw(p, env, episode, slot, role == 2 ? D_REQ_I : D_REQ_X);
        double e = role == 1 ? std_exp(w.z, w.w) : std_exp(w.x, w.y);
        x1 = p.inv_rate * shfl_f64<W>(e, 0);
        x2 = p.call * shfl_f64<W>(e, 1);
        r = (int)bounded(shfl_u32<W>(w.x, 2), 7);
        n = (int)bounded(shfl_u32<W>(w.y, 2), (uint32_t)p.N);
    }
}

// Register image of one env slice.
template <int EPL>
struct SEnv {
    double lat0[EPL];
    uint32_t em[EPL], ed[EPL];
    float olat[EPL], ocpu[EPL];  // observed endpoint latency / cpu (float32 obs columns 4, 2)
    double t, dt, total, last_r;
    uint64_t sum_lat, sum_cpu;  // exact fixed-point episode sums (xsum_add)
    uint32_t sum_hi;
    uint64_t topo, zcap, acc2, acc3;
    uint64_t nz0, nz1;  // node-zone words 0 and 1 (nodes < 64), prefetched with the state
    Scal s;
};

// get_state() (:688-758): rows [zone, zone_cpu_cap, cpu, topo_lat, lat, req_zone, thr, dt]
// The env's R x 32-byte block is written as contiguous runs: store c covers float4s
// cW .. cW + W - 1 of the block (rows cW/2 .. cW/2 + W/2 - 1), lane l the float4 2r + h of
// row r = cW/2 + (l >> 1), h = l & 1.  Row r < E is endpoint r, held by lane r % W in
// slot r / W = c >> 1, so each lane's halves come from lane (c & 1) W/2 + (l >> 1) by a
// lane shuffle; the reject row (r = E) is the same on every lane.
// (put(q, o): float4 q of the env's block; slice_write_obs streams it to out, lb_dqn_steps
// keeps it in LDS)
template <int W, int EPL, typename Put>
__device__ __forceinline__ void slice_obs_rows(const Params& p, int lane, const SEnv<EPL>& v, Put&& put) {
    const float rz = (float)v.s.rz, thr = (float)threshold(v.s.thr_idx), dt = (float)v.dt;
    const int n4 = 2 * p.R, h = lane & 1;
#pragma unroll
    for (int k = 0; k <= EPL; ++k) {
        // this lane's endpoint of slot k (garbage-free zeros past the valid range)
        float4 a = make_float4(0.f, 0.f, 0.f, 0.f), b = a;
        if (k < EPL) {
            const int z = em_zone(v.em[k]);
            a = make_float4((float)z, (float)zcap_val(v.zcap, z), v.ocpu[k], (float)topo_val(v.topo, z, v.s.rz));
            b = make_float4(v.olat[k], rz, thr, dt);
        }
#pragma unroll
        for (int c = 2 * k; c < 2 * k + 2; ++c) {
            if (c * W >= n4) continue;           // uniform over the env's lanes
            const int q = c * W + lane;          // float4 index inside the env's block
            const int r = q >> 1;                // row
            // shuffles with every lane of the slice active (a source lane must not be masked)
            const int src = (c & 1) * (W / 2) + (lane >> 1);
            const float4 sa = make_float4(__shfl(a.x, src, W), __shfl(a.y, src, W), __shfl(a.z, src, W),
                                          __shfl(a.w, src, W));
            const float4 sb = make_float4(__shfl(b.x, src, W), __shfl(b.y, src, W), __shfl(b.z, src, W),
                                          __shfl(b.w, src, W));
            // rows past E: the reject row (r == E, present iff R > E); later rows are past R
            const float4 o = (r < p.E && k < EPL) ? (h ? sb : sa)
                                                  : (h ? make_float4(-1.f, rz, thr, dt) : make_float4(-1.f, -1.f, -1.f, -1.f));
            if (q < n4) put(q, o);
        }
    }
}
template <int W, int EPL>
__device__ __forceinline__ void slice_write_obs(const Params& p, float* out, int64_t env, int lane,
                                                const SEnv<EPL>& v) {
    float4* base = reinterpret_cast<float4*>(out + env * (int64_t)p.R * 8);
    slice_obs_rows<W, EPL>(p, lane, v, [&](int q, float4 o) { st_stream(base + q, o); });
}

// get_state() for the 4 envs of a wave (W = 16) as ONE contiguous run: the envs' R x 32-byte
// blocks are consecutive, so the wave's 4 blocks are 128·R bytes starting at a multiple of
// 128·R (envs 4w .. 4w + 3): every store instruction covers whole 128-byte lines.  Per-env
// runs started mid-line (R x 32 B = 2,080 B at E = 64), and the nontemporal stores reached
// HBM as partial lines.  The rows go through a per-wave LDS image (wave-local: LDS
// instructions of one wave complete in order).  Only for full waves (env0 + 4 <= B).
template <int EPL>
__device__ __forceinline__ void slice_write_obs_wave(const Params& p, float* out, int64_t env0, int wl,
                                                     const SEnv<EPL>& v, float4* st) {
    constexpr int W = 16;
    const int el = wl / W, lane = wl % W, n4 = 2 * p.R;
    const float rz = (float)v.s.rz, thr = (float)threshold(v.s.thr_idx), dt = (float)v.dt;
    float4* mine = st + el * n4;
#pragma unroll
    for (int k = 0; k < EPL; ++k) {
        const int r = lane + k * W;
        if (r < p.E) {
            const int z = em_zone(v.em[k]);
            mine[2 * r] = make_float4((float)z, (float)zcap_val(v.zcap, z), v.ocpu[k], (float)topo_val(v.topo, z, v.s.rz));
            mine[2 * r + 1] = make_float4(v.olat[k], rz, thr, dt);
        }
    }
    if (lane == 0 && p.R > p.E) {  // the reject row
        mine[2 * p.E] = make_float4(-1.f, -1.f, -1.f, -1.f);
        mine[2 * p.E + 1] = make_float4(-1.f, rz, thr, dt);
    }
    float4* base = reinterpret_cast<float4*>(out + env0 * (int64_t)p.R * 8);
    for (int f = wl; f < 4 * n4; f += 64) st_stream(base + f, st[f]);
}

template <int W, int EPL>
__device__ __forceinline__ void slice_load(const Params& p, int64_t env, int lane, SEnv<EPL>& v) {
#pragma unroll
    for (int k = 0; k < EPL; ++k) {
        int64_t i = eidx(p, env, lane + k * W);
        v.lat0[k] = p.lat0[i];
        v.em[k] = p.emeta[i];
        v.ed[k] = p.edyn[i];
    }
    v.t = p.t[env];
    v.s = sc_unpack(p.sc[env]);
    v.zcap = p.zcap[env];
    v.acc2 = p.acc2[env];
    v.acc3 = p.acc3[env];
    v.topo = p.topo[env];
    v.nz0 = p.nzone[env];
    v.nz1 = p.NZW > 1 ? p.nzone[p.B + env] : 0;
    v.sum_lat = p.sum_lat[env];
    v.sum_cpu = p.sum_cpu[env];
    v.sum_hi = p.sum_hi[env];
    v.total = p.total[env];
    v.last_r = p.reward_fn != LB_REWARD_NAIVE ? p.last_r[env] : 0.0;
}

template <int EPL>
__device__ __forceinline__ void slice_store_scalars(const Params& p, int64_t env, const SEnv<EPL>& v) {
    p.t[env] = v.t;
    p.sc[env] = sc_pack(v.s);
    p.acc2[env] = v.acc2;
    p.acc3[env] = v.acc3;
    p.sum_lat[env] = v.sum_lat;
    p.sum_cpu[env] = v.sum_cpu;
    p.sum_hi[env] = v.sum_hi;
    p.total[env] = v.total;
    if (p.reward_fn != LB_REWARD_NAIVE) p.last_r[env] = v.last_r;
}

// the request part of next_request() (:1131-1163); the dequeue part is folded into the LUTs
template <int W, bool TRACE, int EPL>
__device__ __forceinline__ void slice_next_request(const Params& p, int64_t env, int lane, bool from_reset,
                                                   SEnv<EPL>& v) {
    double x1, x2;
    int r, n;
    slice_request_draws<W, TRACE>(p, env, (uint32_t)(v.acc3 >> 32), (uint32_t)v.s.step, lane, from_reset,
                                  x1, x2, r, n);
    double arrival = v.t + x1;
    double departure = arrival + x2;
    v.dt = departure - arrival;
    v.t = arrival;
    v.s.thr_idx = (r + 6) % 7;  // endpoint_list[r - 1] (:1117)
    const uint64_t word = n < 32 ? v.nz0 : (n < 64 ? v.nz1 : p.nzone[(n >> 5) * p.B + env]);
    v.s.rz = (int)((word >> (2 * (n & 31))) & 3);
}

// reset() (:290-400) into registers, then the per-episode state stores (STORE = false: a
// multi-step kernel that keeps the env in registers writes it back itself).
template <int W, int EPL, bool TRACE, bool STORE = true>
__device__ __forceinline__ void slice_reset(const Params& p, int64_t env, int lane, SEnv<EPL>& v) {
    const uint32_t episode = (uint32_t)(v.acc3 >> 32) + 1;
    // nodes (:349-373): zone capacity and the 2-bit zone of every node, one 32-node word
    // at a time (lane l takes nodes l, l+W, ... of the word)
    uint64_t zc = 0;
    for (int w = 0; w < p.NZW; ++w) {
        uint64_t word = 0;
        for (int n = 32 * w + lane; n < 32 * (w + 1) && n < p.N; n += W) {
            int ty, zo, cpu;
            node_draw<TRACE>(p, env, episode, n, ty, zo, cpu);
            zc += (uint64_t)node_cpu_int(ty) << (16 * zo);
            word |= (uint64_t)zo << (2 * (n & 31));
        }
        word = slice_or64<W>(word);
        if (w == 0) v.nz0 = word;
        if (w == 1) v.nz1 = word;
        if (STORE && lane == 0) p.nzone[w * p.B + env] = word;
    }
    if (p.NZW < 2) v.nz1 = 0;
    zc = slice_sum64<W>(zc);
    // endpoints (:328, :379-386)
    int node[EPL];
#pragma unroll
    for (int k = 0; k < EPL; ++k) {
        int e = lane + k * W;
        node[k] = 0;
        v.lat0[k] = 0.0;
        if (e < p.E) {
            if constexpr (TRACE) {
                v.lat0[k] = p.tr.reset_lat0[env * p.E + e];
                node[k] = p.tr.reset_enode[env * p.E + e];
            } else {
                U4 w = draw(p, env, episode, (uint32_t)e, D_EP);
                v.lat0[k] = 1.0 + 99.0 * u53(w.x, w.y);
                node[k] = (int)bounded(w.z, 24);
            }
        }
    }
    // owner slot = first endpoint hosted on the same node (shares that node's CPU)
    int owner[EPL];
#pragma unroll
    for (int k = 0; k < EPL; ++k) owner[k] = lane + k * W;
    for (int e2 = 0; e2 < p.E; ++e2) {
        int nd2 = shfl_u32<W>((uint32_t)sel<EPL>(node, e2 / W), e2 % W);
#pragma unroll
        for (int k = 0; k < EPL; ++k)
            if (nd2 == node[k] && e2 < owner[k]) owner[k] = e2;
    }
#pragma unroll
    for (int k = 0; k < EPL; ++k) {
        int e = lane + k * W;
        v.em[k] = 0;
        v.ed[k] = 0;
        v.olat[k] = 0.f;
        v.ocpu[k] = 0.f;
        if (e < p.E) {
            int ty, zo, cpu;
            node_draw<TRACE>(p, env, episode, node[k], ty, zo, cpu);
            v.em[k] = em_pack(zo, owner[k], ty, cpu, node[k]);
            v.olat[k] = (float)v.lat0[k];
            v.ocpu[k] = (float)cpu;
        }
        if (STORE && e < p.EP) {  // (the thread-per-env layout has no padding slots: EP = E)
            const int64_t i = eidx(p, env, e);
            p.lat0[i] = v.lat0[k];
            p.emeta[i] = v.em[k];
            p.edyn[i] = 0;
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
    slice_next_request<W, TRACE, EPL>(p, env, lane, true, v);
    if (STORE && lane == 0) {
        p.topo[env] = topo;
        p.zcap[env] = zc;
    }
}

template <int W, int EPL, bool TRACE>
__global__ __launch_bounds__(BLOCK) void k_reset_slice(Params p) {
    const int lane = threadIdx.x % W;
    const int64_t env = (int64_t)blockIdx.x * (BLOCK / W) + threadIdx.x / W;
    if (env >= p.B) return;
    if (p.reset_mask && !p.reset_mask[env]) return;
    SEnv<EPL> v;
    v.t = p.t[env];
    v.acc3 = p.acc3[env];
    v.s = sc_unpack(p.sc[env]);
    slice_reset<W, EPL, TRACE>(p, env, lane, v);
    if (p.obs) slice_write_obs<W, EPL>(p, p.obs, env, lane, v);
    if (lane == 0) slice_store_scalars<EPL>(p, env, v);
}

// lanes per env of the thread-per-env step's auto-reset (k_step_tpe, lbk8s_tpe.h)
constexpr int RS_W = 8;

// One step() (:403-513) of the slice's env held in registers, in three parts:
//   slice_prep   the action decoded and the selected endpoint's 4 table values gathered
//                (issued, not waited for);
//   slice_apply  take_action, reward, next_request(), done and the VecEnv auto-reset
//                (terminal obs, episode stats, reset()), on the registers;
//   slice_obs    get_state() of the step's result.
// The single-step kernel runs them in order; the rollout issues step k + 1's gathers before
// step k's obs / reward / done stores, which they would otherwise wait behind (s_waitcnt
// vmcnt retires a wave's memory operations in issue order, stores included).
struct SPrep {
    int a, ai, oA, jA, Mn, jn;
    uint32_t emA;
    double lat0A, lut_selA, sel_cpu, next_lat, next_cpu;
};
template <int W, int EPL>
__device__ __forceinline__ SPrep slice_prep(const Params& p, const SEnv<EPL>& v, int a) {
    const int E = p.E;
    SPrep r;
    r.a = a;
    const bool accept = a >= -E && a < E;
    r.ai = accept ? (a < 0 ? a + E : a) : 0;
    const int src = r.ai % W, sk = r.ai / W;
    r.emA = shfl_u32<W>(sel<EPL>(v.em, sk), src);
    const uint32_t edA = shfl_u32<W>(sel<EPL>(v.ed, sk), src);
    r.lat0A = shfl_f64<W>(sel<EPL>(v.lat0, sk), src);
    r.oA = em_owner(r.emA);
    const uint32_t edO = shfl_u32<W>(sel<EPL>(v.ed, r.oA / W), r.oA % W);
    r.jA = ed_j(edA);
    r.Mn = ed_M(edO) < CMAX ? ed_M(edO) + 1 : CMAX;
    r.jn = r.jA < CMAX ? r.jA + 1 : CMAX;
    const int k0A = (int)r.lat0A, c0A = em_c0(r.emA);
    // selected endpoint before (selected_*) and after (inc+dec) this step's update
    r.lut_selA = p.lat_lut[(r.jA) * LAT_ROWS + k0A];
    r.sel_cpu = p.cpu_lut[(ed_m(edA)) * CPU_ROWS + c0A];
    r.next_lat = p.lat_lut[(r.jn) * LAT_ROWS + k0A];
    r.next_cpu = p.cpu_lut[(r.Mn) * CPU_ROWS + c0A];
    return r;
}
// the observed values of every endpoint from the history counters (table rows 0 are the
// initial values: only endpoints selected this episode (j > 0) / refreshed (m > 0) gather)
template <int EPL>
__device__ __forceinline__ void slice_observe(const Params& p, SEnv<EPL>& v) {
#pragma unroll
    for (int k = 0; k < EPL; ++k) {
        const int j = ed_j(v.ed[k]), m = ed_m(v.ed[k]);
        double l = v.lat0[k], c = (double)em_c0(v.em[k]);
        if (j) l = p.lat_lut[j * LAT_ROWS + (int)v.lat0[k]];
        if (m) c = p.cpu_lut[m * CPU_ROWS + em_c0(v.em[k])];
        v.olat[k] = (float)l;
        v.ocpu[k] = (float)c;
    }
}
// take_action (:578-686), reward, next_request (:1131-1163), done (:472) and the auto-reset;
// returns the reward, done in `done`.  STORE_ED: write the changed history counters back at
// once (the single-step kernel; a multi-step kernel keeps them in registers).
template <int W, int EPL, bool TRACE, bool STORE_ED>
__device__ __forceinline__ double slice_apply(const Params& p, int64_t env, int lane, SEnv<EPL>& v, const SPrep& pr,
                                              bool& done) {
    const int E = p.E, a = pr.a, ai = pr.ai, oA = pr.oA, jA = pr.jA, Mn = pr.Mn, jn = pr.jn;
    v.s.step = v.s.step < 0xFFFF ? v.s.step + 1 : 0xFFFF;
    const bool accept = a >= -E && a < E;
    const bool reject = a == E;
    if (a < -E) v.s.bad = 1;  // reference: IndexError; here: treated as unrecognised
    if (!v.s.reset_done) v.s.bad = 1;
    double reward;
    if (accept) {
        const int zA = em_zone(pr.emA);
        const double sel_lat = jA == 0 ? pr.lat0A : pr.lut_selA;
        const int tl = topo_val(v.topo, v.s.rz, zA);
        // O(E) Gini numerator update for avg_load_served[ai] += 1 (:631)
        int cnt = 0;
#pragma unroll
        for (int k = 0; k < EPL; ++k) {
            int e = lane + k * W;
            if (e < E && e != ai && ed_j(v.ed[k]) <= jA) ++cnt;
        }
        cnt = slice_sum<W>(cnt);
        uint32_t gnum = (uint32_t)(v.acc2 >> 32) + (uint32_t)(2 * (2 * cnt - (E - 1)));
        uint32_t sum_topo = (uint32_t)v.acc2 + (uint32_t)tl;
        v.acc2 = ((uint64_t)gnum << 32) | sum_topo;
        v.acc3 += (uint64_t)node_cost(em_type(pr.emA));
        v.s.acc = v.s.acc < 0xFFFF ? v.s.acc + 1 : 0xFFFF;
        if (v.s.rz == zA) v.s.intra = v.s.intra < 0xFFFF ? v.s.intra + 1 : 0xFFFF;
        xsum_add(v.sum_lat, v.sum_cpu, v.sum_hi, sel_lat, pr.sel_cpu, tl, v.s.rz != zA);
        // increase_resources / increase_endpoint_latency (:674-677) and the same step's
        // decrease in next_request() (:1137-1143) -> the history counters advance
#pragma unroll
        for (int k = 0; k < EPL; ++k) {
            int e = lane + k * W;
            // unconditional select-stores: a conditional store per k lets the compiler
            // fold them into one runtime-indexed store (and move the arrays to LDS)
            const uint32_t edo = e == oA ? (v.ed[k] & ~(0x3FFu << 20)) | ((uint32_t)Mn << 20) : v.ed[k];
            const bool hit = e == ai;
            v.ed[k] = hit ? (edo & (0x3FFu << 20)) | ((uint32_t)Mn << 10) | (uint32_t)jn : edo;
            v.olat[k] = hit ? (float)pr.next_lat : v.olat[k];
            v.ocpu[k] = hit ? (float)pr.next_cpu : v.ocpu[k];
        }
        v.s.penalty = 0;
        reward = accept_reward(p, sel_lat, tl, pr.sel_cpu, v.acc2, v.s.acc);
        v.last_r = reward;
    } else if (reject) {
        v.s.penalty = 1;
        reward = p.reward_fn == LB_REWARD_LATENCY ? -1000.0 : -1.0;
        v.last_r = reward;
    } else {  // unrecognised action (:685-686): penalty and selected_* stay stale
        reward = p.reward_fn == LB_REWARD_NAIVE ? (v.s.penalty ? -1.0 : 1.0) : v.last_r;
    }
    v.total += reward;

    // ---- next_request (:1131-1163), done (:472), auto-reset
    slice_next_request<W, TRACE, EPL>(p, env, lane, false, v);
    done = v.s.step == p.L;
    if (done && p.auto_reset) {
        if (p.term_obs) slice_write_obs<W, EPL>(p, p.term_obs, env, lane, v);
        if (p.ep_stats && lane == 0)
            write_stats_row(p, p.ep_stats + env * LB_ST_K, v.s, v.acc2, v.acc3, v.total, v.sum_lat, v.sum_cpu, v.sum_hi);
        slice_reset<W, EPL, TRACE>(p, env, lane, v);
    } else if (STORE_ED && accept) {
#pragma unroll
        for (int k = 0; k < EPL; ++k) {
            int e = lane + k * W;
            if (e == ai || e == oA) p.edyn[eidx(p, env, e)] = v.ed[k];
        }
    }
    return reward;
}
// get_state() of the step's result: the wave's 4 envs as whole lines through LDS (W = 16), or
// per env
// NWB: waves per block (the LDS stage has one region per wave); 0: not every slice of the
// wave steps a live env of the caller's (per-env stores)
template <int W, int EPL, int NWB = BLOCK / 64>
__device__ __forceinline__ void slice_obs(const Params& p, int64_t env, int lane, const SEnv<EPL>& v, float* obs_out) {
    if constexpr (W == 16 && NWB > 0) {
        // whole-line stores of the wave's 4 envs when all 4 are live
        __shared__ float4 obs_stage[NWB][8 * (16 * EPL + 1)];
        const int wl = threadIdx.x & 63;
        const int64_t env0 = env - wl / W;
        if (env0 + 4 <= p.B) {
            slice_write_obs_wave<EPL>(p, obs_out, env0, wl, v, obs_stage[threadIdx.x >> 6]);
            return;
        }
    }
    slice_write_obs<W, EPL>(p, obs_out, env, lane, v);
}

// one step() (:403-513) of the slice's env held in registers (the single-step kernel's order):
// obs / reward / done of this step out (NULL = skip)
template <int W, int EPL, bool TRACE, bool STORE_ED, int NWB = BLOCK / 64>
__device__ __forceinline__ void slice_step_body(const Params& p, int64_t env, int lane, SEnv<EPL>& v, int a,
                                                float* obs_out, float* reward_out, uint8_t* done_out,
                                                double* rew64_out) {
    const SPrep pr = slice_prep<W, EPL>(p, v, a);
    slice_observe<EPL>(p, v);
    bool done;
    const double reward = slice_apply<W, EPL, TRACE, STORE_ED>(p, env, lane, v, pr, done);
    if (lane == 0) {
        if (reward_out) reward_out[env] = (float)reward;
        if (rew64_out) rew64_out[env] = reward;
        if (done_out) done_out[env] = (uint8_t)done;
    }
    if (obs_out) slice_obs<W, EPL, NWB>(p, env, lane, v, obs_out);
}

// step() (:403-513) fused with next_request(), get_state(), reward, done and auto-reset.
template <int W, int EPL, bool TRACE>
__global__ __launch_bounds__(BLOCK) void k_step_slice(Params p) {
    const int lane = threadIdx.x % W;
    const int64_t env = (int64_t)blockIdx.x * (BLOCK / W) + threadIdx.x / W;
    if (env >= p.B) return;
    SEnv<EPL> v;
    slice_load<W, EPL>(p, env, lane, v);
    const int a = p.actions ? p.actions[env] : random_action(p, env, v.acc3, v.s.step);  // fused random policy
    slice_step_body<W, EPL, TRACE, true>(p, env, lane, v, a, p.obs, p.reward, p.done, p.rew64);
    if (lane == 0) slice_store_scalars<EPL>(p, env, v);
}

// envs/baselines.py (:6-35) on the slice's registers: argmin topology latency / argmax
// zone cpu capacity / argmin endpoint cpu over feasible = mask[:-1] (masks are all True,
// :808-821, so the endpoints e < A - 1), first index on ties; or the uniform random action.
// Same values as k_policy / lb_policy.
template <int W, int EPL>
__device__ __forceinline__ int slice_policy(const Params& p, int64_t env, int lane, const SEnv<EPL>& v, int kind) {
    if (kind == LB_POLICY_RANDOM) return random_action(p, env, v.acc3, v.s.step);
    const int nf = p.A - 1;
    if (nf <= 0) return p.A - 1;
    double best = 0.0;
    int bi = 1 << 30;
#pragma unroll
    for (int k = 0; k < EPL; ++k) {
        const int e = lane + k * W;
        if (e >= nf) continue;
        const int z = em_zone(v.em[k]);
        double val;
        if (kind == LB_POLICY_TOPOLOGY_GREEDY) val = (double)topo_val(v.topo, z, v.s.rz);
        else if (kind == LB_POLICY_ZONE_CPU_GREEDY) val = -(double)zcap_val(v.zcap, z);
        else val = p.cpu_lut[ed_m(v.ed[k]) * CPU_ROWS + em_c0(v.em[k])];
        if (bi == (1 << 30) || val < best) { best = val; bi = e; }
    }
#pragma unroll
    for (int m = W / 2; m >= 1; m >>= 1) {  // (value, index) minimum over the slice, lower index on ties
        const double ob = __shfl_xor(best, m, W);
        const int oi = __shfl_xor(bi, m, W);
        const bool take = oi != (1 << 30) && (bi == (1 << 30) || ob < best || (ob == best && oi < bi));
        best = take ? ob : best;
        bi = take ? oi : bi;
    }
    return bi;
}

// lb_rollout: K steps per launch under an on-device policy, the env state held in
// registers between steps; step k's obs / reward / done go to slot k of the caller's
// buffers.  Bit for bit K x (lb_policy + lb_step) (tests/test_gpu_api.py).
// ET / RT / NZWT / RF > 0 (>= 0 for RF): the shape is a compile-time constant (config 4's E = 64,
// R = 65, N <= 32, multi reward): a local copy of the parameters with those fields fixed lets
// every loop over the endpoints, rows and node words unroll and the reward's other kinds fold
// away, which took the per-step uniform values the compiler kept in (spilled) SGPRs down.
template <int W, int EPL, int ET = 0, int RT = 0, int NZWT = 0, int RF = -1>
__global__ __launch_bounds__(BLOCK) void k_rollout_slice(Params pa, int kind, int K, int32_t* act_out) {
    Params p = pa;
    if (ET > 0) p.E = ET;
    if (RT > 0) p.R = RT;
    if (NZWT > 0) p.NZW = NZWT;
    if (RF >= 0) p.reward_fn = RF;
    const int lane = threadIdx.x % W;
    const int64_t env = (int64_t)blockIdx.x * (BLOCK / W) + threadIdx.x / W;
    if (env >= p.B) return;
    SEnv<EPL> v;
    slice_load<W, EPL>(p, env, lane, v);
    // the observed values live in registers for the whole launch: a step changes only the
    // selected endpoint's (slice_apply), a reset sets them all (slice_reset)
    slice_observe<EPL>(p, v);
    const int64_t obs_slot = p.B * (int64_t)p.R * 8;
    int a = slice_policy<W, EPL>(p, env, lane, v, kind);
    SPrep pr = slice_prep<W, EPL>(p, v, a);
    for (int k = 0; k < K; ++k) {
        bool done;
        const double reward = slice_apply<W, EPL, false, false>(p, env, lane, v, pr, done);
        const int ak = a;
        if (k + 1 < K) {  // step k + 1's gathers, issued before step k's stores
            a = slice_policy<W, EPL>(p, env, lane, v, kind);
            pr = slice_prep<W, EPL>(p, v, a);
        }
        if (lane == 0) {
            if (act_out) act_out[k * p.B + env] = ak;
            if (p.reward) p.reward[k * p.B + env] = (float)reward;
            if (p.done) p.done[k * p.B + env] = (uint8_t)done;
        }
        if (p.obs) slice_obs<W, EPL>(p, env, lane, v, p.obs + k * obs_slot);
    }
#pragma unroll
    for (int k = 0; k < EPL; ++k) {
        const int e = lane + k * W;
        if (e < p.E) p.edyn[eidx(p, env, e)] = v.ed[k];
    }
    if (lane == 0) slice_store_scalars<EPL>(p, env, v);
}

}  // namespace lbk
