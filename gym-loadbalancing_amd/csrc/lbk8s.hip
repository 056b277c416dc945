// lbk8s.hip — MI355X (gfx950) kernels + C ABI for the vectorized LoadBalancerK8sEnv.
//
// Reference hot path: /root/reference/envs/loadbalancer_k8s_env.py (reset :290-400,
// step :403-513, take_action :578-686, get_reward :516-567, get_state :688-758,
// next_request :1131-1163) and envs/utils.py (gini :132-143, endpoint list :33-64).
// Design notes: DESIGN.md.  Public ABI: include/lbk8s.h.
//
// Mapping: one env = one W-lane slice of a wave (W = pow2 >= E, <= 64); a lane owns
// endpoint(s) e = lane + k*W, k < EPL.  Per-env scalars are read by every lane of the
// slice (same-address loads coalesce) and written by lane 0.
//
// State representation (the "history-count" form).  Because an accepted
// request is enqueued and dequeued inside the SAME step (its departure_time is never
// set), every accept applies inc-then-dec to one endpoint latency and one
// node CPU.  Hence
//   endpoint_latency[e] = lat0[e]                 if e was never selected this episode
//                       = LAT[trunc(lat0[e])][j]  after j selections,
//   node_cpu[h]         = CPU[c0(h)][M_h]         after M_h selections of endpoints on h,
//   endpoint_cpu[e]     = CPU[c0(h)][m_e]         m_e = M_h at e's last refresh,
// with LAT / CPU float64 tables built once by the same IEEE operations the reference
// applies (k_luts).  avg_load_served[e] == j_e.  The hot state is therefore lat0 (f64,
// read-only within an episode) plus two 32-bit words per endpoint; only one of them is
// written per step.  Compile with -ffp-contract=off: the reference's float64 math is
// plain IEEE mul/div/add and FMA contraction would change results.

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>

#include "lbk8s.h"

namespace {

constexpr int BLOCK = 256;
constexpr int JCAP = 1024;        // LUT columns; per-episode counters saturate at 1023
constexpr int CMAX = JCAP - 1;
constexpr int LAT_ROWS = 501;     // trunc(initial latency) in [0, 500]
constexpr int CPU_ROWS = 128;     // initial node cpu in [0, 127]
constexpr int NZW_MAX = 8;        // node-zone words of 32 nodes -> num_nodes <= 256
constexpr int EMAX = 256;

// Philox domains — the framework's draw map; mirrored by the oracle.
enum : uint32_t { D_INIT = 1, D_NODE = 2, D_EP = 3, D_TOPO = 4, D_REQ_X = 5, D_REQ_I = 6,
                  D_ACT = 7, D_REQ_X2 = 8 };

// ---- bit layouts -------------------------------------------------------------------
// emeta (static per episode): zone[0:2) owner[2:10) type[10:13) c0[13:20) node[20:28)
// edyn  (per step):           j[0:10)   m[10:20)    M[20:30)
// sc    (u64): step[0:16) acc[16:32) intra[32:48) req_zone[48:50) thr_idx[50:53)
//              penalty[53] reset_done[54] bad_action[55]
// acc2  (u64): sum_topo[0:32) gini_num[32:64)
// acc3  (u64): sum_cost[0:32) episode[32:64)
// topo  (u64): 6 x 9-bit off-diagonal values of the 4x4 zone block, pairs
//              (0,1)(0,2)(0,3)(1,2)(1,3)(2,3)
// zcap  (u64): 4 x 16-bit zone cpu capacity
__device__ __forceinline__ int em_zone(uint32_t m) { return m & 3; }
__device__ __forceinline__ int em_owner(uint32_t m) { return (m >> 2) & 0xFF; }
__device__ __forceinline__ int em_type(uint32_t m) { return (m >> 10) & 7; }
__device__ __forceinline__ int em_c0(uint32_t m) { return (m >> 13) & 0x7F; }
__device__ __forceinline__ int em_node(uint32_t m) { return (m >> 20) & 0xFF; }
__device__ __forceinline__ uint32_t em_pack(int zone, int owner, int type, int c0, int node) {
    return (uint32_t)zone | ((uint32_t)owner << 2) | ((uint32_t)type << 10) | ((uint32_t)c0 << 13) |
           ((uint32_t)node << 20);
}
__device__ __forceinline__ int ed_j(uint32_t d) { return d & 0x3FF; }
__device__ __forceinline__ int ed_m(uint32_t d) { return (d >> 10) & 0x3FF; }
__device__ __forceinline__ int ed_M(uint32_t d) { return (d >> 20) & 0x3FF; }

struct Scal {
    int step, acc, intra, rz, thr_idx, penalty, reset_done, bad;
};
__device__ __forceinline__ Scal sc_unpack(uint64_t s) {
    Scal r;
    r.step = (int)(s & 0xFFFF);
    r.acc = (int)((s >> 16) & 0xFFFF);
    r.intra = (int)((s >> 32) & 0xFFFF);
    r.rz = (int)((s >> 48) & 3);
    r.thr_idx = (int)((s >> 50) & 7);
    r.penalty = (int)((s >> 53) & 1);
    r.reset_done = (int)((s >> 54) & 1);
    r.bad = (int)((s >> 55) & 1);
    return r;
}
__device__ __forceinline__ uint64_t sc_pack(const Scal& r) {
    return (uint64_t)r.step | ((uint64_t)r.acc << 16) | ((uint64_t)r.intra << 32) |
           ((uint64_t)r.rz << 48) | ((uint64_t)r.thr_idx << 50) | ((uint64_t)r.penalty << 53) |
           ((uint64_t)r.reset_done << 54) | ((uint64_t)r.bad << 55);
}

// utils.get_endpoint_list() thresholds {400,200,150,250,450,375,500} / 25, 5 bits each
__device__ __forceinline__ int threshold(int idx) {
    constexpr uint64_t P = 16ull | (8ull << 5) | (6ull << 10) | (10ull << 15) | (18ull << 20) |
                           (15ull << 25) | (20ull << 30);
    return 25 * (int)((P >> (5 * idx)) & 31);
}
// DEFAULT_NODE_TYPES cpu {2,2,2,4,8} and cost {1,2,4,8,16} (:35-39)
__device__ __forceinline__ int node_cpu_int(int t) { return t < 3 ? 2 : (t == 3 ? 4 : 8); }
__device__ __forceinline__ int node_cost(int t) { return 1 << t; }

__device__ __forceinline__ int pair_index(int i, int j) {  // i < j < 4
    return i == 0 ? j - 1 : (i == 1 ? j + 1 : 5);
}
__device__ __forceinline__ int topo_val(uint64_t topo, int a, int b) {
    if (a == b) return 1;
    int i = a < b ? a : b, j = a < b ? b : a;
    return (int)((topo >> (9 * pair_index(i, j))) & 0x1FF);
}
__device__ __forceinline__ int zcap_val(uint64_t zc, int z) { return (int)((zc >> (16 * z)) & 0xFFFF); }

// ---- RNG ---------------------------------------------------------------------------
struct U4 { uint32_t x, y, z, w; };

__device__ __forceinline__ U4 philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                     uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int i = 0; i < 10; ++i) {
        uint32_t hi0 = __umulhi(0xD2511F53u, c0), lo0 = 0xD2511F53u * c0;
        uint32_t hi1 = __umulhi(0xCD9E8D57u, c2), lo1 = 0xCD9E8D57u * c2;
        uint32_t n0 = hi1 ^ c1 ^ k0;
        uint32_t n2 = hi0 ^ c3 ^ k1;
        c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
    return {c0, c1, c2, c3};
}
__device__ __forceinline__ uint32_t bounded(uint32_t w, uint32_t n) {
    return (uint32_t)(((uint64_t)w * n) >> 32);
}
__device__ __forceinline__ double u53(uint32_t hi, uint32_t lo) {
    uint64_t x = (((uint64_t)hi << 32) | lo) >> 11;
    return (double)x * (1.0 / 9007199254740992.0);
}
// log(x), x in (0,1]: fdlibm's reduction + polynomial with plain IEEE ops (bitwise
// identical to the oracle's host build; both compiled without FMA contraction).
__device__ __forceinline__ double fd_log(double x) {
    const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10;
    const double Lg1 = 6.666666666666735130e-01, Lg2 = 3.999999999940941908e-01,
                 Lg3 = 2.857142874366239149e-01, Lg4 = 2.222219843214978396e-01,
                 Lg5 = 1.818357216161805012e-01, Lg6 = 1.531383769920937332e-01,
                 Lg7 = 1.479819860511658591e-01;
    uint64_t bits = (uint64_t)__double_as_longlong(x);
    int k = (int)((bits >> 52) & 0x7ff) - 1023;
    double m = __longlong_as_double((long long)((bits & 0x000fffffffffffffULL) | 0x3ff0000000000000ULL));
    if (m > 1.4142135623730951) { m = m * 0.5; k += 1; }
    double f = m - 1.0;
    double s = f / (2.0 + f);
    double z = s * s, w = z * z;
    double t1 = w * (Lg2 + w * (Lg4 + w * Lg6));
    double t2 = z * (Lg1 + w * (Lg3 + w * (Lg5 + w * Lg7)));
    double R = t2 + t1;
    double hfsq = 0.5 * f * f;
    double dk = (double)k;
    return dk * ln2_hi - ((hfsq - (s * (hfsq + R) + dk * ln2_lo)) - f);
}
__device__ __forceinline__ double std_exp(uint32_t hi, uint32_t lo) { return -fd_log(1.0 - u53(hi, lo)); }

__device__ __forceinline__ double clamp_cpu(double v) { double m = v < 100.0 ? v : 100.0; return m > 1.0 ? m : 1.0; }
__device__ __forceinline__ double clamp_lat(double v) { double m = v < 500.0 ? v : 500.0; return m > 1.0 ? m : 1.0; }

// ---- kernel parameters ------------------------------------------------------------
struct Params {
    double* lat_lut;   // [LAT_ROWS][JCAP]
    double* cpu_lut;   // [CPU_ROWS][JCAP]
    double* lat0;      // [B*EP]
    uint32_t* emeta;   // [B*EP]
    uint32_t* edyn;    // [B*EP]
    double* t;         // [B]
    uint64_t* sc;      // [B]
    uint64_t* topo;    // [B]
    uint64_t* zcap;    // [B]
    uint64_t* nzone;   // [B*NZW]
    uint64_t* acc2;    // [B]
    uint64_t* acc3;    // [B]
    double* sum_lat;   // [B]
    double* sum_cpu;   // [B]
    double* total;     // [B]
    double* last_r;    // [B]
    int64_t B, env_id_offset;
    int E, Z, N, L, R, EP, NZW, A;
    int reward_fn, rejection, auto_reset;
    double inv_rate, call, lw, cw, gw, init_last_r;
    uint32_t key0, key1;
    // per call
    const int32_t* actions;
    float* obs;
    float* reward;
    uint8_t* done;
    float* term_obs;
    double* ep_stats;
    const uint8_t* reset_mask;
    lb_trace tr;
};

__device__ __forceinline__ U4 draw(const Params& p, int64_t env, uint32_t episode, uint32_t slot,
                                   uint32_t dom) {
    uint64_t gid = (uint64_t)(p.env_id_offset + env);
    return philox((uint32_t)gid, episode, slot, dom | ((uint32_t)(gid >> 32) << 8), p.key0, p.key1);
}

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

template <int EPL, typename T>
__device__ __forceinline__ T sel(const T (&a)[EPL], int k) {
    T v = a[0];
#pragma unroll
    for (int i = 1; i < EPL; ++i)
        if (k == i) v = a[i];
    return v;
}

// next_request()'s draws (:1132-1133, :1116, :1120): lanes split the three Philox blocks.
template <int W, bool TRACE>
__device__ __forceinline__ void request_draws(const Params& p, int64_t env, uint32_t episode,
                                              uint32_t slot, int lane, bool from_reset, double& x1,
                                              double& x2, int& r, int& n) {
    if constexpr (TRACE) {
        if (from_reset) {
            x1 = p.tr.reset_x1[env]; x2 = p.tr.reset_x2[env]; r = p.tr.reset_r[env]; n = p.tr.reset_n[env];
        } else {
            x1 = p.tr.step_x1[env]; x2 = p.tr.step_x2[env]; r = p.tr.step_r[env]; n = p.tr.step_n[env];
        }
    } else if constexpr (W >= 4) {
        const int role = lane & 3;
        const uint32_t dom = role == 0 ? D_REQ_X : (role == 1 ? D_REQ_X2 : D_REQ_I);
        U4 w = draw(p, env, episode, slot, dom);
        double e = std_exp(w.x, w.y);
        x1 = p.inv_rate * shfl_f64<W>(e, 0);
        x2 = p.call * shfl_f64<W>(e, 1);
        r = (int)bounded(shfl_u32<W>(w.x, 2), 7);
        n = (int)bounded(shfl_u32<W>(w.y, 2), (uint32_t)p.N);
    } else {
        U4 a = draw(p, env, episode, slot, D_REQ_X);
        U4 b = draw(p, env, episode, slot, D_REQ_X2);
        U4 c = draw(p, env, episode, slot, D_REQ_I);
        x1 = p.inv_rate * std_exp(a.x, a.y);
        x2 = p.call * std_exp(b.x, b.y);
        r = (int)bounded(c.x, 7);
        n = (int)bounded(c.y, (uint32_t)p.N);
    }
}

template <bool TRACE>
__device__ __forceinline__ void node_draw(const Params& p, int64_t env, uint32_t episode, int n,
                                          int& ty, int& zo, int& cpu) {
    if constexpr (TRACE) {
        int64_t i = env * p.N + n;
        ty = p.tr.reset_ntype[i]; zo = p.tr.reset_nzone[i]; cpu = p.tr.reset_ncpu[i];
    } else {
        U4 w = draw(p, env, episode, (uint32_t)n, D_NODE);
        ty = (int)bounded(w.x, 5); zo = (int)bounded(w.y, 4); cpu = 1 + (int)bounded(w.z, 99);
    }
}

// Register image of one env slice.
template <int EPL>
struct Env {
    double lat0[EPL];
    uint32_t em[EPL], ed[EPL];
    double t, dt, sum_lat, sum_cpu, total, last_r;
    uint64_t topo, zcap, acc2, acc3;
    uint64_t nzw;  // zone word of the current request node (only what obs/step needs)
    Scal s;
};

__device__ __forceinline__ double lat_of(const Params& p, double lat0, uint32_t ed) {
    int j = ed_j(ed);
    return j == 0 ? lat0 : p.lat_lut[(int)lat0 * JCAP + j];
}
__device__ __forceinline__ double cpu_of(const Params& p, uint32_t em, uint32_t ed) {
    int m = ed_m(ed);
    int c0 = em_c0(em);
    return m == 0 ? (double)c0 : p.cpu_lut[c0 * JCAP + m];
}
__device__ __forceinline__ double gini_of(uint64_t acc2, int acc, int E) {   // utils.py:132-143
    if (acc == 0) return 0.0;
    double num = (double)(uint32_t)(acc2 >> 32);
    return num / ((double)(2 * E * E) * ((double)acc / (double)E));
}

// get_state() (:688-758): rows [zone, zone_cpu_cap, cpu, topo_lat, lat, req_zone, thr, dt]
template <int W, int EPL>
__device__ __forceinline__ void write_obs(const Params& p, float* out, int64_t env, int lane,
                                          const Env<EPL>& v) {
    float* base = out + env * (int64_t)p.R * 8;
    const float rz = (float)v.s.rz, thr = (float)threshold(v.s.thr_idx), dt = (float)v.dt;
#pragma unroll
    for (int k = 0; k < EPL; ++k) {
        int e = lane + k * W;
        if (e < p.E) {
            int z = em_zone(v.em[k]);
            float4 a = make_float4((float)z, (float)zcap_val(v.zcap, z), (float)cpu_of(p, v.em[k], v.ed[k]),
                                   (float)topo_val(v.topo, z, v.s.rz));
            float4 b = make_float4((float)lat_of(p, v.lat0[k], v.ed[k]), rz, thr, dt);
            float4* row = reinterpret_cast<float4*>(base + e * 8);
            row[0] = a;
            row[1] = b;
        }
    }
    if (p.rejection && lane == (p.E % W)) {
        float4* row = reinterpret_cast<float4*>(base + p.E * 8);
        row[0] = make_float4(-1.f, -1.f, -1.f, -1.f);
        row[1] = make_float4(-1.f, rz, thr, dt);
    }
}

template <int W, int EPL>
__device__ __forceinline__ void write_stats(const Params& p, double* out, const Env<EPL>& v) {
    const Scal& s = v.s;
    uint32_t sum_topo = (uint32_t)v.acc2;
    out[LB_ST_RETURN] = v.total;
    out[LB_ST_LENGTH] = (double)s.step;
    out[LB_ST_ACCEPTED] = (double)s.acc;
    out[LB_ST_SUM_LATENCY] = v.sum_lat;
    out[LB_ST_SUM_TOPOLOGY] = (double)sum_topo;
    // intra-zone accepts see topology 1 (updated 1); inter ones topology * 1.7 (:582-593)
    out[LB_ST_SUM_TOPOLOGY_UPDATED] = (double)s.intra + 1.7 * (double)(sum_topo - (uint32_t)s.intra);
    out[LB_ST_SUM_COST] = (double)(uint32_t)v.acc3;
    out[LB_ST_SUM_CPU] = v.sum_cpu;
    out[LB_ST_INTRA] = (double)s.intra;
    out[LB_ST_INTER] = (double)(s.acc - s.intra);
    out[LB_ST_GINI] = gini_of(v.acc2, s.acc, p.E);
    out[LB_ST_EPISODE] = (double)(uint32_t)(v.acc3 >> 32);
#pragma unroll
    for (int k = LB_ST_EPISODE + 1; k < LB_ST_K; ++k) out[k] = 0.0;
}

template <int EPL>
__device__ __forceinline__ void load_env(const Params& p, int64_t env, int lane, int W, Env<EPL>& v) {
#pragma unroll
    for (int k = 0; k < EPL; ++k) {
        int64_t i = env * p.EP + lane + k * W;
        v.lat0[k] = p.lat0[i];
        v.em[k] = p.emeta[i];
        v.ed[k] = p.edyn[i];
    }
    v.t = p.t[env];
    v.s = sc_unpack(p.sc[env]);
    v.topo = p.topo[env];
    v.zcap = p.zcap[env];
    v.acc2 = p.acc2[env];
    v.acc3 = p.acc3[env];
    v.sum_lat = p.sum_lat[env];
    v.sum_cpu = p.sum_cpu[env];
    v.total = p.total[env];
    v.last_r = p.reward_fn != LB_REWARD_NAIVE ? p.last_r[env] : 0.0;
}

template <int EPL>
__device__ __forceinline__ void store_scalars(const Params& p, int64_t env, const Env<EPL>& v) {
    p.t[env] = v.t;
    p.sc[env] = sc_pack(v.s);
    p.acc2[env] = v.acc2;
    p.acc3[env] = v.acc3;
    p.sum_lat[env] = v.sum_lat;
    p.sum_cpu[env] = v.sum_cpu;
    p.total[env] = v.total;
    if (p.reward_fn != LB_REWARD_NAIVE) p.last_r[env] = v.last_r;
}

// the request part of next_request() (:1131-1163); the dequeue part is folded into the LUTs
template <int W, bool TRACE, int EPL>
__device__ __forceinline__ void next_request(const Params& p, int64_t env, int lane, bool from_reset,
                                             const uint64_t* nz_regs, Env<EPL>& v) {
    double x1, x2;
    int r, n;
    request_draws<W, TRACE>(p, env, (uint32_t)(v.acc3 >> 32), (uint32_t)v.s.step, lane, from_reset,
                            x1, x2, r, n);
    double arrival = v.t + x1;
    double departure = arrival + x2;
    v.dt = departure - arrival;
    v.t = arrival;
    v.s.thr_idx = (r + 6) % 7;  // endpoint_list[r - 1] (:1117)
    uint64_t word;
    if (nz_regs) {
        word = nz_regs[0];
#pragma unroll
        for (int w = 1; w < NZW_MAX; ++w)
            if ((n >> 5) == w) word = nz_regs[w];
    } else {
        word = p.nzone[env * p.NZW + (n >> 5)];
    }
    v.s.rz = (int)((word >> (2 * (n & 31))) & 3);
}

// reset() (:290-400) into registers, then state stores (lat0/emeta/edyn/topo/zcap/nzone).
template <int W, int EPL, bool TRACE>
__device__ void reset_env(const Params& p, int64_t env, int lane, Env<EPL>& v) {
    const uint32_t episode = (uint32_t)(v.acc3 >> 32) + 1;
    // nodes (:349-373): zone capacity and the 2-bit zone of every node
    uint64_t zc = 0;
    uint64_t nz[NZW_MAX];
#pragma unroll
    for (int w = 0; w < NZW_MAX; ++w) nz[w] = 0;
    for (int n = lane; n < p.N; n += W) {
        int ty, zo, cpu;
        node_draw<TRACE>(p, env, episode, n, ty, zo, cpu);
        zc += (uint64_t)node_cpu_int(ty) << (16 * zo);
        uint64_t bit = (uint64_t)zo << (2 * (n & 31));
#pragma unroll
        for (int w = 0; w < NZW_MAX; ++w)
            if ((n >> 5) == w) nz[w] |= bit;
    }
    zc = slice_sum64<W>(zc);
#pragma unroll
    for (int w = 0; w < NZW_MAX; ++w) nz[w] = slice_or64<W>(nz[w]);
    // endpoints (:328, :379-386)
    int node[EPL];
#pragma unroll
    for (int k = 0; k < EPL; ++k) {
        int e = lane + k * W;
        node[k] = 0;
        v.lat0[k] = 0.0;
        v.em[k] = 0;
        v.ed[k] = 0;
        if (e < p.E) {
            double lat;
            int nd;
            if constexpr (TRACE) {
                lat = p.tr.reset_lat0[env * p.E + e];
                nd = p.tr.reset_enode[env * p.E + e];
            } else {
                U4 w = draw(p, env, episode, (uint32_t)e, D_EP);
                lat = 1.0 + 99.0 * u53(w.x, w.y);
                nd = (int)bounded(w.z, 24);
            }
            node[k] = nd;
            v.lat0[k] = lat;
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
        if (e < p.E) {
            int ty, zo, cpu;
            node_draw<TRACE>(p, env, episode, node[k], ty, zo, cpu);
            v.em[k] = em_pack(zo, owner[k], ty, cpu, node[k]);
        }
        int64_t i = env * p.EP + e;
        p.lat0[i] = v.lat0[k];
        p.emeta[i] = v.em[k];
        p.edyn[i] = 0;
    }
    // topology (:331-338): symmetric, diag 1; the 4x4 zone block is all that is observable
    uint64_t topo = 0;
    {
        int val[6];
        if constexpr (TRACE) {
            const int32_t* d = p.tr.reset_topo + env * (int64_t)p.Z * (p.Z - 1);
            int q = 0;
            for (int i = 0; i < 4; ++i)
                for (int j = i + 1; j < 4; ++j) val[q++] = d[j * (p.Z - 1) + i];  // last writer (z1=j, z2=i)
        } else {
            U4 a = draw(p, env, episode, 0, D_TOPO), b = draw(p, env, episode, 1, D_TOPO);
            uint32_t w6[6] = {a.x, a.y, a.z, a.w, b.x, b.y};
#pragma unroll
            for (int q = 0; q < 6; ++q) val[q] = 1 + (int)bounded(w6[q], 499);
        }
#pragma unroll
        for (int q = 0; q < 6; ++q) topo |= (uint64_t)(val[q] & 0x1FF) << (9 * q);
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
    next_request<W, TRACE, EPL>(p, env, lane, true, nz, v);
    if (lane == 0) {
        p.topo[env] = topo;
        p.zcap[env] = zc;
    }
    for (int w = lane; w < p.NZW; w += W) {
        uint64_t word = nz[0];
#pragma unroll
        for (int q = 1; q < NZW_MAX; ++q)
            if (w == q) word = nz[q];
        p.nzone[env * p.NZW + w] = word;
    }
}

// ---- kernels ----------------------------------------------------------------------------

// LAT[k][j]: endpoint latency after j selections from trunc(initial) = k (:1013-1023 then
// :1052-1060 in the same step); CPU[c][M]: node cpu after M selections (:861-887, :937-960).
__global__ void k_luts(double* lat_lut, double* cpu_lut) {
    int row = blockIdx.x * blockDim.x + threadIdx.x;
    if (row < LAT_ROWS) {
        double* o = lat_lut + (int64_t)row * JCAP;
        double v = (double)row;
        o[0] = v;
        for (int j = 1; j < JCAP; ++j) {
            double inc = clamp_lat(trunc(v) * 1.5);
            v = clamp_lat(trunc(inc) / 1.15);
            o[j] = v;
        }
    } else if (row < LAT_ROWS + CPU_ROWS) {
        int c = row - LAT_ROWS;
        double* o = cpu_lut + (int64_t)c * JCAP;
        double w = (double)c;
        o[0] = w;
        for (int m = 1; m < JCAP; ++m) {
            w = clamp_cpu(clamp_cpu(w * 1.15) / 1.15);
            o[m] = w;
        }
    }
}

__global__ void k_init(Params p, int trace) {
    int64_t env = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (env >= p.B) return;
    for (int e = 0; e < p.EP; ++e) {
        int64_t i = env * p.EP + e;
        p.lat0[i] = 0.0;
        p.emeta[i] = 0;
        p.edyn[i] = 0;
    }
    double t;
    if (trace) {
        t = p.tr.t0[env];
    } else {
        U4 w = draw(p, env, 0, 0, D_INIT);
        t = 0.0 + p.inv_rate * std_exp(w.x, w.y);  // __init__'s next_request() (:267)
    }
    p.t[env] = t;
    p.sc[env] = 0;
    p.topo[env] = 0;
    p.zcap[env] = 0;
    for (int w = 0; w < p.NZW; ++w) p.nzone[env * p.NZW + w] = 0;
    p.acc2[env] = 0;
    p.acc3[env] = 0;
    p.sum_lat[env] = 0.0;
    p.sum_cpu[env] = 0.0;
    p.total[env] = 0.0;
    p.last_r[env] = p.init_last_r;
}

template <int W, int EPL, bool TRACE>
__global__ __launch_bounds__(BLOCK) void k_reset(Params p) {
    const int lane = threadIdx.x % W;
    const int64_t env = (int64_t)blockIdx.x * (BLOCK / W) + threadIdx.x / W;
    if (env >= p.B) return;
    if (p.reset_mask && !p.reset_mask[env]) return;
    Env<EPL> v;
    v.t = p.t[env];
    v.acc3 = p.acc3[env];
    v.s = sc_unpack(p.sc[env]);
    reset_env<W, EPL, TRACE>(p, env, lane, v);
    if (p.obs) write_obs<W, EPL>(p, p.obs, env, lane, v);
    if (lane == 0) store_scalars<EPL>(p, env, v);
}

// step() (:403-513) fused with next_request(), get_state(), reward, done and auto-reset.
template <int W, int EPL, bool TRACE>
__global__ __launch_bounds__(BLOCK) void k_step(Params p) {
    const int lane = threadIdx.x % W;
    const int64_t env = (int64_t)blockIdx.x * (BLOCK / W) + threadIdx.x / W;
    if (env >= p.B) return;
    const int E = p.E;
    Env<EPL> v;
    load_env<EPL>(p, env, lane, W, v);
    const int a = p.actions[env];

    // take_action (:578-686)
    v.s.step = v.s.step < 0xFFFF ? v.s.step + 1 : 0xFFFF;
    const bool accept = a >= -E && a < E;
    const bool reject = a == E;
    if (a < -E) v.s.bad = 1;  // reference: IndexError; here: treated as unrecognised
    if (!v.s.reset_done) v.s.bad = 1;
    double reward;
    int dirty_a = -1, dirty_o = -1;
    if (accept) {
        const int ai = a < 0 ? a + E : a;
        const int src = ai % W, sk = ai / W;
        const uint32_t emA = shfl_u32<W>(sel<EPL>(v.em, sk), src);
        const uint32_t edA = shfl_u32<W>(sel<EPL>(v.ed, sk), src);
        const double lat0A = shfl_f64<W>(sel<EPL>(v.lat0, sk), src);
        const int oA = em_owner(emA);
        const uint32_t edO = shfl_u32<W>(sel<EPL>(v.ed, oA / W), oA % W);
        const int zA = em_zone(emA), jA = ed_j(edA);
        const double sel_lat = lat_of(p, lat0A, edA);
        const double sel_cpu = cpu_of(p, emA, edA);
        const int tl = topo_val(v.topo, v.s.rz, zA);
        // O(E) Gini numerator update: avg_load_served[ai] += 1 (:631)
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
        v.acc3 += (uint64_t)node_cost(em_type(emA));
        v.s.acc = v.s.acc < 0xFFFF ? v.s.acc + 1 : 0xFFFF;
        if (v.s.rz == zA) v.s.intra = v.s.intra < 0xFFFF ? v.s.intra + 1 : 0xFFFF;
        v.sum_lat += sel_lat;
        v.sum_cpu += sel_cpu;
        // increase_resources / increase_endpoint_latency now, the decrease in next_request()
        const int Mn = ed_M(edO) < CMAX ? ed_M(edO) + 1 : CMAX;
        const int jn = jA < CMAX ? jA + 1 : CMAX;
#pragma unroll
        for (int k = 0; k < EPL; ++k) {
            int e = lane + k * W;
            if (e == oA) v.ed[k] = (v.ed[k] & ~(0x3FFu << 20)) | ((uint32_t)Mn << 20);
            if (e == ai) v.ed[k] = (v.ed[k] & (0x3FFu << 20)) | ((uint32_t)Mn << 10) | (uint32_t)jn;
        }
        dirty_a = ai;
        dirty_o = oA;
        v.s.penalty = 0;
        switch (p.reward_fn) {  // get_reward (:516-567), float64, reference op order
        case LB_REWARD_NAIVE: reward = 1.0; break;
        case LB_REWARD_LATENCY: reward = -(sel_lat + (double)tl); break;
        case LB_REWARD_FAIRNESS: reward = 1.0 - gini_of(v.acc2, v.s.acc, E); break;
        default: {
            double cur = ((sel_lat + (double)tl) - 2.0) / 998.0;
            double cpu = (sel_cpu - 1.0) / 99.0;
            double g = gini_of(v.acc2, v.s.acc, E);
            reward = p.lw * (1.0 - cur) + p.cw * (1.0 - cpu) + p.gw * (1.0 - g);
        }
        }
        v.last_r = reward;
    } else if (reject) {
        v.s.penalty = 1;
        reward = p.reward_fn == LB_REWARD_LATENCY ? -1000.0 : -1.0;
        v.last_r = reward;
    } else {  // unrecognised action (:685-686): penalty and selected_* stay stale
        reward = p.reward_fn == LB_REWARD_NAIVE ? (v.s.penalty ? -1.0 : 1.0) : v.last_r;
    }
    v.total += reward;

    next_request<W, TRACE, EPL>(p, env, lane, false, nullptr, v);
    const bool done = v.s.step == p.L;
    if (lane == 0) {
        if (p.reward) p.reward[env] = (float)reward;
        if (p.done) p.done[env] = (uint8_t)done;
    }
    if (done && p.auto_reset) {
        if (p.term_obs) write_obs<W, EPL>(p, p.term_obs, env, lane, v);
        if (p.ep_stats && lane == 0) write_stats<W, EPL>(p, p.ep_stats + env * LB_ST_K, v);
        reset_env<W, EPL, TRACE>(p, env, lane, v);
    } else {
#pragma unroll
        for (int k = 0; k < EPL; ++k) {
            int e = lane + k * W;
            if (e == dirty_a || e == dirty_o) p.edyn[env * p.EP + e] = v.ed[k];
        }
    }
    if (p.obs) write_obs<W, EPL>(p, p.obs, env, lane, v);
    if (lane == 0) store_scalars<EPL>(p, env, v);
}

// envs/baselines.py (:6-35): greedy over feasible = mask[:-1] (masks are all True,
// :808-821), first index on ties (numpy argmin/argmax); or uniform random.
template <int W, int EPL>
__global__ __launch_bounds__(BLOCK) void k_policy(Params p, int kind, int32_t* out) {
    const int lane = threadIdx.x % W;
    const int64_t env = (int64_t)blockIdx.x * (BLOCK / W) + threadIdx.x / W;
    if (env >= p.B) return;
    if (kind == LB_POLICY_RANDOM) {
        if (lane == 0) {
            Scal s = sc_unpack(p.sc[env]);
            U4 w = draw(p, env, (uint32_t)(p.acc3[env] >> 32), (uint32_t)s.step, D_ACT);
            out[env] = (int32_t)bounded(w.x, (uint32_t)p.A);
        }
        return;
    }
    const int nf = p.A - 1;
    Scal s = sc_unpack(p.sc[env]);
    uint64_t topo = p.topo[env], zc = p.zcap[env];
    double best = 0.0;
    int bi = 0x7FFFFFFF;
#pragma unroll
    for (int k = 0; k < EPL; ++k) {
        int e = lane + k * W;
        if (e < nf) {
            int64_t i = env * p.EP + e;
            uint32_t em = p.emeta[i];
            double val;
            if (kind == LB_POLICY_TOPOLOGY_GREEDY) val = (double)topo_val(topo, em_zone(em), s.rz);
            else if (kind == LB_POLICY_ZONE_CPU_GREEDY) val = -(double)zcap_val(zc, em_zone(em));
            else val = cpu_of(p, em, p.edyn[i]);
            if (bi == 0x7FFFFFFF || val < best) { best = val; bi = e; }
        }
    }
#pragma unroll
    for (int m = W / 2; m >= 1; m >>= 1) {
        double ob = __shfl_xor(best, m, W);
        int oi = __shfl_xor(bi, m, W);
        if (oi != 0x7FFFFFFF && (bi == 0x7FFFFFFF || ob < best || (ob == best && oi < bi))) {
            best = ob;
            bi = oi;
        }
    }
    if (lane == 0) out[env] = nf <= 0 ? p.A - 1 : bi;
}

template <int W, int EPL>
__global__ __launch_bounds__(BLOCK) void k_field(Params p, int field, double* out) {
    const int lane = threadIdx.x % W;
    const int64_t env = (int64_t)blockIdx.x * (BLOCK / W) + threadIdx.x / W;
    if (env >= p.B) return;
    Scal s = sc_unpack(p.sc[env]);
    if (field >= LB_FIELD_CURRENT_TIME) {
        if (lane != 0) return;
        double v = 0.0;
        switch (field) {
        case LB_FIELD_CURRENT_TIME: v = p.t[env]; break;
        case LB_FIELD_CURRENT_STEP: v = (double)s.step; break;
        case LB_FIELD_REQUEST_ZONE: v = (double)s.rz; break;
        case LB_FIELD_REQUEST_THRESHOLD: v = (double)threshold(s.thr_idx); break;
        default: v = 0.0; break;
        }
        out[env] = v;
        return;
    }
    uint64_t topo = p.topo[env], zc = p.zcap[env];
#pragma unroll
    for (int k = 0; k < EPL; ++k) {
        int e = lane + k * W;
        if (e >= p.E) continue;
        int64_t i = env * p.EP + e;
        uint32_t em = p.emeta[i], ed = p.edyn[i];
        double v;
        switch (field) {
        case LB_FIELD_ENDPOINT_LATENCY: v = lat_of(p, p.lat0[i], ed); break;
        case LB_FIELD_ENDPOINT_CPU: v = cpu_of(p, em, ed); break;
        case LB_FIELD_ENDPOINT_TOPOLOGY_LATENCY: v = (double)topo_val(topo, em_zone(em), s.rz); break;
        case LB_FIELD_ENDPOINT_ZONE_CPU_CAPACITY: v = (double)zcap_val(zc, em_zone(em)); break;
        case LB_FIELD_ENDPOINT_ZONE: v = (double)em_zone(em); break;
        case LB_FIELD_ENDPOINT_NODE: v = (double)em_node(em); break;
        default: v = (double)ed_j(ed); break;  // LB_FIELD_LOAD_SERVED
        }
        out[env * p.E + e] = v;
    }
}

__global__ void k_stats(Params p, double* out) {
    int64_t env = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (env >= p.B) return;
    Env<1> v;
    v.s = sc_unpack(p.sc[env]);
    v.acc2 = p.acc2[env];
    v.acc3 = p.acc3[env];
    v.sum_lat = p.sum_lat[env];
    v.sum_cpu = p.sum_cpu[env];
    v.total = p.total[env];
    write_stats<1, 1>(p, out + env * LB_ST_K, v);
}

__global__ void k_status(Params p, uint32_t* flags) {
    int64_t env = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t f = 0;
    if (env < p.B) {
        Scal s = sc_unpack(p.sc[env]);
        if (s.bad) f |= LB_STATUS_BAD_ACTION;
        if (!s.reset_done) f |= LB_STATUS_NOT_RESET;
    }
    if (f) atomicOr(flags, f);
}

// ---- host side ---------------------------------------------------------------------------
thread_local std::string g_err;

int fail(const char* msg) {
    g_err = msg;
    return -1;
}

struct Geo {
    int W, EPL, EP, NZW;
};

Geo geometry(const lb_config* c) {
    Geo g;
    int E = c->num_endpoints;
    g.W = E <= 4 ? 4 : E <= 8 ? 8 : E <= 16 ? 16 : E <= 32 ? 32 : 64;
    g.EPL = E <= 64 ? 1 : E <= 128 ? 2 : 4;
    g.EP = g.W * g.EPL;
    g.NZW = (c->num_nodes + 31) / 32;
    return g;
}

uint64_t align_up(uint64_t x) { return (x + 255) & ~(uint64_t)255; }

struct Offsets {
    uint64_t lat_lut, cpu_lut, lat0, emeta, edyn, t, sc, topo, zcap, nzone, acc2, acc3, sum_lat,
        sum_cpu, total, last_r, end;
};

Offsets offsets(const lb_config* c, int64_t B) {
    Geo g = geometry(c);
    Offsets o;
    uint64_t x = 0;
    auto take = [&](uint64_t bytes) { uint64_t r = x; x = align_up(x + bytes); return r; };
    o.lat_lut = take((uint64_t)LAT_ROWS * JCAP * 8);
    o.cpu_lut = take((uint64_t)CPU_ROWS * JCAP * 8);
    uint64_t BE = (uint64_t)B * g.EP;
    o.lat0 = take(BE * 8);
    o.emeta = take(BE * 4);
    o.edyn = take(BE * 4);
    o.t = take(B * 8);
    o.sc = take(B * 8);
    o.topo = take(B * 8);
    o.zcap = take(B * 8);
    o.nzone = take((uint64_t)B * g.NZW * 8);
    o.acc2 = take(B * 8);
    o.acc3 = take(B * 8);
    o.sum_lat = take(B * 8);
    o.sum_cpu = take(B * 8);
    o.total = take(B * 8);
    o.last_r = take(B * 8);
    o.end = x;
    return o;
}

double initial_last_reward(const lb_config* c) {
    // get_reward() right after reset(): penalty False, selected latency 0.0, topology 0.0,
    // cpu 1.0, all loads 0 (:297-327) — what an unrecognised first action returns.
    switch (c->reward_fn) {
    case LB_REWARD_NAIVE: return 1.0;
    case LB_REWARD_LATENCY: return -(0.0 + 0.0);
    case LB_REWARD_FAIRNESS: return 1.0 - 0.0;
    default: {
        volatile double cur = ((0.0 + 0.0) - 2.0) / 998.0;
        volatile double cpu = (1.0 - 1.0) / 99.0;
        volatile double a = c->latency_weight * (1.0 - cur);
        volatile double b = c->cpu_weight * (1.0 - cpu);
        volatile double g = c->gini_weight * (1.0 - 0.0);
        volatile double ab = a + b;
        return ab + g;
    }
    }
}

int validate(const lb_config* c) {
    if (!c) return fail("lb_config is NULL");
    if (c->num_endpoints < 1 || c->num_endpoints > EMAX) return fail("num_endpoints must be in [1, 256]");
    if (c->num_zones < 4)
        return fail("IndexError: num_zones < 4 (zone ids are drawn in [0,4), loadbalancer_k8s_env.py:354)");
    if (c->num_nodes < 24)
        return fail("IndexError: num_nodes < 24 (endpoint hosts are drawn in [0,24), loadbalancer_k8s_env.py:380)");
    if (c->num_nodes > 32 * NZW_MAX) return fail("num_nodes must be <= 256");
    if (c->episode_length < 1 || c->episode_length > CMAX) return fail("episode_length must be in [1, 1023]");
    if (c->reward_fn < 0 || c->reward_fn > 3) return fail("unknown reward_fn");
    if (c->rng_mode != LB_RNG_PHILOX && c->rng_mode != LB_RNG_TRACE) return fail("unknown rng_mode");
    if (!(c->arrival_rate > 0.0)) return fail("arrival_rate must be > 0");
    return 0;
}

Params make_params(void* state, const lb_config* c, int64_t B) {
    Geo g = geometry(c);
    Offsets o = offsets(c, B);
    char* base = (char*)state;
    Params p;
    memset(&p, 0, sizeof(p));
    p.lat_lut = (double*)(base + o.lat_lut);
    p.cpu_lut = (double*)(base + o.cpu_lut);
    p.lat0 = (double*)(base + o.lat0);
    p.emeta = (uint32_t*)(base + o.emeta);
    p.edyn = (uint32_t*)(base + o.edyn);
    p.t = (double*)(base + o.t);
    p.sc = (uint64_t*)(base + o.sc);
    p.topo = (uint64_t*)(base + o.topo);
    p.zcap = (uint64_t*)(base + o.zcap);
    p.nzone = (uint64_t*)(base + o.nzone);
    p.acc2 = (uint64_t*)(base + o.acc2);
    p.acc3 = (uint64_t*)(base + o.acc3);
    p.sum_lat = (double*)(base + o.sum_lat);
    p.sum_cpu = (double*)(base + o.sum_cpu);
    p.total = (double*)(base + o.total);
    p.last_r = (double*)(base + o.last_r);
    p.B = B;
    p.env_id_offset = c->env_id_offset;
    p.E = c->num_endpoints;
    p.Z = c->num_zones;
    p.N = c->num_nodes;
    p.L = c->episode_length;
    p.R = c->num_endpoints + (c->rejection_allowed ? 1 : 0);
    p.A = p.R;
    p.EP = g.EP;
    p.NZW = g.NZW;
    p.reward_fn = c->reward_fn;
    p.rejection = c->rejection_allowed ? 1 : 0;
    p.auto_reset = c->auto_reset ? 1 : 0;
    p.inv_rate = 1.0 / c->arrival_rate;
    p.call = c->call_duration;
    p.lw = c->latency_weight;
    p.cw = c->cpu_weight;
    p.gw = c->gini_weight;
    p.init_last_r = initial_last_reward(c);
    p.key0 = (uint32_t)c->seed;
    p.key1 = (uint32_t)(c->seed >> 32);
    return p;
}

int check_launch() {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        g_err = std::string("HIP launch failed: ") + hipGetErrorString(e);
        return -2;
    }
    return 0;
}

#define LB_DISPATCH(W_, EPL_, BODY)                                               \
    do {                                                                          \
        if (W_ == 4 && EPL_ == 1) { constexpr int W = 4, EPL = 1; BODY; }         \
        else if (W_ == 8 && EPL_ == 1) { constexpr int W = 8, EPL = 1; BODY; }    \
        else if (W_ == 16 && EPL_ == 1) { constexpr int W = 16, EPL = 1; BODY; }  \
        else if (W_ == 32 && EPL_ == 1) { constexpr int W = 32, EPL = 1; BODY; }  \
        else if (W_ == 64 && EPL_ == 1) { constexpr int W = 64, EPL = 1; BODY; }  \
        else if (W_ == 64 && EPL_ == 2) { constexpr int W = 64, EPL = 2; BODY; }  \
        else if (W_ == 64 && EPL_ == 4) { constexpr int W = 64, EPL = 4; BODY; }  \
        else return fail("unsupported geometry");                                 \
    } while (0)

unsigned slice_blocks(int64_t B, int W) {
    int64_t per = BLOCK / W;
    return (unsigned)((B + per - 1) / per);
}

}  // namespace

extern "C" {

int lb_abi_version(void) { return LBK8S_ABI_VERSION; }

const char* lb_last_error(void) { return g_err.c_str(); }

int lb_validate_config(const lb_config* cfg) { return validate(cfg); }

int lb_state_bytes(const lb_config* cfg, int64_t num_envs, uint64_t* out_bytes) {
    if (int r = validate(cfg)) return r;
    if (num_envs < 1 || !out_bytes) return fail("num_envs must be >= 1 and out_bytes non-NULL");
    *out_bytes = offsets(cfg, num_envs).end;
    return 0;
}

int lb_init(void* state, const lb_config* cfg, int64_t num_envs, const lb_trace* trace, void* stream) {
    if (int r = validate(cfg)) return r;
    if (!state || num_envs < 1) return fail("state NULL or num_envs < 1");
    const bool tr = cfg->rng_mode == LB_RNG_TRACE;
    if (tr && (!trace || !trace->t0)) return fail("trace mode: lb_init needs trace->t0");
    Params p = make_params(state, cfg, num_envs);
    if (tr) p.tr = *trace;
    hipStream_t s = (hipStream_t)stream;
    hipLaunchKernelGGL(k_luts, dim3((LAT_ROWS + CPU_ROWS + 127) / 128), dim3(128), 0, s, p.lat_lut, p.cpu_lut);
    if (int r = check_launch()) return r;
    hipLaunchKernelGGL(k_init, dim3((unsigned)((num_envs + 255) / 256)), dim3(256), 0, s, p, tr ? 1 : 0);
    return check_launch();
}

int lb_reset(void* state, const lb_config* cfg, int64_t num_envs, const uint8_t* reset_mask,
             float* obs_out, const lb_trace* trace, void* stream) {
    if (int r = validate(cfg)) return r;
    if (!state || num_envs < 1) return fail("state NULL or num_envs < 1");
    const bool tr = cfg->rng_mode == LB_RNG_TRACE;
    if (tr && (!trace || !trace->reset_lat0 || !trace->reset_topo || !trace->reset_ntype ||
               !trace->reset_nzone || !trace->reset_ncpu || !trace->reset_enode || !trace->reset_x1 ||
               !trace->reset_x2 || !trace->reset_r || !trace->reset_n))
        return fail("trace mode: lb_reset needs every reset_* trace array");
    Params p = make_params(state, cfg, num_envs);
    if (tr) p.tr = *trace;
    p.obs = obs_out;
    p.reset_mask = reset_mask;
    Geo g = geometry(cfg);
    hipStream_t s = (hipStream_t)stream;
    LB_DISPATCH(g.W, g.EPL, {
        if (tr) hipLaunchKernelGGL((k_reset<W, EPL, true>), dim3(slice_blocks(num_envs, W)), dim3(BLOCK), 0, s, p);
        else hipLaunchKernelGGL((k_reset<W, EPL, false>), dim3(slice_blocks(num_envs, W)), dim3(BLOCK), 0, s, p);
    });
    return check_launch();
}

int lb_step(void* state, const lb_config* cfg, int64_t num_envs, const int32_t* actions,
            float* obs_out, float* reward_out, uint8_t* done_out, float* terminal_obs_out,
            double* ep_stats_out, const lb_trace* trace, void* stream) {
    if (int r = validate(cfg)) return r;
    if (!state || num_envs < 1 || !actions) return fail("state/actions NULL or num_envs < 1");
    const bool tr = cfg->rng_mode == LB_RNG_TRACE;
    if (tr && (!trace || !trace->step_x1 || !trace->step_x2 || !trace->step_r || !trace->step_n))
        return fail("trace mode: lb_step needs trace->step_* arrays");
    if (tr && cfg->auto_reset &&
        (!trace->reset_lat0 || !trace->reset_topo || !trace->reset_ntype || !trace->reset_nzone ||
         !trace->reset_ncpu || !trace->reset_enode || !trace->reset_x1 || !trace->reset_x2 ||
         !trace->reset_r || !trace->reset_n))
        return fail("trace mode with auto_reset: lb_step needs the reset_* arrays (any step may end an episode)");
    Params p = make_params(state, cfg, num_envs);
    if (tr) p.tr = *trace;
    p.actions = actions;
    p.obs = obs_out;
    p.reward = reward_out;
    p.done = done_out;
    p.term_obs = terminal_obs_out;
    p.ep_stats = ep_stats_out;
    Geo g = geometry(cfg);
    hipStream_t s = (hipStream_t)stream;
    LB_DISPATCH(g.W, g.EPL, {
        if (tr) hipLaunchKernelGGL((k_step<W, EPL, true>), dim3(slice_blocks(num_envs, W)), dim3(BLOCK), 0, s, p);
        else hipLaunchKernelGGL((k_step<W, EPL, false>), dim3(slice_blocks(num_envs, W)), dim3(BLOCK), 0, s, p);
    });
    return check_launch();
}

int lb_policy(const void* state, const lb_config* cfg, int64_t num_envs, int32_t kind,
              int32_t* actions_out, void* stream) {
    if (int r = validate(cfg)) return r;
    if (!state || !actions_out || num_envs < 1) return fail("state/actions_out NULL");
    if (kind < 0 || kind > LB_POLICY_RANDOM) return fail("unknown policy kind");
    Params p = make_params(const_cast<void*>(state), cfg, num_envs);
    Geo g = geometry(cfg);
    hipStream_t s = (hipStream_t)stream;
    LB_DISPATCH(g.W, g.EPL, {
        hipLaunchKernelGGL((k_policy<W, EPL>), dim3(slice_blocks(num_envs, W)), dim3(BLOCK), 0, s, p,
                           (int)kind, actions_out);
    });
    return check_launch();
}

int lb_get_field(const void* state, const lb_config* cfg, int64_t num_envs, int32_t field, double* out,
                 void* stream) {
    if (int r = validate(cfg)) return r;
    if (!state || !out || num_envs < 1) return fail("state/out NULL");
    if (field < 0 || field >= LB_FIELD_COUNT) return fail("unknown field");
    if (field == LB_FIELD_DT) return fail("dt is not stored (it only feeds obs column 7)");
    Params p = make_params(const_cast<void*>(state), cfg, num_envs);
    Geo g = geometry(cfg);
    hipStream_t s = (hipStream_t)stream;
    LB_DISPATCH(g.W, g.EPL, {
        hipLaunchKernelGGL((k_field<W, EPL>), dim3(slice_blocks(num_envs, W)), dim3(BLOCK), 0, s, p,
                           (int)field, out);
    });
    return check_launch();
}

int lb_get_stats(const void* state, const lb_config* cfg, int64_t num_envs, double* stats_out, void* stream) {
    if (int r = validate(cfg)) return r;
    if (!state || !stats_out || num_envs < 1) return fail("state/stats_out NULL");
    Params p = make_params(const_cast<void*>(state), cfg, num_envs);
    hipLaunchKernelGGL(k_stats, dim3((unsigned)((num_envs + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       p, stats_out);
    return check_launch();
}

int lb_status(const void* state, const lb_config* cfg, int64_t num_envs, uint32_t* flags_out, void* stream) {
    if (int r = validate(cfg)) return r;
    if (!state || !flags_out || num_envs < 1) return fail("state/flags_out NULL");
    Params p = make_params(const_cast<void*>(state), cfg, num_envs);
    hipStream_t s = (hipStream_t)stream;
    if (hipMemsetAsync(flags_out, 0, sizeof(uint32_t), s) != hipSuccess) return fail("hipMemsetAsync failed");
    hipLaunchKernelGGL(k_status, dim3((unsigned)((num_envs + 255) / 256)), dim3(256), 0, s, p, flags_out);
    return check_launch();
}

}  // extern "C"
