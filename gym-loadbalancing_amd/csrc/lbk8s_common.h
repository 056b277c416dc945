// lbk8s_common.h — shared device code of the vectorized LoadBalancerK8sEnv kernels:
// constants, packed-state bit layouts, Philox RNG, the float64 IEEE helpers, and the
// kernel parameter block.  Included by lbk8s.hip only.
//
// Reference: /root/reference/envs/loadbalancer_k8s_env.py (constants :17-79) and
// envs/utils.py (endpoint thresholds :33-64, gini :132-143).
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
// applies (k_luts).  avg_load_served[e] == j_e.  Per endpoint the hot state is lat0
// (f64, fixed within an episode) plus two 32-bit words; one word is written per accept.
// Everything is compiled with -ffp-contract=off: the reference's float64 math is plain
// IEEE mul/div/add and FMA contraction would change bits.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "lbk8s.h"

namespace lbk {

constexpr int BLOCK = 256;
constexpr int JCAP = 1024;        // LUT columns; per-episode counters saturate at 1023
constexpr int CMAX = JCAP - 1;
constexpr int LAT_ROWS = 501;     // trunc(initial latency) in [0, 500]; tables are [JCAP][ROWS]
constexpr int CPU_ROWS = 128;     // initial node cpu in [0, 127]
constexpr int NZW_MAX = 8;        // node-zone words of 32 nodes -> num_nodes <= 256
constexpr int EMAX = 256;
constexpr int TPE_E = 8;          // thread-per-env path: E <= 8 endpoints in registers
constexpr int RO_REC_BYTES = 160; // k_rollout_tpe's next-episode record per env (lbk8s_tpe.h)

// Philox domains — the framework's draw map; restated by the oracle.
enum : uint32_t { D_INIT = 1, D_NODE = 2, D_EP = 3, D_TOPO = 4, D_REQ_X = 5, D_REQ_I = 6,
                  D_ACT = 7, D_DQN_EXPLORE = 8, D_DQN_SAMPLE = 9 };

// ---- bit layouts -------------------------------------------------------------------
// emeta (static per episode): zone[0:2) owner[2:10) type[10:13) c0[13:20) node[20:28)
// edyn  (per step):           j[0:10)   m[10:20)    M[20:30)
// sc    (u64): step[0:16) acc[16:32) intra[32:48) req_zone[48:50) thr_idx[50:53)
//              penalty[53] reset_done[54] bad_action[55]
// acc2  (u64): sum_topo[0:32) gini_num[32:64)
// acc3  (u64): sum_cost[0:32) episode[32:64)
// topo  (u64): 6 x 9-bit off-diagonal values of the 4x4 zone block, pairs
//              (0,1)(0,2)(0,3)(1,2)(1,3)(2,3)   (zone ids are drawn in [0,4): :205,:354)
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

// Philox4x32-10 (Salmon, Moraes, Dror, Shaw, SC'11), the Random123 default and SURVEY §7's
// choice; the round function and count are pinned by the Random123 philox4x32_10 known
// answers through the oracle.  (Rounds 1-3 used 7 rounds; an interleaved A/B on the rollout
// kernel measured 10 rounds within 0.4-1.5% of 7, profiles/r03_ablation.jsonl.)
#ifndef LB_PHILOX_ROUNDS  // (an A/B build may override it: tools/roll_variants.py --lib)
#define LB_PHILOX_ROUNDS 10
#endif
__device__ __forceinline__ U4 philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                     uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int i = 0; i < LB_PHILOX_ROUNDS; ++i) {
        // 32x32 -> 64-bit products: one v_mad_u64_u32 each instead of a mul_hi / mul_lo pair
        // (a Philox-only micro-bench: 1.33x the blocks per second; the rollout ~1%)
        const uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
        const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        uint32_t n0 = hi1 ^ c1 ^ k0;
        uint32_t n2 = hi0 ^ c3 ^ k1;
        c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
    return {c0, c1, c2, c3};
}
__device__ __forceinline__ uint32_t bounded(uint32_t w, uint32_t n) {  // Lemire multiply-high
    return (uint32_t)(((uint64_t)w * n) >> 32);
}
__device__ __forceinline__ double u53(uint32_t hi, uint32_t lo) {
    uint64_t x = (((uint64_t)hi << 32) | lo) >> 11;
    return (double)x * (1.0 / 9007199254740992.0);
}
// log(x), x in (0,1]: fdlibm's e_log.c reduction + polynomial with plain IEEE ops (bitwise
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
    double* lat0;      // endpoint arrays, element (env, e) at e*es + env*ee
    uint32_t* emeta;
    uint32_t* edyn;
    double* t;         // [B]
    uint64_t* sc;      // [B]
    uint64_t* topo;    // [B]
    uint64_t* zcap;    // [B]
    uint64_t* nzone;   // [NZW][B]  (word w of env at w*B + env)
    uint64_t* acc2;    // [B]
    uint64_t* acc3;    // [B]
    uint64_t* sum_lat; // [B] exact fixed-point sums (fix52, low 64 bits)
    uint64_t* sum_cpu; // [B]
    uint32_t* sum_hi;  // [B] their carries and the updated-topology residual D (xsum_add)
    double* total;     // [B]
    double* last_r;    // [B]
    double* rew64;     // [B] float64 reward of the last lb_step (lb_reward64: VecMonitor's return)
    uint4* rec;        // [B][RO_REC_BYTES / 16] next-episode records (thread-per-env rollout scratch)
    int64_t B, env_id_offset, es, ee;
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

// Streaming stores for the observation stream (written once per step, consumed later
// by the learner): nontemporal, so they do not displace state lines from L2 / MALL.
// Measured on MI355X at 2^20 default envs: step 0.191 -> 0.108 ms (A/B builds, profiles/r01_ablation.jsonl).
typedef float f4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void st_stream(float4* p, float4 v) {
    __builtin_nontemporal_store(f4v{v.x, v.y, v.z, v.w}, reinterpret_cast<f4v*>(p));
}

__device__ __forceinline__ int64_t eidx(const Params& p, int64_t env, int e) {
    return (int64_t)e * p.es + env * p.ee;
}

__device__ __forceinline__ U4 draw(const Params& p, int64_t env, uint32_t episode, uint32_t slot,
                                   uint32_t dom) {
    uint64_t gid = (uint64_t)(p.env_id_offset + env);
    return philox((uint32_t)gid, episode, slot, dom | ((uint32_t)(gid >> 32) << 8), p.key0, p.key1);
}

// the env's uniform random action for this step (action_space.sample()): lb_policy's
// LB_POLICY_RANDOM and lb_step's fused random policy (actions == NULL) draw the same value
__device__ __forceinline__ int32_t random_action_raw(uint64_t gid, uint64_t acc3, uint32_t step, uint32_t key0,
                                                     uint32_t key1, int A) {
    const U4 w = philox((uint32_t)gid, (uint32_t)(acc3 >> 32), step, D_ACT | ((uint32_t)(gid >> 32) << 8), key0, key1);
    return (int32_t)bounded(w.x, (uint32_t)A);
}
__device__ __forceinline__ int32_t random_action(const Params& p, int64_t env, uint64_t acc3, uint32_t step) {
    return random_action_raw((uint64_t)(p.env_id_offset + env), acc3, step, p.key0, p.key1, p.A);
}
// the DQN's explore decision at vector step t (lb_dqn_act): eps = linear_schedule(t), one
// uniform keyed by (seed, t) for every env
__device__ __forceinline__ bool dqn_explores(const lb_dqn_explore& ex, int64_t t) {
    const double eps = fmax(ex.slope * (double)t + ex.start_e, ex.end_e);  // linear_schedule (:32-34)
    const U4 w = philox((uint32_t)t, (uint32_t)((uint64_t)t >> 32), 0u, D_DQN_EXPLORE, (uint32_t)ex.seed,
                        (uint32_t)(ex.seed >> 32));
    return u53(w.x, w.y) < eps;
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

// the episode's 4x4 topology block from its two D_TOPO blocks (reset() :331-338)
__device__ __forceinline__ uint64_t scen_topo(const Params& p, int64_t env, uint32_t episode) {
    U4 a = draw(p, env, episode, 0, D_TOPO), b = draw(p, env, episode, 1, D_TOPO);
    return (uint64_t)(1 + bounded(a.x, 499)) | ((uint64_t)(1 + bounded(a.y, 499)) << 9) |
           ((uint64_t)(1 + bounded(a.z, 499)) << 18) | ((uint64_t)(1 + bounded(a.w, 499)) << 27) |
           ((uint64_t)(1 + bounded(b.x, 499)) << 36) | ((uint64_t)(1 + bounded(b.y, 499)) << 45);
}

__device__ __forceinline__ double lat_of(const Params& p, double lat0, uint32_t ed) {
    int j = ed_j(ed);
    return j == 0 ? lat0 : p.lat_lut[(j) * LAT_ROWS + (int)lat0];
}
__device__ __forceinline__ double cpu_of(const Params& p, uint32_t em, uint32_t ed) {
    return p.cpu_lut[(ed_m(ed)) * CPU_ROWS + em_c0(em)];
}
__device__ __forceinline__ double gini_of(uint64_t acc2, int acc, int E) {   // utils.py:132-143
    if (acc == 0) return 0.0;
    double num = (double)(uint32_t)(acc2 >> 32);
    return num / ((double)(2 * E * E) * ((double)acc / (double)E));
}

// get_reward() (:516-567) for an accepted request, float64, reference operation order
__device__ __forceinline__ double accept_reward(const Params& p, double sel_lat, int tl, double sel_cpu,
                                                uint64_t acc2, int acc) {
    switch (p.reward_fn) {
    case LB_REWARD_NAIVE: return 1.0;
    case LB_REWARD_LATENCY: return -(sel_lat + (double)tl);
    case LB_REWARD_FAIRNESS: return 1.0 - gini_of(acc2, acc, p.E);
    default: {
        double cur = ((sel_lat + (double)tl) - 2.0) / 998.0;  // normalize(., 2, 1000)
        double cpu = (sel_cpu - 1.0) / 99.0;                  // normalize(., 1, 100)
        double g = gini_of(acc2, acc, p.E);
        return p.lw * (1.0 - cur) + p.cw * (1.0 - cpu) + p.gw * (1.0 - g);
    }
    }
}

// ---- exact episode sums -------------------------------------------------------------
// The reference's per-episode means are statistics.mean over lists of float64 values
// (loadbalancer_k8s_env.py:451-454, :491-506): an exact rational sum, correctly rounded
// once.  Every listed value (endpoint latency in [1, 500], endpoint cpu in [1, 100], an
// updated topology latency fl(t * 1.7) in [1.7, 848.3]) is a float64 in [1, 1024), hence a
// multiple of 2^-52 below 2^62 * 2^-52: it is accumulated EXACTLY as a fixed-point integer
// fix52(x) = x * 2^52.  Episodes hold at most 1023 accepts (the history counters' range), so
//   latency: lo u64 + 7 carry bits   (sum < 1023 * 500 * 2^52 < 2^71)
//   cpu:     lo u64 + 5 carry bits   (sum < 1023 * 100 * 2^52 < 2^69)
// and the updated topology sum needs no 64-bit word at all: with M = fix52(1.7) each term
// is t * M - d(t), d(t) = t * M - fix52(fl(t * 1.7)) in [-202, 246] for t in [1, 499], so
// the sum is intra * 2^52 + M * (sum_topo - intra) - D with D = sum of d, |D| < 2^18.
// The carry word packs  lat carries [0,7) | cpu carries [7,12) | D (two's complement) [12,32).
constexpr uint64_t FIX_17 = 7656119366529843ull;  // fix52(1.7) = fl(1.7) * 2^52
constexpr int XH_CPU = 7, XH_D = 12;

__device__ __forceinline__ uint64_t fix52(double x) {  // x in [1, 1024): x * 2^52, exactly
    const uint64_t b = (uint64_t)__double_as_longlong(x);
    const int e = (int)(b >> 52) - 1023;
    return ((b & 0x000fffffffffffffull) | 0x0010000000000000ull) << e;
}
// one accepted request's appends (:626-632): latency and cpu of the selected endpoint; an
// inter-zone request's updated topology latency fl(tl * 1.7) adds its residual d(tl) to D
__device__ __forceinline__ void xsum_add(uint64_t& lat, uint64_t& cpu, uint32_t& hi, double sel_lat,
                                         double sel_cpu, int tl, bool inter) {
    const uint64_t fl = fix52(sel_lat), fc = fix52(sel_cpu);
    lat += fl;
    cpu += fc;
    uint32_t h = hi + (lat < fl ? 1u : 0u) + (cpu < fc ? (1u << XH_CPU) : 0u);
    if (inter) h += (uint32_t)((uint64_t)tl * FIX_17 - fix52((double)tl * 1.7)) << XH_D;
    hi = h;
}
// the exact sum (carries * 2^64 + lo) * 2^-52 as an unevaluated pair: s = the correctly
// rounded float64 sum, r = the exact remainder (sum = s + r as rationals)
__device__ __forceinline__ void xsum_pair(uint64_t lo, uint32_t carries, double& s, double& r) {
    const double xh = (double)carries * 0x1p64 + (double)(uint32_t)(lo >> 32) * 0x1p32;
    const double xl = (double)(uint32_t)lo;  // xh: <= 39 significant bits, exact
    const double sum = xh + xl;              // one rounding
    const double rem = xl - (sum - xh);      // Fast2Sum: xh is 0 or a multiple of 2^32 > xl
    s = sum * 0x1p-52;  // exact scaling
    r = rem * 0x1p-52;
}

// ep_stats row (include/lbk8s.h LB_ST_*) from the accumulators
__device__ __forceinline__ void write_stats_row(const Params& p, double* out, const Scal& s, uint64_t acc2,
                                                uint64_t acc3, double total, uint64_t sum_lat,
                                                uint64_t sum_cpu, uint32_t sum_hi) {
    uint32_t sum_topo = (uint32_t)acc2;
    double ls, lr, cs, cr;
    xsum_pair(sum_lat, sum_hi & 0x7Fu, ls, lr);
    xsum_pair(sum_cpu, (sum_hi >> XH_CPU) & 0x1Fu, cs, cr);
    out[LB_ST_RETURN] = total;
    out[LB_ST_LENGTH] = (double)s.step;
    out[LB_ST_ACCEPTED] = (double)s.acc;
    out[LB_ST_SUM_LATENCY] = ls;
    out[LB_ST_SUM_TOPOLOGY] = (double)sum_topo;
    // intra-zone accepts see topology 1 (updated 1); inter ones topology * 1.7 (:582-593)
    // (float64 approximation; the exact sum comes with LB_ST_SUM_TOPOLOGY_UPDATED_D)
    out[LB_ST_SUM_TOPOLOGY_UPDATED] = (double)s.intra + 1.7 * (double)(sum_topo - (uint32_t)s.intra);
    out[LB_ST_SUM_COST] = (double)(uint32_t)acc3;
    out[LB_ST_SUM_CPU] = cs;
    out[LB_ST_INTRA] = (double)s.intra;
    out[LB_ST_INTER] = (double)(s.acc - s.intra);
    out[LB_ST_GINI] = gini_of(acc2, s.acc, p.E);
    out[LB_ST_EPISODE] = (double)(uint32_t)(acc3 >> 32);
    out[LB_ST_SUM_LATENCY_REM] = lr;
    out[LB_ST_SUM_CPU_REM] = cr;
    out[LB_ST_SUM_TOPOLOGY_UPDATED_D] = (double)((int32_t)sum_hi >> XH_D);
    out[LB_ST_K - 1] = 0.0;
}

}  // namespace lbk
