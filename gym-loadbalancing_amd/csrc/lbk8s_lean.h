// lbk8s_lean.h — k_rollout_lean: lb_rollout on the thread-per-env layout for the bench's and
// config 1's launches (E = 8 / R = 9 with N <= 32 and E = 6 / R = 7 with N <= 64, episodes at
// least as long as the launch, whole waves of 64 envs, every output written).
//
// k_rollout_img's step (lbk8s_rollout.h: one lane per env for the whole launch, the 40-word
// LDS image of the observation rows, the next episodes drawn before the first step),
// re-laid around one rule of the memory pipeline (MI355X_MICROARCH.md):
//
//   s_waitcnt vmcnt(N) retires a wave's vector-memory operations in ISSUE order, stores
//   included, so the data of a load waits for every store its wave issued before it.
//
// A step stores ~19 KB per wave (obs block, rewards, done flags).  Every load of the loop is
// therefore issued BEFORE the stores it would otherwise wait behind:
//   * step k + 1's 4 table gathers right after its action, step k's obs / reward / done /
//     action stores after them (spread over step k + 1's request draws), and the gathers
//     waited for at the end of that step (a counted vmcnt behind the step's own stores);
//   * the record of an env that ends at step k + 1 (the next episode, drawn before the first
//     step) is fetched in iteration k, next to the gathers: 10 lanes x 16 bytes per env, one
//     unconditional load instruction for up to FAST envs, landing in 4 registers per lane; at
//     its end the wave drops it into the env's own image region and the env restarts from
//     there, in place;
//   * the terminal observations leave as one store per group of 64 / 2R envs (lane = piece),
//     the groups' episode-statistics rows as one store per group, staged in LDS.
// Addresses are scalar buffer descriptors plus 32-bit lane offsets (raw buffer
// instructions): no 64-bit per-lane address lives in a register, and the compiler cannot
// strength-reduce the per-step output addresses into per-lane pointers.  Every 16-byte
// store has soffset 0 (buf_st_f4: an SGPR soffset is unsafe on gfx950, see there).
// Compile-time E, R, node-zone words and reward kind keep registers and SGPRs down; empty
// asm statements launder values the compiler would hoist out of the step loop and spill.
// The record layout is this kernel's own (lean_write_record: scenario words first, the
// initial latencies last, so the in-place restart never overwrites a word it still needs).
// Bit for bit K x (lb_policy + lb_step) and the C oracle (tests/test_gpu_lean.py,
// tests/test_gpu_api.py, tests/test_gpu_parity.py): the same draws and float64 operations
// in the same order.
#pragma once

#include "lbk8s_rollout.h"

namespace lbk {

typedef __amdgpu_buffer_rsrc_t Rsrc;
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// raw buffer descriptor over [base, base + 4 GiB): stride 0, gfx9 data format word
__device__ __forceinline__ Rsrc rsrc_of(const void* base) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, -1, 0x00020000);
}
// the output stores' cache policy: nontemporal (gfx940+: sc0 = 1, nt = 2, sc1 = 16; nt sc1, sc1 and
// plain stores measured slower at 2^20 envs, profiles/r05_ab_store_policy.jsonl)
constexpr int BUF_NT = 2;

// Hoisting guards of the step loop.  At 4 waves per SIMD (128 VGPRs) loop-invariant values the
// compiler hoists out of the step loop spill, so they are laundered through empty asm and
// recomputed per step.
#define LB_GUARD_S(...) asm volatile("" : "+s"(__VA_ARGS__))
#define LB_GUARD_V(...) asm volatile("" : "+v"(__VA_ARGS__))

__device__ __forceinline__ double buf_ld_f64(Rsrc r, uint32_t off) {
    return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0));
}
__device__ __forceinline__ uint4 buf_ld_u128(Rsrc r, uint32_t off) {
    const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
    return make_uint4(v.x, v.y, v.z, v.w);
}
// 16-byte stores with every offset in the lane's VGPR and soffset 0.  An SGPR soffset is not
// safe on gfx950: the compiler's hazard recognizer treats such a store's data registers as free
// once it has issued (its >64-bit store-data rule excludes that form), and under load an f64
// VALU write several instructions later still changed the stored data of a quarter of the lanes
// (lanes 12-15 of every 16; 16 wait states did not help, soffset 0 or a global store did)
template <int AUX>
__device__ __forceinline__ void buf_st_f4(float4 v, Rsrc r, uint32_t voff) {
    const u32x4 d{__float_as_uint(v.x), __float_as_uint(v.y), __float_as_uint(v.z), __float_as_uint(v.w)};
    __builtin_amdgcn_raw_buffer_store_b128(d, r, voff, 0, AUX);
}

// draw() with the Philox key laundered through an opaque copy: the 10 rounds' keys are then
// recomputed by 2 scalar adds per round in every call instead of being hoisted out of the step
// loop as 20 SGPRs (which spilled, and were read back with v_readlane in every round)
__device__ __forceinline__ U4 draw_o(const Params& p, int64_t env, uint32_t episode, uint32_t slot, uint32_t dom) {
    uint32_t k0 = p.key0, k1 = p.key1;
    LB_GUARD_S(k0);
    LB_GUARD_S(k1);
    const uint64_t gid = (uint64_t)(p.env_id_offset + env);
    // (the counter words too: their loop-invariant parts, hoisted per draw domain, spilled)
    uint32_t c0 = (uint32_t)gid, hi = (uint32_t)(gid >> 32) << 8;
    LB_GUARD_V(c0);
    LB_GUARD_V(hi);
    return philox(c0, episode, slot, dom | hi, k0, k1);
}
// two blocks with one key schedule (the request's X and I blocks of a step: same counter but
// the domain word): the 10 rounds' key additions are issued once for both, and the two
// independent chains interleave.  Each block equals draw_o's.
__device__ __forceinline__ void draw2_o(const Params& p, int64_t env, uint32_t episode, uint32_t slot, uint32_t dom_a,
                                        uint32_t dom_b, U4& a, U4& b) {
    uint32_t k0 = p.key0, k1 = p.key1;
    LB_GUARD_S(k0);
    LB_GUARD_S(k1);
    const uint64_t gid = (uint64_t)(p.env_id_offset + env);
    uint32_t c0 = (uint32_t)gid, hi = (uint32_t)(gid >> 32) << 8;
    LB_GUARD_V(c0);
    LB_GUARD_V(hi);
    uint32_t a0 = c0, a1 = episode, a2 = slot, a3 = dom_a | hi;
    uint32_t b0 = c0, b1 = episode, b2 = slot, b3 = dom_b | hi;
#pragma unroll
    for (int i = 0; i < LB_PHILOX_ROUNDS; ++i) {  // (philox()'s round, twice)
        const uint64_t pa0 = (uint64_t)0xD2511F53u * a0, pa1 = (uint64_t)0xCD9E8D57u * a2;
        const uint64_t pb0 = (uint64_t)0xD2511F53u * b0, pb1 = (uint64_t)0xCD9E8D57u * b2;
        const uint32_t na0 = (uint32_t)(pa1 >> 32) ^ a1 ^ k0, na2 = (uint32_t)(pa0 >> 32) ^ a3 ^ k1;
        const uint32_t nb0 = (uint32_t)(pb1 >> 32) ^ b1 ^ k0, nb2 = (uint32_t)(pb0 >> 32) ^ b3 ^ k1;
        a0 = na0; a1 = (uint32_t)pa1; a2 = na2; a3 = (uint32_t)pa0;
        b0 = nb0; b1 = (uint32_t)pb1; b2 = nb2; b3 = (uint32_t)pb0;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    a = {a0, a1, a2, a3};
    b = {b0, b1, b2, b3};
}

template <int KIND>
__device__ __forceinline__ int lean_policy(const Params& p, int64_t env, const TEnv& tv, const uint32_t (&em)[TPE_E],
                                           const uint32_t (&ed)[TPE_E]) {
    if constexpr (KIND == LB_POLICY_RANDOM) {  // random_action's draw
        const U4 w = draw_o(p, env, (uint32_t)(tv.acc3 >> 32), (uint32_t)tv.s.step, D_ACT);
        return (int)bounded(w.x, (uint32_t)p.A);
    }
    return tpe_policy<KIND>(p, env, tv, em, ed);
}

// topology latency between zones a and b (topo_val), branch-free
__device__ __forceinline__ int topo_bf(uint64_t topo, int a, int b) {
    const int i = a < b ? a : b, j = a < b ? b : a;
    const int val = (int)((topo >> (9 * ((i * (7 - i)) / 2 + j - i - 1))) & 0x1FF);
    return a == b ? 1 : val;
}

// the next step, prepared: its action with the request's threshold index and zone packed
// in one word (a | thr_idx << 8 | rz << 12; the on-device policies draw a in [0, A)), the
// selected endpoint's 4 table values, and next_request()'s clock already advanced (arrival
// and dt from the clock the step will see: nothing changes it in between)
struct LPrepL {
    uint32_t arz;  // a | thr_idx << 8 | rz << 12 | owner(a) << 14 | zone(a) << 17 | type(a) << 19
    uint32_t jm;   // loads: j(a) | M(owner) + 1 (capped) << 10 | M(a) << 20
    double sel_lat, sel_cpu, next_lat, next_cpu, arr;
    float dt;
};

// lean_apply with the packed preparation (the same operations in the same order)
template <int ET, int RT, int RF>
__device__ __forceinline__ double lean_apply_l(const Params& p, const LPrepL& pr, LEnv& v,
                                               const uint32_t (&em)[TPE_E], uint32_t (&ed)[TPE_E], uint32_t* me) {
    constexpr int E = ET;
    const int rf = RF >= 0 ? RF : p.reward_fn;
    const int a = (int)(pr.arz & 0xFFu);
    const bool accept = a < E, reject = a == E;
    const int ai = accept ? a : 0;
    if (!((v.s1 >> S1_RD) & 1)) v.s1 |= 1u << S1_BAD;
    // (the selected endpoint's fields as the preparation found them: nothing changed them since)
    const int oA = (int)((pr.arz >> 14) & 7u);
    const int jA = (int)(pr.jm & 0x3FFu), Mn = (int)((pr.jm >> 10) & 0x3FFu), MA = (int)(pr.jm >> 20);
    const int jn = jA < CMAX ? jA + 1 : CMAX;
    double reward;
    if (accept) {
        int cnt = 0;  // #{e != ai : loads[e] <= loads[ai]} for the O(E) Gini update
#pragma unroll
        for (int e = 0; e < TPE_E; ++e)
            if (e < E && e != ai && ed_j(ed[e]) <= jA) ++cnt;
        const int rz = (int)((v.s1 >> S1_RZ) & 3), zA = (int)((pr.arz >> 17) & 3u);
        const int tl = topo_bf(v.topo, rz, zA);
        const uint32_t gnum = (uint32_t)(v.acc2 >> 32) + (uint32_t)(2 * (2 * cnt - (E - 1)));
        v.acc2 = ((uint64_t)gnum << 32) | (uint32_t)((uint32_t)v.acc2 + (uint32_t)tl);
        v.acc3 += (uint64_t)node_cost((int)((pr.arz >> 19) & 7u));
        v.s0 += 1u << 16;                 // acc (<= step <= L <= 1023: no saturation)
        if (rz == zA) v.s1 += 1;          // intra
        xsum_add(v.sum_lat, v.sum_cpu, v.sum_hi, pr.sel_lat, pr.sel_cpu, tl, rz != zA);
        const uint32_t edA_new = ((oA == ai ? (uint32_t)Mn : (uint32_t)MA) << 20) |
                                 ((uint32_t)Mn << 10) | (uint32_t)jn;
#pragma unroll
        for (int e = 0; e < TPE_E; ++e) {  // select-stores over constant indices
            const uint32_t edo = e == oA ? (ed[e] & ~(0x3FFu << 20)) | ((uint32_t)Mn << 20) : ed[e];
            ed[e] = e == ai ? edA_new : edo;
        }
        img_sel(me, ai, (float)pr.next_cpu, (float)pr.next_lat);
        v.s1 &= ~(1u << S1_PEN);
        reward = rf == LB_REWARD_NAIVE ? 1.0 : accept_reward(p, pr.sel_lat, tl, pr.sel_cpu, v.acc2, (int)(v.s0 >> 16));
        v.last_r = reward;
    } else if (reject) {
        v.s1 |= 1u << S1_PEN;
        reward = rf == LB_REWARD_LATENCY ? -1000.0 : -1.0;
        v.last_r = reward;
    } else {  // unrecognised action (:685-686): penalty and selected_* stay stale
        reward = rf == LB_REWARD_NAIVE ? (((v.s1 >> S1_PEN) & 1) ? -1.0 : 1.0) : v.last_r;
    }
    v.total += reward;
    // next_request (:1131-1163), prepared
    v.dt = pr.dt;
    v.t = pr.arr;
    v.s1 = (v.s1 & ~((3u << S1_RZ) | (7u << S1_THR))) | (((pr.arz >> 12) & 3u) << S1_RZ) |
           (((pr.arz >> 8) & 7u) << S1_THR);
    img_request(me, v, em, E);
    return reward;
}

// ---- the lean record: RO_REC_BYTES = 160 per env in the state blob's record area ----------
//   words 0..7 emeta (em_pack) | 8,9 topo | 10,11 zcap | 12,13 nz0 | 14,15 nz1 | 16,17 x1 |
//   18,19 x2 | 20 thr_idx | rz << 8 | 21..23 - | 24..39 lat0 (f64) of endpoints 0..7
constexpr uint32_t LREC_LAT0 = 96;  // byte offset of lat0[0]
// after the restart (which reads the record into the image region), words 12..23 hold the ended
// episode's accumulators until the launch's end: total, acc2 | sum_lat, sum_cpu | cost (acc3's
// low word), sum_hi, s0, s1
constexpr uint32_t LREC_ACC = 12;
__device__ __forceinline__ float4 u4f(double a, uint64_t b) {
    const uint64_t x = (uint64_t)__double_as_longlong(a);
    return make_float4(__uint_as_float((uint32_t)x), __uint_as_float((uint32_t)(x >> 32)), __uint_as_float((uint32_t)b),
                       __uint_as_float((uint32_t)(b >> 32)));
}
__device__ __forceinline__ float4 u4f(uint64_t a, uint64_t b) {
    return make_float4(__uint_as_float((uint32_t)a), __uint_as_float((uint32_t)(a >> 32)), __uint_as_float((uint32_t)b),
                       __uint_as_float((uint32_t)(b >> 32)));
}

// reset()'s draws for one env (the same map and owner rule as tpe_write_record), 8 lanes.
// Each Philox block is drawn once per env: lane l draws nodes l, l + 8, ... (the first three
// of them, nodes < 24, packed and handed to the endpoint lanes whose host they are, instead of
// a second draw of the host node per endpoint), endpoint l, and ONE of the episode's four
// remaining blocks by its role: lanes 0 / 1 the request's X block (x1 / x2: one log each),
// lane 2 its I block, lanes 3 / 4 the topology blocks (8 Philox blocks per lane before: 5).
template <int W>
__device__ __forceinline__ void lean_write_record(const Params& p, int64_t env, uint32_t episode, int lane) {
    static_assert(W == 8, "eight lanes per record (the node packing covers nodes < 24 = 3 x 8)");
    uint64_t zc = 0, nz0 = 0, nz1 = 0;
    uint32_t hp01 = 0, hp2 = 0;  // this lane's nodes lane, lane + 8 (16 bits each), lane + 16: ty | zo << 3 | cpu << 5
    for (int w = 0; w < p.NZW; ++w) {  // nodes (:349-373)
        uint64_t word = 0;
        int j = 0;
        for (int n = 32 * w + lane; n < 32 * (w + 1) && n < p.N; n += W, ++j) {
            int ty, zo, cpu;
            node_draw<false>(p, env, episode, n, ty, zo, cpu);
            zc += (uint64_t)node_cpu_int(ty) << (16 * zo);
            word |= (uint64_t)zo << (2 * (n & 31));
            const uint32_t hp = (uint32_t)ty | ((uint32_t)zo << 3) | ((uint32_t)cpu << 5);
            if (w == 0 && j == 0) hp01 |= hp;
            if (w == 0 && j == 1) hp01 |= hp << 16;
            if (w == 0 && j == 2) hp2 = hp;
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
    // the host node's draws, from the lane that drew it (node n: lane n % 8, its (n / 8)-th draw)
    const uint32_t ha = shfl_u32<W>(hp01, node & 7), hb = shfl_u32<W>(hp2, node & 7);
    const uint32_t hp = (node >> 3) == 0 ? (ha & 0xFFFFu) : (node >> 3) == 1 ? (ha >> 16) : hb;
    uint32_t* out = reinterpret_cast<uint32_t*>(p.rec + env * (RO_REC_BYTES / 16));
    if (lane < p.E) {
        const int ty = (int)(hp & 7u), zo = (int)((hp >> 3) & 3u), cpu = (int)((hp >> 5) & 0x7Fu);
        const uint64_t lb = (uint64_t)__double_as_longlong(lat0);
        *reinterpret_cast<uint2*>(out + 24 + 2 * lane) = make_uint2((uint32_t)lb, (uint32_t)(lb >> 32));
        out[lane] = em_pack(zo, owner, ty, cpu, node);
    }
    // the topology (:331-338) and next_request() closing reset() (:397): one block per lane
    const int role = lane;
    const U4 w = draw(p, env, episode, role == 4 ? 1u : 0u,
                      role == 2 ? D_REQ_I : (role == 3 || role == 4) ? D_TOPO : D_REQ_X);
    const double e = role == 1 ? std_exp(w.z, w.w) : std_exp(w.x, w.y);
    const double x1 = p.inv_rate * shfl_f64<W>(e, 0), x2 = p.call * shfl_f64<W>(e, 1);
    const int r = (int)bounded(shfl_u32<W>(w.x, 2), 7), n = (int)bounded(shfl_u32<W>(w.y, 2), (uint32_t)p.N);
    const uint32_t a0 = shfl_u32<W>(w.x, 3), a1 = shfl_u32<W>(w.y, 3), a2 = shfl_u32<W>(w.z, 3),
                   a3 = shfl_u32<W>(w.w, 3), b0 = shfl_u32<W>(w.x, 4), b1 = shfl_u32<W>(w.y, 4);
    if (lane == 0) {
        const uint64_t topo = (uint64_t)(1 + bounded(a0, 499)) | ((uint64_t)(1 + bounded(a1, 499)) << 9) |
                              ((uint64_t)(1 + bounded(a2, 499)) << 18) | ((uint64_t)(1 + bounded(a3, 499)) << 27) |
                              ((uint64_t)(1 + bounded(b0, 499)) << 36) | ((uint64_t)(1 + bounded(b1, 499)) << 45);
        const int rz = (int)(((n < 32 ? nz0 : nz1) >> (2 * (n & 31))) & 3);
        const uint64_t wd[6] = {topo, zc, nz0, nz1, (uint64_t)__double_as_longlong(x1),
                                (uint64_t)__double_as_longlong(x2)};
#pragma unroll
        for (int j = 0; j < 6; ++j)
            *reinterpret_cast<uint2*>(out + 8 + 2 * j) = make_uint2((uint32_t)wd[j], (uint32_t)(wd[j] >> 32));
        out[20] = (uint32_t)((r + 6) % 7) | ((uint32_t)rz << 8);
    }
}

// The next episodes of the envs in grp (<= 8 of them) from their records, staged (by the wave)
// in each env's own image region, rebuilt in place by the wave: 8 lanes per env build its
// endpoint rows (zone / capacity pair, initial cpu and latency) and its emeta register words
// (lem), and each env's own lane ("mine") loads its scalars and the lem words.  Words of the
// staged record: 0..7 emeta, 8..20 scalars, 24..39 lat0; the rows land on words 0..31 and the
// lem words on 32..39, which the env's lane then overwrites with the reject row and the
// request block (it reads them first).
template <int ET, int RT, int NG>  // NG: at most NG envs in grp (the ctz walk stops there)
__device__ __forceinline__ void lean_restart_group(const Params& p, const LDims<ET, RT>& d, uint32_t* wimg,
                                                   uint64_t grp, int lane, bool mine, LEnv& v,
                                                   uint32_t (&em)[TPE_E], uint32_t (&ed)[TPE_E], uint32_t* me) {
    // the scalars of each restarting env, by its own lane, before any row overwrites them
    if (mine) {
        const uint4* q = reinterpret_cast<const uint4*>(me);
        const uint4 s0 = q[2], s1 = q[3], s2 = q[4];
        const uint32_t s3 = me[20];
        v.topo = (uint64_t)s0.x | ((uint64_t)s0.y << 32);
        v.zcap = (uint64_t)s0.z | ((uint64_t)s0.w << 32);
        v.nz0 = (uint64_t)s1.x | ((uint64_t)s1.y << 32);
        v.nz1 = (uint64_t)s1.z | ((uint64_t)s1.w << 32);
        const uint32_t episode = (uint32_t)(v.acc3 >> 32) + 1;
        v.acc3 = (uint64_t)episode << 32;
        v.acc2 = 0;
        v.sum_lat = 0;
        v.sum_cpu = 0;
        v.sum_hi = 0;
        v.total = 0.0;
        v.last_r = p.init_last_r;
        v.s0 = 0;  // step, acc
        // intra 0, penalty 0, reset_done 1, bad kept (the status word)
        v.s1 = (v.s1 & (1u << S1_BAD)) | (1u << S1_RD) | ((s3 & 7u) << S1_THR) | (((s3 >> 8) & 3u) << S1_RZ);
        const double x1 = __longlong_as_double((long long)((uint64_t)s2.x | ((uint64_t)s2.y << 32)));
        const double x2 = __longlong_as_double((long long)((uint64_t)s2.z | ((uint64_t)s2.w << 32)));
        const double arrival = v.t + x1;
        const double departure = arrival + x2;
        v.dt = (float)(departure - arrival);
        v.t = arrival;
    }
    // endpoint e of the g-th env of grp on lane 8 g + e
    const int e = lane & 7, g = lane >> 3;
    int el = -1;
    {
        uint64_t m = grp;
#pragma unroll
        for (int i = 0; i < NG; ++i) {
            const int b = m ? (int)__builtin_ctzll(m) : -1;
            if (g == i) el = b;
            m &= m - 1;
        }
    }
    const bool helper = el >= 0 && e < ET;
    uint32_t* ri = wimg + (el < 0 ? 0 : el) * IMG_W;
    uint32_t mw = 0, l0lo = 0, l0hi = 0, zlo = 0, zhi = 0;
    if (helper) {
        mw = ri[e];
        l0lo = ri[24 + 2 * e];
        l0hi = ri[25 + 2 * e];
        zlo = ri[10];
        zhi = ri[11];
    }
    wave_lds_sync();  // (every read of the staged records is back before the first row is written)
    if (helper) {
        const double l0 = __longlong_as_double((long long)((uint64_t)l0lo | ((uint64_t)l0hi << 32)));
        const int z = em_zone(mw);
        const uint64_t zcap = (uint64_t)zlo | ((uint64_t)zhi << 32);
        // (the row's topology word is written with the request block below)
        *reinterpret_cast<uint4*>(ri + 4 * e) =
            make_uint4(img_zc(z, zcap_val(zcap, z)), 0u, __float_as_uint((float)em_c0(mw)), __float_as_uint((float)l0));
        ri[32 + e] = lem_make(mw, l0);  // table rows 0: the initial values
    }
    wave_lds_sync();
    if (mine) {
        const uint4 a = *reinterpret_cast<const uint4*>(me + 32), b = *reinterpret_cast<const uint4*>(me + 36);
        const uint32_t lw[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
        for (int i = 0; i < TPE_E; ++i) {
            em[i] = i < ET ? lw[i] : 0u;
            ed[i] = 0u;
        }
        *reinterpret_cast<uint4*>(me + 4 * d.E) = make_uint4(IMG_ZC_REJECT, F32_M1, F32_M1, F32_M1);
        img_request(me, v, em, d.E);
    }
}

// lane -> (env, record chunk) of the record fetch: lanes 10 i .. 10 i + 9 fetch the record
// of the i-th lowest env of m (i < NJ <= 6: the callers' groups hold at most NJ envs);
// returns the env's lane or -1
template <int NJ>
__device__ __forceinline__ int rec_fetch_env(uint64_t m, int lane, int& chunk) {
    static_assert(NJ <= 6, "64 lanes: 6 records of 10 chunks");
    const int i = lane / 10;
    chunk = lane - 10 * i;
    int el = -1;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
        const int b = m ? (int)__builtin_ctzll(m) : -1;
        if (i == j) el = b;
        m &= m - 1;
    }
    return el;
}
constexpr int REC_FETCH_MAX = 6;

// the ep_stats row's inputs (write_stats_row's accumulators)
struct Acc {
    double total;
    uint64_t acc2, acc3, sum_lat, sum_cpu;
    uint32_t sum_hi, s0, s1;
};
// the ep_stats row (write_stats_row's values, the LB_ST_* column order) into the lane's LDS
// image region, 16 doubles = words 0..31
template <int ET>
__device__ __forceinline__ void stats_row_lds(uint32_t* me, const Acc& a) {
    static_assert(LB_ST_RETURN == 0 && LB_ST_LENGTH == 1 && LB_ST_ACCEPTED == 2 && LB_ST_SUM_LATENCY == 3 &&
                      LB_ST_SUM_TOPOLOGY == 4 && LB_ST_SUM_TOPOLOGY_UPDATED == 5 && LB_ST_SUM_COST == 6 &&
                      LB_ST_SUM_CPU == 7 && LB_ST_INTRA == 8 && LB_ST_INTER == 9 && LB_ST_GINI == 10 &&
                      LB_ST_EPISODE == 11 && LB_ST_SUM_LATENCY_REM == 12 && LB_ST_SUM_CPU_REM == 13 &&
                      LB_ST_SUM_TOPOLOGY_UPDATED_D == 14 && LB_ST_K == 16,
                  "ep_stats column order");
    const Scal s = sc_unpack((uint64_t)a.s0 | ((uint64_t)a.s1 << 32));
    const uint32_t sum_topo = (uint32_t)a.acc2;
    auto put = [&](int i, double x, double y) {
        const uint64_t lo = (uint64_t)__double_as_longlong(x), hi = (uint64_t)__double_as_longlong(y);
        *reinterpret_cast<uint4*>(me + 4 * i) = make_uint4((uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32));
    };
    double ls, lr, cs, cr;
    put(0, a.total, (double)s.step);
    xsum_pair(a.sum_lat, a.sum_hi & 0x7Fu, ls, lr);
    put(1, (double)s.acc, ls);
    put(2, (double)sum_topo, (double)s.intra + 1.7 * (double)(sum_topo - (uint32_t)s.intra));
    xsum_pair(a.sum_cpu, (a.sum_hi >> XH_CPU) & 0x1Fu, cs, cr);
    put(3, (double)(uint32_t)a.acc3, cs);
    put(4, (double)s.intra, (double)(s.acc - s.intra));
    put(5, gini_of(a.acc2, s.acc, ET), (double)(uint32_t)(a.acc3 >> 32));
    put(6, lr, cr);
    put(7, (double)((int32_t)a.sum_hi >> XH_D), 0.0);
}
// the i-th lowest set bit of m (i < 8), or -1
__device__ __forceinline__ int nth_env8(uint64_t m, int i) {
    int el = -1;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int b = m ? (int)__builtin_ctzll(m) : -1;
        if (i == j) el = b;
        m &= m - 1;
    }
    return el;
}
__device__ __forceinline__ u32x4 lds_u4(const uint32_t* a) {
    const uint4 q = *reinterpret_cast<const uint4*>(a);
    return u32x4{q.x, q.y, q.z, q.w};
}

// one group of terminal observations: lane l reads piece l % P of env l / P of the group
// (the (l / P)-th lowest set bit of m), or -1 / nothing for lanes past the group
template <int P>
__device__ __forceinline__ int term_group_env(uint64_t m, int lane) {
    constexpr int G = 64 / P;
    const int g = lane / P;
    int el = -1;
#pragma unroll
    for (int i = 0; i < G; ++i) {
        const int b = m ? (int)__builtin_ctzll(m) : -1;
        if (g == i) el = b;
        m &= m - 1;
    }
    return el;
}
template <int P>
__device__ __forceinline__ uint64_t drop_low(uint64_t m) {  // m without its G = 64 / P lowest bits
#pragma unroll
    for (int i = 0; i < 64 / P; ++i) m &= m - 1;
    return m;
}
__device__ __forceinline__ float4 term_piece(const uint32_t* wimg, int el, int pc) {
    const char* base = reinterpret_cast<const char*>(wimg) + el * (IMG_W * 4);
    const uint4 A = *reinterpret_cast<const uint4*>(base + 16 * (pc >> 1));
    const uint4 S = *reinterpret_cast<const uint4*>(base + 4 * IMG_S);
    return img_piece(A, S, (pc & 1) != 0);
}

// piece 64 it + lane of the wave's obs block from its image: env e = piece / P by a multiply
// (exact below 64 P pieces), row = (piece - P e) / 2, half = lane parity (P, 64 it even):
//   row block at 160 e + 16 row = (160 - 8 P) e + 16 (32 it + lane / 2), request block at 160 e + 144
template <int P>
__device__ __forceinline__ float4 lean_piece(const uint32_t* wimg, int lane, int it, bool h) {
    constexpr uint32_t MAG = (65536u + P - 1) / P;
    static_assert(P % 2 == 0 && 64u * P * (MAG * P - 65536u) < 65536u, "piece / P by multiply, exact below 64 P");
    const uint32_t e = ((uint32_t)lane * MAG + (uint32_t)it * (64u * MAG)) >> 16;
    const char* b = reinterpret_cast<const char*>(wimg);
    const uint4 A = *reinterpret_cast<const uint4*>(b + e * (uint32_t)(IMG_W * 4 - 8 * P) + 16u * (uint32_t)(lane >> 1) +
                                                    512u * (uint32_t)it);
    const uint4 S = *reinterpret_cast<const uint4*>(b + e * (uint32_t)(IMG_W * 4) + 4u * IMG_S);
    return img_piece(A, S, h);
}

// per-wave timeline stamps: diagnostic builds only (-DLB_TIMELINE: tools/diag, tools/timeline_lean.py)
#ifdef LB_TIMELINE
#include "../../tools/diag/lbk8s_lean_timeline.h"
#else
#define LB_LTL(k, i) ((void)0)
#define LB_LTL_HDR(slot) ((void)0)
#define LB_LTL_HWID() ((void)0)
#endif

// One wave per block: a block's LDS and wave slot are released the moment its wave ends, so
// the next wave starts there at once (with 4-wave blocks a finished wave's slot waited for its
// three siblings: 74 % of the wave slots were in use over a 20-step launch)
constexpr int LEAN_NB = 64;

// The split layout (CW = 1: k_rollout_lean_split, lb_rollout's launches of at most
// LEAN_SPLIT_MAX_K steps): each block pairs the env wave with a copy wave.  The env wave never
// issues an observation store: at each step it leaves the step's reward / done (/ action)
// words next to its image and meets the copy wave at two LDS-only barriers, A (image and words
// ready) and B (the copy wave has read them into its registers); between them it prepares the
// next step.  The copy wave then issues the step's obs block, reward and done stores while the
// env wave computes.  (The env work alone runs 26-30 us per step at 2^20 envs, the store stream
// alone 46-55, the two in one wave 63-66; split, the env waves are half as many per SIMD, and
// the 20-step launch gains 3-4%, the 100-step one loses 1-2%: profiles/r05_ab_split.jsonl.)
// Round 6: the copy wave also draws every step's Philox blocks one step ahead -- the random
// policy's action and the next request's X / I blocks with their two float64 logs, a third of
// the env wave's per-step chain -- and hands them over in LDS (split_draws); the env wave's
// preparation reads them.  The copy wave replays the env's step count and episode itself (an
// env ends at most once in a launch, L >= K, at step count L).  Bit for bit the same draws
// (tests/test_gpu_lean_oracle.py); 131,072 envs 9.21 -> 8.86 us per step (profiles/r06_ab_*).
// the split layout's draw buffers (after the reward / done / action words in sstage): per step
// parity b, 64 x1 and 64 x2 (f64) and 64 words a | r << 8 | n << 16 (byte offsets from sstage)
constexpr uint32_t SD_BASE = 3 * 64 * 4, SD_BUF = 64 * 20, SD_X2 = 64 * 8, SD_W = 64 * 16;
__device__ __forceinline__ double* sd_x1(uint32_t* sst, int b) {
    return reinterpret_cast<double*>(reinterpret_cast<char*>(sst) + SD_BASE + b * SD_BUF);
}
__device__ __forceinline__ double* sd_x2(uint32_t* sst, int b) { return sd_x1(sst, b) + 64; }
__device__ __forceinline__ uint32_t* sd_w(uint32_t* sst, int b) {
    return reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(sst) + SD_BASE + b * SD_BUF + SD_W);
}
// the draws of one env's next step (prep's, lbk8s_lean.h): the random policy's action at slot
// cs, the request's X and I blocks at slot cs + 1 of episode ep -> the draw buffer
template <int KIND>
__device__ __forceinline__ void split_draws(const Params& p, int64_t env, uint32_t ep, uint32_t cs, uint32_t* sst,
                                            int b, int lane) {
    uint32_t a = 0;
    if constexpr (KIND == LB_POLICY_RANDOM) a = bounded(draw_o(p, env, ep, cs, D_ACT).x, (uint32_t)p.A);
    U4 wx, wi;
    draw2_o(p, env, ep, cs + 1, D_REQ_X, D_REQ_I, wx, wi);
    sd_x1(sst, b)[lane] = p.inv_rate * std_exp(wx.x, wx.y);
    sd_x2(sst, b)[lane] = p.call * std_exp(wx.z, wx.w);
    sd_w(sst, b)[lane] = a | (bounded(wi.x, 7) << 8) | (bounded(wi.y, (uint32_t)p.N) << 16);
}

template <int P, bool ACT, int CW, int KIND>
__device__ __forceinline__ void lean_copier(const Params& p, int K, int32_t* act_out, uint32_t (*simg)[64 * IMG_W],
                                            uint32_t* sst, int64_t env0) {
    const int lane = threadIdx.x & 63;
    const bool h = (lane & 1) != 0;
    uint32_t cs = 0, cep = 0;  // the env's step count and episode before the next step (split_draws)
    // the next episodes of the block's envs that end inside the launch, into their records (the
    // env wave's prologue in the single-wave layout; here beside the env wave's state loads and
    // image): 8 lanes per record, 8 records per pass, then barrier P
#pragma unroll
    for (int c = 0; c < CW; ++c) {
        const int64_t env = env0 + 64 * c + lane;
        const uint64_t sc = p.sc[env], acc3 = p.acc3[env];
        cs = (uint32_t)(sc & 0xFFFF);
        cep = (uint32_t)(acc3 >> 32);
        const int to_done = p.L - (int)(sc & 0xFFFF);
        uint64_t mm = __ballot(to_done >= 1 && to_done <= K);
        const uint32_t epi = (uint32_t)(acc3 >> 32) + 1;
        const int g = lane / RS_W, gl = lane % RS_W;
        while (mm) {  // (wave-uniform)
            const int el = nth_env8(mm, g);
            const uint32_t ep = (uint32_t)__shfl((int)epi, el < 0 ? 0 : el);
            if (el >= 0) lean_write_record<RS_W>(p, env0 + 64 * c + el, ep, gl);
#pragma unroll
            for (int j = 0; j < 8; ++j) mm &= mm - 1;
        }
    }
    split_draws<KIND>(p, env0 + lane, cep, cs, sst, 0, lane);  // step 0's
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (the records are written before P)
    block_lds_sync();  // P
    for (int k = 0; k < K; ++k) {
        // the env after step k (an env ends at most once in the launch, L >= K: restart at L),
        // then step k + 1's draws into buffer (k + 1) & 1 (its last reader, the env wave's
        // preparation of step k - 1, finished before barrier B of step k - 2 / the prologue)
        if (++cs == (uint32_t)p.L) {
            cs = 0;
            ++cep;
        }
        if (k + 1 < K) split_draws<KIND>(p, env0 + lane, cep, cs, sst, (k + 1) & 1, lane);
        block_lds_sync();  // A: step k's images and words are in LDS
        float4 v[CW][P];
        uint32_t rw[CW], dn[CW], ac[CW];
#pragma unroll
        for (int c = 0; c < CW; ++c) {
#pragma unroll
            for (int it = 0; it < P; ++it) v[c][it] = lean_piece<P>(simg[c], lane, it, h);
            rw[c] = sst[192 * c + lane];
            dn[c] = sst[192 * c + 64 + lane];
            ac[c] = ACT ? sst[192 * c + 128 + lane] : 0u;
        }
        block_lds_sync();  // B: read (the env waves may rewrite them)
        const Rsrc out = rsrc_of(p.obs + (int64_t)k * p.B * (P / 2) * 8);
        const Rsrc rwo = rsrc_of(p.reward + (int64_t)k * p.B), dno = rsrc_of(p.done + (int64_t)k * p.B);
#pragma unroll
        for (int c = 0; c < CW; ++c) {
            const uint32_t envi = (uint32_t)(env0 + 64 * c + lane);
            const uint32_t obs_wave = (uint32_t)((env0 + 64 * c) * P * 16);
#pragma unroll
            for (int it = 0; it < P; ++it)
                buf_st_f4<BUF_NT>(v[c][it], out, (uint32_t)lane * 16u + obs_wave + 1024u * (uint32_t)it);
            __builtin_amdgcn_raw_buffer_store_b32(rw[c], rwo, envi * 4u, 0, BUF_NT);
            __builtin_amdgcn_raw_buffer_store_b8((uint8_t)dn[c], dno, envi, 0, BUF_NT);
            if (ACT) __builtin_amdgcn_raw_buffer_store_b32(ac[c], rsrc_of(act_out + (int64_t)k * p.B), envi * 4u, 0, 0);
        }
    }
}

// (the LDS arrays are the kernels': LDS declared in a device function is lowered as
// module-level, and the compiler then assumes occupancy 1 and spends registers accordingly)
template <int KIND, int ET, int RT, int NZW, bool NAIVE, bool ACT, int CW>
__device__ __forceinline__ void lean_body(Params p, int K, int32_t* act_out, uint32_t (*simg)[64 * IMG_W],
                                          uint32_t* sstage) {
    static_assert(CW == 0 || CW == 1, "one env wave per copy wave (two: the copy wave's registers for both blocks spilled)");
    constexpr bool SPLIT = CW > 0;
    constexpr int NB = SPLIT ? 64 * (CW + 1) : LEAN_NB, NW = SPLIT ? CW : NB / 64, P = 2 * RT, GT = 64 / P;
    constexpr int FAST = GT < REC_FETCH_MAX ? GT : REC_FETCH_MAX;  // restarts per step of the fast path
    static_assert(ET >= 1 && ET <= TPE_E && (RT == ET || RT == ET + 1), "compile-time geometry");
    (void)NW;
    const LDims<ET, RT> d(p);
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    // block -> env group (blocks are dealt round-robin over the 8 XCDs; giving each XCD a
    // contiguous eighth of the groups measured within noise: profiles/r05_ab_xcd.jsonl)
    const int64_t blk = blockIdx.x;
    if constexpr (SPLIT) {
        if (wv == CW) {  // the copy wave (its block's env waves 0 .. CW - 1: envs blockIdx.x * 64 CW ..)
            lean_copier<P, ACT, CW, KIND>(p, K, act_out, simg, sstage, blk * 64 * CW);
            return;
        }
    }
    uint32_t* wimg = simg[wv];
    uint32_t* me = wimg + lane * IMG_W;
    // whole waves only (the host checks B % 64 == 0): every lane of a live wave is a live env,
    // and the waves past B in a partial last block leave (no block barrier follows: every
    // synchronisation below is within the wave; the split layout's blocks are whole)
    const int64_t env0 = blk * (SPLIT ? 64 * CW : NB) + __builtin_amdgcn_readfirstlane(threadIdx.x & ~63);
    if (env0 >= p.B) return;
    LB_LTL_HDR(2);
    LB_LTL_HWID();
    const int64_t env = env0 + lane;
    const uint32_t envi = (uint32_t)env;
    const Rsrc blob = rsrc_of(p.lat_lut);  // tables, lat0 array and records (blob < 4 GiB: host check)
    const uint32_t rec_off = (uint32_t)(reinterpret_cast<const char*>(p.rec) - reinterpret_cast<const char*>(p.lat_lut));
    const uint32_t cpu0 = (uint32_t)(reinterpret_cast<const char*>(p.cpu_lut) - reinterpret_cast<const char*>(p.lat_lut));

    // the state, issued first: its loads are in flight while the records below are drawn
    // (the step counter and the episode word first: the record list needs them)
    LEnv v;
    uint32_t em[TPE_E], ed[TPE_E];
    double l0s[TPE_E];
    {
        const uint64_t sc = p.sc[env];
        v.acc3 = p.acc3[env];
        v.s0 = (uint32_t)sc;
        v.s1 = (uint32_t)(sc >> 32);
#pragma unroll
        for (int e = 0; e < TPE_E; ++e) {
            em[e] = 0u;
            ed[e] = 0u;
            l0s[e] = 0.0;
            if (e < ET) {
                const int64_t i = (int64_t)e * p.B + env;
                l0s[e] = p.lat0[i];
                em[e] = p.emeta[i];  // (the raw emeta word until the records are drawn)
                ed[e] = p.edyn[i];
            }
        }
        v.t = p.t[env];
        v.zcap = p.zcap[env];
        v.acc2 = p.acc2[env];
        v.topo = p.topo[env];
        v.nz0 = p.nzone[env];
        // (the second node-zone word exists only when the config has more than 32 nodes: the
        // NZW = 2 instantiation also serves E = 6 configs with N <= 32, whose nzone array
        // holds one word per env)
        v.nz1 = NZW > 1 && p.NZW > 1 ? p.nzone[p.B + env] : 0;
        v.sum_lat = p.sum_lat[env];
        v.sum_cpu = p.sum_cpu[env];
        v.sum_hi = p.sum_hi[env];
        v.total = p.total[env];
        v.last_r = NAIVE ? 0.0 : p.last_r[env];
        v.dt = 0.f;
    }

    // the next episodes of the envs that end inside the launch, into their records (split
    // layout: the copy wave draws them)
    if constexpr (!SPLIT) {
        const int to_done = p.L - (int)(v.s0 & 0xFFFF);
        const bool fin = to_done >= 1 && to_done <= K;
        const uint64_t fm = __ballot(fin);
        if (fin) {
            uint32_t* it = wimg + 2 * __popcll(fm & ((1ull << lane) - 1));
            it[0] = (uint32_t)lane;
            it[1] = (uint32_t)(v.acc3 >> 32) + 1;
        }
        wave_lds_sync();
        const int nf = __popcll(fm), g = lane / RS_W, gl = lane % RS_W;
        for (int r0 = 0; r0 < nf; r0 += 64 / RS_W) {
            const int i = r0 + g;
            if (i < nf) lean_write_record<RS_W>(p, env0 + (int64_t)wimg[2 * i], wimg[2 * i + 1], gl);
        }
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    }
    LB_LTL_HDR(4);

    // the observation image from the state (table reads of the current latency and cpu)
    {
        float olat[TPE_E], ocpu[TPE_E];
#pragma unroll
        for (int e = 0; e < TPE_E; ++e) {
            olat[e] = 0.f;
            ocpu[e] = 0.f;
            if (e < ET) {
                const uint32_t m = em[e];
                em[e] = lem_make(m, l0s[e]);
                olat[e] = (float)lat_of(p, l0s[e], ed[e]);
                ocpu[e] = (float)cpu_of(p, m, ed[e]);
            }
        }
        img_endpoints(me, d, em, v.zcap, olat, ocpu);
    }

    // the state loads have landed (a wait the compiler sees: values it loaded before the
    // loop and uses on some paths only were otherwise still pending at the loop header,
    // where its wait for them drained the stores of the previous step)
    __builtin_amdgcn_s_waitcnt(0xF70);  // vmcnt(0)
    LB_LTL_HDR(5);
    bool new_episode = false;
    uint32_t l0off = (uint32_t)(reinterpret_cast<const char*>(p.lat0) - reinterpret_cast<const char*>(p.lat_lut)) +
                     envi * 8u;
    uint32_t l0step = (uint32_t)p.B * 8u;
    const uint32_t obs_wave = (uint32_t)(env0 * P * 16);  // byte offset of the wave's obs block in a slot

    // record prefetch of the envs that end at the next step (<= FAST of them: else the slow
    // path in the loop fetches them itself)
    uint4 qn = make_uint4(0u, 0u, 0u, 0u);
    // (one load in every step, on every lane: lanes without a record to fetch read the wave's
    // first record chunk, one cache line.  A conditional load merged into qn's register
    // through a copy, and the compiler drained the whole queue for that copy)
    auto fetch_next = [&](int steps_done) {
        const uint64_t mn = __ballot((int)(steps_done + 1) == p.L);
        int chunk, ln = lane;
        LB_GUARD_V(ln);  // (recomputed per step: hoisted, the lane's chunk and slot spilled)
        const int el = rec_fetch_env<FAST>(mn, ln, chunk);
        const uint32_t w0 = rec_off + (uint32_t)env0 * RO_REC_BYTES;
        qn = buf_ld_u128(blob, el >= 0 ? w0 + (uint32_t)el * RO_REC_BYTES + 16u * chunk : w0);
    };

    LPrepL pr;
    auto prep = [&](const int j, auto&& between) {
        (void)j;
        // the next step's action, its endpoint's 4 table gathers, the record prefetch, then the
        // request draws with the previous step's stores spread over between(0..5)
        LPrepL r;
        TEnv tv;
        tv.topo = v.topo;
        tv.zcap = v.zcap;
        tv.acc3 = v.acc3;
        tv.s.rz = (int)((v.s1 >> S1_RZ) & 3);
        const int step = (int)(v.s0 & 0xFFFF);
        tv.s.step = step;
        // (split layout: the copy wave drew this step's action and request one step ahead)
        const uint32_t dw = SPLIT ? sd_w(sstage, j & 1)[lane] : 0u;
        const int a = SPLIT && KIND == LB_POLICY_RANDOM ? (int)(dw & 0xFFu) : lean_policy<KIND>(p, env, tv, em, ed);
        const bool accept = a < ET;
        const int ai = accept ? a : 0;
        const uint32_t emA = pick8(em, ai), edA = pick8(ed, ai);
        const int oA = em_owner(emA);
        const uint32_t edO = pick8(ed, oA);
        const int jA = ed_j(edA);
        const int Mn = ed_M(edO) < CMAX ? ed_M(edO) + 1 : CMAX;
        const int jn = jA < CMAX ? jA + 1 : CMAX;
        const int k0A = lem_k0(emA), c0A = em_c0(emA);
        // selected_endpoint_latency: lat0 on a first selection (LAT row 0 holds trunc(lat0))
        r.sel_lat = buf_ld_f64(blob, jA == 0 ? l0off + (uint32_t)ai * l0step : (uint32_t)(jA * LAT_ROWS + k0A) * 8u);
        r.sel_cpu = buf_ld_f64(blob, cpu0 + (uint32_t)(ed_m(edA) * CPU_ROWS + c0A) * 8u);
        r.next_lat = buf_ld_f64(blob, (uint32_t)(jn * LAT_ROWS + k0A) * 8u);
        r.next_cpu = buf_ld_f64(blob, cpu0 + (uint32_t)(Mn * CPU_ROWS + c0A) * 8u);
        fetch_next(step);
        // (each stage's stores are pinned between computed values: "memory" barriers that
        // name the values just computed, so neither the compiler's IR passes nor its
        // scheduler can bunch the stores or sink the computation past them)
        asm volatile("" ::: "memory");
        between(0);
        asm volatile("" ::: "memory");
        double x1, x2;
        int rr, n;
        if constexpr (SPLIT) {
            x1 = sd_x1(sstage, j & 1)[lane];
            x2 = sd_x2(sstage, j & 1)[lane];
            rr = (int)((dw >> 8) & 0xFFu);
            n = (int)(dw >> 16);
        } else {
        const uint32_t episode = (uint32_t)(v.acc3 >> 32), slot = (uint32_t)(step + 1);
        U4 wx, wi;
        draw2_o(p, env, episode, slot, D_REQ_X, D_REQ_I, wx, wi);
        asm volatile("" ::"v"(wx.x), "v"(wx.y), "v"(wx.z), "v"(wx.w), "v"(wi.x), "v"(wi.y) : "memory");
        between(1);
        asm volatile("" ::: "memory");
        x1 = p.inv_rate * std_exp(wx.x, wx.y);
        asm volatile("" ::"v"(x1) : "memory");
        between(2);
        asm volatile("" ::: "memory");
        x2 = p.call * std_exp(wx.z, wx.w);
        rr = (int)bounded(wi.x, 7);
        n = (int)bounded(wi.y, (uint32_t)p.N);
        }
        // next_request()'s clock (:1135-1139): the same operations as at the step
        r.arr = v.t + x1;
        r.dt = (float)((r.arr + x2) - r.arr);
        asm volatile("" ::"v"(r.arr), "v"(r.dt) : "memory");
        between(3);
        asm volatile("" ::: "memory");
        const uint64_t word = (NZW > 1 && n >= 32) ? v.nz1 : v.nz0;
        const uint32_t rz = (uint32_t)((word >> (2 * (n & 31))) & 3);
        r.arz = (uint32_t)a | ((uint32_t)((rr + 6) % 7) << 8) | (rz << 12) | ((uint32_t)oA << 14) |
                ((uint32_t)em_zone(emA) << 17) | ((uint32_t)em_type(emA) << 19);
        r.jm = (uint32_t)jA | ((uint32_t)Mn << 10) | ((uint32_t)ed_M(edA) << 20);
        asm volatile("" ::"v"(r.arz) : "memory");
        between(4);
        asm volatile("" ::: "memory");
        between(5);
        return r;
    };
    if constexpr (SPLIT) block_lds_sync();  // P: the copy wave's records are written (the prefetch below reads them)
    pr = prep(0, [](int) {});
    // (its loads land here, before the loop: pending at the loop header, they made every
    // wait for the preparation's values inside the loop a vmcnt(0) or close to it)
    asm volatile("" : "+v"(pr.sel_lat), "+v"(pr.sel_cpu), "+v"(pr.next_lat), "+v"(pr.next_cpu), "+v"(qn.x), "+v"(qn.y),
                 "+v"(qn.z), "+v"(qn.w));

    // one step (k): apply, auto-reset, then step k + 1's preparation with step k's stores
    auto iter = [&](const int k) {
        LB_LTL(k, 0);
        // issue priority by progress (k_rollout_img): a wave behind the others goes first
        {
            const int pl = 3 - (4 * k) / K;
            if (pl >= 3) __builtin_amdgcn_s_setprio(3);
            else if (pl == 2) __builtin_amdgcn_s_setprio(2);
            else if (pl == 1) __builtin_amdgcn_s_setprio(1);
            else __builtin_amdgcn_s_setprio(0);
        }
        const int a_k = (int)(pr.arz & 0xFFu);
        v.s0 += 1;  // step (<= L: the episode ends there)
        const bool done = (int)(v.s0 & 0xFFFF) == p.L;  // (:472)
        const double reward = lean_apply_l<ET, RT, NAIVE ? (int)LB_REWARD_NAIVE : -1>(p, pr, v, em, ed, me);
        const uint64_t m = __ballot(done);
        LB_LTL(k, 1);
        if (m) {  // VecEnv auto-reset: episode stats + terminal obs, then the record's episode
            // (the stores below are younger than the prefetched record, so waiting for it does
            // not wait for them; the next gathers do, but a few 16-byte stores issued just
            // before them cost about nothing next to the gathers' own round trip)
            wave_lds_sync();  // (apply's image writes, read by other lanes below)
            // groups of up to FAST ending envs: their terminal observations (one store), their
            // records into their image regions (prefetched when the whole step is one group,
            // else loaded here: a block of its own, so the wait for the prefetched record stays
            // a counted vmcnt instead of a vmcnt(0) behind the stores above), the restarts in place
            const int pc = lane % P;
            bool pre = __popcll(m) <= FAST;
            for (uint64_t mm = m; mm;) {  // (wave-uniform)
                uint64_t grp = mm;
#pragma unroll
                for (int j = 0; j < FAST; ++j) mm &= mm - 1;
                grp &= ~mm;
                const int tel = term_group_env<P>(grp, lane);
                if (tel >= 0)
                    buf_st_f4<BUF_NT>(term_piece(wimg, tel, pc), rsrc_of(p.term_obs),
                                      (uint32_t)((env0 + tel) * P + pc) * 16u);
                const bool mine = done && ((grp >> lane) & 1);
                int chunk;
                const int rl = rec_fetch_env<FAST>(grp, lane, chunk);
                uint4* dst = reinterpret_cast<uint4*>(wimg + rl * IMG_W + 4 * chunk);
                wave_lds_sync();  // (the rows are read before the records overwrite them)
                if (pre) {
                    if (rl >= 0) *dst = qn;
                } else {
                    if (rl >= 0) *dst = buf_ld_u128(blob, rec_off + (uint32_t)(env0 + rl) * RO_REC_BYTES + 16u * chunk);
                }
                // the ended episode's accumulators, for its episode-statistics row at the launch's
                // end (an env ends at most once in a launch: L >= K), into words 12..23 of its
                // record, which only the restart reads (they are in the image region now)
                if (mine) {
                    const uint32_t o = rec_off + envi * RO_REC_BYTES + 4u * LREC_ACC;
                    buf_st_f4<0>(u4f(v.total, v.acc2), blob, o);
                    buf_st_f4<0>(u4f(v.sum_lat, v.sum_cpu), blob, o + 16u);
                    buf_st_f4<0>(make_float4(__uint_as_float((uint32_t)v.acc3), __uint_as_float(v.sum_hi),
                                             __uint_as_float(v.s0), __uint_as_float(v.s1)),
                                 blob, o + 32u);
                }
                wave_lds_sync();
                lean_restart_group<ET, RT, FAST>(p, d, wimg, grp, lane, mine, v, em, ed, me);
                if (mine) {
                    new_episode = true;
                    l0off = rec_off + envi * RO_REC_BYTES + LREC_LAT0;
                    l0step = 8u;
                }
                pre = false;
            }
        }
        LB_LTL(k, 2);
        if constexpr (SPLIT) {  // the copy wave stores step k's outputs
            sstage[192 * wv + lane] = __float_as_uint((float)reward);
            sstage[192 * wv + 64 + lane] = done ? 1u : 0u;
            if (ACT) sstage[192 * wv + 128 + lane] = (uint32_t)a_k;
            block_lds_sync();  // A
            LB_LTL(k, 3);
            if (k + 1 < K) {
                pr = prep(k + 1, [](int) {});
                asm volatile("" : "+v"(pr.sel_lat), "+v"(pr.sel_cpu), "+v"(pr.next_lat), "+v"(pr.next_cpu),
                             "+v"(qn.x), "+v"(qn.y), "+v"(qn.z), "+v"(qn.w));
            }
            LB_LTL(k, 4);
            block_lds_sync();  // B (the image and words are read)
            LB_LTL(k, 5);
            return;
        }
        // step k's outputs leave after step k + 1's gathers, spread over its request draws
        const Rsrc out = rsrc_of(p.obs + k * (int64_t)p.B * RT * 8);
        const Rsrc rw = rsrc_of(p.reward + (int64_t)k * p.B), dn = rsrc_of(p.done + (int64_t)k * p.B);
        wave_lds_sync();
        // copy-out by pieces: store instruction it writes float4s 64 it .. 64 it + 63 of the
        // wave's obs block (a piece = half a row: lane parity = half), fully coalesced (lanes
        // storing whole rows, 32 bytes apart, ran 2.3x slower)
        const bool h = (lane & 1) != 0;
        auto stores = [&](int stage) {
            if (stage == 0) {
                LB_LTL(k, 3);
                if (ACT) __builtin_amdgcn_raw_buffer_store_b32((uint32_t)a_k, rsrc_of(act_out + (int64_t)k * p.B),
                                                               envi * 4u, 0, 0);
                __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint((float)reward), rw, envi * 4u, 0, BUF_NT);
                __builtin_amdgcn_raw_buffer_store_b8((uint8_t)done, dn, envi, 0, BUF_NT);
            }
            constexpr int per = (P + PREP_STAGES - 1) / PREP_STAGES;
            // (the wave's base offset from an opaque copy: hoisted out of the step loop, the
            // per-store offsets were 2R SGPRs, spilled and read back with v_readlane per store)
            uint32_t so = obs_wave + 1024u * (uint32_t)(stage * per);
            LB_GUARD_S(so);
            int ln = lane;  // (opaque: the pieces' LDS addresses are loop-invariant, and hoisted they spilled)
            LB_GUARD_V(ln);
#pragma unroll
            for (int it = stage * per; it < (stage + 1) * per && it < P; ++it) {
                buf_st_f4<BUF_NT>(lean_piece<P>(wimg, ln, it, h), out,
                                  (uint32_t)ln * 16u + so + 1024u * (uint32_t)(it - stage * per));
            }
        };
        if (k + 1 < K) {
            pr = prep(k + 1, stores);
            LB_LTL(k, 4);
            // the loads land here, behind the step's stores (a counted wait), and the values
            // the next step reads are this statement's, not the loads': none is pending at the
            // loop header, where a merge of the paths made the compiler's wait a vmcnt(0)
            asm volatile("" : "+v"(pr.sel_lat), "+v"(pr.sel_cpu), "+v"(pr.next_lat), "+v"(pr.next_cpu), "+v"(qn.x),
                         "+v"(qn.y), "+v"(qn.z), "+v"(qn.w));
            LB_LTL(k, 5);
        } else {
            for (int s = 0; s < PREP_STAGES; ++s) stores(s);
        }
        wave_lds_sync();  // (the next step rewrites the image)
    };
    // (the first step is peeled off the loop: the loop is then entered, like its back edge,
    // with the gathers followed by a step's stores in flight, and the compiler's wait for
    // the gathers is a counted vmcnt instead of the vmcnt(0) the loop entry's shape forced)
    LB_LTL_HDR(0);
    if (K > 0) iter(0);
    for (int k = 1; k < K; ++k) iter(k);
    // (the write-back's addresses from an opaque copy of the env index: the compiler would
    // otherwise keep the launch start's 64-bit addresses alive across the loop)
    LB_LTL_HDR(1);
    // the episode-statistics rows of the envs that ended in the launch (write_stats_row's values),
    // from the accumulators their lanes saved at the restart: one pass for the wave, each lane
    // its row into its image region (the image is not read again), then 8 lanes (16 bytes each)
    // per 128-byte row, one store instruction per 8 envs
    {
        const uint64_t endm = __ballot(new_episode);
        if (endm) {
            if (new_episode) {
                const uint32_t o = rec_off + envi * RO_REC_BYTES + 4u * LREC_ACC;
                const uint4 q0 = buf_ld_u128(blob, o), q1 = buf_ld_u128(blob, o + 16u), q2 = buf_ld_u128(blob, o + 32u);
                auto u64 = [](uint32_t lo, uint32_t hi) { return (uint64_t)lo | ((uint64_t)hi << 32); };
                const uint64_t acc3 = ((uint64_t)((uint32_t)(v.acc3 >> 32) - 1u) << 32) | q2.x;  // (the ended episode)
                stats_row_lds<ET>(me, Acc{__longlong_as_double((long long)u64(q0.x, q0.y)), u64(q0.z, q0.w), acc3,
                                          u64(q1.x, q1.y), u64(q1.z, q1.w), q2.y, q2.z, q2.w});
            }
            wave_lds_sync();
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int el = 8 * i + (lane >> 3), c = lane & 7;
                if ((endm >> el) & 1)
                    __builtin_amdgcn_raw_buffer_store_b128(lds_u4(wimg + el * IMG_W + 4 * c), rsrc_of(p.ep_stats),
                                                           (uint32_t)(env0 + el) * (uint32_t)(8 * LB_ST_K) + 16u * (uint32_t)c,
                                                           0, 0);
            }
        }
    }
    int64_t ew = env;
    asm volatile("" : "+v"(ew));
#pragma unroll
    for (int e = 0; e < TPE_E; ++e)
        if (e < ET) p.edyn[(int64_t)e * p.B + ew] = ed[e];
    if (new_episode) {  // the scenario of the episode started in the launch, from its record
        const uint32_t* w = reinterpret_cast<const uint32_t*>(p.rec + ew * (RO_REC_BYTES / 16));
#pragma unroll
        for (int e = 0; e < TPE_E; ++e) {
            if (e >= ET) continue;
            const int64_t i = (int64_t)e * p.B + ew;
            p.lat0[i] = __longlong_as_double((long long)((uint64_t)w[24 + 2 * e] | ((uint64_t)w[25 + 2 * e] << 32)));
            p.emeta[i] = w[e];
        }
        p.topo[ew] = v.topo;
        p.zcap[ew] = (uint64_t)w[10] | ((uint64_t)w[11] << 32);
        p.nzone[ew] = v.nz0;
        if (NZW > 1 && p.NZW > 1) p.nzone[p.B + ew] = v.nz1;
    }
    p.t[ew] = v.t;
    p.sc[ew] = (uint64_t)v.s0 | ((uint64_t)v.s1 << 32);
    p.acc2[ew] = v.acc2;
    p.acc3[ew] = v.acc3;
    p.sum_lat[ew] = v.sum_lat;
    p.sum_cpu[ew] = v.sum_cpu;
    p.sum_hi[ew] = v.sum_hi;
    p.total[ew] = v.total;
    if (!NAIVE) p.last_r[ew] = v.last_r;
    LB_LTL_HDR(3);
}

template <int KIND, int ET, int RT, int NZW, bool NAIVE, bool ACT>
__global__ __launch_bounds__(LEAN_NB, 4) void k_rollout_lean(Params p, int K, int32_t* act_out) {
    __shared__ __attribute__((aligned(16))) uint32_t simg[LEAN_NB / 64][64 * IMG_W];
    lean_body<KIND, ET, RT, NZW, NAIVE, ACT, 0>(p, K, act_out, simg, nullptr);
}
// the split layout: 128-thread blocks (env wave + copy wave)
// (4 waves per SIMD: 128 VGPRs; 2 and 3 measured equal, profiles/r05_ab_occupancy.jsonl)
template <int KIND, int ET, int RT, int NZW, bool NAIVE, bool ACT, int CW>
__global__ __launch_bounds__(64 * (CW + 1), 4) void k_rollout_lean_split(Params p, int K,
                                                                                       int32_t* act_out) {
    __shared__ __attribute__((aligned(16))) uint32_t simg[CW][64 * IMG_W];
    // each env wave's step reward, done, action words; then the draw buffers
    __shared__ __attribute__((aligned(16))) uint32_t sstage[CW * 3 * 64 + 2 * SD_BUF / 4];
    lean_body<KIND, ET, RT, NZW, NAIVE, ACT, CW>(p, K, act_out, simg, sstage);
}

}  // namespace lbk
