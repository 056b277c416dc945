// lbk8s_rollout.h — lb_rollout on the thread-per-env layout (E <= 8, N <= 64) for episodes at
// least as long as the launch (L >= K: an env ends at most once per launch; the bench's
// L = 100 and config 1's): k_rollout_img.
//
// One lane = one env for all K steps of the launch, as k_rollout_tpe (lbk8s_tpe.h), laid out
// for occupancy.  k_rollout_tpe held the whole env in registers (178-190 VGPRs) and staged all
// 64 envs' rows in LDS every step (78 KB per block): two waves per SIMD, 2^20 envs in eight
// block generations.  Here (128 VGPRs, 40 KB per block: four waves per SIMD, four generations)
//   * the endpoints' initial latencies (16 VGPRs) are not held: a step needs lat0 only when
//     it selects an endpoint for the first time, and then gathers it (from the state's lat0
//     array, or from the episode's record for an episode started inside the launch) in the
//     same load as the table value it replaces; the table row trunc(lat0) lives in the emeta
//     register instead of the node id (lem layout below);
//   * the step / counters / flags are two 32-bit words (the state's sc), not 8 registers;
//   * the observed values (latency / cpu of every endpoint, zone capacities, dt, the request's
//     topology row) live in a compact per-env LDS image (40 words) that a step updates in 3
//     words, and the copy-out decodes the float4 pieces from it straight into full-line
//     stores (k_rollout_tpe built 18 float4 per env per step in registers and LDS);
//   * the records of the envs that end inside the launch are drawn before the env state is
//     loaded, and per-lane addresses are 32-bit offsets from uniform bases.
// Everything else is k_rollout_tpe's PRE path: the next episodes of the envs that end inside
// the launch are drawn before the first step into per-env records (tpe_write_record), the
// step that ends an episode starts the next one from its record, and the next step's action,
// table gathers and request draws are issued before the current step's rows are stored.
// Measured against k_rollout_tpe (tools/roll_variants.py, 2^20 staggered default envs,
// interleaved): see DESIGN.md §4.  At the bench's shapes lb_rollout now runs k_rollout_lean
// (lbk8s_lean.h); this kernel takes the other thread-per-env launches with L >= K.
// Tried and dropped (same file): each lane storing its own rows (scattered 16-byte
// nontemporal stores: 12x slower; plain stores 2x), half the pieces of every env per pass
// (144-byte runs: 1.7-2.8x slower), 32 envs' whole rows per pass (2 waves per SIMD: equal to
// k_rollout_tpe).
// Bit for bit K x (lb_policy + lb_step) and the C oracle (tests/test_gpu_api.py,
// tests/test_gpu_parity.py).
#pragma once

#include "lbk8s_common.h"
#include "lbk8s_slice.h"
#include "lbk8s_tpe.h"

namespace lbk {

#ifdef LB_TIMELINE
static __device__ uint64_t* g_timeline;  // [waves][K + 2] s_memrealtime (100 MHz) stamps, or NULL
#endif

// lem (the rollout's emeta register): zone[0:2) owner[2:10) type[10:13) c0[13:20) k0[20:29)
// with k0 = trunc(lat0), the endpoint's LAT row (the node id is not needed inside the launch)
__device__ __forceinline__ int lem_k0(uint32_t m) { return (int)(m >> 20); }
__device__ __forceinline__ uint32_t lem_make(uint32_t em, double lat0) {
    return (em & 0xFFFFFu) | ((uint32_t)(int)lat0 << 20);
}

// sc as two words: s0 = step | acc << 16, s1 = intra | rz << 16 | thr_idx << 18 |
// penalty << 21 | reset_done << 22 | bad << 23 (the high word of sc_pack's layout)
constexpr uint32_t S1_RZ = 16, S1_THR = 18, S1_PEN = 21, S1_RD = 22, S1_BAD = 23;

struct LEnv {
    double t, total, last_r;
    uint64_t acc2, acc3, topo, zcap, nz0, nz1;
    uint64_t sum_lat, sum_cpu;
    uint32_t sum_hi, s0, s1;
    float dt;
};

struct LPrep {
    int a;
    double sel_lat, sel_cpu, next_lat, next_cpu;
    double x1, x2;
    int r, n;
};

// base + a 32-bit byte offset: a uniform (SGPR) base and one offset VGPR per lane (the
// "saddr" global addressing form) instead of a 64-bit address pair per lane and pointer
template <typename T>
__device__ __forceinline__ T* at(T* base, uint32_t byte_off) {
    return reinterpret_cast<T*>(reinterpret_cast<char*>(base) + byte_off);
}
template <typename T>
__device__ __forceinline__ const T* at(const T* base, uint32_t byte_off) {
    return reinterpret_cast<const T*>(reinterpret_cast<const char*>(base) + byte_off);
}
// a[i] for a lane-varying i < TPE_E as an OR of masked elements.  (A select chain
// `r = i == e ? a[e] : r` was folded by the compiler into an indexed load, which put the
// whole array in scratch memory: a scratch load and an s_waitcnt vmcnt(0) -- a wait for
// every obs store of the wave in flight -- twice per step.  2^20 staggered envs: K = 20
// 69.4 -> 66.8 us per step, K = 100 55.7 -> 54.8, one box, interleaved A/B.)
__device__ __forceinline__ uint32_t pick8(const uint32_t (&a)[TPE_E], int i) {
    uint32_t r = 0;
#pragma unroll
    for (int e = 0; e < TPE_E; ++e) r |= (i == e) ? a[e] : 0u;
    return r;
}
template <int ET, int RT>
struct LDims {
    const int E, R;
    __device__ __forceinline__ LDims(const Params& p) : E(ET > 0 ? ET : p.E), R(ET > 0 ? RT : p.R) {}
};

// ---- k_rollout_img's per-env LDS image (IMG_W = 40 words, 16-byte row blocks)
//   row block r at word 4r (r < E an endpoint; r = E the reject row, constant):
//     [zc, topology, cpu, latency]   zc = the f16 pair (zone, zone cpu capacity) -- small
//     integers (capacity <= 64 nodes x 8 cpus), exact in f16; the reject row's -1, -1 --
//     then the endpoint's topology latency to the request's zone and its observed cpu and
//     latency (f32)
//   shared block at word IMG_S: [req_zone, threshold, dt, -] (f32; 16-byte aligned, one
//   12-byte LDS read)
// Piece j of an env's obs (row j / 2, half j % 2) from its image:
//   half 0 = (zone, capacity, cpu, topology) = (lo(zc), hi(zc), word 2, word 1) of row j / 2
//   half 1 = (latency, req_zone, threshold, dt) = (word 3 of the row block, shared 0..2)
// A store instruction of the copy-out covers 64 consecutive pieces of the wave's block and
// P = 2R is even, so every lane stores the same half in every store (its lane parity): two
// 16-byte LDS reads, the f16 pair's two conversions and four selects on a loop-invariant
// flag per piece.  A step writes the selected endpoint's cpu + latency (one 8-byte write),
// the shared block (one 16-byte write) and the topology column (E words).
constexpr int IMG_S = 4 * (TPE_E + 1), IMG_W = IMG_S + 4;  // 36, 40
constexpr uint32_t IMG_ZC_REJECT = 0xBC00BC00u;          // f16 pair (-1, -1)
constexpr uint32_t F32_M1 = 0xBF800000u;                 // -1.f

__device__ __forceinline__ uint32_t img_zc(int zone, int cap) {
    const _Float16 z = (_Float16)zone, c = (_Float16)cap;
    return (uint32_t)__builtin_bit_cast(uint16_t, z) | ((uint32_t)__builtin_bit_cast(uint16_t, c) << 16);
}

// topology latency between zones z (compile-time) and rz (topo_val), branch-free: the
// pair (i, j) = (min, max) of 4 zones is bit field i (7 - i) / 2 + j - i - 1 of the packed block
template <int Z>
__device__ __forceinline__ uint32_t topo_to(uint64_t topo, int rz) {
    const int i = Z < rz ? Z : rz, j = Z < rz ? rz : Z;
    const uint32_t val = (uint32_t)(topo >> (9 * ((i * (7 - i)) / 2 + j - i - 1))) & 0x1FFu;
    return rz == Z ? 1u : val;
}
__device__ __forceinline__ void img_request(uint32_t* me, const LEnv& v, const uint32_t (&em)[TPE_E], int E) {
    const int rz = (int)((v.s1 >> S1_RZ) & 3);
    // the four zones' topology latencies to the request zone, then a two-level select per
    // endpoint on its zone bits.  (Written as a nested ?: over topo_val calls, the column
    // compiled into exec-mask branches around each endpoint's write: ~15 instructions
    // including SALU mask updates per endpoint per step.)
    uint32_t t0 = __float_as_uint((float)topo_to<0>(v.topo, rz)), t1 = __float_as_uint((float)topo_to<1>(v.topo, rz));
    uint32_t t2 = __float_as_uint((float)topo_to<2>(v.topo, rz)), t3 = __float_as_uint((float)topo_to<3>(v.topo, rz));
    asm volatile("" : "+v"(t0), "+v"(t1), "+v"(t2), "+v"(t3));
    *reinterpret_cast<uint4*>(me + IMG_S) =
        make_uint4(__float_as_uint((float)rz), __float_as_uint((float)threshold((int)((v.s1 >> S1_THR) & 7))),
                   __float_as_uint(v.dt), 0u);
#pragma unroll
    for (int e = 0; e < TPE_E; ++e) {
        if (e >= E) continue;
        const uint32_t z = em[e] & 3u;
        const uint32_t lo = (z & 1u) ? t1 : t0, hi = (z & 1u) ? t3 : t2;
        me[4 * e + 1] = (z & 2u) ? hi : lo;
    }
}
// the selected endpoint's new observed cpu and latency (words 2, 3 of its row block)
__device__ __forceinline__ void img_sel(uint32_t* me, int e, float cpu, float lat) {
    *reinterpret_cast<uint2*>(me + 4 * e + 2) = make_uint2(__float_as_uint(cpu), __float_as_uint(lat));
}
// piece of row block A / shared block S for a lane storing half h
__device__ __forceinline__ float4 img_piece(const uint4& A, const uint4& S, bool h) {
    const float zf = (float)__builtin_bit_cast(_Float16, (uint16_t)(A.x & 0xFFFFu));
    const float cf = (float)__builtin_bit_cast(_Float16, (uint16_t)(A.x >> 16));
    return make_float4(h ? __uint_as_float(A.w) : zf, h ? __uint_as_float(S.x) : cf,
                       h ? __uint_as_float(S.y) : __uint_as_float(A.z), h ? __uint_as_float(S.z) : __uint_as_float(A.y));
}

// Copy-out cursor of a lane: the env (LDS byte offset ea of its image inside the wave's
// image, index el) and row r2 of the lane's piece in the current store instruction.  One
// store instruction further = 64 pieces = 32 rows further: r2 += 32 % R, el += 32 / R, and
// one env more when r2 wraps.
struct ImgCursor {
    uint32_t ea;
    int r2, el;
};
template <int ET, int RT>
__device__ __forceinline__ ImgCursor img_cursor(const LDims<ET, RT>& d, int lane) {
    int ln = lane;
    // (opaque per call: the cursor of every store is a function of the lane only, and
    // hoisting them out of the step loop would hold 2R of them in registers all launch)
    asm volatile("" : "+v"(ln));
    const int el = ln / (2 * d.R), r2 = (ln - el * 2 * d.R) >> 1;
    return ImgCursor{(uint32_t)el * (uint32_t)(IMG_W * 4), r2, el};
}
template <int ET, int RT>
__device__ __forceinline__ void img_advance(const LDims<ET, RT>& d, ImgCursor& c) {
    const int dr = 32 % d.R, de = 32 / d.R;
    c.r2 += dr;
    c.ea += (uint32_t)(de * IMG_W * 4);
    c.el += de;
    if (c.r2 >= d.R) {
        c.r2 -= d.R;
        c.ea += IMG_W * 4;
        c.el += 1;
    }
}
__device__ __forceinline__ float4 img_read_piece(const uint32_t* wimg, const ImgCursor& c, bool h) {
    const char* b = reinterpret_cast<const char*>(wimg) + c.ea;
    const uint4 A = *reinterpret_cast<const uint4*>(b + 16 * c.r2);
    const uint4 S = *reinterpret_cast<const uint4*>(b + 4 * IMG_S);
    return img_piece(A, S, h);
}

// the next step's action (policy on the current state), its selected endpoint's 4 table
// values (the lat0 of a first selection instead of LAT[0]) and its request draws
// between(stage), stage = 0..PREP_STAGES-1, runs between the stages of the computation (the
// rollout issues the previous step's obs stores there, so they spread over the step's work)
constexpr int PREP_STAGES = 6;
struct NoInterleave {
    __device__ __forceinline__ void operator()(int) const {}
};
template <int KIND, int ET, int RT, typename F = NoInterleave>
__device__ __forceinline__ LPrep lean_prep(const Params& p, const LDims<ET, RT>& d, int64_t ev, const LEnv& v,
                                           const uint32_t (&em)[TPE_E], const uint32_t (&ed)[TPE_E],
                                           uint32_t l0off, uint32_t l0step, F&& between = F()) {
    LPrep r;
    TEnv tv;  // the policy's view (tpe_policy)
    tv.topo = v.topo;
    tv.zcap = v.zcap;
    tv.acc3 = v.acc3;
    tv.s.rz = (int)((v.s1 >> S1_RZ) & 3);
    tv.s.step = (int)(v.s0 & 0xFFFF);
    const int a = tpe_policy<KIND>(p, ev, tv, em, ed);
    r.a = a;
    between(0);
    const int E = d.E;
    const bool accept = a >= -E && a < E;
    const int ai = accept ? (a < 0 ? a + E : a) : 0;
    const uint32_t emA = pick8(em, ai), edA = pick8(ed, ai);
    const int oA = em_owner(emA);
    const uint32_t edO = pick8(ed, oA);
    const int jA = ed_j(edA);
    const int Mn = ed_M(edO) < CMAX ? ed_M(edO) + 1 : CMAX;
    const int jn = jA < CMAX ? jA + 1 : CMAX;
    const int k0A = lem_k0(emA), c0A = em_c0(emA);
    // selected_endpoint_latency: lat0 on a first selection (LAT row 0 holds trunc(lat0))
    // (every table, lat0 array and record lives in the state blob, which starts at lat_lut)
    const uint32_t cpu0 = (uint32_t)(reinterpret_cast<const char*>(p.cpu_lut) - reinterpret_cast<const char*>(p.lat_lut));
    r.sel_lat = *at(p.lat_lut, jA == 0 ? l0off + (uint32_t)ai * l0step : (uint32_t)(jA * LAT_ROWS + k0A) * 8u);
    r.sel_cpu = *at(p.lat_lut, cpu0 + (uint32_t)(ed_m(edA) * CPU_ROWS + c0A) * 8u);
    r.next_lat = *at(p.lat_lut, (uint32_t)(jn * LAT_ROWS + k0A) * 8u);
    r.next_cpu = *at(p.lat_lut, cpu0 + (uint32_t)(Mn * CPU_ROWS + c0A) * 8u);
    between(1);
    const int step = (int)(v.s0 & 0xFFFF);
    // next_request()'s draws (tpe_request_draws' map), the two float64 logs one after the
    // other: interleaved they held two log chains' temporaries at once
    const uint32_t episode = (uint32_t)(v.acc3 >> 32), slot = (uint32_t)(step + 1);
    const U4 wx = draw(p, ev, episode, slot, D_REQ_X);
    between(2);
    r.x1 = p.inv_rate * std_exp(wx.x, wx.y);
    __builtin_amdgcn_sched_barrier(0);
    between(3);
    r.x2 = p.call * std_exp(wx.z, wx.w);
    __builtin_amdgcn_sched_barrier(0);
    between(4);
    const U4 wi = draw(p, ev, episode, slot, D_REQ_I);
    r.r = (int)bounded(wi.x, 7);
    r.n = (int)bounded(wi.y, (uint32_t)p.N);
    between(5);
    return r;
}

// step() (:403-513) after the step counter advanced: take_action (:578-686), reward
// (:516-567), next_request() (:1131-1163) from the prepared values; returns the reward
// The selected endpoint's new observed latency / cpu, dt and the request words go to this
// lane's LDS image (me).
// RF: the reward function when known at compile time (LB_REWARD_*), -1 = p.reward_fn
template <int ET, int RT, int RF = -1>
__device__ __forceinline__ double lean_apply(const Params& p, const LDims<ET, RT>& d, const LPrep& pr, LEnv& v,
                                             const uint32_t (&em)[TPE_E], uint32_t (&ed)[TPE_E], uint32_t* me) {
    const int rf = RF >= 0 ? RF : p.reward_fn;
    const int E = d.E, a = pr.a;
    const bool accept = a >= -E && a < E, reject = a == E;
    const int ai = accept ? (a < 0 ? a + E : a) : 0;
    if (a < -E || !((v.s1 >> S1_RD) & 1)) v.s1 |= 1u << S1_BAD;
    const uint32_t emA = pick8(em, ai), edA = pick8(ed, ai);
    const int oA = em_owner(emA);
    const uint32_t edO = pick8(ed, oA);
    const int jA = ed_j(edA);
    const int Mn = ed_M(edO) < CMAX ? ed_M(edO) + 1 : CMAX;
    const int jn = jA < CMAX ? jA + 1 : CMAX;
    double reward;
    if (accept) {
        int cnt = 0;  // #{e != ai : loads[e] <= loads[ai]} for the O(E) Gini update
#pragma unroll
        for (int e = 0; e < TPE_E; ++e)
            if (e < E && e != ai && ed_j(ed[e]) <= jA) ++cnt;
        const int rz = (int)((v.s1 >> S1_RZ) & 3), zA = em_zone(emA);
        const int tl = topo_val(v.topo, rz, zA);
        const uint32_t gnum = (uint32_t)(v.acc2 >> 32) + (uint32_t)(2 * (2 * cnt - (E - 1)));
        v.acc2 = ((uint64_t)gnum << 32) | (uint32_t)((uint32_t)v.acc2 + (uint32_t)tl);
        v.acc3 += (uint64_t)node_cost(em_type(emA));
        v.s0 += 1u << 16;                 // acc (<= step <= L <= 1023: no saturation)
        if (rz == zA) v.s1 += 1;          // intra
        xsum_add(v.sum_lat, v.sum_cpu, v.sum_hi, pr.sel_lat, pr.sel_cpu, tl, rz != zA);
        // increase_resources / increase_endpoint_latency (:674-677) and the same step's
        // decrease in next_request() (:1137-1143): the history counters advance
        const uint32_t edA_new = ((oA == ai ? (uint32_t)Mn : (uint32_t)ed_M(edA)) << 20) |
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
    // next_request (:1131-1163)
    const double arrival = v.t + pr.x1;
    const double departure = arrival + pr.x2;
    v.dt = (float)(departure - arrival);
    v.t = arrival;
    const uint64_t word = pr.n < 32 ? v.nz0 : v.nz1;
    const uint32_t rz = (uint32_t)((word >> (2 * (pr.n & 31))) & 3);
    v.s1 = (v.s1 & ~((3u << S1_RZ) | (7u << S1_THR))) | (rz << S1_RZ) | ((uint32_t)((pr.r + 6) % 7) << S1_THR);
    img_request(me, v, em, E);
    return reward;
}

__device__ __forceinline__ Scal lean_scal(const LEnv& v) {
    return sc_unpack((uint64_t)v.s0 | ((uint64_t)v.s1 << 32));
}

// ---- k_rollout_img: the rollout with the env's observation rows kept as a compact LDS
// image (IMG_W = 40 words per env, above) instead of registers + a per-step row image.
// The step writes what changed (the selected endpoint's cpu + latency, the shared request
// block, the topology column), and the copy-out decodes float4 pieces from the image
// straight into full-line stores of the wave's contiguous obs block (a piece q of the wave:
// env q / 2R, piece q % 2R; 64 consecutive pieces per store instruction).  Registers hold
// no observed values and no row pieces; LDS holds 10 KB per wave (4 blocks of 4 waves per
// CU), so occupancy is set by the step state alone.  Round 3 replaced the 35-word image
// whose pieces were decoded with 64-bit addressing and a division per store (~35 VALU per
// piece) by the 16-byte row blocks and the per-lane cursor (~16): 1,680 -> 1,402 VALU per
// wave-step (PMC), 2^20 staggered envs 80.2-81.6 -> 77.9-78.1 us per step at K = 20.

// the env's row blocks at the launch start (the observed values of the loaded state) and
// the constant reject row
template <int ET, int RT>
__device__ __forceinline__ void img_endpoints(uint32_t* me, const LDims<ET, RT>& d, const uint32_t (&em)[TPE_E],
                                              uint64_t zcap, const float (&lat)[TPE_E], const float (&cpu)[TPE_E]) {
#pragma unroll
    for (int e = 0; e < TPE_E; ++e) {
        if (e >= d.E) continue;
        const int z = em_zone(em[e]);
        me[4 * e] = img_zc(z, zcap_val(zcap, z));
        img_sel(me, e, cpu[e], lat[e]);
    }
    *reinterpret_cast<uint4*>(me + 4 * d.E) = make_uint4(IMG_ZC_REJECT, F32_M1, F32_M1, F32_M1);
}

// the wave's obs rows, store instructions [it0, it1) of the copy-out into out (the wave's
// block of nenv envs x P float4: store it covers float4s 64 it .. 64 it + 63); c is the
// lanes' cursor at it0 and is advanced past it1.  FLAGGED: only envs whose bit is set in m
// (the terminal observations of the envs that finished).
template <bool FLAGGED, int ET, int RT>
__device__ __forceinline__ void img_copy(const LDims<ET, RT>& d, const uint32_t* wimg, float4* outw, int nenv,
                                         int lane, ImgCursor& c, int it0, int it1, uint64_t m = 0) {
    const bool h = (lane & 1) != 0;
    const int P = 2 * d.R;
    if (!FLAGGED && nenv == 64) {  // a full wave: every lane stores
        for (int it = it0; it < it1; ++it) {
            st_stream(at(outw + 64 * it, (uint32_t)lane * 16u), img_read_piece(wimg, c, h));
            img_advance(d, c);
        }
        return;
    }
    for (int it = it0; it < it1; ++it) {
        bool go = 64 * it + lane < nenv * P;
        if constexpr (FLAGGED) {
            const int lo = (64 * it) / P, hi = (64 * it + 63) / P;  // envs this store touches
            const uint64_t span = (hi >= 63 ? ~0ull : ((2ull << hi) - 1)) & ~((1ull << lo) - 1);
            go = go && (m & span) && ((m >> c.el) & 1);
        }
        if (go) st_stream(at(outw + 64 * it, (uint32_t)lane * 16u), img_read_piece(wimg, c, h));
        img_advance(d, c);
    }
}

// lean_start_episode for the image kernel: the record's endpoints in two halves (fewer
// registers in flight), each written to the image at once, then the scalars
template <int ET, int RT>
__device__ __forceinline__ void img_start_episode(const Params& p, const LDims<ET, RT>& d, const uint4* rp, LEnv& v,
                                                  uint32_t (&em)[TPE_E], uint32_t (&ed)[TPE_E], uint32_t* me) {
    const uint32_t* rw = reinterpret_cast<const uint32_t*>(rp);
    const uint4 tq[4] = {rp[6], rp[7], rp[8], rp[9]};  // words 24..39: topo, zcap, nz0, nz1, x1, x2, thr | rz
    const uint64_t zcap = (uint64_t)tq[0].z | ((uint64_t)tq[0].w << 32);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const uint4 l01 = rp[2 * h], l23 = rp[2 * h + 1], mq = rp[4 + h];
        const uint32_t lw[8] = {l01.x, l01.y, l01.z, l01.w, l23.x, l23.y, l23.z, l23.w};
        const uint32_t mw[4] = {mq.x, mq.y, mq.z, mq.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int e = 4 * h + i;
            ed[e] = 0u;
            em[e] = 0u;
            if (e >= d.E) continue;
            const double l0 = __longlong_as_double((long long)((uint64_t)lw[2 * i] | ((uint64_t)lw[2 * i + 1] << 32)));
            em[e] = lem_make(mw[i], l0);
            const int z = em_zone(mw[i]);
            me[4 * e] = img_zc(z, zcap_val(zcap, z));
            img_sel(me, e, (float)em_c0(mw[i]), (float)l0);  // table rows 0: the initial values
        }
    }
    (void)rw;
    v.topo = (uint64_t)tq[0].x | ((uint64_t)tq[0].y << 32);
    v.zcap = zcap;
    v.nz0 = (uint64_t)tq[1].x | ((uint64_t)tq[1].y << 32);
    v.nz1 = (uint64_t)tq[1].z | ((uint64_t)tq[1].w << 32);
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
    v.s1 = (v.s1 & (1u << S1_BAD)) | (1u << S1_RD) | ((tq[3].x & 7u) << S1_THR) | (((tq[3].x >> 8) & 3u) << S1_RZ);
    const double x1 = __longlong_as_double((long long)((uint64_t)tq[2].x | ((uint64_t)tq[2].y << 32)));
    const double x2 = __longlong_as_double((long long)((uint64_t)tq[2].z | ((uint64_t)tq[2].w << 32)));
    const double arrival = v.t + x1;
    const double departure = arrival + x2;
    v.dt = (float)(departure - arrival);
    v.t = arrival;
    img_request(me, v, em, d.E);
}

template <int NB, int KIND, int ET, int RT, int MINW = 1>
__global__ __launch_bounds__(NB, MINW) void k_rollout_img(Params p, int K, int32_t* act_out) {
    constexpr int NW = NB / 64;
    __shared__ __attribute__((aligned(16))) uint32_t simg[NW][64 * IMG_W];
    const LDims<ET, RT> d(p);
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint32_t* wimg = simg[wv];
    uint32_t* me = wimg + lane * IMG_W;
    // (the wave's first env, wave-uniform: its output blocks are scalar bases)
    const int64_t env0 = (int64_t)blockIdx.x * NB + __builtin_amdgcn_readfirstlane(threadIdx.x & ~63);
    const int64_t env = env0 + lane;
    const bool live = env < p.B;
    const int64_t ev = live ? env : 0;  // dead lanes step env 0's copy and store nothing
    const int E = d.E, R = d.R, P = 2 * R;
    const int nenv = p.B - env0 < 64 ? (int)(p.B - env0) : 64;

    // first (with nothing else live), the next episodes of the envs that end inside the
    // launch, into their records (8 lanes per env); the list lives in the image region
    // before the image is built
    {
        const int to_done = p.L - (int)(p.sc[ev] & 0xFFFF);
        const bool fin = live && to_done >= 1 && to_done <= K;
        const uint64_t fm = __ballot(fin);
        if (fin) {
            uint32_t* it = wimg + 2 * __popcll(fm & ((1ull << lane) - 1));
            it[0] = (uint32_t)lane;
            it[1] = (uint32_t)(p.acc3[ev] >> 32) + 1;
        }
        wave_lds_sync();
        const int nf = __popcll(fm), g = lane / RS_W, gl = lane % RS_W;
        for (int r0 = 0; r0 < nf; r0 += 64 / RS_W) {
            const int i = r0 + g;
            if (i < nf) tpe_write_record<RS_W>(p, env0 + (int64_t)wimg[2 * i], wimg[2 * i + 1], gl);
        }
        // the records are read back by other lanes of this wave; the list region becomes
        // the image
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    }

    LEnv v;
    uint32_t em[TPE_E], ed[TPE_E];
    float olat[TPE_E], ocpu[TPE_E];  // launch start and episode starts only (then the image)
#pragma unroll
    for (int e = 0; e < TPE_E; ++e) {
        em[e] = 0u;
        ed[e] = 0u;
        olat[e] = 0.f;
        ocpu[e] = 0.f;
        if (e < E) {
            const int64_t i = (int64_t)e * p.B + ev;
            const double l0 = p.lat0[i];
            const uint32_t m = p.emeta[i];
            ed[e] = p.edyn[i];
            em[e] = lem_make(m, l0);
            olat[e] = (float)lat_of(p, l0, ed[e]);
            ocpu[e] = (float)cpu_of(p, m, ed[e]);
        }
    }
    v.t = p.t[ev];
    {
        const uint64_t sc = p.sc[ev];
        v.s0 = (uint32_t)sc;
        v.s1 = (uint32_t)(sc >> 32);
    }
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
    v.dt = 0.f;

    img_endpoints(me, d, em, v.zcap, olat, ocpu);

    bool new_episode = false;
    const uint32_t envi = (uint32_t)ev;
    const uint4* rec = at(p.rec, envi * (uint32_t)RO_REC_BYTES);
    const char* blob = reinterpret_cast<const char*>(p.lat_lut);
    uint32_t l0off = (uint32_t)(reinterpret_cast<const char*>(p.lat0) - blob) + envi * 8u;
    uint32_t l0step = (uint32_t)p.B * 8u;
    const int64_t obs_slot = p.B * (int64_t)R * 8;

    LPrep pr = lean_prep<KIND>(p, d, ev, v, em, ed, l0off, l0step);
#ifdef LB_TIMELINE  // diagnostic build (tools/timeline.py): each wave's step start times
    const int64_t gw = (int64_t)blockIdx.x * NW + wv;
    if (g_timeline && lane == 0) g_timeline[gw * (K + 2)] = __builtin_amdgcn_s_memrealtime();
#endif
    for (int k = 0; k < K; ++k) {
#ifdef LB_TIMELINE
        if (g_timeline && lane == 0) g_timeline[gw * (K + 2) + 1 + k] = __builtin_amdgcn_s_memrealtime();
#endif
        // issue priority by progress: a wave behind the others in its launch goes first.
        // (The default oldest-first lets the four waves of a block drift apart, and a block's
        // LDS is released only when its slowest wave ends: 18-28% of the wave slots sat idle
        // mid-launch, tools/timeline.py.)  2^20 staggered envs, K = 20: 77.7-78.0 -> 74.1-74.9
        // us per step; K = 100 equal (profiles/r03_ablation.jsonl).
        {
            const int pl = 3 - (4 * k) / K;
            if (pl >= 3) __builtin_amdgcn_s_setprio(3);
            else if (pl == 2) __builtin_amdgcn_s_setprio(2);
            else if (pl == 1) __builtin_amdgcn_s_setprio(1);
            else __builtin_amdgcn_s_setprio(0);
        }
        if (act_out && live) *at(act_out + (int64_t)k * p.B, envi * 4u) = pr.a;
        v.s0 += 1;  // step (<= L: the episode ends there)
        const bool done = live && (int)(v.s0 & 0xFFFF) == p.L;  // (:472)
        const double reward = lean_apply(p, d, pr, v, em, ed, me);
        if (live) {
            // (nontemporal like the obs: 1-1.5% per step at 2^20 envs, profiles/r03_ablation.jsonl)
            if (p.reward) __builtin_nontemporal_store((float)reward, at(p.reward + (int64_t)k * p.B, envi * 4u));
            if (p.done) __builtin_nontemporal_store((uint8_t)done, at(p.done + (int64_t)k * p.B, envi));
        }
        const uint64_t m = __ballot(done);
        if (m) {  // VecEnv auto-reset: terminal obs + episode stats, then the record's episode
            if (done && p.ep_stats)
                write_stats_row(p, at(p.ep_stats, envi * (uint32_t)(8 * LB_ST_K)), lean_scal(v), v.acc2, v.acc3,
                                v.total, v.sum_lat, v.sum_cpu, v.sum_hi);
            if (p.term_obs) {
                wave_lds_sync();
                ImgCursor tc = img_cursor(d, lane);
                // (an opaque scalar base: the stores' addresses are the same every step, and
                // hoisting them out of the step loop would hold 2R address pairs all launch)
                int64_t toff = env0 * P;
                asm volatile("" : "+s"(toff));
                float4* tob = reinterpret_cast<float4*>(p.term_obs) + toff;
                img_copy<true>(d, wimg, tob, nenv, lane, tc, 0, P, m);
            }
            if (done) {
                wave_lds_sync();  // (the copy-out read the terminal image)
                img_start_episode(p, d, rec, v, em, ed, me);
                new_episode = true;
                l0off = (uint32_t)(reinterpret_cast<const char*>(rec) - blob);
                l0step = 8u;
            }
        }
        // step k's obs rows leave while step k + 1's action, gathers and draws are computed:
        // the stores of a wave spread over its step instead of one burst at the end
        float4* outw = p.obs ? reinterpret_cast<float4*>(p.obs + k * obs_slot) + env0 * P : nullptr;
        if (outw) wave_lds_sync();
        ImgCursor cur = img_cursor(d, lane);
        auto stores = [&](int stage) {
            if (!outw) return;
            const int per = (P + PREP_STAGES - 1) / PREP_STAGES;
            const int it0 = stage * per, it1 = it0 + per < P ? it0 + per : P;
            img_copy<false>(d, wimg, outw, nenv, lane, cur, it0, it1);
        };
        if (k + 1 < K) {
            pr = lean_prep<KIND>(p, d, ev, v, em, ed, l0off, l0step, stores);
        } else {
            for (int st = 0; st < PREP_STAGES; ++st) stores(st);
        }
        if (outw) wave_lds_sync();  // (the next step rewrites the image)
    }
#ifdef LB_TIMELINE
    if (g_timeline && lane == 0) g_timeline[gw * (K + 2) + K + 1] = __builtin_amdgcn_s_memrealtime();
#endif
    if (!live) return;
#pragma unroll
    for (int e = 0; e < TPE_E; ++e)
        if (e < E) p.edyn[(int64_t)e * p.B + env] = ed[e];
    if (new_episode) {  // the scenario of the episode started in the launch, from its record
        const uint32_t* w = reinterpret_cast<const uint32_t*>(rec);
#pragma unroll
        for (int e = 0; e < TPE_E; ++e) {
            if (e >= E) continue;
            const int64_t i = (int64_t)e * p.B + env;
            p.lat0[i] = __longlong_as_double((long long)((uint64_t)w[2 * e] | ((uint64_t)w[2 * e + 1] << 32)));
            p.emeta[i] = w[16 + e];
        }
        p.topo[env] = v.topo;
        p.zcap[env] = v.zcap;
        p.nzone[env] = v.nz0;
        if (p.NZW > 1) p.nzone[p.B + env] = v.nz1;
    }
    p.t[env] = v.t;
    p.sc[env] = (uint64_t)v.s0 | ((uint64_t)v.s1 << 32);
    p.acc2[env] = v.acc2;
    p.acc3[env] = v.acc3;
    p.sum_lat[env] = v.sum_lat;
    p.sum_cpu[env] = v.sum_cpu;
    p.sum_hi[env] = v.sum_hi;
    p.total[env] = v.total;
    if (p.reward_fn != LB_REWARD_NAIVE) p.last_r[env] = v.last_r;
}

}  // namespace lbk
