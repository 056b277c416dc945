// lbk8s_ds_train.h — fused deep-sets backward for the PPO / DQN updates on MI355X.
//
// Reference: the update's autograd through envs/deep_sets_agent_original.py:56-106
// (EquivariantLayer y = Lambda(x) - Gamma(max_set x), the actor Eq-ReLU-Eq-ELU-Eq and the
// critic Eq-ELU-Eq-ELU-Eq-mean), as driven by envs/ppo_deepset.py:227-263.
//
// Split of the training step:
//   * k_deepsets_fwd<TS, P, true> (lbk8s_deepsets.h) writes the logits, the critic's psi
//     mean and the hidden activations h1, h2 (actor) / c1, c2 (critic) row-major.
//   * torch evaluates rho, the PPO loss and its gradient w.r.t. logits and psi mean.
//   * k_ds_train_bwd (here), one launch per head: each wave (one per SIMD) walks its
//     sets in 16-row steps, pass 1 of one set beside pass 2 of the previous (below):
//       pass 1 (h2, h1; VALU, lane = feature): every set-wise max and its FIRST argmax row
//         (torch.max's index), the set sums the Gamma / Lambda3 gradients need, and the
//         set sum of dz2 in closed form: sum_r dz2[r][o] = Lambda3[o] sum_r dl[r]
//         elu'(h2[r][o]) - g3 Gamma3[o] elu'(max_r h2[r][o]) (the critic: u, vv);
//       pass 2 (MFMA), per 16-row tile: dz2 from h2; dLambda2 += dz2^T h1 over the rows;
//         the data gradient dz1 = (dz2 Lambda2 - [r == argmax] Gamma2^T sum dz2) act'(h1);
//         dLambda1 += dz1^T obs.
//     The weight-gradient accumulators stay in registers across all the sets a wave
//     visits; at the end the block sums its waves in LDS in a fixed order and writes one
//     slot, and k_ds_wgrad_reduce sums the slots in a fixed order: no per-row gradient
//     reaches HBM, and the result does not depend on timing.  Per-set vectors (set-wise
//     max, gradient sums over the set, the last-layer products) give every Gamma gradient
//     and the rank-1 last-layer gradients as small GEMMs over the sets.
// Fragment order of the weight image is that of lbk8s_deepsets.h (at k-step k, lane l
// holds features 16(k >> 2) + 4(l >> 4) + (k & 3)).
#pragma once

#include "lbk8s_deepsets.h"

namespace lbk {

// backward weight image: transposed 64x64 matrices in fragment order, then the actor's
// last-layer rows in natural order
enum : int {
    DSB_A2LT = 0, DSB_A2GT = 4096, DSB_C2LT = 8192, DSB_C2GT = 12288, DSB_C3LT = 16384, DSB_C3GT = 20480,
    DSB_A3L = 24576, DSB_A3G = 24640, DSB_FLOATS = 24704,
};
// per-set vector block (floats); every 64-wide entry is indexed by input feature
enum : int {
    DSV_MAX0 = 0,     // [8]  max over the set of the observation (forward)
    DSV_GA3 = 8,      // actor: sum_r dlogit[r] h2[r]           (Lambda3 gradient)
    DSV_MAX2A = 72,   //        max_set h2 (forward)             (Gamma3)
    DSV_GS2A = 136,   //        sum_r dz2[r]                     (Gamma2)
    DSV_MAX1A = 200,  //        max_set h1                       (Gamma2)
    DSV_GS1A = 264,   //        sum_r dz1[r]                     (Gamma1)
    DSV_CS2 = 328,    // critic: sum_r c2[r]                     (Lambda3: rank 1, d psi = dmean / R)
    DSV_MAX2C = 392,  //         max_set c2                      (Gamma3)
    DSV_GS2C = 456,   //         sum_r dz2[r]
    DSV_MAX1C = 520,  //         max_set c1
    DSV_GS1C = 584,   //         sum_r dz1[r]
    DSV_ID1A = 648,   // [64] u16: first argmax row of max_set h1 / h2 / c1 / c2 (forward)
    DSV_ID2A = 680,
    DSV_ID1C = 712,
    DSV_ID2C = 744,
    DSV_P1A = 776,    // actor: layer 1's pooled term per feature, V act'(MAX1)
    DSV_P1C = 840,    // critic
    DSV_FLOATS = 904,
};
static_assert(DSV_MAX1A == LB_DSV_MAX1A && DSV_MAX2A == LB_DSV_MAX2A && DSV_MAX1C == LB_DSV_MAX1C &&
                  DSV_MAX2C == LB_DSV_MAX2C && DSV_ID1A == LB_DSV_ID1A && DSV_ID2A == LB_DSV_ID2A &&
                  DSV_ID1C == LB_DSV_ID1C && DSV_ID2C == LB_DSV_ID2C && DSV_P1A == LB_DSV_P1A && DSV_P1C == LB_DSV_P1C &&
                  DSV_MAX0 == LB_DSV_MAX0 && DSV_FLOATS == LB_DS_SETVEC_FLOATS,
              "per-set vector layout and header disagree");

constexpr int DSB_BLOCK = 512;                       // 8 waves: 2 per SIMD, one block per CU
constexpr int DSW_FLOATS = 4608;                     // per head: dLambda2 [64][64], dLambda1 [64][8]
constexpr int DSW_GRID = 256;                        // fixed grid (any B): one block per CU
constexpr int DSW_SLOTS = DSW_GRID;                  // one partial-sum slot per block
constexpr int DST_FLOATS = 1280;                     // per-wave LDS tile buffer (floats)

struct DSBwdParams {
    const float* obs;          // [B][R][8]
    const float* wb;           // backward weight image [DSB_FLOATS]
    const float* save_actor;   // [2][B][R][64] h1, h2
    const float* save_critic;  // [2][B][R][64] c1, c2
    const float* dlogits;      // [B][R]
    const float* dmean;        // [B][64]
    float* wpart;              // [DSW_SLOTS][2][DSW_FLOATS] per-block weight-gradient partials
    float* setvec;             // [B][DSV_FLOATS]
    int64_t B;
    int R;
    int actor, critic;
};

// d act / d z from the activation's output: ReLU (ACT 1) y > 0; ELU (ACT 2) y > 0 ? 1 : y + 1
template <int ACT>
__device__ __forceinline__ float dact(float y) {
    return ACT == 1 ? (y > 0.f ? 1.f : 0.f) : (y > 0.f ? 1.f : y + 1.f);
}

// ---- the backward kernel
//
// Two waves per SIMD (8 per CU, 256 registers each: one wave's vector and memory work
// issues while the other's matrix instructions run).  A wave walks its sets (env0, env0 +
// nwaves, ...) 16 rows at a time.  The set-wise maxima and their first argmax rows come
// from the training forward (setvec MAX*, ID*), so each set is read once:
//   per set, before its first tile: the set vectors c1, c2 (below), from the actor's
//     dlogits (g3 = sum_r dl[r]) or the critic's dmean (lane-per-feature matrix-vector
//     products against natural-order weights in LDS);
//   per 16-row tile, in the W layout (lane (col, grp) holds rows 4c + grp, c < 4, and
//     features 4col .. 4col + 3, which is the operand layout of dLambda2 += dz2^T h1 and
//     dLambda1 += dz1^T obs, contractions over rows, so those MFMAs read registers):
//     dz2; dLambda2; the data gradient dz1 = (dz2 Lambda2) act'(h1) (contraction over
//     features: dz2 goes through a per-wave LDS transpose into the MFMA's other operand
//     layout and the result back, Lambda2^T from LDS); dLambda1; the set sums S, G of h2
//     terms and of dz1;
//   per set, after its last tile: sum_r dz2 in closed form, V = Gamma2^T sum_r dz2, layer
//     1's pooled term (dz1 at row ID1[o] of feature o carries -V[o] act'(MAX1[o]): one row
//     per feature, folded into sum_r dz1 and, with the obs row at ID1[o], into dLambda1), the set
//     sums out.
// Each set's small inputs (dlogits or dmean, ID2, MAX2) are loaded one set ahead.
//
// Per feature o, dz2[r][o] = (c1[o] - [r == ID2[o]] c2[o]) elu'(h2[r][o]) with actor
// c1 = dl[r] Lambda3[o] (row-dependent through dl), c2 = g3 Gamma3[o];
// critic c1 = u[o] = (Lambda3^T dmean)[o] / R, c2 = vv[o] = (Gamma3^T dmean)[o].  Its set
// sum is closed-form: sum_r dz2[r][o] = c1 S[o] - c2 elu'(MAX2[o]) with
// S = sum_r w[r] elu'(h2[r][o]) = sum_r w[r] min(h2[r][o], 0) + sum_r w[r] (ELU output y:
// elu' = y > 0 ? 1 : y + 1 = min(y, 0) + 1), w = dl (actor) / 1 (critic).
constexpr int DSB_WAVES = DSB_BLOCK / 64;
constexpr int DSB_NAT = 3 * 4096 + 128;  // natural-order weights (below)
constexpr int DSB_CV = 192;              // per-wave set vectors (below)

// one 16-row tile of the backward's inputs in the W layout, as loaded: rows past R read
// row R - 1 (finite values, in bounds) and every use masks them, so no instruction touches
// the registers before the tile is used
struct Tile2 {
    float4 a[4];  // h2 / c2 of row 16t + 4c + grp, features 4col .. 4col + 3
    float4 h[4];  // h1 / c1
    float x[4];   // observation feature col & 7 of row 16t + 4c + grp
    float d[4];   // the actor's dlogit of row 16t + 4c + grp
};
// a set's small inputs, loaded one set ahead
struct SetIn {
    float dls;       // actor: this lane's share of sum_r dlogits (rows lane, lane + 64, ...)
    float dm;        // critic: dmean[lane]
    uint2 id2;       // ID2 rows (u16) of features 4col .. 4col + 3
    float4 mx2;      // MAX2 of features 4col .. 4col + 3
    float mx1;       // MAX1 of feature lane
    uint32_t id1;    // ID1 row of feature lane (layer 1's pooled term, below)
};

template <int HEAD>
__device__ __forceinline__ void load_tile2(const DSBwdParams& p, const float* in1, const float* in2, int64_t env, int t,
                                           int col, int grp, Tile2& s) {
    const int R = p.R;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const int64_t er = env * (int64_t)R + min(16 * t + 4 * c + grp, R - 1);
        // (the activations are read once: nontemporal loads keep them out of the caches)
        const dsf4 a4 = __builtin_nontemporal_load(reinterpret_cast<const dsf4*>(in2 + er * 64 + 4 * col));
        const dsf4 h4 = __builtin_nontemporal_load(reinterpret_cast<const dsf4*>(in1 + er * 64 + 4 * col));
        s.a[c] = make_float4(a4[0], a4[1], a4[2], a4[3]);
        s.h[c] = make_float4(h4[0], h4[1], h4[2], h4[3]);
        s.x[c] = p.obs[er * 8 + (col & 7)];
        s.d[c] = HEAD == 0 ? p.dlogits[er] : 0.f;
    }
}

template <int HEAD>
__device__ __forceinline__ void load_setin(const DSBwdParams& p, int64_t env, int lane, int col, SetIn& s) {
    const int R = p.R;
    const float* sv = p.setvec + env * (int64_t)DSV_FLOATS;
    if (HEAD == 0) {
        const float* dl = p.dlogits + env * (int64_t)R;
        float a = 0.f;  // (summed in row order per lane, then across the lanes)
        for (int r = lane; r < R; r += 64) a += dl[r];
        s.dls = a;
    } else {
        s.dm = p.dmean[env * 64 + lane];
    }
    s.id2 = *reinterpret_cast<const uint2*>(reinterpret_cast<const uint16_t*>(sv + (HEAD == 0 ? DSV_ID2A : DSV_ID2C)) +
                                            4 * col);
    s.mx2 = *reinterpret_cast<const float4*>(sv + (HEAD == 0 ? DSV_MAX2A : DSV_MAX2C) + 4 * col);
    s.mx1 = sv[(HEAD == 0 ? DSV_MAX1A : DSV_MAX1C) + lane];
    s.id1 = reinterpret_cast<const uint16_t*>(sv + (HEAD == 0 ? DSV_ID1A : DSV_ID1C))[lane];
}

// lane-per-feature matrix-vector product out[lane] = sum_i M[i][lane] x[i], M natural
// order ([i][o], 64 x 64) in LDS, x a 64-float LDS vector (broadcast reads)
__device__ __forceinline__ float matvec64(const float* M, const float* x, int lane, float xs = 1.f) {
    float acc = 0.f;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        const float4 v = *reinterpret_cast<const float4*>(x + 4 * j);
        acc += M[(4 * j) * 64 + lane] * (v.x * xs);
        acc += M[(4 * j + 1) * 64 + lane] * (v.y * xs);
        acc += M[(4 * j + 2) * 64 + lane] * (v.z * xs);
        acc += M[(4 * j + 3) * 64 + lane] * (v.w * xs);
    }
    return acc;
}

// One launch per head (HEAD 0 actor, 1 critic).
template <int HEAD>
__global__ __launch_bounds__(DSB_BLOCK, 1) void k_ds_train_bwd(DSBwdParams p) {
    constexpr int ACT1 = HEAD == 0 ? 1 : 2;  // activation after layer 1: ReLU (actor) / ELU (critic)
    // natural-order weights [i][o] (W[out i][in o]): Gamma2 at 0; the critic's Lambda3,
    // Gamma3 at 4096, 8192; the actor's Lambda3 / Gamma3 rows at 12288 / 12352
    __shared__ __attribute__((aligned(16))) float NAT[DSB_NAT];
    // Lambda2^T in fragment order (the data gradient's A operands)
    __shared__ __attribute__((aligned(16))) float LT[4096];
    // per wave: the 16-row tile transposes (16 x 16 float4), and the block's reduction
    __shared__ __attribute__((aligned(16))) float TB[DSB_WAVES][DST_FLOATS];
    // per wave: [0, 64) broadcast scratch, c1 [64, 128), c2 [128, 192) of the current set
    __shared__ __attribute__((aligned(16))) float CV[DSB_WAVES][DSB_CV];
    // per wave: layer 1's pooled term in dLambda1, lane o's row (8 floats), summed over its sets
    __shared__ __attribute__((aligned(16))) float POOL[DSB_WAVES][64 * 8];
    {
        // fragment image -> natural order: fragment (nt, k), lane l holds W^T[o][i] with
        // o = 16nt + (l & 15), i = 16(k >> 2) + 4(l >> 4) + (k & 3)
        const float* srcs[3] = {p.wb + (HEAD == 0 ? DSB_A2GT : DSB_C2GT), p.wb + DSB_C3LT, p.wb + DSB_C3GT};
        const int nm = HEAD == 0 ? 1 : 3;
        for (int idx = threadIdx.x; idx < 4096 * nm; idx += DSB_BLOCK) {
            const int m = idx >> 12, i = (idx >> 6) & 63, o = idx & 63;
            const int k = 4 * (i >> 4) + (i & 3), l = (o & 15) + 16 * ((i >> 2) & 3);
            NAT[idx] = srcs[m][((o >> 4) * 16 + k) * 64 + l];
        }
        if (HEAD == 0)
            for (int i = threadIdx.x; i < 128; i += DSB_BLOCK) NAT[12288 + i] = p.wb[DSB_A3L + i];
        // Lambda2^T fragments regrouped by k quad: LT[((nt * 4 + kq) * 64 + lane) * 4 + kk] is
        // fragment (nt, 4kq + kk) of lane, one float4 read per (nt, kq)
        const float* src = p.wb + (HEAD == 0 ? DSB_A2LT : DSB_C2LT);
        for (int i = threadIdx.x; i < 4096; i += DSB_BLOCK)
            LT[i] = src[(4 * (i >> 8) + (i & 3)) * 64 + ((i >> 2) & 63)];
    }
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t nwaves = (int64_t)gridDim.x * DSB_WAVES;
    float* la = TB[wv];
    float* cv = CV[wv];
    float4* pool = reinterpret_cast<float4*>(POOL[wv]) + 2 * lane;
    pool[0] = make_float4(0.f, 0.f, 0.f, 0.f);
    pool[1] = make_float4(0.f, 0.f, 0.f, 0.f);
    const int R = p.R, ntl = (R + 15) / 16;
    const int nct = ((R - 1) % 16) / 4 + 1;  // 4-row groups of the last tile that hold set rows
    const bool one_row = R % 16 == 1;        // the last tile holds one set row (below)
    const int col = lane & 15, grp = lane >> 4;
    const int64_t plane = p.B * (int64_t)R * 64;
    const float* in1 = HEAD == 0 ? p.save_actor : p.save_critic;  // h1 / c1
    const float* in2 = in1 + plane;                                 // h2 / c2
    dsf4 w2[4][4], w1[4];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) w2[mt][nt] = dsf4{0.f, 0.f, 0.f, 0.f};
        w1[mt] = dsf4{0.f, 0.f, 0.f, 0.f};
    }
    const int64_t env0 = (int64_t)blockIdx.x * DSB_WAVES + wv;
    const int64_t n = env0 < p.B ? (p.B - 1 - env0) / nwaves + 1 : 0;  // this wave's sets
    if (n > 0) {
        auto env_of = [&](int64_t j) { return env0 + j * nwaves; };
        // per-set state (W layout: this lane's rows, features 4col .. 4col + 3)
        float S4[4], G4[4], gs1[4], g3 = 0.f;
        float4 xid0, xid1;  // the obs row at ID1 of this lane's feature
        uint2 id2w = make_uint2(0u, 0u);
        float4 mx2v;
        float mx1l = 0.f;
#pragma unroll
        for (int m = 0; m < 4; ++m) S4[m] = G4[m] = gs1[m] = 0.f;
        SetIn pre;
        load_setin<HEAD>(p, env_of(0), lane, col, pre);

        // the set vectors of set j (c1, c2 to LDS), then set j + 1's inputs requested
        auto prologue = [&](int64_t j) {
            const SetIn cur = pre;
            if (j + 1 < n) load_setin<HEAD>(p, env_of(j + 1), lane, col, pre);
            id2w = cur.id2;
            mx2v = cur.mx2;
            mx1l = cur.mx1;
            // the obs row at ID1 of this lane's feature (used by the epilogue: in flight
            // across the set's tiles)
            {
                const float4* xr = reinterpret_cast<const float4*>(p.obs + (env_of(j) * (int64_t)R + cur.id1) * 8);
                xid0 = xr[0];
                xid1 = xr[1];
            }
            float c1, c2;
            if (HEAD == 0) {
                float s = cur.dls;
#pragma unroll
                for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
                g3 = s;
                c1 = NAT[12288 + lane];
                c2 = g3 * NAT[12352 + lane];
            } else {
                cv[lane] = cur.dm;
                c1 = matvec64(NAT + 4096, cv, lane, 1.0f / (float)R);
                c2 = matvec64(NAT + 8192, cv, lane);
            }
            cv[64 + lane] = c1;
            cv[128 + lane] = c2;
        };
        // the set sums of set j out, V = Gamma2^T sum_r dz2
        auto epilogue = [&](int64_t j) {
            float* sv = p.setvec + env_of(j) * (int64_t)DSV_FLOATS;
            // the four row groups (lanes col, col + 16, col + 32, col + 48) summed
#pragma unroll
            for (int m = 0; m < 4; ++m) {
                S4[m] += __shfl_xor(S4[m], 16);
                S4[m] += __shfl_xor(S4[m], 32);
                G4[m] += __shfl_xor(G4[m], 16);
                G4[m] += __shfl_xor(G4[m], 32);
                gs1[m] += __shfl_xor(gs1[m], 16);
                gs1[m] += __shfl_xor(gs1[m], 32);
            }
            const float4 c1v = *reinterpret_cast<const float4*>(cv + 64 + 4 * col);
            const float4 c2v = *reinterpret_cast<const float4*>(cv + 128 + 4 * col);
            const float c1a[4] = {c1v.x, c1v.y, c1v.z, c1v.w}, c2a[4] = {c2v.x, c2v.y, c2v.z, c2v.w};
            const float ma[4] = {mx2v.x, mx2v.y, mx2v.z, mx2v.w};
            const float wsum = HEAD == 0 ? g3 : (float)R;
            float gs[4];
#pragma unroll
            for (int m = 0; m < 4; ++m) gs[m] = c1a[m] * (S4[m] + wsum) - c2a[m] * dact<2>(ma[m]);
            if (grp == 0) {
                *reinterpret_cast<float4*>(sv + (HEAD == 0 ? DSV_GS2A : DSV_GS2C) + 4 * col) =
                    make_float4(gs[0], gs[1], gs[2], gs[3]);
                *reinterpret_cast<float4*>(sv + (HEAD == 0 ? DSV_GA3 : DSV_CS2) + 4 * col) =
                    make_float4(G4[0], G4[1], G4[2], G4[3]);
                *reinterpret_cast<float4*>(cv + 4 * col) = make_float4(gs[0], gs[1], gs[2], gs[3]);
            }
            // layer 1's pooled term: dz1 at row ID1[o] of feature o also carries -v[o]
            // act'(MAX1[o]) with v = Gamma2^T sum_r dz2 (h1 at that row is the max); it
            // changes that row's share of sum_r dz1 and of dLambda1 (its obs row)
            const float v = matvec64(NAT, cv, lane);
            const float corr = v * dact<ACT1>(mx1l);
            cv[lane] = corr;
            const float4 cw = *reinterpret_cast<const float4*>(cv + 4 * col);
            gs1[0] -= cw.x;
            gs1[1] -= cw.y;
            gs1[2] -= cw.z;
            gs1[3] -= cw.w;
            if (grp == 0)
                *reinterpret_cast<float4*>(sv + (HEAD == 0 ? DSV_GS1A : DSV_GS1C) + 4 * col) =
                    make_float4(gs1[0], gs1[1], gs1[2], gs1[3]);
            sv[(HEAD == 0 ? DSV_P1A : DSV_P1C) + lane] = corr;
            // ... and in dLambda1: dLambda1[o][c] -= corr[o] obs[ID1[o]][c] (lane o; subtracted
            // from the block's slot after the waves' sums)
            {
                float4 q0 = pool[0], q1 = pool[1];
                q0.x += corr * xid0.x;
                q0.y += corr * xid0.y;
                q0.z += corr * xid0.z;
                q0.w += corr * xid0.w;
                q1.x += corr * xid1.x;
                q1.y += corr * xid1.y;
                q1.z += corr * xid1.z;
                q1.w += corr * xid1.w;
                pool[0] = q0;
                pool[1] = q1;
            }
#pragma unroll
            for (int m = 0; m < 4; ++m) S4[m] = G4[m] = gs1[m] = 0.f;
        };
        // one 16-row tile of the current set
        // nc: the tile's 4-row groups that hold set rows (the weight-gradient products skip
        // the others)
        auto compute = [&](int t, Tile2& c, int nc) {
#pragma clang fp contract(fast)
            // Lambda2^T and the set vectors re-read from LDS per tile: an opaque offset keeps
            // the compiler from hoisting the loop-invariant reads into registers
            uint32_t wo = 0;
            asm volatile("" : "+s"(wo));
            const float* LTt = LT + wo;
            const float* cvt = cv + wo;
            const float4 c1v = *reinterpret_cast<const float4*>(cvt + 64 + 4 * col);
            const float4 c2v = *reinterpret_cast<const float4*>(cvt + 128 + 4 * col);
            // dz2 = (w c1 - [r == ID2] c2) elu'(h2); rows past R have w = 0 and are never an
            // argmax, so their dz2 (and dz1) is 0; the set sums S, G of the h2 terms
            float4 dz[4];
#pragma unroll
            for (int cc = 0; cc < 4; ++cc) {
                const int row = 16 * t + 4 * cc + grp;
                const float w = row < R ? (HEAD == 0 ? c.d[cc] : 1.f) : 0.f;
                float x[4];
                const float y[4] = {c.a[cc].x, c.a[cc].y, c.a[cc].z, c.a[cc].w};
                const float c1a[4] = {c1v.x, c1v.y, c1v.z, c1v.w}, c2a[4] = {c2v.x, c2v.y, c2v.z, c2v.w};
#pragma unroll
                for (int m = 0; m < 4; ++m) {
                    const float mn = fminf(y[m], 0.f);
                    const uint32_t idw = m < 2 ? id2w.x : id2w.y;
                    const float u = w * c1a[m] - (row == (int)((idw >> (16 * (m & 1))) & 0xffffu) ? c2a[m] : 0.f);
                    x[m] = u * mn + u;
                    S4[m] += w * mn;
                    G4[m] += w * y[m];  // actor: sum dl h2 (Lambda3); critic: sum c2
                }
                dz[cc] = make_float4(x[0], x[1], x[2], x[3]);
            }
            // the tile through LDS into the data gradient's k layout (row = col): float4 q of
            // row rho at rho * 16 + (q ^ rho), conflict-free both ways
            float4* T4 = reinterpret_cast<float4*>(la);
            if (!(one_row && t == ntl - 1))
#pragma unroll
                for (int cc = 0; cc < 4; ++cc) {
                    const int rho = 4 * cc + grp;
                    T4[rho * 16 + (col ^ rho)] = dz[cc];
                }
            // dLambda2 += dz2^T h1 straight from registers (W layout = the MFMA operands)
#pragma unroll
            for (int cs = 0; cs < 4; ++cs) {
                if (cs >= nc) break;
                const float av[4] = {dz[cs].x, dz[cs].y, dz[cs].z, dz[cs].w};
                const float bv[4] = {c.h[cs].x, c.h[cs].y, c.h[cs].z, c.h[cs].w};
#pragma unroll
                for (int mt = 0; mt < 4; ++mt)
#pragma unroll
                    for (int nt = 0; nt < 4; ++nt) w2[mt][nt] = mfma4(av[mt], bv[nt], w2[mt][nt]);
            }
            float4 pre1 = make_float4(0.f, 0.f, 0.f, 0.f);
            if (one_row && t == ntl - 1) {
                // a last tile holding one set row (R = 16 t + 1: config 4's 65), row 16 t on the
                // lanes of row group 0: its dz2 Lambda2 as lane dot products -- lane (col, grp)
                // sums inputs 16kq + 4grp + kk of outputs 16nt + col from the same Lambda2^T
                // fragments, the four row groups added -- instead of 64 MFMAs on one live row
                float* v = la + 1024;  // (past the transpose's 256 float4)
                if (grp == 0) *reinterpret_cast<float4*>(v + 4 * col) = dz[0];
                float dv[16];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const float4 d = *reinterpret_cast<const float4*>(v + 16 * q + 4 * grp);
                    dv[4 * q] = d.x;
                    dv[4 * q + 1] = d.y;
                    dv[4 * q + 2] = d.z;
                    dv[4 * q + 3] = d.w;
                }
                float po[4];
#pragma unroll
                for (int nt = 0; nt < 4; ++nt) {
                    float a = 0.f;
#pragma unroll
                    for (int kq = 0; kq < 4; ++kq) {
                        const float4 l = *reinterpret_cast<const float4*>(LTt + ((nt * 4 + kq) * 64 + lane) * 4);
                        a += l.x * dv[4 * kq] + l.y * dv[4 * kq + 1] + l.z * dv[4 * kq + 2] + l.w * dv[4 * kq + 3];
                    }
                    a += __shfl_xor(a, 16);
                    po[nt] = a + __shfl_xor(a, 32);
                }
                // to the W layout (features 4col .. 4col + 3 on row group 0)
                if (grp == 0)
#pragma unroll
                    for (int nt = 0; nt < 4; ++nt) v[64 + 16 * nt + col] = po[nt];
                const float4 q4 = *reinterpret_cast<const float4*>(v + 64 + 4 * col);
                if (grp == 0) pre1 = q4;
            } else {
            // dz2 in k layout (lane: row col, features 16q + 4grp .. + 3 at k = 4q ..)
            float dk[16];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const float4 v = T4[col * 16 + ((4 * q + grp) ^ col)];
                dk[4 * q] = v.x;
                dk[4 * q + 1] = v.y;
                dk[4 * q + 2] = v.z;
                dk[4 * q + 3] = v.w;
            }
            // dz1 pre-activation = dz2 Lambda2: the four output tiles' chains interleaved
            dsf4 eacc[4];
#pragma unroll
            for (int nt = 0; nt < 4; ++nt) eacc[nt] = dsf4{0.f, 0.f, 0.f, 0.f};
            float4 Lf[4], Ln[4];
#pragma unroll
            for (int nt = 0; nt < 4; ++nt) Ln[nt] = *reinterpret_cast<const float4*>(LTt + (nt * 4 * 64 + lane) * 4);
#pragma unroll
            for (int kq = 0; kq < 4; ++kq) {
#pragma unroll
                for (int nt = 0; nt < 4; ++nt) {
                    Lf[nt] = Ln[nt];
                    if (kq < 3) Ln[nt] = *reinterpret_cast<const float4*>(LTt + ((nt * 4 + kq + 1) * 64 + lane) * 4);
                }
#pragma unroll
                for (int kk = 0; kk < 4; ++kk)
#pragma unroll
                    for (int nt = 0; nt < 4; ++nt) {
                        const float l = kk == 0 ? Lf[nt].x : kk == 1 ? Lf[nt].y : kk == 2 ? Lf[nt].z : Lf[nt].w;
                        eacc[nt] = mfma4(l, dk[4 * kq + kk], eacc[nt]);
                    }
            }
            // back to the W layout: output tile nt, lane (row col, grp) holds features
            // 16nt + 4grp .. + 3 = float4 q = 4nt + grp of row col
#pragma unroll
            for (int nt = 0; nt < 4; ++nt)
                T4[col * 16 + ((4 * nt + grp) ^ col)] = make_float4(eacc[nt][0], eacc[nt][1], eacc[nt][2], eacc[nt][3]);
            }
            // dz1 = pre act'(h1) (W layout; the pooled term is added per set), its set sum,
            // dLambda1 += dz1^T obs (B columns 8..15 zero)
#pragma unroll
            for (int cc = 0; cc < 4; ++cc) {
                const int rho = 4 * cc + grp;
                const float4 pre = (one_row && t == ntl - 1) ? (cc == 0 ? pre1 : make_float4(0.f, 0.f, 0.f, 0.f))
                                                             : T4[rho * 16 + (col ^ rho)];
                const float pa[4] = {pre.x, pre.y, pre.z, pre.w};
                const float ha[4] = {c.h[cc].x, c.h[cc].y, c.h[cc].z, c.h[cc].w};
                float d1[4];
#pragma unroll
                for (int m = 0; m < 4; ++m) {
                    d1[m] = ACT1 == 1 ? (ha[m] > 0.f ? pa[m] : 0.f) : pa[m] * fminf(ha[m], 0.f) + pa[m];
                    gs1[m] += d1[m];
                }
                if (cc < nc) {
                    const float xv = col < 8 ? c.x[cc] : 0.f;
#pragma unroll
                    for (int mt = 0; mt < 4; ++mt) w1[mt] = mfma4(d1[mt], xv, w1[mt]);
                }
            }
        };

        // the stream of tiles g = j * ntl + t, j < n
        const int64_t steps = n * ntl;
        int64_t j = 0;
        int t = 0;
        auto step = [&]() {
            if (t == 0) prologue(j);
            Tile2 cur;
            load_tile2<HEAD>(p, in1, in2, env_of(j), t, col, grp, cur);
            compute(t, cur, t == ntl - 1 ? nct : 4);
            if (t == ntl - 1) {
                epilogue(j);
                t = 0;
                ++j;
            } else {
                ++t;
            }
        };
        for (int64_t g = 0; g < steps; ++g) step();
    }
    // the block's waves summed in LDS in a fixed order, one slot per block
    __syncthreads();
    float* red = &TB[0][0];
    static_assert(sizeof(TB) / sizeof(float) >= DSW_FLOATS, "reduction buffer");
    for (int w = 0; w < DSB_WAVES; ++w) {
        if (wv == w) {
            // accumulator (mt, nt) reg i of lane (col, grp): output feature 16grp + 4i + mt,
            // input feature 4col + nt (the W layout's feature order); dLambda1 column col
#pragma unroll
            for (int mt = 0; mt < 4; ++mt)
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int o = 16 * grp + 4 * i + mt;
#pragma unroll
                    for (int nt = 0; nt < 4; ++nt) {
                        float& r = red[o * 64 + 4 * col + nt];
                        r = w == 0 ? w2[mt][nt][i] : r + w2[mt][nt][i];
                    }
                    if (col < 8) {
                        float& r = red[4096 + o * 8 + col];
                        r = w == 0 ? w1[mt][i] : r + w1[mt][i];
                    }
                }
            // (the wave's own LDS accesses complete in order)
            const float4 q0 = pool[0], q1 = pool[1];
            const float pq[8] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w};
#pragma unroll
            for (int c = 0; c < 8; ++c) red[4096 + lane * 8 + c] -= pq[c];
        }
        __syncthreads();
    }
    float* slot = p.wpart + (int64_t)blockIdx.x * (2 * DSW_FLOATS) + HEAD * DSW_FLOATS;
    for (int i = threadIdx.x; i < DSW_FLOATS; i += DSB_BLOCK) slot[i] = red[i];
}

// sum of the per-wave partials: out[j] = sum_s wpart[s][j], j < 2 * DSW_FLOATS; zeros for
// a head that was not run.  Block = 64 outputs x 8 slot groups (each thread sums every 8th
// slot), combined through LDS in a fixed order: deterministic, and 1,152 blocks x 128
// loads per thread instead of one 1,024-long chain per output.
constexpr int DSR_COLS = 64, DSR_GROUPS = 8;
constexpr int DSR_BLOCKS = (2 * DSW_FLOATS + DSR_COLS - 1) / DSR_COLS;
__device__ __forceinline__ void ds_wgrad_reduce_body(const float* wpart, float* out, int actor, int critic, int blk,
                                                     float (*part)[DSR_COLS]) {
    const int c = threadIdx.x % DSR_COLS, g = threadIdx.x / DSR_COLS;
    const int j = blk * DSR_COLS + c;
    const bool live = j < 2 * DSW_FLOATS && (j < DSW_FLOATS ? actor : critic);
    float s0 = 0.f, s1 = 0.f;
    if (live)
        for (int s = g; s < DSW_SLOTS; s += 2 * DSR_GROUPS) {
            s0 += wpart[(int64_t)s * (2 * DSW_FLOATS) + j];
            s1 += wpart[(int64_t)(s + DSR_GROUPS) * (2 * DSW_FLOATS) + j];
        }
    part[g][c] = s0 + s1;
    __syncthreads();
    if (g == 0 && j < 2 * DSW_FLOATS) {
        float t = 0.f;
#pragma unroll
        for (int k = 0; k < DSR_GROUPS; ++k) t += part[k][c];
        out[j] = live ? t : 0.f;
    }
}
__global__ __launch_bounds__(DSR_COLS * DSR_GROUPS) void k_ds_wgrad_reduce(const float* wpart, float* out, int actor,
                                                                           int critic) {
    __shared__ float part[DSR_GROUPS][DSR_COLS];
    ds_wgrad_reduce_body(wpart, out, actor, critic, blockIdx.x, part);
}

// PPO loss head (envs/ppo_deepset.py:227-263 on a minibatch): per set, from the logits
// and the value, the clipped policy loss, the (clipped) value loss, the Categorical
// entropy, approx_kl and clipfrac terms, and the loss's gradient w.r.t. every logit and the
// value — autograd's tie rules included (torch.max of two tensors splits the gradient
// evenly on ties; clamp passes it on the closed interval; masked logits are -1e8 and get
// none).  One wave per set, rows r and r + 64 on lane r.  adv: already normalised.
struct PPOHeadParams {
    const float* logits;    // [M][R]
    const uint8_t* masks;   // [M][R] or NULL
    const float* actions;   // [M] (float, as PPO's storage keeps them)
    const float* oldlogp;   // [M]
    const float* adv;       // [M]
    const float* ret;       // [M]
    const float* vold;      // [M]
    const float* value;     // [M]
    float* dlogits;         // [M][R]
    float* dvalue;          // [M]
    float* terms;           // [M][6]: pg, max(v terms), entropy, kl, clipped, loss
    int64_t M;
    int R;
    float clip, ent_coef, vf_coef, inv_m;
    int clip_vloss;
};

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
    return v;
}

// rows lane + 64 j of a set, j < PH_J: R <= 64 PH_J (LB_DS_MAX_ELEMENTS_TRAIN = 257)
constexpr int PH_J = 5;
__global__ __launch_bounds__(256) void k_ppo_head(PPOHeadParams p) {
    const int lane = threadIdx.x & 63;
    const int64_t nw = (int64_t)gridDim.x * (blockDim.x / 64);
    const int R = p.R;
    for (int64_t s = (int64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6); s < p.M; s += nw) {
        const float* lg = p.logits + s * R;
        bool v[PH_J], m[PH_J];
        float l[PH_J], lp[PH_J], pr[PH_J];
        float lmax = -INFINITY;
#pragma unroll
        for (int j = 0; j < PH_J; ++j) {
            const int r = lane + 64 * j;
            v[j] = r < R;
            m[j] = v[j] && (!p.masks || p.masks[s * R + r]);
            l[j] = v[j] ? (m[j] ? lg[r] : -1e8f) : -INFINITY;
            lmax = fmaxf(lmax, l[j]);
        }
        const float mx = wave_max(lmax);
        float es = 0.f;
#pragma unroll
        for (int j = 0; j < PH_J; ++j) es += v[j] ? expf(l[j] - mx) : 0.f;
        const float lse = mx + logf(wave_sum(es));
        float hs = 0.f;
#pragma unroll
        for (int j = 0; j < PH_J; ++j) {
            lp[j] = l[j] - lse;
            pr[j] = v[j] ? expf(lp[j]) : 0.f;
            hs += v[j] ? pr[j] * lp[j] : 0.f;
        }
        const float H = -wave_sum(hs);
        const int a = (int)p.actions[s];
        float lpa = lp[0];
#pragma unroll
        for (int j = 1; j < PH_J; ++j) lpa = (a >> 6) == j ? lp[j] : lpa;
        const float nlp = __shfl(lpa, a & 63);
        const float logratio = nlp - p.oldlogp[s];
        const float ratio = expf(logratio);
        const float A = p.adv[s];
        const float lo = 1.f - p.clip, hi = 1.f + p.clip;
        const float rc = fminf(fmaxf(ratio, lo), hi);
        const float pg1 = -A * ratio, pg2 = -A * rc;
        const float w1 = pg1 > pg2 ? 1.f : (pg1 == pg2 ? 0.5f : 0.f);
        const float inr = (ratio >= lo && ratio <= hi) ? 1.f : 0.f;
        const float g_nlp = p.inv_m * (w1 * (-A) + (1.f - w1) * (-A) * inr) * ratio;
        const float ge = p.ent_coef * p.inv_m;
#pragma unroll
        for (int j = 0; j < PH_J; ++j) {
            const int r = lane + 64 * j;
            if (v[j]) p.dlogits[s * R + r] = m[j] ? g_nlp * ((r == a ? 1.f : 0.f) - pr[j]) + ge * pr[j] * (lp[j] + H) : 0.f;
        }
        if (lane == 0) {
            const float v = p.value[s], rt = p.ret[s], vo = p.vold[s];
            const float vu = (v - rt) * (v - rt);
            float vt = vu, gv;
            if (p.clip_vloss) {
                const float d = v - vo;
                const float vc = vo + fminf(fmaxf(d, -p.clip), p.clip);
                const float vcl = (vc - rt) * (vc - rt);
                vt = fmaxf(vu, vcl);
                const float wu = vu > vcl ? 1.f : (vu == vcl ? 0.5f : 0.f);
                const float inv = (d >= -p.clip && d <= p.clip) ? 1.f : 0.f;
                gv = wu * 2.f * (v - rt) + (1.f - wu) * 2.f * (vc - rt) * inv;
            } else {
                gv = 2.f * (v - rt);
            }
            p.dvalue[s] = p.vf_coef * 0.5f * p.inv_m * gv;
            const float pgt = fmaxf(pg1, pg2);
            float* t = p.terms + s * 6;
            t[0] = pgt;
            t[1] = vt;
            t[2] = H;
            t[3] = (ratio - 1.f) - logratio;
            t[4] = fabsf(ratio - 1.f) > p.clip ? 1.f : 0.f;
            t[5] = pgt - p.ent_coef * H + p.vf_coef * 0.5f * vt;
        }
    }
}

// DQN loss head (dqn_deepset.py:180-187) in one launch, one wave per sample:
// td = r + gamma max_r q_next[r] (1 - done) (the target network's max; float32 in the
// reference's operation order), old = q[a], sq_err = (td - old)^2 (F.mse_loss's terms), and
// the loss's gradient w.r.t. q: 2 (old - td) / M at column a, 0 elsewhere (gather's backward).
struct DQNHeadParams {
    const float* q;       // [M][R] Q(obs) of the network being trained
    const float* q_next;  // [M][R] the target network's Q(next_obs)
    const int64_t* actions;
    const float* rewards;
    const float* dones;
    int64_t M;
    int R;
    float gamma, two_over_m;
    float* dq;      // [M][R]
    float* sq_err;  // [M]
    float* td;      // [M] or NULL
    float* old;     // [M] or NULL
    float* loss;    // [1] or NULL: mean of sq_err (k_dqn_head_block only)
};
__global__ __launch_bounds__(256) void k_dqn_head(DQNHeadParams p) {
    const int lane = threadIdx.x & 63;
    const int64_t nw = (int64_t)gridDim.x * (blockDim.x / 64);
    const int R = p.R;
    for (int64_t s = (int64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6); s < p.M; s += nw) {
        float m = -INFINITY;
        for (int r = lane; r < R; r += 64) m = fmaxf(m, p.q_next[s * R + r]);
        const float tmax = wave_max(m);
        const float td = p.rewards[s] + p.gamma * tmax * (1.f - p.dones[s]);
        const int a = (int)p.actions[s];
        const float old = p.q[s * R + a];
        const float d = td - old;
        const float g = p.two_over_m * (old - td);
        for (int r = lane; r < R; r += 64) p.dq[s * R + r] = r == a ? g : 0.f;
        if (lane == 0) {
            p.sq_err[s] = d * d;
            if (p.td) p.td[s] = td;
            if (p.old) p.old[s] = old;
        }
    }
}

// the same head for up to DQN_HEAD_BLOCK_MAX samples in one block, one lane per sample, and
// the loss (the mean of the squared errors, summed in float64 in a fixed tree) in the same
// launch: the DQN's 128-sample train step then needs no separate mean kernel
constexpr int DQN_HEAD_BLOCK_MAX = 1024;
__global__ __launch_bounds__(DQN_HEAD_BLOCK_MAX) void k_dqn_head_block(DQNHeadParams p) {
    __shared__ double part[DQN_HEAD_BLOCK_MAX / 64];
    const int s = threadIdx.x, R = p.R;
    double sq = 0.0;
    if (s < p.M) {
        float m = -INFINITY;
        for (int r = 0; r < R; ++r) m = fmaxf(m, p.q_next[(int64_t)s * R + r]);
        const float td = p.rewards[s] + p.gamma * m * (1.f - p.dones[s]);
        const int a = (int)p.actions[s];
        const float old = p.q[(int64_t)s * R + a];
        const float d = td - old;
        const float g = p.two_over_m * (old - td);
        for (int r = 0; r < R; ++r) p.dq[(int64_t)s * R + r] = r == a ? g : 0.f;
        const float e = d * d;
        p.sq_err[s] = e;
        if (p.td) p.td[s] = td;
        if (p.old) p.old[s] = old;
        sq = (double)e;
    }
    for (int o = 32; o > 0; o >>= 1) sq += __shfl_down(sq, o);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = sq;
    __syncthreads();
    if (threadIdx.x == 0) {
        double t = 0.0;
        for (int w = 0; w < (int)(blockDim.x >> 6); ++w) t += part[w];
        *p.loss = (float)(t / (double)p.M);
    }
}

// lb_ds_pack_backward: one thread per image float; transposed fragment order for the
// 64x64 matrices (lane l of fragment (nt, k) holds W^T[16nt + (l & 15)][in(k, l >> 4)])
__device__ __forceinline__ void ds_pack_bwd_one(const lb_ds_weights& w, float* out, int i) {
    if (i >= DSB_FLOATS) return;
    if (i >= DSB_A3L) {
        const int j = i - DSB_A3L;
        const float* v = j < 64 ? w.actor_lambda[2] : w.actor_gamma[2];
        out[i] = v[j & 63];
        return;
    }
    const float* srcs[6] = {w.actor_lambda[1], w.actor_gamma[1], w.critic_lambda[1],
                            w.critic_gamma[1], w.critic_lambda[2], w.critic_gamma[2]};
    const float* src = srcs[i >> 12];
    const int idx = i & 4095;
    const int f = idx >> 6, lane = idx & 63;
    const int nt = f >> 4, k = f & 15;
    const int row = 16 * nt + (lane & 15);                        // output of W^T = input of W
    const int in = 16 * (k >> 2) + 4 * (lane >> 4) + (k & 3);     // input of W^T = output of W
    out[i] = src ? src[in * 64 + row] : 0.f;
}
__global__ void k_ds_pack_bwd(lb_ds_weights w, float* out) {
    ds_pack_bwd_one(w, out, blockIdx.x * blockDim.x + threadIdx.x);
}
// lb_ds_pack_pair: both images of the same weights in one launch (the first blocks the forward
// image, the rest the backward image); a DQN train period packs them once at its start
constexpr int DS_PACK_BLOCKS = (DS_IMG_FLOATS + 255) / 256, DSB_PACK_BLOCKS = (DSB_FLOATS + 255) / 256;
__global__ void k_ds_pack_pair(lb_ds_weights w, float* out, float* bout) {
    if ((int)blockIdx.x < DS_PACK_BLOCKS) ds_pack_one(w, out, blockIdx.x * 256 + threadIdx.x);
    else ds_pack_bwd_one(w, bout, (blockIdx.x - DS_PACK_BLOCKS) * 256 + threadIdx.x);
}

// ---- lb_ds_set_grads: out[m][n] = scale * sum_s A(s, m) B(s, n), one job per weight
// gradient (fused_train.py's _over_sets and sums), the sets staged through LDS in chunks
struct SetGradJob {
    const float* a;  // amode 0: A(s, m) = a[s lda + m]; 1: A = 1; 2: A(s, 0) = sum_{r < alen} a[s lda + r]
    int lda, M, amode, alen;
    const float* b;  // B(s, n) = b[s ldb + n]
    int ldb, N;
    float scale;
    float* out;      // [M][N]
};
constexpr int SG_JOBS = 8, SG_CH = 64, SG_THREADS = 512, SG_PER = SG_CH * 64 / SG_THREADS;
constexpr int SG_TILES = 64 * 64 / SG_THREADS;  // blocks per job
struct SetGradParams {
    SetGradJob job[SG_JOBS];
    int64_t S;
};

// a chunk's loads are all issued before the first is used (the DQN's 128 sets: two chunks,
// two memory round trips per block); the row sums take 4 lanes per set
// (block (bx, by): job by, outputs bx SG_THREADS ..; sa, sb: the block's LDS chunk buffers)
__device__ __forceinline__ void ds_set_grads_body(const SetGradParams& p, int bx, int by, float (*sa)[64],
                                                  float (*sb)[64]) {
    const SetGradJob j = p.job[by];
    const int tile = bx * SG_THREADS;
    if (tile >= j.M * j.N) return;  // (block-uniform)
    const int e = tile + threadIdx.x;
    const bool on = e < j.M * j.N;
    const int m = on ? e / j.N : 0, n = on ? e % j.N : 0;
    float acc = 0.f;
    for (int64_t s0 = 0; s0 < p.S; s0 += SG_CH) {
        const int cs = p.S - s0 < SG_CH ? (int)(p.S - s0) : SG_CH;
        float rb[SG_PER], ra[SG_PER];
#pragma unroll
        for (int q = 0; q < SG_PER; ++q) {
            const int i = threadIdx.x + q * SG_THREADS, s = i >> 6, c = i & 63;
            rb[q] = (s < cs && c < j.N) ? j.b[(s0 + s) * j.ldb + c] : 0.f;
            ra[q] = (s < cs && c < j.M && j.amode == 0) ? j.a[(s0 + s) * j.lda + c] : 1.f;
        }
        float rs = 0.f;
        if (j.amode == 2) {  // lane (set threadIdx / 4, part threadIdx % 4): rows part, part + 4, ...
            const int s = threadIdx.x >> 2, part = threadIdx.x & 3;
            if (s < cs) {
                const float* row = j.a + (s0 + s) * j.lda;
                float t0 = 0.f, t1 = 0.f;
                int r = part;
                for (; r + 4 < j.alen; r += 8) {
                    t0 += row[r];
                    t1 += row[r + 4];
                }
                if (r < j.alen) t0 += row[r];
                rs = t0 + t1;
            }
            rs += __shfl_xor(rs, 1);
            rs += __shfl_xor(rs, 2);
        }
        __syncthreads();  // (the previous chunk is consumed)
#pragma unroll
        for (int q = 0; q < SG_PER; ++q) {
            const int i = threadIdx.x + q * SG_THREADS;
            sb[i >> 6][i & 63] = rb[q];
            if (j.amode != 2 || (i & 63) != 0) sa[i >> 6][i & 63] = ra[q];  // (row sums: below)
        }
        if (j.amode == 2 && (threadIdx.x & 3) == 0 && (int)(threadIdx.x >> 2) < cs) sa[threadIdx.x >> 2][0] = rs;
        __syncthreads();
        if (on)
            for (int s = 0; s < cs; ++s) acc += sa[s][m] * sb[s][n];
    }
    if (on) j.out[e] = j.scale * acc;
}
__global__ __launch_bounds__(SG_THREADS) void k_ds_set_grads(SetGradParams p) {
    __shared__ float sa[SG_CH][64], sb[SG_CH][64];
    ds_set_grads_body(p, blockIdx.x, blockIdx.y, sa, sb);
}
// lb_ds_train_backward_sets: the weight-gradient slot reduction and the set-gradient jobs in one
// launch (blocks below DSR_BLOCKS reduce, the rest are k_ds_set_grads' blocks): the DQN train
// step's two last launches after the backward
static_assert(SG_THREADS == DSR_COLS * DSR_GROUPS, "one block size for both parts");
__global__ __launch_bounds__(SG_THREADS) void k_ds_wgrad_reduce_sets(const float* wpart, float* out, int actor,
                                                                    int critic, SetGradParams sg) {
    __shared__ float part[DSR_GROUPS][DSR_COLS];
    __shared__ float sa[SG_CH][64], sb[SG_CH][64];
    if ((int)blockIdx.x < DSR_BLOCKS) {
        ds_wgrad_reduce_body(wpart, out, actor, critic, blockIdx.x, part);
    } else {
        const int v = blockIdx.x - DSR_BLOCKS;
        ds_set_grads_body(sg, v % SG_TILES, v / SG_TILES, sa, sb);
    }
}

// ---- lb_ds_over_sets: out[m][n] = scale * sum_s A(s, m) B(s, n) over a large batch of sets
// (the PPO minibatch's 51,200), every job in two launches.  The sums over the sets of the
// training step -- the Gamma gradients (sum_r dz)^T max_set(h), the critic's Lambda3, rho's
// two weight gradients and the bias sums -- were chunked torch GEMMs plus a reduction each
// (~20 + 10 us per product: ~0.25 ms per minibatch).  Here one wave owns one job's whole output
// over one span of OS_SPAN sets on v_mfma_f32_16x16x4_f32 with the sets as the K dimension, its
// partial sums to workspace[span][job output]; k_ds_over_sets_reduce adds the spans in
// ascending order (deterministic) and scales.
// Operand layout: a job of M > 16 outputs takes four 16-row tiles i with output m = 4c + i on
// tile row c, so lane (c, q) reads A(s, 4c .. 4c + 3) of set s = s0 + 4k + q as one float4 and
// feeds the four tiles (the same for N > 16 and the columns); M, N <= 16: one tile, m = c.
// A 64 x 64 job: two float4 loads per 16 independent MFMAs, every input read once.
struct OverSetsJob {
    const float* a;  // A(s, m) = a[s lda + m]; NULL: A(s, 0) = 1 (M == 1: a plain sum of B)
    int64_t lda;
    const float* b;  // B(s, n) = b[s ldb + n]
    int64_t ldb;
    int M, N;
    float scale;
    float* out;      // [M][N]
    int ooff;        // offset of the job's outputs in a span's workspace row
    int vec;         // bit 0 (1): a (b) 16-byte aligned with lda (ldb) % 4 == 0: float4 operand loads
};
constexpr int OS_JOBS = 16, OS_SPAN = LB_DS_OVER_SETS_SPAN, OS_D = 8;
struct OverSetsParams {
    OverSetsJob job[OS_JOBS];
    int njobs, row;  // row: workspace floats per span (the sum of the jobs' M N)
    int64_t S;
    float* work;     // [spans][row]
};

// this lane's operand values of set s for the T tiles (T = 4: outputs 4c .. 4c + 3; T = 1:
// output c), zero past the job's outputs or the span
template <int T>
__device__ __forceinline__ void os_load(const float* p, int64_t ld, int K, bool vec, int c, int64_t s, bool in,
                                        float (&v)[T]) {
    if constexpr (T == 4) {
        if (vec && in && 4 * c + 3 < K) {  // (vec: p 16-byte aligned, ld % 4 == 0)
            const float4 q = *reinterpret_cast<const float4*>(p + s * ld + 4 * c);
            v[0] = q.x;
            v[1] = q.y;
            v[2] = q.z;
            v[3] = q.w;
        } else {
#pragma unroll
            for (int i = 0; i < 4; ++i) v[i] = (in && 4 * c + i < K) ? p[s * ld + 4 * c + i] : 0.f;
        }
    } else {
        v[0] = (in && c < K) ? (p ? p[s * ld + c] : 1.f) : 0.f;
    }
}

template <int MT, int NT>
__device__ __forceinline__ void os_job(const OverSetsJob& j, int64_t s0, int64_t s1, float* w, int lane) {
    const int c = lane & 15, q = lane >> 4;
    dsf4 acc[MT][NT];
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[i][t] = dsf4{0.f, 0.f, 0.f, 0.f};
    // (a wave-uniform trip count: the MFMA takes every lane; sets past the span's end load 0).
    // The operands of OS_D steps are in flight ahead of the MFMAs (a block holds at most four
    // jobs' waves, so the latency is hidden in the wave, not by occupancy)
    const int steps = (int)((s1 - s0 + 3) / 4);
    float av[OS_D][MT], bv[OS_D][NT];
#pragma unroll
    for (int d = 0; d < OS_D; ++d) {
        const int64_t s = s0 + 4 * d + q;
        os_load<MT>(j.a, j.lda, j.M, j.vec & 1, c, s, s < s1, av[d]);
        os_load<NT>(j.b, j.ldb, j.N, j.vec & 2, c, s, s < s1, bv[d]);
    }
    for (int k = 0; k < steps; k += OS_D) {
#pragma unroll
        for (int d = 0; d < OS_D; ++d) {
            if (k + d < steps) {
#pragma unroll
                for (int i = 0; i < MT; ++i)
#pragma unroll
                    for (int t = 0; t < NT; ++t)
                        acc[i][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[d][i], bv[d][t], acc[i][t], 0, 0, 0);
            }
            const int64_t s = s0 + 4 * (k + d + OS_D) + q;
            os_load<MT>(j.a, j.lda, j.M, j.vec & 1, c, s, s < s1, av[d]);
            os_load<NT>(j.b, j.ldb, j.N, j.vec & 2, c, s, s < s1, bv[d]);
        }
    }
    // tile (i, t) register r of lane (c, q): tile row 4q + r, tile column c
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int m = MT == 4 ? 4 * (4 * q + r) + i : 4 * q + r, n = NT == 4 ? 4 * c + t : c;
                if (m < j.M && n < j.N) w[m * j.N + n] = acc[i][t][r];
            }
}

__global__ __launch_bounds__(256) void k_ds_over_sets(OverSetsParams p) {
    const int wj = blockIdx.x * 4 + (threadIdx.x >> 6);  // this wave's job
    if (wj >= p.njobs) return;                           // (wave-uniform)
    const OverSetsJob j = p.job[wj];
    const int64_t s0 = (int64_t)blockIdx.y * OS_SPAN;
    const int64_t s1 = s0 + OS_SPAN < p.S ? s0 + OS_SPAN : p.S;
    float* w = p.work + (int64_t)blockIdx.y * p.row + j.ooff;
    const int lane = threadIdx.x & 63;
    if (j.M > 16) {
        if (j.N > 16) os_job<4, 4>(j, s0, s1, w, lane);
        else os_job<4, 1>(j, s0, s1, w, lane);
    } else {
        if (j.N > 16) os_job<1, 4>(j, s0, s1, w, lane);
        else os_job<1, 1>(j, s0, s1, w, lane);
    }
}

// out[e] = scale * sum over the spans of the partial sums: block = 64 outputs x OS_RG span
// groups (thread (e, g) adds spans g, g + OS_RG, ... in order), the groups combined in LDS in
// a fixed order (deterministic)
constexpr int OS_RG = 8;
__global__ __launch_bounds__(64 * OS_RG) void k_ds_over_sets_reduce(OverSetsParams p, int spans) {
    __shared__ float part[OS_RG][64];
    const int o = threadIdx.x & 63, g = threadIdx.x >> 6;
    const int e = blockIdx.x * 64 + o;
    float acc = 0.f;
    if (e < p.row)
        for (int z = g; z < spans; z += OS_RG) acc += p.work[(int64_t)z * p.row + e];
    part[g][o] = acc;
    __syncthreads();
    if (g != 0 || e >= p.row) return;
    float t = part[0][o];
#pragma unroll
    for (int i = 1; i < OS_RG; ++i) t += part[i][o];
    int ji = 0;
    while (ji + 1 < p.njobs && e >= p.job[ji + 1].ooff) ++ji;
    const OverSetsJob& j = p.job[ji];
    j.out[e - j.ooff] = j.scale * t;
}

}  // namespace lbk
