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
//   * k_ds_train_bwd (here), one wave per set, 8 waves per CU (2 per SIMD, so one wave's
//     vector work runs beside the other's matrix work), the set streamed 16 rows at a time
//     in two passes:
//       pass 1 (h2, h1): every set-wise max and its FIRST argmax row (torch.max's index)
//         in one sweep, the set sums the Gamma / Lambda3 gradients need, and the set sum
//         of dz2 in closed form: sum_r dz2[r][o] = Lambda3[o] sum_r dl[r] elu'(h2[r][o])
//         - g3 Gamma3[o] elu'(max_r h2[r][o]) (the critic: u, vv for Lambda3, Gamma3);
//       pass 2, per 16-row tile: dz2 from h2; dLambda2 += dz2^T h1 (MFMA over rows: the
//         tiles go through a per-wave LDS transpose); the data gradient dz1 = (dz2
//         Lambda2 - [r == argmax] Gamma2^T sum dz2) act'(h1) (f32 MFMA); dLambda1 += dz1^T obs.
//     The weight-gradient accumulators stay in registers across all the sets a wave
//     visits; at the end the block sums its 8 waves in LDS in a fixed order and writes one
//     slot, and k_ds_wgrad_reduce sums the slots in a fixed order: no per-row gradient
//     reaches HBM, and the result does not depend on timing.  Per-set vectors (set-wise
//     max, gradient sums over the set, the last-layer products) give every Gamma gradient
//     and the rank-1 last-layer gradients as small GEMMs over the sets.
// Layout conventions (fragment order, accumulator layout) are those of lbk8s_deepsets.h:
// lane l holds set element (l & 15) of each 16-row tile, and at k-step k the features
// 16(k >> 2) + 4(l >> 4) + (k & 3).
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
    DSV_MAX0 = 0,     // [8]  max over the set of the observation
    DSV_GA3 = 8,      // actor: sum_r dlogit[r] h2[r]           (Lambda3 gradient)
    DSV_MAX2A = 72,   //        max_set h2                       (Gamma3)
    DSV_GS2A = 136,   //        sum_r dz2[r]                     (Gamma2)
    DSV_MAX1A = 200,  //        max_set h1                       (Gamma2)
    DSV_GS1A = 264,   //        sum_r dz1[r]                     (Gamma1)
    DSV_CS2 = 328,    // critic: sum_r c2[r]                     (Lambda3: rank 1, d psi = dmean / R)
    DSV_MAX2C = 392,  //         max_set c2                      (Gamma3)
    DSV_GS2C = 456,   //         sum_r dz2[r]
    DSV_MAX1C = 520,  //         max_set c1
    DSV_GS1C = 584,   //         sum_r dz1[r]
    DSV_FLOATS = 648,
};

constexpr int DSB_BLOCK = 512;                       // 8 waves: 2 per SIMD, one block per CU
constexpr int DSW_FLOATS = 4608;                     // per head: dLambda2 [64][64], dLambda1 [64][8]
constexpr int DSW_GRID = 256;                        // fixed grid (any B): one block per CU
constexpr int DSW_SLOTS = DSW_GRID;                  // one partial-sum slot per block
constexpr int DST_STRIDE = 80;                       // LDS transpose row stride (floats)
constexpr int DSB_LDS_W = 16384;                     // head weights in LDS (the critic's four 64x64)

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

// element (row, feature f) of a staged 16-row tile: rows 80 floats apart, the feature index
// XOR-swizzled by 4 (row & 7) (groups of 4 features stay contiguous), so the row-major
// float4 stores of 8 consecutive rows and the transposed reads (4 rows x 16 features per
// 32 lanes) are bank-conflict free.  TBOff holds that index for each access pattern in
// closed form: a few lane offsets, the rest compile-time constants.
struct TBOff {
    int rd;        // transposed reads, row 4c + grp, feature col + 16m:  rd + 320c + 16 (m ^ (c & 1))
    int we, wo;    // row-major float4 stores, row col, features 16nt + 4grp:  (nt even ? we : wo) + 16nt
    int w80, w81;  // observation stores, row col, feature 4kk + grp (kk = 0, 1)
    int r8;        // observation reads, row 4c + grp, feature col & 7:  r8 + 320c + 16 (c & 1)
};
__device__ __forceinline__ TBOff tb_offsets(int col, int grp) {
    static_assert(DST_STRIDE == 80, "closed forms assume 80-float rows");
    TBOff o;
    const int b = (col >> 2) & 1, base0 = col * DST_STRIDE + 4 * (grp ^ (col & 3));
    o.rd = grp * DST_STRIDE + (col ^ (4 * grp));
    o.we = base0 + 16 * b;
    o.wo = base0 - 16 * b;
    o.w80 = col * DST_STRIDE + grp + 4 * (col & 7);
    o.w81 = col * DST_STRIDE + grp + 4 * (1 ^ (col & 7));
    o.r8 = grp * DST_STRIDE + ((col & 7) ^ (4 * grp));
    return o;
}

// one 16-row tile of a [B][R][64] plane in fragment layout (lane: row 16t + col, features
// 16nt + 4grp + i); rows past R read row R - 1 (in bounds, no branch) and are zeroed
__device__ __forceinline__ void load_tile(const float* plane, float (&h)[16], int64_t env, int R, int row, int grp) {
    const bool ok = row < R;
    const float* q = plane + (env * (int64_t)R + (ok ? row : R - 1)) * 64 + 4 * grp;
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
        const float4 v = *reinterpret_cast<const float4*>(q + 16 * nt);
        h[4 * nt] = ok ? v.x : 0.f;
        h[4 * nt + 1] = ok ? v.y : 0.f;
        h[4 * nt + 2] = ok ? v.z : 0.f;
        h[4 * nt + 3] = ok ? v.w : 0.f;
    }
}

// a 16-feature vector in k layout (every lane of a row holds it): column-0 lanes store it
__device__ __forceinline__ void store_vec(float* dst, const float (&v)[16], int col, int grp) {
    if (col != 0) return;
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
        *reinterpret_cast<float4*>(dst + 16 * nt + 4 * grp) = make_float4(v[4 * nt], v[4 * nt + 1], v[4 * nt + 2], v[4 * nt + 3]);
}

// argmax rows (< 80) of 16 features, one byte each: id[k >> 2] byte (k & 3)
__device__ __forceinline__ int id_of(const int (&id)[4], int k) { return (id[k >> 2] >> (8 * (k & 3))) & 0xff; }

// d act / d z from the activation's output: ReLU (ACT 1) y > 0; ELU (ACT 2) y > 0 ? 1 : y + 1
template <int ACT>
__device__ __forceinline__ float dact(float y) {
    return ACT == 1 ? (y > 0.f ? 1.f : 0.f) : (y > 0.f ? 1.f : y + 1.f);
}

// per-lane running (max, first row) of a pass-1 sweep -> the set's max and FIRST argmax row
// (torch.max's index) per feature: the max over the 16 lanes of the row group, then the
// smallest row among the lanes that hold it
__device__ __forceinline__ void finish_argmax(float (&m)[16], const float (&r)[16], int (&id)[4]) {
    float M[16], c[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) M[k] = m[k];
    row_reduce<true>(M);
#pragma unroll
    for (int k = 0; k < 16; ++k) c[k] = m[k] == M[k] ? -r[k] : -1e9f;
    row_reduce<true>(c);
#pragma unroll
    for (int k = 0; k < 16; ++k) m[k] = M[k];
#pragma unroll
    for (int q = 0; q < 4; ++q)
        id[q] = (int)(-c[4 * q]) | ((int)(-c[4 * q + 1]) << 8) | ((int)(-c[4 * q + 2]) << 16) | ((int)(-c[4 * q + 3]) << 24);
}

// stage one 16-row tile (this lane: row col, features 16nt + 4grp + i) in LDS
__device__ __forceinline__ void stage_tile(float* buf, const float (&v)[16], const TBOff& o) {
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
        *reinterpret_cast<float4*>(buf + (nt % 2 == 0 ? o.we : o.wo) + 16 * nt) =
            make_float4(v[4 * nt], v[4 * nt + 1], v[4 * nt + 2], v[4 * nt + 3]);
}

// acc[mt][nt] += dz^T h over one staged 16-row tile: MFMA k-step c contracts rows
// 4c..4c+3; A[m][kk] = dz[4c + kk][16mt + m], B[kk][n] = h[4c + kk][16nt + n]
__device__ __forceinline__ void wgrad64(const float* la, const float* lb, dsf4 (&acc)[4][4], const TBOff& o) {
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        float av[4], bv[4];
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            const int i = o.rd + 320 * c + 16 * (m ^ (c & 1));
            av[m] = la[i];
            bv[m] = lb[i];
        }
#pragma unroll
        for (int mt = 0; mt < 4; ++mt)
#pragma unroll
            for (int nt = 0; nt < 4; ++nt) acc[mt][nt] = mfma4(av[mt], bv[nt], acc[mt][nt]);
    }
}

// acc[mt] += dz^T obs over one staged tile (dz1 in la): the tile's observation rows (this
// lane: features grp and 4 + grp of row col) are staged in lb, B columns 8..15 read as zero
__device__ __forceinline__ void wgrad8(const float* la, float* lb, const float (&x0)[2], dsf4 (&acc)[4], int col,
                                       const TBOff& o) {
    lb[o.w80] = x0[0];
    lb[o.w81] = x0[1];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const float x = lb[o.r8 + 320 * c + 16 * (c & 1)];
        const float xv = col < 8 ? x : 0.f;
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) acc[mt] = mfma4(la[o.rd + 320 * c + 16 * (mt ^ (c & 1))], xv, acc[mt]);
    }
}

// One launch per head (HEAD 0 actor, 1 critic).
template <int HEAD>
__global__ __launch_bounds__(DSB_BLOCK, 1) void k_ds_train_bwd(DSBwdParams p) {
    constexpr int ACT1 = HEAD == 0 ? 1 : 2;  // activation after layer 1: ReLU (actor) / ELU (critic)
    __shared__ __attribute__((aligned(16))) float W[DSB_LDS_W];
    __shared__ __attribute__((aligned(16))) float TB[DSB_BLOCK / 64][2][16 * DST_STRIDE];
    // the head's weights: [0, 8192) Lambda2^T, Gamma2^T (fragment order); the actor's
    // Lambda3 / Gamma3 rows at 8192 / 8256, the critic's Lambda3^T / Gamma3^T at 8192 / 12288
    {
        const int n = HEAD == 0 ? 8192 : 16384;
        const float* src = p.wb + (HEAD == 0 ? DSB_A2LT : DSB_C2LT);
        for (int i = threadIdx.x * 4; i < n; i += DSB_BLOCK * 4)
            *reinterpret_cast<float4*>(W + i) = *reinterpret_cast<const float4*>(src + i);
        if (HEAD == 0)
            for (int i = threadIdx.x; i < 128; i += DSB_BLOCK) W[8192 + i] = p.wb[DSB_A3L + i];
    }
    __syncthreads();
    const float* LT = W;  // (Gamma2^T at W + 4096)
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t nwaves = (int64_t)gridDim.x * (DSB_BLOCK / 64);
    float* la = TB[wv][0];
    float* lb = TB[wv][1];
    const int R = p.R, ntl = (R + 15) / 16;
    const int col = lane & 15, grp = lane >> 4;
    const TBOff tbo = tb_offsets(col, grp);
    const int64_t plane = p.B * (int64_t)R * 64;
    const float* in1 = HEAD == 0 ? p.save_actor : p.save_critic;  // h1 / c1
    const float* in2 = in1 + plane;                                 // h2 / c2
    const bool do_max0 = HEAD == 0 || !p.actor;
    dsf4 w2[4][4], w1[4];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) w2[mt][nt] = dsf4{0.f, 0.f, 0.f, 0.f};
        w1[mt] = dsf4{0.f, 0.f, 0.f, 0.f};
    }
    for (int64_t env = (int64_t)blockIdx.x * (DSB_BLOCK / 64) + wv; env < p.B; env += nwaves) {
        float* sv = p.setvec + env * DSV_FLOATS;
        // weights re-read from LDS per set (an opaque offset: no loop-invariant hoisting)
        uint32_t wso = 0;
        asm volatile("" : "+s"(wso));
        const float* Ws = W + wso;
        // ---- pass 1: set-wise maxima + first argmax rows, set sums
        float mx2[16], r2[16], mx1[16], r1[16], S[16], G[16], g3 = 0.f;
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            mx2[k] = mx1[k] = -INFINITY;
            r2[k] = r1[k] = 0.f;
            S[k] = G[k] = 0.f;
        }
        for (int t = 0; t < ntl; ++t) {
            const int row = 16 * t + col;
            const bool ok = row < R;
            const float fr = (float)row;
            float a[16], h[16];
            load_tile(in2, a, env, R, row, grp);
            load_tile(in1, h, env, R, row, grp);
            float w = ok ? 1.f : 0.f;  // actor: dlogit of the row (0 past R); critic: row validity
            if (HEAD == 0) {
                const float d = p.dlogits[env * R + (ok ? row : R - 1)];
                w = ok ? d : 0.f;
                g3 += w;
            }
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                const bool u2 = ok && a[k] > mx2[k];  // strict: rows ascend, the first maximum stays
                mx2[k] = u2 ? a[k] : mx2[k];
                r2[k] = u2 ? fr : r2[k];
                S[k] += w * dact<2>(a[k]);
                G[k] += HEAD == 0 ? w * a[k] : a[k];  // actor: sum dl h2 (Lambda3); critic: sum c2
                const bool u1 = ok && h[k] > mx1[k];
                mx1[k] = u1 ? h[k] : mx1[k];
                r1[k] = u1 ? fr : r1[k];
            }
        }
        int id2[4], id1[4];
        finish_argmax(mx2, r2, id2);
        finish_argmax(mx1, r1, id1);
        row_reduce<false>(S);
        row_reduce<false>(G);
        store_vec(sv + (HEAD == 0 ? DSV_MAX2A : DSV_MAX2C), mx2, col, grp);
        store_vec(sv + (HEAD == 0 ? DSV_GA3 : DSV_CS2), G, col, grp);
        store_vec(sv + (HEAD == 0 ? DSV_MAX1A : DSV_MAX1C), mx1, col, grp);
        // per feature o, dz2[r][o] = (c1[o] - [r == argmax] c2[o]) elu'(h2[r][o]) with
        // actor c1 = dl[r] Lambda3[o] (row-dependent through dl), c2 = g3 Gamma3[o];
        // critic c1 = u[o] = (Lambda3^T dmean)[o] / R, c2 = vv[o] = (Gamma3^T dmean)[o]
        float c1[16], c2[16];
        if (HEAD == 0) {
            float gv[4] = {g3, 0.f, 0.f, 0.f};
            row_reduce<false>(gv);
            g3 = gv[0];
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                const int f = 16 * (k >> 2) + 4 * grp + (k & 3);
                c1[k] = Ws[8192 + f];
                c2[k] = g3 * Ws[8256 + f];
            }
        } else {
            float gm[16];
            const float* q = p.dmean + env * 64 + 4 * grp;
#pragma unroll
            for (int nt = 0; nt < 4; ++nt) {
                const float4 v = *reinterpret_cast<const float4*>(q + 16 * nt);
                gm[4 * nt] = v.x;
                gm[4 * nt + 1] = v.y;
                gm[4 * nt + 2] = v.z;
                gm[4 * nt + 3] = v.w;
            }
            const float invR = 1.0f / (float)R;
#pragma unroll
            for (int nt = 0; nt < 4; ++nt) {
                dsf4 uu = {0.f, 0.f, 0.f, 0.f}, w = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int k = 0; k < 16; ++k) {
                    uu = mfma4(Ws[8192 + (nt * 16 + k) * 64 + lane], gm[k] * invR, uu);
                    w = mfma4(Ws[12288 + (nt * 16 + k) * 64 + lane], gm[k], w);
                }
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    c1[4 * nt + i] = uu[i];
                    c2[4 * nt + i] = w[i];
                }
            }
        }
        // sum over the set of dz2, in closed form from pass 1's sums (S = sum of dl elu'(h2)
        // for the actor, of elu'(c2) over the set's rows for the critic)
        float gs[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) gs[k] = c1[k] * S[k] - c2[k] * dact<2>(mx2[k]);
        store_vec(sv + (HEAD == 0 ? DSV_GS2A : DSV_GS2C), gs, col, grp);
        // v = Gamma2^T (sum dz2): the pooled part of the layer-1 data gradient
        float v[16];
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) {
            dsf4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int k = 0; k < 16; ++k) acc = mfma4(Ws[4096 + (nt * 16 + k) * 64 + lane], gs[k], acc);
#pragma unroll
            for (int i = 0; i < 4; ++i) v[4 * nt + i] = acc[i];
        }
        // ---- pass 2, per tile: dz2, dLambda2 += dz2^T h1, dz1, dLambda1 += dz1^T obs
        float gs1[16], m0[2] = {-INFINITY, -INFINITY};
#pragma unroll
        for (int k = 0; k < 16; ++k) gs1[k] = 0.f;
        for (int t = 0; t < ntl; ++t) {
            // Lambda2^T re-read from LDS per tile: an opaque offset keeps the compiler from
            // hoisting its 64 loop-invariant fragments into registers (which spilled)
            uint32_t wo = 0;
            asm volatile("" : "+s"(wo));
            const float* LTt = LT + wo;
            const int row = 16 * t + col;
            const bool ok = row < R;
            float a[16], h[16], x0[2];
            load_tile(in2, a, env, R, row, grp);
            load_tile(in1, h, env, R, row, grp);
            {
                const float* x = p.obs + (env * (int64_t)R + (ok ? row : R - 1)) * 8;
                x0[0] = ok ? x[grp] : 0.f;
                x0[1] = ok ? x[4 + grp] : 0.f;
            }
            float d = 0.f;
            if (HEAD == 0) {
                const float dv = p.dlogits[env * R + (ok ? row : R - 1)];
                d = ok ? dv : 0.f;
            }
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                const float x = (HEAD == 0 ? d * c1[k] : c1[k]) - (row == id_of(id2, k) ? c2[k] : 0.f);
                a[k] = ok ? x * dact<2>(a[k]) : 0.f;
            }
            stage_tile(la, a, tbo);
            stage_tile(lb, h, tbo);
            wgrad64(la, lb, w2, tbo);
#pragma unroll
            for (int nt = 0; nt < 4; ++nt) {
                dsf4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int k = 0; k < 16; ++k) acc = mfma4(LTt[(nt * 16 + k) * 64 + lane], a[k], acc);
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int kk = 4 * nt + i;
                    const float x = acc[i] - (row == id_of(id1, kk) ? v[kk] : 0.f);
                    h[kk] = ok ? x * dact<ACT1>(h[kk]) : 0.f;
                }
            }
#pragma unroll
            for (int k = 0; k < 16; ++k) gs1[k] += h[k];
            if (do_max0 && ok) {
                m0[0] = max2(m0[0], x0[0]);
                m0[1] = max2(m0[1], x0[1]);
            }
            stage_tile(la, h, tbo);
            wgrad8(la, lb, x0, w1, col, tbo);
        }
        row_reduce<false>(gs1);
        store_vec(sv + (HEAD == 0 ? DSV_GS1A : DSV_GS1C), gs1, col, grp);
        if (do_max0) {
            row_reduce<true>(m0);
            if (col == 0) {
                sv[DSV_MAX0 + grp] = m0[0];
                sv[DSV_MAX0 + 4 + grp] = m0[1];
            }
        }
    }
    // the block's 8 waves summed in LDS in a fixed order, one slot per block
    __syncthreads();
    float* red = &TB[0][0][0];
    static_assert(sizeof(TB) / sizeof(float) >= DSW_FLOATS, "reduction buffer");
    for (int w = 0; w < DSB_BLOCK / 64; ++w) {
        if (wv == w) {
#pragma unroll
            for (int mt = 0; mt < 4; ++mt)
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int o = 16 * mt + 4 * grp + i;
#pragma unroll
                    for (int nt = 0; nt < 4; ++nt) {
                        float& r = red[o * 64 + 16 * nt + col];
                        r = w == 0 ? w2[mt][nt][i] : r + w2[mt][nt][i];
                    }
                    if (col < 8) {
                        float& r = red[4096 + o * 8 + col];
                        r = w == 0 ? w1[mt][i] : r + w1[mt][i];
                    }
                }
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
__global__ __launch_bounds__(DSR_COLS * DSR_GROUPS) void k_ds_wgrad_reduce(const float* wpart, float* out, int actor,
                                                                           int critic) {
    __shared__ float part[DSR_GROUPS][DSR_COLS];
    const int c = threadIdx.x % DSR_COLS, g = threadIdx.x / DSR_COLS;
    const int j = blockIdx.x * DSR_COLS + c;
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

__global__ __launch_bounds__(256) void k_ppo_head(PPOHeadParams p) {
    const int lane = threadIdx.x & 63;
    const int64_t nw = (int64_t)gridDim.x * (blockDim.x / 64);
    const int R = p.R;
    for (int64_t s = (int64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6); s < p.M; s += nw) {
        const float* lg = p.logits + s * R;
        const int r0 = lane, r1 = lane + 64;
        const bool v0 = r0 < R, v1 = r1 < R;
        const bool m0 = v0 && (!p.masks || p.masks[s * R + r0]);
        const bool m1 = v1 && (!p.masks || p.masks[s * R + r1]);
        const float l0 = v0 ? (m0 ? lg[r0] : -1e8f) : -INFINITY;
        const float l1 = v1 ? (m1 ? lg[r1] : -1e8f) : -INFINITY;
        const float mx = wave_max(fmaxf(l0, l1));
        const float e0 = v0 ? expf(l0 - mx) : 0.f, e1 = v1 ? expf(l1 - mx) : 0.f;
        const float lse = mx + logf(wave_sum(e0 + e1));
        const float lp0 = l0 - lse, lp1 = l1 - lse;
        const float p0 = v0 ? expf(lp0) : 0.f, p1 = v1 ? expf(lp1) : 0.f;
        const float H = -wave_sum((v0 ? p0 * lp0 : 0.f) + (v1 ? p1 * lp1 : 0.f));
        const int a = (int)p.actions[s];
        const float nlp = __shfl(a < 64 ? lp0 : lp1, a & 63);
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
        if (v0) p.dlogits[s * R + r0] = m0 ? g_nlp * ((r0 == a ? 1.f : 0.f) - p0) + ge * p0 * (lp0 + H) : 0.f;
        if (v1) p.dlogits[s * R + r1] = m1 ? g_nlp * ((r1 == a ? 1.f : 0.f) - p1) + ge * p1 * (lp1 + H) : 0.f;
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

// lb_ds_pack_backward: one thread per image float; transposed fragment order for the
// 64x64 matrices (lane l of fragment (nt, k) holds W^T[16nt + (l & 15)][in(k, l >> 4)])
__global__ void k_ds_pack_bwd(lb_ds_weights w, float* out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
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

}  // namespace lbk
