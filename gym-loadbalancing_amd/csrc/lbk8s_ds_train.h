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
//   * k_ds_train_bwd (here), one wave per set: back through every equivariant layer in
//     registers — the set-wise max's argmax is recomputed from the saved activation, the
//     activation derivative is taken from the activation itself (ReLU: y > 0; ELU: y > 0 ?
//     1 : y + 1), the data gradient of each 64x64 layer is an f32 MFMA against the
//     transposed Lambda.  The two big weight gradients of each head, dLambda2 = dz2^T h1
//     (64x64) and dLambda1 = dz1^T obs (64x8), are accumulated over all the sets a wave
//     visits by MFMA (contraction over rows: each 16-row tile is transposed through a
//     per-wave LDS buffer) in accumulator registers, written once per wave into a slot of
//     a workspace, and summed over slots by k_ds_wgrad_reduce: no per-row gradient ever
//     reaches HBM.  Per-set vectors (set-wise max, gradient sums over the set, the
//     last-layer products) give every Gamma gradient and the rank-1 last-layer gradients
//     as small GEMMs over the sets.
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

constexpr int DSB_BLOCK = 256;                       // 4 waves, 1 per SIMD: 512 registers per lane
constexpr int DSW_FLOATS = 4608;                     // per head: dLambda2 [64][64], dLambda1 [64][8]
constexpr int DSW_SLOTS = 1024;                      // one per wave of the fixed grid
constexpr int DSW_GRID = DSW_SLOTS / (DSB_BLOCK / 64);
constexpr int DST_STRIDE = 80;                       // LDS transpose row stride (floats): 16 banks per row group

struct DSBwdParams {
    const float* obs;          // [B][R][8]
    const float* wb;           // backward weight image [DSB_FLOATS]
    const float* save_actor;   // [2][B][R][64] h1, h2
    const float* save_critic;  // [2][B][R][64] c1, c2
    const float* dlogits;      // [B][R]
    const float* dmean;        // [B][64]
    float* wpart;              // [DSW_SLOTS][2][DSW_FLOATS] per-wave weight-gradient partials
    float* setvec;             // [B][DSV_FLOATS]
    int64_t B;
    int R;
    int actor, critic;
};

template <int TS>
__device__ __forceinline__ void load_rows(const float* plane, float (&h)[TS][16], int64_t env, int R, int col,
                                          int grp) {
#pragma unroll
    for (int t = 0; t < TS; ++t) {
        const int row = 16 * t + col;
        if (row < R) {
            const float* q = plane + (env * (int64_t)R + row) * 64 + 4 * grp;
#pragma unroll
            for (int nt = 0; nt < 4; ++nt) {
                const float4 v = *reinterpret_cast<const float4*>(q + 16 * nt);
                h[t][4 * nt] = v.x;
                h[t][4 * nt + 1] = v.y;
                h[t][4 * nt + 2] = v.z;
                h[t][4 * nt + 3] = v.w;
            }
        } else {
#pragma unroll
            for (int k = 0; k < 16; ++k) h[t][k] = 0.f;
        }
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

// per feature: max over the set's valid rows and the FIRST row attaining it (torch.max's
// index, where the reference's autograd sends the pooled gradient)
template <int TS>
__device__ __forceinline__ void set_max_idx(const float (&h)[TS][16], float (&mx)[16], int (&id)[4], int col, int R) {
    float m[16], c[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        float v = -INFINITY;
#pragma unroll
        for (int t = 0; t < TS; ++t)
            if (16 * t + col < R) v = max2(v, h[t][k]);
        m[k] = v;
    }
    row_reduce<true>(m);
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        float v = -1e9f;  // max of -row == min row
#pragma unroll
        for (int t = 0; t < TS; ++t) {
            const int row = 16 * t + col;
            if (row < R && h[t][k] == m[k]) v = max2(v, -(float)row);
        }
        c[k] = v;
    }
    row_reduce<true>(c);
#pragma unroll
    for (int k = 0; k < 16; ++k) mx[k] = m[k];
#pragma unroll
    for (int q = 0; q < 4; ++q)
        id[q] = (int)(-c[4 * q]) | ((int)(-c[4 * q + 1]) << 8) | ((int)(-c[4 * q + 2]) << 16) | ((int)(-c[4 * q + 3]) << 24);
}

// sum over the set (rows past R hold 0)
template <int TS>
__device__ __forceinline__ void set_sum(const float (&h)[TS][16], float (&s)[16]) {
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        float v = 0.f;
#pragma unroll
        for (int t = 0; t < TS; ++t) v += h[t][k];
        s[k] = v;
    }
    row_reduce<false>(s);
}

// d act / d z from the activation's output: ReLU (ACT 1) y > 0; ELU (ACT 2) y > 0 ? 1 : y + 1
template <int ACT>
__device__ __forceinline__ float dact(float y) {
    return ACT == 1 ? (y > 0.f ? 1.f : 0.f) : (y > 0.f ? 1.f : y + 1.f);
}

// Back through a 64 -> 64 equivariant layer z = Lambda h - Gamma max_set(h), h = act(z_prev):
// g = dz (this layer), gs = sum_r dz; h (in: the layer input, out: dz of the layer below)
//   dh[r][i] = sum_o Lambda[o][i] dz[r][o] - [r == argmax_i] sum_o Gamma[o][i] gs[o]
//   dz_prev  = dh * act'(h)
template <int TS, int ACT>
__device__ __forceinline__ void eq_back64(const float* LT, const float* GT, const float (&g)[TS][16],
                                          const float (&gs)[16], float (&h)[TS][16], const int (&id)[4], int lane,
                                          int col, int R) {
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
        dsf4 v = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int k = 0; k < 16; ++k) v = mfma4(GT[(nt * 16 + k) * 64 + lane], gs[k], v);
#pragma unroll
        for (int t = 0; t < TS; ++t) {
            dsf4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int k = 0; k < 16; ++k) acc = mfma4(LT[(nt * 16 + k) * 64 + lane], g[t][k], acc);
            const int row = 16 * t + col;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int kk = 4 * nt + i;
                const float x = acc[i] - (row == id_of(id, kk) ? v[i] : 0.f);
                h[t][kk] = row < R ? x * dact<ACT>(h[t][kk]) : 0.f;
            }
        }
    }
}

// stage one 16-row tile (this lane: row col, features 16nt + 4grp + i) row-major in LDS
__device__ __forceinline__ void stage_tile(float* buf, const float (&v)[16], int col, int grp) {
    float* q = buf + col * DST_STRIDE + 4 * grp;
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
        *reinterpret_cast<float4*>(q + 16 * nt) = make_float4(v[4 * nt], v[4 * nt + 1], v[4 * nt + 2], v[4 * nt + 3]);
}

// acc[mt][nt] += dz^T h over one staged 16-row tile: MFMA k-step c contracts rows
// 4c..4c+3; A[m][kk] = dz[4c + kk][16mt + m], B[kk][n] = h[4c + kk][16nt + n]
__device__ __forceinline__ void wgrad64(const float* la, const float* lb, dsf4 (&acc)[4][4], int col, int grp) {
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        float av[4], bv[4];
        const int r = (4 * c + grp) * DST_STRIDE + col;
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            av[m] = la[r + 16 * m];
            bv[m] = lb[r + 16 * m];
        }
#pragma unroll
        for (int mt = 0; mt < 4; ++mt)
#pragma unroll
            for (int nt = 0; nt < 4; ++nt) acc[mt][nt] = mfma4(av[mt], bv[nt], acc[mt][nt]);
    }
}

// acc[mt] += dz^T obs over one staged tile: the tile's observation rows (h0: this lane holds
// features 4kk + grp of row col) are staged next to it, B columns 8..15 read as zero
template <int TS>
__device__ __forceinline__ void wgrad8(const float* la, float* lb, const float (&h0)[TS][2], int t, dsf4 (&acc)[4],
                                       int col, int grp) {
    lb[col * DST_STRIDE + grp] = h0[t][0];
    lb[col * DST_STRIDE + 4 + grp] = h0[t][1];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const int r = (4 * c + grp) * DST_STRIDE + col;
        const float xv = col < 8 ? lb[r] : 0.f;
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) acc[mt] = mfma4(la[r + 16 * mt], xv, acc[mt]);
    }
}

// a set's observation in fragment layout: h0[t][kk] = feature 4kk + grp of row 16t + col
template <int TS>
__device__ __forceinline__ void load_obs(const float* obs, int64_t env, int R, int col, int grp, float (&h0)[TS][2]) {
    const float* x = obs + env * (int64_t)R * 8;
#pragma unroll
    for (int t = 0; t < TS; ++t) {
        const int row = 16 * t + col;
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) h0[t][kk] = row < R ? x[row * 8 + 4 * kk + grp] : 0.f;
    }
}

// the head's upstream gradient for one set: actor dlogits rows (dl), critic dmean (gm, k layout)
template <int TS, int HEAD>
__device__ __forceinline__ void load_upstream(const DSBwdParams& p, int64_t env, int col, int grp, float (&dl)[TS],
                                              float (&gm)[16]) {
    if (HEAD == 0) {
#pragma unroll
        for (int t = 0; t < TS; ++t) {
            const int row = 16 * t + col;
            dl[t] = row < p.R ? p.dlogits[env * p.R + row] : 0.f;
        }
    } else {
        const float* q = p.dmean + env * 64 + 4 * grp;
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) {
            const float4 v = *reinterpret_cast<const float4*>(q + 16 * nt);
            gm[4 * nt] = v.x;
            gm[4 * nt + 1] = v.y;
            gm[4 * nt + 2] = v.z;
            gm[4 * nt + 3] = v.w;
        }
    }
}

__device__ __forceinline__ void wpart_store(float* wp, const dsf4 (&a2)[4][4], const dsf4 (&a1)[4], int col, int grp) {
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int o = 16 * mt + 4 * grp + i;
#pragma unroll
            for (int nt = 0; nt < 4; ++nt) wp[o * 64 + 16 * nt + col] = a2[mt][nt][i];
            if (col < 8) wp[4096 + o * 8 + col] = a1[mt][i];
        }
}

// One launch per head (HEAD 0 actor, 1 critic): a head's 80 accumulator registers, its two
// activation tiles and the set-wise bookkeeping fit the 512 registers of a wave.  With one
// wave per SIMD nothing else hides memory latency, so the loop is software-pipelined: the
// next set's layer-2 input is loaded as soon as the layer-2 tile is dead (after the data
// gradient), its layer-1 input and observation once the dLambda1 tiles are done.
template <int TS, int HEAD>
__global__ __launch_bounds__(DSB_BLOCK, 1) void k_ds_train_bwd(DSBwdParams p) {
    __shared__ __attribute__((aligned(16))) float W[DSB_FLOATS];
    __shared__ __attribute__((aligned(16))) float TB[DSB_BLOCK / 64][2][16 * DST_STRIDE];
    for (int i = threadIdx.x * 4; i < DSB_FLOATS; i += DSB_BLOCK * 4)
        *reinterpret_cast<float4*>(W + i) = *reinterpret_cast<const float4*>(p.wb + i);
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const int64_t wave = (int64_t)blockIdx.x * (DSB_BLOCK / 64) + (threadIdx.x >> 6);
    const int64_t nwaves = (int64_t)gridDim.x * (DSB_BLOCK / 64);
    float* la = TB[threadIdx.x >> 6][0];
    float* lb = TB[threadIdx.x >> 6][1];
    const int R = p.R;
    const int col = lane & 15, grp = lane >> 4;
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
    float a[TS][16], h[TS][16], h0[TS][2], dl[TS], gm[16];
    int64_t env = wave;
    if (env < p.B) {
        load_rows<TS>(in2, a, env, R, col, grp);
        load_upstream<TS, HEAD>(p, env, col, grp, dl, gm);
        load_rows<TS>(in1, h, env, R, col, grp);
        load_obs<TS>(p.obs, env, R, col, grp, h0);
    }
    for (; env < p.B; env += nwaves) {
        const int64_t nxt = env + nwaves;
        float* sv = p.setvec + env * DSV_FLOATS;
        float mx[16], gs[16];
        int id[4];
        if (HEAD == 0) {
            set_max_idx<TS>(a, mx, id, col, R);
            store_vec(sv + DSV_MAX2A, mx, col, grp);
            // Lambda3 product and the set sum of dlogits, in one row reduction
            float red[20];
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                float v = 0.f;
#pragma unroll
                for (int t = 0; t < TS; ++t) v += dl[t] * a[t][k];
                red[k] = v;
            }
            {
                float v = 0.f;
#pragma unroll
                for (int t = 0; t < TS; ++t) v += dl[t];
                red[16] = v;
                red[17] = red[18] = red[19] = 0.f;
            }
            row_reduce<false>(red);
            {
                float ga[16];
#pragma unroll
                for (int k = 0; k < 16; ++k) ga[k] = red[k];
                store_vec(sv + DSV_GA3, ga, col, grp);
            }
            const float g3 = red[16];
            // dz2 = (dlogit Lambda3 - [r == argmax] g3 Gamma3) * elu'(h2)
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                const int f = 16 * (k >> 2) + 4 * grp + (k & 3);
                const float l3 = W[DSB_A3L + f], gg = g3 * W[DSB_A3G + f];
#pragma unroll
                for (int t = 0; t < TS; ++t) {
                    const int row = 16 * t + col;
                    const float x = dl[t] * l3 - (row == id_of(id, k) ? gg : 0.f);
                    a[t][k] = row < R ? x * dact<2>(a[t][k]) : 0.f;
                }
            }
        } else {
            // d psi[r] = dmean / R on every row: u = Lambda3^T dmean / R (row-independent),
            // vv = Gamma3^T (sum_r d psi[r]) = Gamma3^T dmean
            float u[16], vv[16];
            const float invR = 1.0f / (float)R;
#pragma unroll
            for (int nt = 0; nt < 4; ++nt) {
                dsf4 uu = {0.f, 0.f, 0.f, 0.f}, w = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int k = 0; k < 16; ++k) {
                    uu = mfma4(W[DSB_C3LT + (nt * 16 + k) * 64 + lane], gm[k] * invR, uu);
                    w = mfma4(W[DSB_C3GT + (nt * 16 + k) * 64 + lane], gm[k], w);
                }
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    u[4 * nt + i] = uu[i];
                    vv[4 * nt + i] = w[i];
                }
            }
            set_max_idx<TS>(a, mx, id, col, R);
            store_vec(sv + DSV_MAX2C, mx, col, grp);
            set_sum<TS>(a, gs);
            store_vec(sv + DSV_CS2, gs, col, grp);
#pragma unroll
            for (int k = 0; k < 16; ++k)
#pragma unroll
                for (int t = 0; t < TS; ++t) {
                    const int row = 16 * t + col;
                    const float x = u[k] - (row == id_of(id, k) ? vv[k] : 0.f);
                    a[t][k] = row < R ? x * dact<2>(a[t][k]) : 0.f;
                }
        }
        set_sum<TS>(a, gs);
        store_vec(sv + (HEAD == 0 ? DSV_GS2A : DSV_GS2C), gs, col, grp);
        set_max_idx<TS>(h, mx, id, col, R);
        store_vec(sv + (HEAD == 0 ? DSV_MAX1A : DSV_MAX1C), mx, col, grp);
#pragma unroll
        for (int t = 0; t < TS; ++t) {
            stage_tile(la, a[t], col, grp);
            stage_tile(lb, h[t], col, grp);
            wgrad64(la, lb, w2, col, grp);
        }
        if (HEAD == 0) eq_back64<TS, 1>(W + DSB_A2LT, W + DSB_A2GT, a, gs, h, id, lane, col, R);
        else eq_back64<TS, 2>(W + DSB_C2LT, W + DSB_C2GT, a, gs, h, id, lane, col, R);
        if (nxt < p.B) {  // layer-2 tile and upstream gradient are dead: prefetch the next set's
            load_rows<TS>(in2, a, nxt, R, col, grp);
            load_upstream<TS, HEAD>(p, nxt, col, grp, dl, gm);
        }
        set_sum<TS>(h, gs);
        store_vec(sv + (HEAD == 0 ? DSV_GS1A : DSV_GS1C), gs, col, grp);
#pragma unroll
        for (int t = 0; t < TS; ++t) {
            stage_tile(la, h[t], col, grp);
            wgrad8<TS>(la, lb, h0, t, w1, col, grp);
        }
        if (do_max0) {
            float m0[2];
            set_max_batched<TS, 1, 2>(h0, m0, col, R);
            if (col == 0) {
                sv[DSV_MAX0 + grp] = m0[0];
                sv[DSV_MAX0 + 4 + grp] = m0[1];
            }
        }
        if (nxt < p.B) {
            load_rows<TS>(in1, h, nxt, R, col, grp);
            load_obs<TS>(p.obs, nxt, R, col, grp, h0);
        }
    }
    // every wave of the fixed grid owns one slot (zeros if it saw no set)
    wpart_store(p.wpart + wave * (2 * DSW_FLOATS) + HEAD * DSW_FLOATS, w2, w1, col, grp);
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
