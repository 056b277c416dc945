// lbk8s_deepsets.h — fused deep-sets forward (actor logits + critic value) for MI355X.
//
// Reference networks: envs/deep_sets_agent_original.py — EquivariantLayer (:56-66),
// EquivariantDeepSet actor (:69-83), InvariantDeepSet critic (:86-106).  One launch reads
// each env's (R x 8) observation once and produces its R logits and its value.
//
// MFMA formulation (f32 in / f32 accumulate, v_mfma_f32_16x16x4_f32, exact f32 products):
// every layer is computed TRANSPOSED, D[feature][set element] = W · H, so a layer's
// accumulator tile — lane l holds features 4(l>>4)+i (i<4) of set element l&15 — is, after
// the activation, already the B operand of the next layer: k-step (t, i) of the next layer
// consumes features {16t + 4q + i : q = l>>4}.  The weights are packed host-side in that
// k order ("fragment order", lbk8s/fused.py), one 256-byte fragment per (output tile,
// k-step), and staged once per block in LDS.  The set-wise max of a layer input is a
// 16-lane max over the lanes of one lane group (plus an elementwise max over set tiles);
// replicated over the 16 columns it is the B operand of the Gamma pass, whose result
// (every column equal) initialises the accumulator: acc = -Gamma·max + Lambda·H.
// Invalid set columns (padding past R) are excluded from the max and the mean.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "lbk8s.h"

namespace lbk {

typedef float dsf4 __attribute__((ext_vector_type(4)));

struct DSParams {
    const float* obs;     // [B][R][8]
    const float* wfrag;   // fragment-ordered weights (see lbk8s/fused.py)
    float* logits;        // [B][R]
    float* value;         // [B]
    int64_t B;
    int R;
    int actor, critic;    // which heads to evaluate (DQN: actor only)
};

// fragment layout of the packed weights (floats).  A matrix with KS input k-steps and NT
// 16-row output tiles occupies NT*KS fragments of 64 floats; fragment (nt, k), lane l holds
// W[16nt + (l&15)][in(k, l>>4)], in(k, q) = 4k + q for the 8 obs features and
// 16(k>>2) + 4q + (k&3) for 64 hidden features (rows >= out_features are zero).
enum : int {
    DS_A1L = 0, DS_A1G = 512, DS_A2L = 1024, DS_A2G = 5120, DS_A3L = 9216, DS_A3G = 10240,
    DS_C1L = 11264, DS_C1G = 11776, DS_C2L = 12288, DS_C2G = 16384, DS_C3L = 20480, DS_C3G = 24576,
    DS_R1W = 28672, DS_R1B = 32768, DS_R2W = 32832, DS_R2B = 33856, DS_FLOATS = 33860,
};

constexpr int DS_BLOCK = 512;       // 8 waves: 2 per SIMD
constexpr int DS_LDS_FLOATS = DS_FLOATS;  // 132 KiB of weight fragments: one block per CU

__device__ __forceinline__ dsf4 mfma4(float a, float b, dsf4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ float group_max16(float v) {
#pragma unroll
    for (int m = 8; m >= 1; m >>= 1) v = fmaxf(v, __shfl_xor(v, m, 64));
    return v;
}
__device__ __forceinline__ float group_sum16(float v) {
#pragma unroll
    for (int m = 8; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
    return v;
}

__device__ __forceinline__ float act_elu(float x) { return x > 0.f ? x : expm1f(x); }
__device__ __forceinline__ float act_relu(float x) { return x > 0.f ? x : 0.f; }

// set-wise max of a fragment set: per k-step, max over valid columns of every set tile,
// then over the 16 lanes of the lane group -> the value replicated in every column
template <int TS, int KS>
__device__ __forceinline__ void set_max(const float (&h)[TS][KS], float (&mx)[KS], int lane, int R) {
#pragma unroll
    for (int k = 0; k < KS; ++k) {
        float v = -INFINITY;
#pragma unroll
        for (int s = 0; s < TS; ++s)
            if (16 * s + (lane & 15) < R) v = fmaxf(v, h[s][k]);
        mx[k] = group_max16(v);
    }
}

// one equivariant layer with 64 outputs: out = act(Lambda·h - Gamma·max_set(h))
// KS = input k-steps (2 for the 8-feature obs, 16 for 64 features)
template <int TS, int KS, int ACT>
__device__ __forceinline__ void eq_layer64(const float* L, const float* G, const float (&h)[TS][KS],
                                           const float (&mx)[KS], float (&out)[TS][16], int lane) {
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
        dsf4 g = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int k = 0; k < KS; ++k) g = mfma4(G[(nt * KS + k) * 64 + lane], mx[k], g);
#pragma unroll
        for (int s = 0; s < TS; ++s) {
            dsf4 acc = -g;
#pragma unroll
            for (int k = 0; k < KS; ++k) acc = mfma4(L[(nt * KS + k) * 64 + lane], h[s][k], acc);
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                float x = acc[i];
                out[s][4 * nt + i] = ACT == 1 ? act_relu(x) : (ACT == 2 ? act_elu(x) : x);
            }
        }
    }
}

template <int TS>
__global__ __launch_bounds__(DS_BLOCK, 2) void k_deepsets_fwd(DSParams p) {
    __shared__ __attribute__((aligned(16))) float W[DS_LDS_FLOATS];
    // stage the weight fragments (once per block; blocks are persistent)
    for (int i = threadIdx.x * 4; i < DS_FLOATS; i += DS_BLOCK * 4)
        *reinterpret_cast<float4*>(W + i) = *reinterpret_cast<const float4*>(p.wfrag + i);
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const int64_t wave = (int64_t)blockIdx.x * (DS_BLOCK / 64) + (threadIdx.x >> 6);
    const int64_t nwaves = (int64_t)gridDim.x * (DS_BLOCK / 64);
    const int R = p.R;
    const int col = lane & 15, grp = lane >> 4;
    for (int64_t env = wave; env < p.B; env += nwaves) {
        // obs -> layer-1 B fragments: k-step kk holds feature 4kk + grp of set element col
        const float* x = p.obs + env * (int64_t)R * 8;
        float h0[TS][2];
#pragma unroll
        for (int s = 0; s < TS; ++s) {
            const int row = 16 * s + col;
#pragma unroll
            for (int kk = 0; kk < 2; ++kk) h0[s][kk] = row < R ? x[row * 8 + 4 * kk + grp] : 0.f;
        }
        float m0[2];
        set_max<TS, 2>(h0, m0, lane, R);

        float h1[TS][16], m1[16], h2[TS][16], m2[16];
        // ---- actor: Eq(8->64) ReLU Eq(64->64) ELU Eq(64->1)
        if (p.actor) {
            eq_layer64<TS, 2, 1>(W + DS_A1L, W + DS_A1G, h0, m0, h1, lane);
            set_max<TS, 16>(h1, m1, lane, R);
            eq_layer64<TS, 16, 2>(W + DS_A2L, W + DS_A2G, h1, m1, h2, lane);
            set_max<TS, 16>(h2, m2, lane, R);
            const float* L = W + DS_A3L;
            const float* G = W + DS_A3G;
            dsf4 g = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int k = 0; k < 16; ++k) g = mfma4(G[k * 64 + lane], m2[k], g);
#pragma unroll
            for (int s = 0; s < TS; ++s) {
                dsf4 acc = -g;
#pragma unroll
                for (int k = 0; k < 16; ++k) acc = mfma4(L[k * 64 + lane], h2[s][k], acc);
                const int row = 16 * s + col;
                if (grp == 0 && row < R) p.logits[env * R + row] = acc[0];  // output feature 0
            }
        }
        if (!p.critic) continue;

        // ---- critic: psi = Eq ELU Eq ELU Eq, mean over the set, rho = Linear ELU Linear
        eq_layer64<TS, 2, 2>(W + DS_C1L, W + DS_C1G, h0, m0, h1, lane);
        set_max<TS, 16>(h1, m1, lane, R);
        eq_layer64<TS, 16, 2>(W + DS_C2L, W + DS_C2G, h1, m1, h2, lane);
        set_max<TS, 16>(h2, m2, lane, R);
        eq_layer64<TS, 16, 0>(W + DS_C3L, W + DS_C3G, h2, m2, h1, lane);
        float mean[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            float v = 0.f;
#pragma unroll
            for (int s = 0; s < TS; ++s)
                if (16 * s + col < R) v += h1[s][k];
            mean[k] = group_sum16(v) / (float)R;
        }
        float r1[16];
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) {
            dsf4 acc;
#pragma unroll
            for (int i = 0; i < 4; ++i) acc[i] = W[DS_R1B + 16 * nt + 4 * grp + i];
#pragma unroll
            for (int k = 0; k < 16; ++k) acc = mfma4(W[DS_R1W + (nt * 16 + k) * 64 + lane], mean[k], acc);
#pragma unroll
            for (int i = 0; i < 4; ++i) r1[4 * nt + i] = act_elu(acc[i]);
        }
        dsf4 v = {W[DS_R2B], 0.f, 0.f, 0.f};
#pragma unroll
        for (int k = 0; k < 16; ++k) v = mfma4(W[DS_R2W + k * 64 + lane], r1[k], v);
        if (lane == 0) p.value[env] = v[0];
    }
}

// lb_ds_pack: one thread per fragment float
struct DSPackRegion {
    int off, nout, kin, ks;
};

__device__ __forceinline__ float ds_frag_value(const float* w, int nout, int kin, int ks, int idx) {
    const int f = idx >> 6, lane = idx & 63;
    const int nt = f / ks, k = f - nt * ks;
    const int row = 16 * nt + (lane & 15), q = lane >> 4;
    const int in = kin == 8 ? 4 * k + q : 16 * (k >> 2) + 4 * q + (k & 3);
    return (w && row < nout) ? w[row * kin + in] : 0.f;
}

__global__ void k_ds_pack(lb_ds_weights w, float* out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= DS_FLOATS) return;
    // regions in layout order: (start, pointer, out features, in features, k-steps)
    const int starts[16] = {DS_A1L, DS_A1G, DS_A2L, DS_A2G, DS_A3L, DS_A3G, DS_C1L, DS_C1G,
                            DS_C2L, DS_C2G, DS_C3L, DS_C3G, DS_R1W, DS_R1B, DS_R2W, DS_R2B};
    int r = 15;
    while (r > 0 && i < starts[r]) --r;
    const int idx = i - starts[r];
    float v = 0.f;
    switch (r) {
        case 0: v = ds_frag_value(w.actor_lambda[0], 64, 8, 2, idx); break;
        case 1: v = ds_frag_value(w.actor_gamma[0], 64, 8, 2, idx); break;
        case 2: v = ds_frag_value(w.actor_lambda[1], 64, 64, 16, idx); break;
        case 3: v = ds_frag_value(w.actor_gamma[1], 64, 64, 16, idx); break;
        case 4: v = ds_frag_value(w.actor_lambda[2], 1, 64, 16, idx); break;
        case 5: v = ds_frag_value(w.actor_gamma[2], 1, 64, 16, idx); break;
        case 6: v = ds_frag_value(w.critic_lambda[0], 64, 8, 2, idx); break;
        case 7: v = ds_frag_value(w.critic_gamma[0], 64, 8, 2, idx); break;
        case 8: v = ds_frag_value(w.critic_lambda[1], 64, 64, 16, idx); break;
        case 9: v = ds_frag_value(w.critic_gamma[1], 64, 64, 16, idx); break;
        case 10: v = ds_frag_value(w.critic_lambda[2], 64, 64, 16, idx); break;
        case 11: v = ds_frag_value(w.critic_gamma[2], 64, 64, 16, idx); break;
        case 12: v = ds_frag_value(w.rho_w1, 64, 64, 16, idx); break;
        case 13: v = w.rho_b1 ? w.rho_b1[idx] : 0.f; break;
        case 14: v = ds_frag_value(w.rho_w2, 1, 64, 16, idx); break;
        default: v = (w.rho_b2 && idx == 0) ? w.rho_b2[0] : 0.f; break;
    }
    out[i] = v;
}

}  // namespace lbk
