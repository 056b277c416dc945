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
// (every column equal) initialises the accumulator: acc = (-Gamma)·max + Lambda·H, with
// -Gamma stored by the pack kernel.
// Invalid set columns (padding past R) are excluded from the max and the mean.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "lbk8s.h"
#include "lbk8s_common.h"

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
    // training forward (TRAIN = true) only: activations kept for lb_ds_train_backward
    float* save_actor;    // [2][B][R][64]: actor h1 (after ReLU), h2 (after ELU)
    float* save_critic;   // [2][B][R][64]: critic c1, c2 (after ELU)
    float* psi_mean;      // [B][64]: critic psi output averaged over the set (rho runs in torch)
    float* setvec;        // [B][LB_DS_SETVEC_FLOATS]: set-wise maxima of the layer inputs and
                          // their first argmax rows (LB_DSV_MAX*, LB_DSV_ID*), for the backward
    // greedy action (inference only): actions[b] = first argmax over rows of
    // (masks[b][r] ? logits[b][r] : -1e8) (dqn_deepset.py:134-142); NULL = skip
    int32_t* actions;
    const uint8_t* masks;  // [B][R] or NULL (all valid)
    // argmax mode, lb_dqn_act: the DQN's explore decision first (ex_on); exploring, every env
    // takes its uniform random action (the env state's episode / step words) and no Q value
    // is computed
    int ex_on;
    lb_dqn_explore ex;
    const uint64_t* ex_acc3;
    const uint64_t* ex_sc;
    int64_t ex_env_offset;
    uint32_t ex_key0, ex_key1;
};

// lb_dqn_act's decision: true when this launch explores (the random actions are written)
__device__ __forceinline__ bool ds_dqn_explore(const DSParams& p) {
    const int64_t t = *p.ex.vstep_in;
    const bool explore = dqn_explores(p.ex, t);
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        *p.ex.explore_out = explore ? 1 : 0;
        *p.ex.vstep_out = t + 1;
    }
    if (!explore) return false;
    for (int64_t env = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; env < p.B; env += (int64_t)gridDim.x * blockDim.x)
        p.actions[env] = random_action_raw((uint64_t)(p.ex_env_offset + env), p.ex_acc3[env],
                                           (uint32_t)(p.ex_sc[env] & 0xFFFF), p.ex_key0, p.ex_key1, p.R);
    return true;
}

// fragment layout of the packed weights (floats).  A matrix with KS input k-steps and NT
// 16-row output tiles occupies NT*KS fragments of 64 floats; fragment (nt, k), lane l holds
// W[16nt + (l&15)][in(k, l>>4)], in(k, q) = 4k + q for the 8 obs features and
// 16(k>>2) + 4q + (k&3) for 64 hidden features (rows >= out_features are zero).
enum : int {
    DS_A1L = 0, DS_A1G = 512, DS_A2L = 1024, DS_A2G = 5120, DS_A3L = 9216, DS_A3G = 10240,
    DS_C1L = 11264, DS_C1G = 11776, DS_C2L = 12288, DS_C2G = 16384, DS_C3L = 20480, DS_C3G = 24576,
    DS_R1W = 28672, DS_R1B = 32768, DS_R2W = 32832, DS_R2B = 33856, DS_FLOATS = 33860,
};

constexpr int DS_BLOCK = 512;             // 8 waves: 2 per SIMD
constexpr int DS_LDS_FLOATS = DS_FLOATS;  // 132 KiB of weight fragments: one block per CU

// The VALU image (round 6), appended to the fragment image at DS_FLOATS, for the forwards with one
// env per wave iteration and at least three 16-element set tiles (R in 33..80: config 4's R = 65).
// There every matrix-VECTOR product of the networks -- each equivariant layer's Gamma term
// (Gamma max_set(h), one vector per set), the critic's layer 3 on the set mean and max, rho --
// filled one of the 16 columns of its MFMA tiles (64 MFMAs each, 33% of the forward's MFMA issue
// at R = 65); here each is 64 lane-wise dot products on the VALU (lane f: output feature f) from
// row-major weights, padded rows (stride 68 / 12 floats: a 16-lane ds_read_b128 group covers the
// 64 banks once).  The set-wise Lambda terms stay on MFMA (their fragments are copied here so the
// image is one contiguous LDS stage).  Gamma matrices are stored negated, as the fragments.
// The actor's last layer (64 -> 1) is two plain 64-vectors (A3V: Lambda3, A3GV: -Gamma3).
// Regions in stage order: the actor's, the critic's, rho's, then the extra-row block (XR, the
// training forward of R = 16 TS + 1 elements, below: the four layers' Lambda row-major).
enum : int {
    VG_RS = 68, VG_RS8 = 12,
    VG_A1L = 0, VG_A2L = 512, VG_A3V = 4608, VG_A3GV = 4672, VG_A1G = 4736, VG_A2G = 5504, VG_ACTOR = 9856,
    VG_C1L = 9856, VG_C2L = 10368, VG_C1G = 14464, VG_C2G = 15232, VG_C3L = 19584, VG_C3G = 23936,
    VG_CRITIC = 28288,
    VG_R1W = 28288, VG_R1B = 32640, VG_R2W = 32704, VG_R2B = 32768, VG_RHO = 32772,
    VG_XA1 = 32772, VG_XA2 = 33540, VG_XC1 = 37892, VG_XC2 = 38660, VG_FLOATS = 43012,
    DS_IMG_FLOATS = DS_FLOATS + VG_FLOATS,
    VG_SCRATCH = 128,  // per wave and env of a wave iteration: the matvec input x[64] and output y[64]
    // the XR forward's LDS: the actor and critic regions, then the extra-row block
    VGX_BASE = VG_CRITIC, VGX_A1 = VGX_BASE, VGX_A2 = VGX_BASE + (VG_XA2 - VG_XA1),
    VGX_C1 = VGX_BASE + (VG_XC1 - VG_XA1), VGX_C2 = VGX_BASE + (VG_XC2 - VG_XA1),
    VGX_END = VGX_BASE + (VG_FLOATS - VG_XA1),
};
// VG: the forwards with one env per wave iteration and >= 3 set tiles, and the greedy-action
// forward (MODE 2: the DQN's Q values) of small sets with one or two envs per iteration -- the
// same arithmetic as k_dqn_step's Q forward, so lb_dqn_act and lb_dqn_step pick the same actions.
// XR: the training forward (MODE 1, VG) of R = 16 TS + 1 set elements (config 4's R = 65: E = 64
// servers and the reject row).  The TS full tiles run as above; the one extra row -- a fifth
// 16-row tile with one live column, 20% of the forward's MFMA issue -- is VALU dot products per
// layer (lane f: output feature f), its outputs folded into the set-wise maxima, argmax rows and
// the psi sum as a last row.
template <int TS, int P, int MODE = 0, bool XR = false>
struct DSGeom {
    static constexpr bool VG = (TS >= 3 && P == 1) || (MODE == 2 && TS == 1 && P <= 2);
    static_assert(!XR || (VG && MODE == 1 && P == 1), "the extra row: one-env VALU-image training forward");
    static constexpr int IMG = XR ? VGX_END : (MODE == 1 ? VG_CRITIC : VG_RHO);
    static constexpr int LDS = VG ? IMG + (DS_BLOCK / 64) * P * VG_SCRATCH : DS_LDS_FLOATS;
};
static_assert(DSGeom<4, 1, 1, true>::LDS * 4 <= 160 * 1024, "XR forward LDS");
// (wave-local LDS ordering: the wave's own writes before its later reads by other lanes)
__device__ __forceinline__ void ds_wave_fence() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
// ELU(alpha=1) without a divergent branch: exp2 on the clamped argument
__device__ __forceinline__ float act_elu(float x) {
    const float e = __builtin_amdgcn_exp2f(fminf(x, 0.f) * 1.4426950408889634f) - 1.0f;
    return x > 0.f ? x : e;
}
__device__ __forceinline__ float act_relu(float x) { return x > 0.f ? x : 0.f; }
// the set's max (lane (col, grp) holds env col mod P's, feature in(k, grp)) into x[KS * 4]
// (P envs: env s's at x + 128 s, written by the lanes of column s)
template <int KS>
__device__ __forceinline__ void vg_put(const float (&mb)[KS], float* x, int col, int grp, int P = 1) {
    if (col >= P) return;
    x += 128 * col;
    if constexpr (KS == 2) {
        x[grp] = mb[0];
        x[4 + grp] = mb[1];
    } else {
#pragma unroll
        for (int t = 0; t < 4; ++t)
            *reinterpret_cast<float4*>(x + 16 * t + 4 * grp) = make_float4(mb[4 * t], mb[4 * t + 1], mb[4 * t + 2], mb[4 * t + 3]);
    }
}
// acc + sum_j W[f][j] x[j] for this lane's output feature f = lane (ascending j)
// (in groups of 16 inputs: the compiler would otherwise issue every LDS read of the row first and
// hold it in registers, 64 VGPRs for a 64-input row)
template <int KIN, int S>
__device__ __forceinline__ float vg_dot(const float* Wrm, const float* x, int lane, float acc) {
    const float* w = Wrm + lane * S;
#pragma unroll
    for (int j = 0; j < KIN; j += 4) {
        const float4 a = *reinterpret_cast<const float4*>(w + j), b = *reinterpret_cast<const float4*>(x + j);
        acc = fmaf(a.x, b.x, acc);
        acc = fmaf(a.y, b.y, acc);
        acc = fmaf(a.z, b.z, acc);
        acc = fmaf(a.w, b.w, acc);
        if ((j & 15) == 12) asm volatile("" : "+v"(acc));
    }
    return acc;
}
// (-Gamma) max_set(h) of each of the P envs by VALU into the scratch: y_s = xs + 128 s + 64.
// Lane f computes output f of every env (P dot products); the caller reads the accumulator
// layout, y_s[16 nt + 4 grp + i], where it initialises the accumulators (vg_init)
// (returns env 0's output f = lane: the XR forward's extra row starts from it)
template <int KS, int P>
__device__ __forceinline__ float vg_gamma(const float* Grm, const float (&mb)[KS], float* xs, int lane) {
    const int col = lane & 15, grp = lane >> 4;
    vg_put<KS>(mb, xs, col, grp, P);
    ds_wave_fence();
    float y0 = 0.f;
#pragma unroll
    for (int s = 0; s < P; ++s) {
        const float y = vg_dot<4 * KS, KS == 2 ? VG_RS8 : VG_RS>(Grm, xs + 128 * s, lane, 0.f);
        xs[128 * s + 64 + lane] = y;
        if (s == 0) y0 = y;
    }
    ds_wave_fence();
    return y0;
}
// XR: the extra row's layer output for feature f = lane, act(Lambda x + (-Gamma) max_set(h)):
// g the Gamma term (vg_gamma), x the row's layer input -- the observation row (KS = 2: lane
// (col, grp) holds features 4kk + grp, put by the column-0 lanes) or the previous layer's
// extra-row output (KS = 16: lane f holds feature f).  Accumulates Gamma first, then the inputs
// in order, as the tiles' chains.  The scratch's earlier reads have completed (eq_layer fences).
template <int KS, int ACT>
__device__ __forceinline__ float vg_xrow(const float* Lrm, const float* x2, float x64, float g, float* xs, int lane) {
    if constexpr (KS == 2) {
        const int col = lane & 15, grp = lane >> 4;
        if (col == 0) {
            xs[grp] = x2[0];
            xs[4 + grp] = x2[1];
        }
    } else {
        xs[lane] = x64;
    }
    ds_wave_fence();
    const float z = vg_dot<4 * KS, KS == 2 ? VG_RS8 : VG_RS>(Lrm, xs, lane, g);
    ds_wave_fence();
    return ACT == 1 ? act_relu(z) : act_elu(z);
}
// the extra row's output (lane f: feature f) in the accumulator layout: xr[k] = feature
// 16 (k >> 2) + 4 grp + (k & 3), the tiles' layout of this lane's row group
__device__ __forceinline__ void vg_xspread(float v, float* xs, int lane, float (&xr)[16]) {
    const int grp = lane >> 4;
    xs[lane] = v;
    ds_wave_fence();
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        const float4 q = *reinterpret_cast<const float4*>(xs + 16 * t + 4 * grp);
        xr[4 * t] = q.x;
        xr[4 * t + 1] = q.y;
        xr[4 * t + 2] = q.z;
        xr[4 * t + 3] = q.w;
    }
    ds_wave_fence();
}
__device__ __forceinline__ dsf4 vg_init(const float* xs, int s, int nt, int grp) {
    return *reinterpret_cast<const dsf4*>(xs + 128 * s + 64 + 16 * nt + 4 * grp);
}

__device__ __forceinline__ dsf4 mfma4(float a, float b, dsf4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// DPP inside a 16-lane row.  Reductions (max / sum over the 16 lanes, every lane gets the
// result) are quad_perm xor 1, xor 2, row_ror 4, row_ror 8, written as v_max/v_add with the
// DPP operand so there is no separate move; four independent values per asm block keep three
// VALU ops between a write and its DPP read (the hazard needs two wait states), and the
// leading s_nop covers whatever the compiler scheduled just before the block.
#define LBK_DPP4(OP, CTRL)                                                              \
    OP " %0, %0, %0 " CTRL " row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"             \
    OP " %1, %1, %1 " CTRL " row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"             \
    OP " %2, %2, %2 " CTRL " row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"             \
    OP " %3, %3, %3 " CTRL " row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
#define LBK_ROW_REDUCE4(OP)                                                             \
    asm volatile("s_nop 1\n\t" LBK_DPP4(OP, "quad_perm:[1,0,3,2]") LBK_DPP4(OP, "quad_perm:[2,3,0,1]") \
                 LBK_DPP4(OP, "row_ror:4") LBK_DPP4(OP, "row_ror:8")                    \
                 : "+v"(a), "+v"(b), "+v"(c), "+v"(d))

__device__ __forceinline__ void row_max4(float& a, float& b, float& c, float& d) { LBK_ROW_REDUCE4("v_max_f32_dpp"); }
__device__ __forceinline__ void row_sum4(float& a, float& b, float& c, float& d) { LBK_ROW_REDUCE4("v_add_f32_dpp"); }

// reduce N values in place, four per block (the tail padded with scratch values)
template <bool MAX, int N>
__device__ __forceinline__ void row_reduce(float (&v)[N]) {
#pragma unroll
    for (int i = 0; i < N; i += 4) {
        float x0 = v[i], x1 = i + 1 < N ? v[i + 1] : 0.f, x2 = i + 2 < N ? v[i + 2] : 0.f,
              x3 = i + 3 < N ? v[i + 3] : 0.f;
        if (MAX) row_max4(x0, x1, x2, x3);
        else row_sum4(x0, x1, x2, x3);
        v[i] = x0;
        if (i + 1 < N) v[i + 1] = x1;
        if (i + 2 < N) v[i + 2] = x2;
        if (i + 3 < N) v[i + 3] = x3;
    }
}

template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xf, 0xf, true));
}
__device__ __forceinline__ float max2(float a, float b) { return a > b ? a : b; }
// value of column S of this lane's 16-lane row (row_newbcast)
template <int S>
__device__ __forceinline__ float from_col(float v) { return dpp<0x150 + S>(v); }

// broadcast from column s (s a loop index of a fully unrolled loop over P <= 4)
template <int P>
__device__ __forceinline__ float from_col_dyn(float v, int s) {
    if (P == 1) return v;  // every column of a single env's result is equal
    switch (s) {
        case 0: return from_col<0>(v);
        case 1: return from_col<1>(v);
        case 2: return from_col<2>(v);
        default: return from_col<3>(v);
    }
}

// A wave iteration holds P envs of TS set tiles each: fragment array h[P*TS][KS], tile
// (s, t) = env s, set elements 16t..16t+15.  Per-env reductions (max, mean) run over that
// env's valid columns; the Gamma pass and rho are BATCHED over the P envs: column c of their
// B operand carries env (c mod P), and each env's result is broadcast back from its column.
// batched B operand of the Gamma pass: per k-step, env (col mod P)'s set-wise max
template <int TS, int P, int KS>
__device__ __forceinline__ void set_max_batched(const float (&h)[P * TS][KS], float (&mb)[KS], int col, int R) {
    float m[KS * P];
#pragma unroll
    for (int k = 0; k < KS; ++k)
#pragma unroll
        for (int s = 0; s < P; ++s) {
            float v = -INFINITY;
#pragma unroll
            for (int t = 0; t < TS; ++t)
                if (16 * t + col < R) v = max2(v, h[s * TS + t][k]);
            m[k * P + s] = v;
        }
    row_reduce<true>(m);
#pragma unroll
    for (int k = 0; k < KS; ++k) {
        float r = m[k * P];
#pragma unroll
        for (int s = 1; s < P; ++s) r = (col % P == s) ? m[k * P + s] : r;
        mb[k] = r;
    }
}

// training forward: each env's set-wise max of the observation per feature (mb from
// set_max_batched, feature 4k + grp) into setvec; lane col == s stores env s
template <int TS, int P>
__device__ __forceinline__ void store_obs_max(const float (&mb)[2], int col, int grp, int64_t env0, int64_t B,
                                              float* setvec) {
#pragma unroll
    for (int s = 0; s < P; ++s) {
        const float m0 = from_col_dyn<P>(mb[0], s), m1 = from_col_dyn<P>(mb[1], s);
        if (col != s || env0 + s >= B) continue;
        float* sv = setvec + (env0 + s) * (int64_t)LB_DS_SETVEC_FLOATS + LB_DSV_MAX0;
        sv[grp] = m0;
        sv[4 + grp] = m1;
    }
}

// training forward: set_max_batched and the first argmax rows in one pass.  Each lane keeps
// its max over its rows and the first row attaining it (strict > over ascending tiles);
// the set's max is the 16 columns' max, its first row the smallest row among the lanes
// holding it.  Both go to setvec (lane col == s stores env s), the batched max to mb.
// XR (xr non-null, P = 1): the extra row R - 1, after every tile row, in the accumulator
// layout; it is the max where strictly greater
template <int TS, int P, int KS>
__device__ __forceinline__ void set_max_store(const float (&h)[P * TS][KS], float (&mb)[KS], int col, int grp, int R,
                                              int64_t env0, int64_t B, float* setvec, int off_max, int off_id,
                                              const float* xr = nullptr) {
    static_assert(KS == 16, "hidden layers");
    float m[KS * P], rr[KS * P];
#pragma unroll
    for (int k = 0; k < KS; ++k)
#pragma unroll
        for (int s = 0; s < P; ++s) {
            float v = -INFINITY, r = 1e9f;
#pragma unroll
            for (int t = 0; t < TS; ++t) {
                const float x = h[s * TS + t][k];
                const bool u = (t < TS - 1 || 16 * t + col < R) && x > v;  // only the last tile has rows past R
                v = u ? x : v;
                r = u ? (float)(16 * t + col) : r;
            }
            m[k * P + s] = v;
            rr[k * P + s] = r;
        }
    float M[KS * P];
#pragma unroll
    for (int i = 0; i < KS * P; ++i) M[i] = m[i];
    row_reduce<true>(M);  // every lane of a row group: the max of each (feature, env)
#pragma unroll
    for (int i = 0; i < KS * P; ++i) m[i] = m[i] == M[i] ? -rr[i] : -1e9f;
    row_reduce<true>(m);  // -(first row)
    if (xr) {
#pragma unroll
        for (int k = 0; k < KS; ++k) {
            const bool u = xr[k] > M[k];
            M[k] = u ? xr[k] : M[k];
            m[k] = u ? -(float)(R - 1) : m[k];
        }
    }
#pragma unroll
    for (int k = 0; k < KS; ++k) {
        float r = M[k * P];
#pragma unroll
        for (int s = 1; s < P; ++s) r = (col % P == s) ? M[k * P + s] : r;
        mb[k] = r;
    }
#pragma unroll
    for (int s = 0; s < P; ++s) {
        if (col != s || env0 + s >= B) continue;
        float* sv = setvec + (env0 + s) * (int64_t)LB_DS_SETVEC_FLOATS;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int f0 = 16 * q + 4 * grp;
            *reinterpret_cast<float4*>(sv + off_max + f0) =
                make_float4(M[(4 * q) * P + s], M[(4 * q + 1) * P + s], M[(4 * q + 2) * P + s], M[(4 * q + 3) * P + s]);
            *reinterpret_cast<uint2*>(reinterpret_cast<uint16_t*>(sv + off_id) + f0) =
                make_uint2((uint32_t)(-m[(4 * q) * P + s]) | ((uint32_t)(-m[(4 * q + 1) * P + s]) << 16),
                           (uint32_t)(-m[(4 * q + 2) * P + s]) | ((uint32_t)(-m[(4 * q + 3) * P + s]) << 16));
        }
    }
}

// out = act(Lambda·h - Gamma·max_set(h)), NT 16-row output tiles (4 for 64 outputs).
// Issue order: the four Gamma chains side by side, then per output tile the P*TS set tiles'
// chains side by side (all four output tiles at once when P*TS <= 2), so consecutive MFMAs
// are independent (a dependent f32 MFMA waits 40 cycles against 32 for issue, and one chain
// at a time left the DPP broadcast of each Gamma result on the critical path).  Every
// element still accumulates Gamma first, then k = 0..KS-1 in order: the same bits.
// VG (DSGeom<TS, P>::VG): G is the row-major Gamma of the VALU image and xs the wave's scratch;
// the Gamma term is then vg_gamma's instead of 4 x KS MFMAs with one useful column (gret: env 0's
// Gamma term of output feature lane, for the XR forward's extra row)
template <int TS, int P, int KS, int ACT, bool VG = false>
__device__ __forceinline__ void eq_layer(const float* L, const float* G, const float (&h)[P * TS][KS],
                                         const float (&mb)[KS], float (&out)[P * TS][16], int lane,
                                         float* xs = nullptr, float* gret = nullptr) {
    constexpr int ST = P * TS;
    dsf4 g[4];  // (MFMA: env s's result in column s; VG: in the scratch, every lane reads its part)
    if constexpr (VG) {
        static_assert(P <= 2, "VALU Gamma: one or two envs per wave iteration");
        const float g0 = vg_gamma<KS, P>(G, mb, xs, lane);
        if (gret) *gret = g0;
    } else {
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) g[nt] = dsf4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int k = 0; k < KS; ++k)
#pragma unroll
            for (int nt = 0; nt < 4; ++nt) g[nt] = mfma4(G[(nt * KS + k) * 64 + lane], mb[k], g[nt]);
    }
    constexpr int NTB = ST <= 2 ? 4 : 1;  // output tiles per pass
#pragma unroll
    for (int nt0 = 0; nt0 < 4; nt0 += NTB) {
        dsf4 acc[NTB][ST];
#pragma unroll
        for (int j = 0; j < NTB; ++j)
#pragma unroll
            for (int s = 0; s < P; ++s) {
                dsf4 init;
                if constexpr (VG) {
                    init = vg_init(xs, s, nt0 + j, lane >> 4);
                } else {
#pragma unroll
                    for (int i = 0; i < 4; ++i) init[i] = from_col_dyn<P>(g[nt0 + j][i], s);
                }
#pragma unroll
                for (int t = 0; t < TS; ++t) acc[j][s * TS + t] = init;
            }
        if constexpr (VG) ds_wave_fence();  // (the scratch is read before a later layer rewrites it)
#pragma unroll
        for (int k = 0; k < KS; ++k)
#pragma unroll
            for (int j = 0; j < NTB; ++j) {
                const float a = L[((nt0 + j) * KS + k) * 64 + lane];
#pragma unroll
                for (int st = 0; st < ST; ++st) acc[j][st] = mfma4(a, h[st][k], acc[j][st]);
            }
#pragma unroll
        for (int j = 0; j < NTB; ++j)
#pragma unroll
            for (int st = 0; st < ST; ++st)
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const float x = acc[j][st][i];
                    out[st][4 * (nt0 + j) + i] = ACT == 1 ? act_relu(x) : (ACT == 2 ? act_elu(x) : x);
                }
    }
}

// the training forward's activation rows stream out with nontemporal stores: 66 KB per set
// at R = 65 (3.4 GB per 51,200-set minibatch), read back once by the backward (R = 65:
// 1.41 -> 1.34 ms per minibatch forward; tools/train_bench.py A/B)
__device__ __forceinline__ void ds_stream(float* q, float a, float b, float c, float d) {
    __builtin_nontemporal_store(dsf4{a, b, c, d}, reinterpret_cast<dsf4*>(q));
}

// store a layer output (accumulator layout) row-major into plane [B][R][64]
template <int TS, int P>
__device__ __forceinline__ void store_rows(float* plane, const float (&h)[P * TS][16], int64_t env0, int64_t B,
                                           int R, int col, int grp) {
#pragma unroll
    for (int s = 0; s < P; ++s)
#pragma unroll
        for (int t = 0; t < TS; ++t) {
            const int row = 16 * t + col;
            if (env0 + s >= B || row >= R) continue;
            float* q = plane + ((env0 + s) * (int64_t)R + row) * 64 + 4 * grp;
#pragma unroll
            for (int nt = 0; nt < 4; ++nt) {
                if (TS >= 3)
                    ds_stream(q + 16 * nt, h[s * TS + t][4 * nt], h[s * TS + t][4 * nt + 1],
                              h[s * TS + t][4 * nt + 2], h[s * TS + t][4 * nt + 3]);
                else  // (small sets: plain stores measured faster, R = 9: 0.43 vs 0.51 ms)
                    *reinterpret_cast<float4*>(q + 16 * nt) =
                        make_float4(h[s * TS + t][4 * nt], h[s * TS + t][4 * nt + 1], h[s * TS + t][4 * nt + 2],
                                    h[s * TS + t][4 * nt + 3]);
            }
        }
}

// XR training forward: the extra row's layer output (lane f: feature f) to row R - 1 of the plane
__device__ __forceinline__ void store_xrow(float* plane, float v, int64_t env, int64_t B, int R, int lane) {
    if (env < B) __builtin_nontemporal_store(v, plane + (env * (int64_t)R + R - 1) * 64 + lane);
}

// one wave iteration's P envs: the observation -> layer-1 B fragments and its set-wise max
// (XR: the extra row R - 1 = 16 TS into xr0, features 4kk + grp, and into the max; xobs: the
// group's observations elsewhere, env env0 + s at xobs + s R 8 -- lb_dqn_steps' LDS copy)
template <int TS, int P, int MODE, bool XR = false>
__device__ __forceinline__ void ds_group_obs(const DSParams& p, int64_t env0, int col, int grp, int R,
                                             float (&h0)[P * TS][2], float (&m0)[2], float (&xr0)[2],
                                             const float* xobs = nullptr) {
    constexpr bool TRAIN = MODE == 1;
    // obs -> layer-1 B fragments: k-step kk holds feature 4kk + grp of set element col
#pragma unroll
    for (int s = 0; s < P; ++s) {
        const bool live = env0 + s < p.B;
        const float* x = xobs ? xobs + s * R * 8 : p.obs + (env0 + s) * (int64_t)R * 8;
#pragma unroll
        for (int t = 0; t < TS; ++t) {
            const int row = 16 * t + col;
#pragma unroll
            for (int kk = 0; kk < 2; ++kk) h0[s * TS + t][kk] = (live && row < R) ? x[row * 8 + 4 * kk + grp] : 0.f;
        }
    }
    set_max_batched<TS, P, 2>(h0, m0, col, R);
    if constexpr (XR) {
        const float* x = p.obs + (env0 * (int64_t)R + 16 * TS) * 8;
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
            xr0[kk] = env0 < p.B ? x[4 * kk + grp] : 0.f;
            m0[kk] = max2(m0[kk], xr0[kk]);
        }
    }
    if (TRAIN) store_obs_max<TS, P>(m0, col, grp, env0, p.B, p.setvec);
}

// one wave iteration's P envs: the actor (or Q network) Eq(8->64) ReLU Eq(64->64) ELU Eq(64->1);
// logits / training rows / the masked greedy action (ARGMAX: lane s < P returns env0 + s's)
// (W: the fragment image, or the VALU image with xs the wave's scratch: DSGeom<TS, P>::VG)
template <int TS, int P, int MODE, bool VG = DSGeom<TS, P, MODE>::VG, bool XR = false>
__device__ __forceinline__ int32_t ds_group_actor(const DSParams& p, const float* W, int lane, int64_t env0, int col,
                                                  int grp, int R, const float (&h0)[P * TS][2], const float (&m0)[2],
                                                  float* xs = nullptr, const float* xr0 = nullptr) {
    constexpr bool TRAIN = MODE == 1, ARGMAX = MODE == 2;
    constexpr int A1L = VG ? VG_A1L : DS_A1L, A1G = VG ? VG_A1G : DS_A1G, A2L = VG ? VG_A2L : DS_A2L,
                  A2G = VG ? VG_A2G : DS_A2G;
    int32_t act = -1;
    float h1[P * TS][16], m1[16], h2[P * TS][16], m2[16];
    // ---- actor: Eq(8->64) ReLU Eq(64->64) ELU Eq(64->1)
    if (p.actor) {
        float g = 0.f, r1 = 0.f, r2 = 0.f, xr[16];  // (XR: the extra row, below)
        eq_layer<TS, P, 2, 1, VG>(W + A1L, W + A1G, h0, m0, h1, lane, xs, XR ? &g : nullptr);
        if constexpr (XR) {
            r1 = vg_xrow<2, 1>(W + VGX_A1, xr0, 0.f, g, xs, lane);
            vg_xspread(r1, xs, lane, xr);
            store_xrow(p.save_actor, r1, env0, p.B, R, lane);
        }
        if (TRAIN) store_rows<TS, P>(p.save_actor, h1, env0, p.B, R, col, grp);
        if (TRAIN)
            set_max_store<TS, P, 16>(h1, m1, col, grp, R, env0, p.B, p.setvec, LB_DSV_MAX1A, LB_DSV_ID1A,
                                     XR ? xr : nullptr);
        else set_max_batched<TS, P, 16>(h1, m1, col, R);
        eq_layer<TS, P, 16, 2, VG>(W + A2L, W + A2G, h1, m1, h2, lane, xs, XR ? &g : nullptr);
        if constexpr (XR) {
            r2 = vg_xrow<16, 2>(W + VGX_A2, nullptr, r1, g, xs, lane);
            vg_xspread(r2, xs, lane, xr);
            store_xrow(p.save_actor + p.B * (int64_t)R * 64, r2, env0, p.B, R, lane);
        }
        if (TRAIN) store_rows<TS, P>(p.save_actor + p.B * (int64_t)R * 64, h2, env0, p.B, R, col, grp);
        if (TRAIN)
            set_max_store<TS, P, 16>(h2, m2, col, grp, R, env0, p.B, p.setvec, LB_DSV_MAX2A, LB_DSV_ID2A,
                                     XR ? xr : nullptr);
        else set_max_batched<TS, P, 16>(h2, m2, col, R);
        // layer 3 (64 -> 1) on the VALU: a 16-row output tile would use 1/16 of an MFMA.
        // Lane (col, grp) dots its 16 features in(k, grp) with Lambda3 / -Gamma3 (the VALU
        // image's vectors, or row 0 of the fragments: column 0 of its row group), then the 4
        // row groups are summed.
        auto l3 = [&](int k, bool gamma) {
            return VG ? W[(gamma ? VG_A3GV : VG_A3V) + 16 * (k >> 2) + 4 * grp + (k & 3)]
                      : W[(gamma ? DS_A3G : DS_A3L) + 16 * grp + 64 * k];
        };
        float gl = 0.f;
#pragma unroll
        for (int k = 0; k < 16; ++k) gl += l3(k, true) * m2[k];
        gl += __shfl_xor(gl, 16);
        gl += __shfl_xor(gl, 32);
        if constexpr (XR) {  // the extra row's logit: lane f's product, summed over the wave
            float v[1] = {W[VG_A3V + lane] * r2};
            row_reduce<false>(v);
            v[0] += __shfl_xor(v[0], 16);
            v[0] += __shfl_xor(v[0], 32);
            if (lane == 0 && env0 < p.B && p.logits) p.logits[env0 * R + R - 1] = gl + v[0];
        }
        float best[P], brow[P];  // this lane's first masked maximum per env (argmax mode)
#pragma unroll
        for (int s = 0; s < P; ++s) {
            const float init = from_col_dyn<P>(gl, s);
            best[s] = -INFINITY;
            brow[s] = 1e9f;
#pragma unroll
            for (int t = 0; t < TS; ++t) {
                float v = 0.f;
#pragma unroll
                for (int k = 0; k < 16; ++k) v += l3(k, false) * h2[s * TS + t][k];
                v += __shfl_xor(v, 16);
                v += __shfl_xor(v, 32);
                const int row = 16 * t + col;
                const bool live = row < R && env0 + s < p.B;
                if (grp == 0 && live && p.logits) p.logits[(env0 + s) * R + row] = init + v;
                if (ARGMAX && live) {
                    const float q = (!p.masks || p.masks[(env0 + s) * R + row]) ? init + v : -1e8f;
                    if (q > best[s]) {
                        best[s] = q;
                        brow[s] = (float)row;
                    }
                }
            }
        }
        if (ARGMAX) {
            // over the 16 columns: the max, then the smallest row attaining it
            float m[P], c[P];
#pragma unroll
            for (int s = 0; s < P; ++s) m[s] = best[s];
            row_reduce<true>(m);
#pragma unroll
            for (int s = 0; s < P; ++s) c[s] = best[s] == m[s] ? -brow[s] : -1e9f;
            row_reduce<true>(c);
            if (lane < P && env0 + lane < p.B) {
                float r = -c[0];
#pragma unroll
                for (int s = 1; s < P; ++s) r = lane == s ? -c[s] : r;
                p.actions[env0 + lane] = (int32_t)r;
                act = (int32_t)r;
            }
        }
    }
    return act;
}

// MODE 0: logits / value; 1: training forward (TRAIN: activations, psi mean); 2: Q values
// and the masked greedy action (ARGMAX; actor only)
// the forward of the blocks blk = 0 .. nblk - 1 (k_deepsets_fwd: the whole grid; k_ds_fwd_pair:
// its half of the grid), W the block's LDS weight region
template <int TS, int P, int MODE, bool XR = false>
__device__ __forceinline__ void ds_fwd_body(const DSParams& p, float* W, int blk, int nblk) {
    constexpr bool TRAIN = MODE == 1, ARGMAX = MODE == 2, VG = DSGeom<TS, P, MODE, XR>::VG;
    // stage the weight image (once per block; blocks are persistent): the fragment image, or
    // the VALU image (VG: the actor's and critic's regions, rho's for the inference forward, the
    // extra-row block for XR); an actor-only launch (DQN) stages only the actor's part
    const int nstage = VG ? ((ARGMAX || !p.critic) ? (int)VG_ACTOR : (int)DSGeom<TS, P, MODE>::IMG)
                          : ((ARGMAX || !p.critic) ? (int)DS_C1L : (int)DS_FLOATS);
    const float* src = p.wfrag + (VG ? DS_FLOATS : 0);
    for (int i = threadIdx.x * 4; i < nstage; i += DS_BLOCK * 4)
        *reinterpret_cast<float4*>(W + i) = *reinterpret_cast<const float4*>(src + i);
    if constexpr (XR)
        for (int i = threadIdx.x * 4; i < VG_FLOATS - VG_XA1; i += DS_BLOCK * 4)
            *reinterpret_cast<float4*>(W + VGX_BASE + i) = *reinterpret_cast<const float4*>(src + VG_XA1 + i);
    __syncthreads();
    float* xs = VG ? W + DSGeom<TS, P, MODE, XR>::IMG + (threadIdx.x >> 6) * P * VG_SCRATCH : nullptr;
    const int lane = threadIdx.x & 63;
    // wave-major numbering: a batch of fewer groups than waves puts one wave on each SIMD
    // of every CU (waves 0-3 of a block sit on its 4 SIMDs) before any SIMD takes a second
    const int64_t wave = (int64_t)(threadIdx.x >> 6) * nblk + blk;
    const int64_t nwaves = (int64_t)nblk * (DS_BLOCK / 64);
    const int R = p.R;
    const int col = lane & 15, grp = lane >> 4;
    const int64_t groups = (p.B + P - 1) / P;
    for (int64_t gi = wave; gi < groups; gi += nwaves) {
        const int64_t env0 = gi * P;
        float h0[P * TS][2], m0[2], xr0[2];
        ds_group_obs<TS, P, MODE, XR>(p, env0, col, grp, R, h0, m0, xr0);
        ds_group_actor<TS, P, MODE, VG, XR>(p, W, lane, env0, col, grp, R, h0, m0, xs, xr0);
        float h1[P * TS][16], m1[16], h2[P * TS][16], m2[16];
        if (ARGMAX || !p.critic) continue;

        // ---- critic: psi = Eq ELU Eq ELU Eq, mean over the set, rho = Linear ELU Linear
        constexpr int C1L = VG ? VG_C1L : DS_C1L, C1G = VG ? VG_C1G : DS_C1G, C2L = VG ? VG_C2L : DS_C2L,
                      C2G = VG ? VG_C2G : DS_C2G;
        float g = 0.f, c1r = 0.f, xr[16];  // (XR: the extra row, as the actor's)
        eq_layer<TS, P, 2, 2, VG>(W + C1L, W + C1G, h0, m0, h1, lane, xs, XR ? &g : nullptr);
        if constexpr (XR) {
            c1r = vg_xrow<2, 2>(W + VGX_C1, xr0, 0.f, g, xs, lane);
            vg_xspread(c1r, xs, lane, xr);
            store_xrow(p.save_critic, c1r, env0, p.B, R, lane);
        }
        if (TRAIN) store_rows<TS, P>(p.save_critic, h1, env0, p.B, R, col, grp);
        if (TRAIN)
            set_max_store<TS, P, 16>(h1, m1, col, grp, R, env0, p.B, p.setvec, LB_DSV_MAX1C, LB_DSV_ID1C,
                                     XR ? xr : nullptr);
        else set_max_batched<TS, P, 16>(h1, m1, col, R);
        eq_layer<TS, P, 16, 2, VG>(W + C2L, W + C2G, h1, m1, h2, lane, xs, XR ? &g : nullptr);
        if constexpr (XR) {
            const float c2r = vg_xrow<16, 2>(W + VGX_C2, nullptr, c1r, g, xs, lane);
            vg_xspread(c2r, xs, lane, xr);  // (xr: c2's extra row, into the max and the sum)
            store_xrow(p.save_critic + p.B * (int64_t)R * 64, c2r, env0, p.B, R, lane);
        }
        if (TRAIN) store_rows<TS, P>(p.save_critic + p.B * (int64_t)R * 64, h2, env0, p.B, R, col, grp);
        if (TRAIN)
            set_max_store<TS, P, 16>(h2, m2, col, grp, R, env0, p.B, p.setvec, LB_DSV_MAX2C, LB_DSV_ID2C,
                                     XR ? xr : nullptr);
        else set_max_batched<TS, P, 16>(h2, m2, col, R);
        // layer 3 has no activation and only its mean over the set is used, so
        // mean_r(Lambda3 c2[r] - Gamma3 max(c2)) = Lambda3 mean_r(c2) - Gamma3 max(c2): one
        // matrix-vector pair on the batched (column c = env c mod P) operands instead of a
        // 64x64 layer over every row
        if constexpr (VG) {  // the pair, rho's two layers: lane f's dot products (xs: x, then y)
            float sm[16];
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                float v = 0.f;
#pragma unroll
                for (int t = 0; t < TS; ++t)
                    if (16 * t + col < R) v += h2[t][k];
                sm[k] = v;
            }
            row_reduce<false>(sm);
            if constexpr (XR) {
#pragma unroll
                for (int k = 0; k < 16; ++k) sm[k] += xr[k];
            }
            const float invR = 1.0f / (float)R;
#pragma unroll
            for (int k = 0; k < 16; ++k) sm[k] *= invR;
            vg_put<16>(m2, xs, col, grp);
            ds_wave_fence();
            float mean = vg_dot<64, VG_RS>(W + VG_C3G, xs, lane, 0.f);  // (-Gamma3) max, then Lambda3 mean
            ds_wave_fence();
            vg_put<16>(sm, xs, col, grp);
            ds_wave_fence();
            mean = vg_dot<64, VG_RS>(W + VG_C3L, xs, lane, mean);
            if (TRAIN) {
                if (env0 < p.B) p.psi_mean[env0 * 64 + lane] = mean;
                ds_wave_fence();
                continue;
            }
            ds_wave_fence();
            xs[lane] = mean;
            ds_wave_fence();
            const float r1 = act_elu(vg_dot<64, VG_RS>(W + VG_R1W, xs, lane, W[VG_R1B + lane]));
            float v[1] = {W[VG_R2W + lane] * r1};
            row_reduce<false>(v);
            v[0] += __shfl_xor(v[0], 16);
            v[0] += __shfl_xor(v[0], 32);
            if (lane == 0 && env0 < p.B) p.value[env0] = W[VG_R2B] + v[0];
            ds_wave_fence();
            continue;
        }
        float mean[16];
        {
            const float invR = 1.0f / (float)R;
            float sm[16 * P], mc[16];
#pragma unroll
            for (int k = 0; k < 16; ++k)
#pragma unroll
                for (int s = 0; s < P; ++s) {
                    float v = 0.f;
#pragma unroll
                    for (int t = 0; t < TS; ++t)
                        if (16 * t + col < R) v += h2[s * TS + t][k];
                    sm[k * P + s] = v;
                }
            row_reduce<false>(sm);
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                float r = sm[k * P];
#pragma unroll
                for (int s = 1; s < P; ++s) r = (col % P == s) ? sm[k * P + s] : r;
                mc[k] = r * invR;
            }
            // (the four output tiles' chains side by side; each element: Gamma then Lambda, k in order)
            dsf4 acc[4];
#pragma unroll
            for (int nt = 0; nt < 4; ++nt) acc[nt] = dsf4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int k = 0; k < 16; ++k)
#pragma unroll
                for (int nt = 0; nt < 4; ++nt) acc[nt] = mfma4(W[DS_C3G + (nt * 16 + k) * 64 + lane], m2[k], acc[nt]);
#pragma unroll
            for (int k = 0; k < 16; ++k)
#pragma unroll
                for (int nt = 0; nt < 4; ++nt) acc[nt] = mfma4(W[DS_C3L + (nt * 16 + k) * 64 + lane], mc[k], acc[nt]);
#pragma unroll
            for (int nt = 0; nt < 4; ++nt)
#pragma unroll
                for (int i = 0; i < 4; ++i) mean[4 * nt + i] = acc[nt][i];
        }
        if (TRAIN) {
            // column c carries env (c mod P): lanes of columns < P store their env's features
            if (col < P && env0 + col < p.B) {
                float* q = p.psi_mean + (env0 + col) * 64 + 4 * grp;
#pragma unroll
                for (int nt = 0; nt < 4; ++nt)
                    *reinterpret_cast<float4*>(q + 16 * nt) =
                        make_float4(mean[4 * nt], mean[4 * nt + 1], mean[4 * nt + 2], mean[4 * nt + 3]);
            }
            continue;
        }
        float r1[16];
        {
            dsf4 acc[4];
#pragma unroll
            for (int nt = 0; nt < 4; ++nt)
#pragma unroll
                for (int i = 0; i < 4; ++i) acc[nt][i] = W[DS_R1B + 16 * nt + 4 * grp + i];
#pragma unroll
            for (int k = 0; k < 16; ++k)
#pragma unroll
                for (int nt = 0; nt < 4; ++nt) acc[nt] = mfma4(W[DS_R1W + (nt * 16 + k) * 64 + lane], mean[k], acc[nt]);
#pragma unroll
            for (int nt = 0; nt < 4; ++nt)
#pragma unroll
                for (int i = 0; i < 4; ++i) r1[4 * nt + i] = act_elu(acc[nt][i]);
        }
        dsf4 v = {W[DS_R2B], 0.f, 0.f, 0.f};
#pragma unroll
        for (int k = 0; k < 16; ++k) v = mfma4(W[DS_R2W + k * 64 + lane], r1[k], v);
        // row 0 of the result: column c = env (c mod P)
        if (grp == 0 && col < P && env0 + col < p.B) p.value[env0 + col] = v[0];
    }
}

template <int TS, int P, int MODE, bool XR = false>
__global__ __launch_bounds__(DS_BLOCK, 2) void k_deepsets_fwd(DSParams p) {
    if (MODE == 2 && p.ex_on && ds_dqn_explore(p)) return;  // (uniform: the DQN step explores)
    __shared__ __attribute__((aligned(16))) float W[DSGeom<TS, P, MODE, XR>::LDS];
    ds_fwd_body<TS, P, MODE, XR>(p, W, blockIdx.x, gridDim.x);
}

// two forwards in one launch (lb_ds_forward_pair: the DQN train step's target-network Q values
// of the next observations and the trained network's training forward): blocks below ga run
// a's inference forward (MODE 0), the rest b's training forward (MODE 1); actor only
template <int TS, int P>
__global__ __launch_bounds__(DS_BLOCK, 2) void k_ds_fwd_pair(DSParams a, DSParams b, int ga) {
    __shared__ __attribute__((aligned(16))) float W[DS_C1L];
    if ((int)blockIdx.x < ga) ds_fwd_body<TS, P, 0>(a, W, blockIdx.x, ga);
    else ds_fwd_body<TS, P, 1>(b, W, blockIdx.x - ga, gridDim.x - ga);
}

// ---- large sets (LB_DS_MAX_ELEMENTS < R <= LB_DS_MAX_ELEMENTS_FWD) ------------------------
// One env per wave iteration; the set is streamed in chunks of DS_CT 16-row tiles (32 elements).  A layer
// needs the set-wise max of its input, so each layer's max is one pass over the chunks that
// recomputes the earlier layers of the chunk: nothing per element leaves registers, at the
// price of layer 1 three times and layer 2 twice for the actor (R up to 257: E <= 256 with
// the reject row).  Same fragments, same per-element math as k_deepsets_fwd.
constexpr int DS_CT = 2;

template <int KS>
__device__ __forceinline__ void chunk_max_acc(const float (&h)[DS_CT][KS], float (&acc)[KS], int row0, int col, int R) {
#pragma unroll
    for (int t = 0; t < DS_CT; ++t)
        if (row0 + 16 * t + col < R)
#pragma unroll
            for (int k = 0; k < KS; ++k) acc[k] = max2(acc[k], h[t][k]);
}

__device__ __forceinline__ void load_obs_chunk(const float* x, int row0, int R, int col, int grp, float (&h0)[DS_CT][2]) {
#pragma unroll
    for (int t = 0; t < DS_CT; ++t) {
        const int row = row0 + 16 * t + col;
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) h0[t][kk] = row < R ? x[row * 8 + 4 * kk + grp] : 0.f;
    }
}

// training (chunked): each lane's running max of its rows per feature and the FIRST row
// attaining it (strict > over ascending rows)
template <int KS>
__device__ __forceinline__ void chunk_argmax_acc(const float (&h)[DS_CT][KS], float (&v)[KS], float (&r)[KS], int row0,
                                                 int col, int R) {
#pragma unroll
    for (int t = 0; t < DS_CT; ++t) {
        const int row = row0 + 16 * t + col;
        if (row >= R) continue;
#pragma unroll
        for (int k = 0; k < KS; ++k) {
            const bool u = h[t][k] > v[k];
            v[k] = u ? h[t][k] : v[k];
            r[k] = u ? (float)row : r[k];
        }
    }
}
// ... then the set's max over the 16 columns (into v, every lane) and the smallest row among
// the lanes holding it, both to setvec (feature 16q + 4grp + i of the accumulator layout)
__device__ __forceinline__ void chunk_argmax_store(float (&v)[16], float (&r)[16], int col, int grp, float* sv,
                                                   int off_max, int off_id) {
    float M[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) M[k] = v[k];
    row_reduce<true>(M);
#pragma unroll
    for (int k = 0; k < 16; ++k) r[k] = v[k] == M[k] ? -r[k] : -1e9f;
    row_reduce<true>(r);
#pragma unroll
    for (int k = 0; k < 16; ++k) v[k] = M[k];
    if (col != 0) return;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int f0 = 16 * q + 4 * grp;
        *reinterpret_cast<float4*>(sv + off_max + f0) = make_float4(M[4 * q], M[4 * q + 1], M[4 * q + 2], M[4 * q + 3]);
        *reinterpret_cast<uint2*>(reinterpret_cast<uint16_t*>(sv + off_id) + f0) =
            make_uint2((uint32_t)(-r[4 * q]) | ((uint32_t)(-r[4 * q + 1]) << 16),
                       (uint32_t)(-r[4 * q + 2]) | ((uint32_t)(-r[4 * q + 3]) << 16));
    }
}
// a chunk's layer output rows (accumulator layout) into plane [B][R][64]
__device__ __forceinline__ void store_rows_chunk(float* plane, const float (&h)[DS_CT][16], int64_t env, int R, int row0,
                                                 int col, int grp) {
#pragma unroll
    for (int t = 0; t < DS_CT; ++t) {
        const int row = row0 + 16 * t + col;
        if (row >= R) continue;
        float* q = plane + (env * (int64_t)R + row) * 64 + 4 * grp;
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) ds_stream(q + 16 * nt, h[t][4 * nt], h[t][4 * nt + 1], h[t][4 * nt + 2], h[t][4 * nt + 3]);
    }
}

// MODE 0: logits / value; 1: training forward (activations, set maxima + first argmax rows,
// psi mean; as k_deepsets_fwd<.., 1>); 2: Q values and the masked greedy action (actor only)
template <int MODE>
__global__ __launch_bounds__(DS_BLOCK, 2) void k_deepsets_fwd_big(DSParams p) {
    constexpr bool ARGMAX = MODE == 2, TRAIN = MODE == 1;
    if (ARGMAX && p.ex_on && ds_dqn_explore(p)) return;
    __shared__ __attribute__((aligned(16))) float W[DS_LDS_FLOATS];
    const int nstage = (ARGMAX || !p.critic) ? DS_C1L : DS_FLOATS;
    for (int i = threadIdx.x * 4; i < nstage; i += DS_BLOCK * 4)
        *reinterpret_cast<float4*>(W + i) = *reinterpret_cast<const float4*>(p.wfrag + i);
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const int64_t wave = (int64_t)blockIdx.x * (DS_BLOCK / 64) + (threadIdx.x >> 6);
    const int64_t nwaves = (int64_t)gridDim.x * (DS_BLOCK / 64);
    const int R = p.R;
    const int col = lane & 15, grp = lane >> 4;
    const int nch = (R + 16 * DS_CT - 1) / (16 * DS_CT);
    for (int64_t env = wave; env < p.B; env += nwaves) {
        const float* x = p.obs + env * (int64_t)R * 8;
        // the weight fragments are re-read from LDS in every chunk: an opaque base pointer
        // per chunk keeps the compiler from hoisting KiBs of loop-invariant loads into
        // registers (which spilled to scratch)
        // (an opaque 32-bit offset into the shared array keeps the loads ds_reads)
        float h0[DS_CT][2], h1[DS_CT][16], h2[DS_CT][16];
        float m0[2] = {-INFINITY, -INFINITY};
        for (int c = 0; c < nch; ++c) {
            load_obs_chunk(x, 16 * DS_CT * c, R, col, grp, h0);
            chunk_max_acc<2>(h0, m0, 16 * DS_CT * c, col, R);
        }
        row_reduce<true>(m0);
        float* sv = TRAIN ? p.setvec + env * (int64_t)LB_DS_SETVEC_FLOATS : nullptr;
        if (TRAIN && col == 0) {
            sv[LB_DSV_MAX0 + grp] = m0[0];
            sv[LB_DSV_MAX0 + 4 + grp] = m0[1];
        }
        if (p.actor) {
            float m1[16], m2[16], r1[16];
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                m1[k] = m2[k] = -INFINITY;
                r1[k] = 1e9f;
            }
            for (int c = 0; c < nch; ++c) {
                uint32_t wo = 0;
                asm volatile("" : "+s"(wo));
                const float* Wc = W + wo;
                load_obs_chunk(x, 16 * DS_CT * c, R, col, grp, h0);
                eq_layer<DS_CT, 1, 2, 1>(Wc + DS_A1L, Wc + DS_A1G, h0, m0, h1, lane);
                if (TRAIN) chunk_argmax_acc<16>(h1, m1, r1, 16 * DS_CT * c, col, R);
                else chunk_max_acc<16>(h1, m1, 16 * DS_CT * c, col, R);
            }
            if (TRAIN) chunk_argmax_store(m1, r1, col, grp, sv, LB_DSV_MAX1A, LB_DSV_ID1A);
            else row_reduce<true>(m1);
#pragma unroll
            for (int k = 0; k < 16; ++k) r1[k] = 1e9f;
            for (int c = 0; c < nch; ++c) {
                uint32_t wo = 0;
                asm volatile("" : "+s"(wo));
                const float* Wc = W + wo;
                load_obs_chunk(x, 16 * DS_CT * c, R, col, grp, h0);
                eq_layer<DS_CT, 1, 2, 1>(Wc + DS_A1L, Wc + DS_A1G, h0, m0, h1, lane);
                eq_layer<DS_CT, 1, 16, 2>(Wc + DS_A2L, Wc + DS_A2G, h1, m1, h2, lane);
                if (TRAIN) chunk_argmax_acc<16>(h2, m2, r1, 16 * DS_CT * c, col, R);
                else chunk_max_acc<16>(h2, m2, 16 * DS_CT * c, col, R);
            }
            if (TRAIN) chunk_argmax_store(m2, r1, col, grp, sv, LB_DSV_MAX2A, LB_DSV_ID2A);
            else row_reduce<true>(m2);
            const float* G = W + DS_A3G + 16 * grp;
            float gl = 0.f;
#pragma unroll
            for (int k = 0; k < 16; ++k) gl += G[k * 64] * m2[k];
            gl += __shfl_xor(gl, 16);
            gl += __shfl_xor(gl, 32);
            float best = -INFINITY, brow = 1e9f;
            for (int c = 0; c < nch; ++c) {
                uint32_t wo = 0;
                asm volatile("" : "+s"(wo));
                const float* Wc = W + wo;
                load_obs_chunk(x, 16 * DS_CT * c, R, col, grp, h0);
                eq_layer<DS_CT, 1, 2, 1>(Wc + DS_A1L, Wc + DS_A1G, h0, m0, h1, lane);
                eq_layer<DS_CT, 1, 16, 2>(Wc + DS_A2L, Wc + DS_A2G, h1, m1, h2, lane);
                if (TRAIN) {
                    store_rows_chunk(p.save_actor, h1, env, R, 16 * DS_CT * c, col, grp);
                    store_rows_chunk(p.save_actor + p.B * (int64_t)R * 64, h2, env, R, 16 * DS_CT * c, col, grp);
                }
#pragma unroll
                for (int t = 0; t < DS_CT; ++t) {
                    float v = 0.f;
#pragma unroll
                    for (int k = 0; k < 16; ++k) v += Wc[DS_A3L + 16 * grp + k * 64] * h2[t][k];
                    v += __shfl_xor(v, 16);
                    v += __shfl_xor(v, 32);
                    const int row = 16 * DS_CT * c + 16 * t + col;
                    if (row >= R) continue;
                    if (grp == 0 && p.logits) p.logits[env * R + row] = gl + v;
                    if (ARGMAX) {
                        const float q = (!p.masks || p.masks[env * R + row]) ? gl + v : -1e8f;
                        if (q > best) {  // rows ascend: the first maximum of this lane wins
                            best = q;
                            brow = (float)row;
                        }
                    }
                }
            }
            if (ARGMAX) {
                float m[1] = {best};
                row_reduce<true>(m);
                float cc[1] = {best == m[0] ? -brow : -1e9f};
                row_reduce<true>(cc);
                if (lane == 0) p.actions[env] = (int32_t)(-cc[0]);
            }
        }
        if (ARGMAX || !p.critic) continue;
        // critic: the max of c1, then the max and the sum of c2, then layer 3 / rho as above
        float mc1[16], mc2[16], sm[16], rc[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            mc1[k] = mc2[k] = -INFINITY;
            sm[k] = 0.f;
            rc[k] = 1e9f;
        }
        for (int c = 0; c < nch; ++c) {
            uint32_t wo = 0;
            asm volatile("" : "+s"(wo));
            const float* Wc = W + wo;
            load_obs_chunk(x, 16 * DS_CT * c, R, col, grp, h0);
            eq_layer<DS_CT, 1, 2, 2>(Wc + DS_C1L, Wc + DS_C1G, h0, m0, h1, lane);
            if (TRAIN) chunk_argmax_acc<16>(h1, mc1, rc, 16 * DS_CT * c, col, R);
            else chunk_max_acc<16>(h1, mc1, 16 * DS_CT * c, col, R);
        }
        if (TRAIN) chunk_argmax_store(mc1, rc, col, grp, sv, LB_DSV_MAX1C, LB_DSV_ID1C);
        else row_reduce<true>(mc1);
#pragma unroll
        for (int k = 0; k < 16; ++k) rc[k] = 1e9f;
        for (int c = 0; c < nch; ++c) {
            uint32_t wo = 0;
            asm volatile("" : "+s"(wo));
            const float* Wc = W + wo;
            load_obs_chunk(x, 16 * DS_CT * c, R, col, grp, h0);
            eq_layer<DS_CT, 1, 2, 2>(Wc + DS_C1L, Wc + DS_C1G, h0, m0, h1, lane);
            eq_layer<DS_CT, 1, 16, 2>(Wc + DS_C2L, Wc + DS_C2G, h1, mc1, h2, lane);
            if (TRAIN) {
                chunk_argmax_acc<16>(h2, mc2, rc, 16 * DS_CT * c, col, R);
                store_rows_chunk(p.save_critic, h1, env, R, 16 * DS_CT * c, col, grp);
                store_rows_chunk(p.save_critic + p.B * (int64_t)R * 64, h2, env, R, 16 * DS_CT * c, col, grp);
            } else {
                chunk_max_acc<16>(h2, mc2, 16 * DS_CT * c, col, R);
            }
#pragma unroll
            for (int t = 0; t < DS_CT; ++t)
                if (16 * DS_CT * c + 16 * t + col < R)
#pragma unroll
                    for (int k = 0; k < 16; ++k) sm[k] += h2[t][k];
        }
        if (TRAIN) chunk_argmax_store(mc2, rc, col, grp, sv, LB_DSV_MAX2C, LB_DSV_ID2C);
        else row_reduce<true>(mc2);
        row_reduce<false>(sm);
        const float invR = 1.0f / (float)R;
        float mean[16];
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) {
            dsf4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int k = 0; k < 16; ++k) acc = mfma4(W[DS_C3G + (nt * 16 + k) * 64 + lane], mc2[k], acc);
#pragma unroll
            for (int k = 0; k < 16; ++k) acc = mfma4(W[DS_C3L + (nt * 16 + k) * 64 + lane], sm[k] * invR, acc);
#pragma unroll
            for (int i = 0; i < 4; ++i) mean[4 * nt + i] = acc[i];
        }
        if (TRAIN) {  // psi mean (rho runs in torch): every column holds the set's value
            if (col == 0) {
                float* q = p.psi_mean + env * 64 + 4 * grp;
#pragma unroll
                for (int nt = 0; nt < 4; ++nt)
                    *reinterpret_cast<float4*>(q + 16 * nt) =
                        make_float4(mean[4 * nt], mean[4 * nt + 1], mean[4 * nt + 2], mean[4 * nt + 3]);
            }
            continue;
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

// the VALU image (VG_*): fragments for the Lambda regions, row-major rows (stride S) elsewhere
__device__ __forceinline__ float vg_rm_value(const float* w, int kin, int S, int idx) {
    const int f = idx / S, j = idx - f * S;
    return (w && j < kin) ? w[f * kin + j] : 0.f;
}
__device__ __forceinline__ void vg_pack_one(const lb_ds_weights& w, float* out, int j) {
    const int starts[20] = {VG_A1L, VG_A2L, VG_A3V, VG_A3GV, VG_A1G, VG_A2G, VG_C1L, VG_C2L, VG_C1G, VG_C2G,
                            VG_C3L, VG_C3G, VG_R1W, VG_R1B, VG_R2W, VG_R2B, VG_XA1, VG_XA2, VG_XC1, VG_XC2};
    int r = 19;
    while (r > 0 && j < starts[r]) --r;
    const int idx = j - starts[r];
    float v = 0.f;
    switch (r) {
        case 0: v = ds_frag_value(w.actor_lambda[0], 64, 8, 2, idx); break;
        case 1: v = ds_frag_value(w.actor_lambda[1], 64, 64, 16, idx); break;
        case 2: v = w.actor_lambda[2] ? w.actor_lambda[2][idx] : 0.f; break;
        case 3: v = w.actor_gamma[2] ? -w.actor_gamma[2][idx] : 0.f; break;
        case 4: v = -vg_rm_value(w.actor_gamma[0], 8, VG_RS8, idx); break;
        case 5: v = -vg_rm_value(w.actor_gamma[1], 64, VG_RS, idx); break;
        case 6: v = ds_frag_value(w.critic_lambda[0], 64, 8, 2, idx); break;
        case 7: v = ds_frag_value(w.critic_lambda[1], 64, 64, 16, idx); break;
        case 8: v = -vg_rm_value(w.critic_gamma[0], 8, VG_RS8, idx); break;
        case 9: v = -vg_rm_value(w.critic_gamma[1], 64, VG_RS, idx); break;
        case 10: v = vg_rm_value(w.critic_lambda[2], 64, VG_RS, idx); break;
        case 11: v = -vg_rm_value(w.critic_gamma[2], 64, VG_RS, idx); break;
        case 12: v = vg_rm_value(w.rho_w1, 64, VG_RS, idx); break;
        case 13: v = w.rho_b1 ? w.rho_b1[idx] : 0.f; break;
        case 14: v = w.rho_w2 ? w.rho_w2[idx] : 0.f; break;
        case 15: v = (w.rho_b2 && idx == 0) ? w.rho_b2[0] : 0.f; break;
        case 16: v = vg_rm_value(w.actor_lambda[0], 8, VG_RS8, idx); break;
        case 17: v = vg_rm_value(w.actor_lambda[1], 64, VG_RS, idx); break;
        case 18: v = vg_rm_value(w.critic_lambda[0], 8, VG_RS8, idx); break;
        default: v = vg_rm_value(w.critic_lambda[1], 64, VG_RS, idx); break;
    }
    out[DS_FLOATS + j] = v;
}

__device__ __forceinline__ void ds_pack_one(const lb_ds_weights& w, float* out, int i) {
    if (i >= DS_IMG_FLOATS) return;
    if (i >= DS_FLOATS) {
        vg_pack_one(w, out, i - DS_FLOATS);
        return;
    }
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
    // Gamma fragments are stored negated: the kernel adds (-Gamma)·max
    const bool gamma = r == 1 || r == 3 || r == 5 || r == 7 || r == 9 || r == 11;
    out[i] = gamma ? -v : v;
}
__global__ void k_ds_pack(lb_ds_weights w, float* out) { ds_pack_one(w, out, blockIdx.x * blockDim.x + threadIdx.x); }

}  // namespace lbk
