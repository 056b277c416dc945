// lbk8s_lean_timeline.h — diagnostic builds only (-DLB_TIMELINE, tools/timeline_lean.py): the
// per-wave stamps of k_rollout_lean(_split).  Included by csrc/lbk8s_lean.h under LB_TIMELINE; the
// product library defines LB_LTL / LB_LTL_HDR as no-ops.
//   per wave (index env0 / 64): LTL_H header words, then LTL_NP s_memtime stamps per step;
//   header: 0 loop start, 1 loop end, 2 entry, 3 exit, 4 records drawn, 5 image built
//   (s_memrealtime, 100 MHz), 6 HW_ID, 7 XCC_ID
#pragma once
constexpr int LTL_NP = 6, LTL_H = 8;
#define LB_LTL(k, i)                                                                                             \
    do {                                                                                                         \
        asm volatile("" ::: "memory");                                                                           \
        if (g_timeline && lane == 0)                                                                             \
            g_timeline[(env0 / 64) * (LTL_H + K * LTL_NP) + LTL_H + (k) * LTL_NP + (i)] = __builtin_amdgcn_s_memtime(); \
        asm volatile("" ::: "memory");                                                                           \
    } while (0)
#define LB_LTL_HDR(slot)                                                                                         \
    do {                                                                                                         \
        if (g_timeline && (threadIdx.x & 63) == 0)                                                               \
            g_timeline[(env0 / 64) * (LTL_H + K * LTL_NP) + (slot)] = __builtin_amdgcn_s_memrealtime();          \
    } while (0)
#define LB_LTL_HWID()                                                                                            \
    do {                                                                                                         \
        if (g_timeline && (threadIdx.x & 63) == 0) {                                                             \
            g_timeline[(env0 / 64) * (LTL_H + K * LTL_NP) + 6] = __builtin_amdgcn_s_getreg((31 << 11) | 4);      \
            g_timeline[(env0 / 64) * (LTL_H + K * LTL_NP) + 7] = __builtin_amdgcn_s_getreg((31 << 11) | 20);     \
        }                                                                                                        \
    } while (0)
