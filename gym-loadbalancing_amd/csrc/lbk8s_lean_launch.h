// lbk8s_lean_launch.h — the host-side interface of k_rollout_lean(_split) (lbk8s_lean.h).
//
// The lean kernels are compiled in their own units, one per on-device policy
// (lbk8s_lean_inst.hip built with -DLB_LEAN_KIND=0..3): 16 instantiations of a large kernel
// per policy, compiled in parallel instead of inside lbk8s.hip.  lbk8s.hip's lb_rollout calls
// launch_lean through the explicit instantiations declared here.
#pragma once

#include <hip/hip_runtime.h>

#include "lbk8s_common.h"

namespace lbk {

// launches of at most LEAN_SPLIT_MAX_K steps take k_rollout_lean_split (an env wave and a copy
// wave per block), longer ones k_rollout_lean (one wave per block): the split layout was 3-4%
// faster at K = 20 and 1-2% slower at K = 100 (profiles/r05_ab_split.jsonl)
constexpr int LEAN_SPLIT_MAX_K = 32;

// k_rollout_lean(_split) over B envs (B % 64 == 0), `steps` vector steps, on stream s
template <int KIND, int ET, int RT, int NZW, bool NAIVE, bool ACT>
void launch_lean(const Params& p, int64_t B, int steps, int32_t* act, hipStream_t s);

#define LB_LEAN_EXTERN(KIND_, NAIVE_, ACT_)                                                                    \
    extern template void launch_lean<KIND_, 8, 9, 1, NAIVE_, ACT_>(const Params&, int64_t, int, int32_t*, hipStream_t); \
    extern template void launch_lean<KIND_, 6, 7, 2, NAIVE_, ACT_>(const Params&, int64_t, int, int32_t*, hipStream_t);
#define LB_LEAN_EXTERN_KIND(KIND_)                                                                             \
    LB_LEAN_EXTERN(KIND_, true, true) LB_LEAN_EXTERN(KIND_, true, false) LB_LEAN_EXTERN(KIND_, false, true)     \
    LB_LEAN_EXTERN(KIND_, false, false)
LB_LEAN_EXTERN_KIND(0)
LB_LEAN_EXTERN_KIND(1)
LB_LEAN_EXTERN_KIND(2)
LB_LEAN_EXTERN_KIND(3)
#undef LB_LEAN_EXTERN_KIND
#undef LB_LEAN_EXTERN

}  // namespace lbk

#ifdef LB_TIMELINE
// (diagnostic builds: each policy unit's stamps buffer)
extern "C" int lbx_set_timeline_lean_0(uint64_t* buf);
extern "C" int lbx_set_timeline_lean_1(uint64_t* buf);
extern "C" int lbx_set_timeline_lean_2(uint64_t* buf);
extern "C" int lbx_set_timeline_lean_3(uint64_t* buf);
#endif
