// lbk8s_lean_inst.hip — the k_rollout_lean(_split) instantiations of ONE on-device policy
// (LB_LEAN_KIND = LB_POLICY_*, set by csrc/Makefile: four objects from this file).  The kernels
// are lbk8s_lean.h's; lb_rollout (lbk8s.hip) launches them through launch_lean.
#include "lbk8s_lean.h"
#include "lbk8s_lean_launch.h"

#ifndef LB_LEAN_KIND
#error "LB_LEAN_KIND (the policy of this unit) must be defined"
#endif

namespace lbk {

template <int KIND, int ET, int RT, int NZW, bool NAIVE, bool ACT>
void launch_lean(const Params& p, int64_t B, int steps, int32_t* act, hipStream_t s) {
    if (steps <= LEAN_SPLIT_MAX_K) {
        hipLaunchKernelGGL((k_rollout_lean_split<KIND, ET, RT, NZW, NAIVE, ACT, 1>), dim3((unsigned)(B / 64)), dim3(128), 0,
                           s, p, steps, act);
        return;
    }
    hipLaunchKernelGGL((k_rollout_lean<KIND, ET, RT, NZW, NAIVE, ACT>), dim3((unsigned)((B + LEAN_NB - 1) / LEAN_NB)),
                       dim3(LEAN_NB), 0, s, p, steps, act);
}

#define LB_LEAN_INST(NAIVE_, ACT_)                                                                                  \
    template void launch_lean<LB_LEAN_KIND, 8, 9, 1, NAIVE_, ACT_>(const Params&, int64_t, int, int32_t*, hipStream_t); \
    template void launch_lean<LB_LEAN_KIND, 6, 7, 2, NAIVE_, ACT_>(const Params&, int64_t, int, int32_t*, hipStream_t);
LB_LEAN_INST(true, true)
LB_LEAN_INST(true, false)
LB_LEAN_INST(false, true)
LB_LEAN_INST(false, false)
#undef LB_LEAN_INST

}  // namespace lbk

#ifdef LB_TIMELINE
#define LB_CAT2(a, b) a##b
#define LB_CAT(a, b) LB_CAT2(a, b)
extern "C" int LB_CAT(lbx_set_timeline_lean_, LB_LEAN_KIND)(uint64_t* buf) {
    return hipMemcpyToSymbol(HIP_SYMBOL(lbk::g_timeline), &buf, sizeof(buf)) == hipSuccess ? 0 : -1;
}
#endif
