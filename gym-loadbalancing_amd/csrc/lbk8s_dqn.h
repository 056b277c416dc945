// lbk8s_dqn.h — lb_dqn_step: one DQN vector step (envs/dqn_deepset.py:122-174) in ONE launch.
//
// The device DQN loop's vector step was three launches: lb_dqn_act (the explore decision, then
// the greedy action of the Q network's fused forward or every env's random action), lb_step
// (the env step) and lb_replay_add (the replay write, obs <- next obs, the finished episodes'
// sums).  Each env's chain -- its Q values, its action, its step, its replay row -- touches no
// other env, so one wave carries it through for P envs at a time: the forward's P sets of a
// wave iteration are exactly P 16-lane env slices of the slice layout's step kernel
// (W = 16, one endpoint per lane: the env layout of E <= 16 at fewer than 32,768 envs).  At
// config 5 (4096 envs) the step and replay kernels were ~5 us each of mostly launch ramp and
// tail (profiles/r03_dqn_kernel_stats_setgrads.csv); here they follow the forward inside the
// same waves.  Same functions, same order per env: bit for bit the three launches
// (tests/test_gpu_dqn_step.py).  The launch takes P = 2 envs per wave iteration (lbk8s.hip:
// dqn_steps_launch; one env per wave measured slower: profiles/r06_dqn_p1_ab.jsonl).
#pragma once

#include "lbk8s_deepsets.h"
#include "lbk8s_slice.h"

namespace lbk {

struct DQNReplay {  // lb_replay_add's buffers
    int64_t slots;
    int f4;  // float4s per observation
    const int64_t* pos_in;
    int64_t* pos_out;
    float4* obs;  // [B][f4] the step's input observations; <- the next observations
    float4* rb_obs;
    float4* rb_next_obs;
    int64_t* rb_actions;
    float* rb_rewards;
    float* rb_dones;
    double* ep_sum;  // [B] or NULL
    double* ep_cnt;
};

// d: the Q forward (lb_dqn_act's DSParams: obs, the actor-only weight image, masks, actions,
// the explore struct); e: the env (lb_step's Params: obs = the next observations, reward,
// done, terminal obs, ep_stats); r: the replay buffer.
//
// nsteps > 1 (lb_dqn_steps): that many vector steps in the one launch.  Within a DQN train
// period the Q network is fixed (the train step follows the period's last vector step) and
// every env's chain touches no other env, so each wave takes its P envs through all the
// steps: step i explores by dqn_explores(t + i) (the same draw for every env), writes replay
// slot pos + i, and leaves obs <- next obs and the env state for step i + 1, which the same
// wave reads back after an s_waitcnt vmcnt(0).  The device words (vstep, pos, explore flag)
// are then written by the launch's last block (sync: a counter the launch leaves at 0), after
// every block has read them: in and out may be the same words.  The counter wraps itself: the
// last block's atomicInc (limit gridDim.x - 1) returns gridDim.x - 1 and stores 0, so a launch
// that starts with *sync == 0 leaves it 0 with no separate store.
constexpr int DQN_OBS_F4 = 34;  // float4s of an observation of R <= 17 rows (dqn_step_fusable: R <= 16)
template <int P>
__global__ __launch_bounds__(DS_BLOCK, 2) void k_dqn_step(DSParams d, Params e, DQNReplay r, int nsteps,
                                                         int32_t* sync) {
    static_assert(P == 1 || P == 2, "envs per wave iteration (the VALU Gamma takes at most two)");
    constexpr int NWB = DS_BLOCK / 64;
    const int64_t t = *d.ex.vstep_in;
    const int64_t pos = *r.pos_in;
    uint32_t exm = 0;  // step i explores: bit i (:127, uniform over the launch)
    for (int i = 0; i < nsteps; ++i)
        if (dqn_explores(d.ex, t + i)) exm |= 1u << i;
    if (!sync && blockIdx.x == 0 && threadIdx.x == 0) {  // (nsteps == 1: in and out differ)
        *d.ex.explore_out = (int32_t)(exm & 1u);
        *d.ex.vstep_out = t + 1;
        *r.pos_out = (pos + 1) % r.slots;
    }
    // the Q network's VALU image (the actor part of VG_*: Lambda fragments, row-major Gamma: the
    // Gamma terms of the P sets of a wave iteration as VALU dot products instead of MFMA tiles
    // with P of 16 columns used), then each wave's scratch
    __shared__ __attribute__((aligned(16))) float W[VG_ACTOR + NWB * P * VG_SCRATCH];
    const uint32_t all = nsteps >= 32 ? ~0u : (1u << nsteps) - 1u;
    if (exm != all) {  // (some step is greedy)
        for (int i = threadIdx.x * 4; i < VG_ACTOR; i += DS_BLOCK * 4)
            *reinterpret_cast<float4*>(W + i) = *reinterpret_cast<const float4*>(d.wfrag + DS_FLOATS + i);
        __syncthreads();
    }
    float* xs = W + VG_ACTOR + (threadIdx.x >> 6) * P * VG_SCRATCH;
    const int lane = threadIdx.x & 63;
    // wave-major numbering, as k_deepsets_fwd: fewer groups than waves put one wave per SIMD
    const int64_t wave = (int64_t)(threadIdx.x >> 6) * gridDim.x + blockIdx.x;
    const int64_t nwaves = (int64_t)gridDim.x * NWB;
    const int R = d.R, col = lane & 15, grp = lane >> 4;
    const int64_t groups = (d.B + P - 1) / P, n4 = e.B * r.f4;
    const int s = lane >> 4, l16 = lane & 15;
    // the group's observations across the launch's steps in LDS, two buffers (step i's input
    // and its next observations): the Q forward and the replay rows read them there, so a step
    // issues its stores and reads nothing back from global memory (round 6: each step waited
    // for its obs stores to land, then re-read them -- two memory round trips per step)
    __shared__ __attribute__((aligned(16))) float4 OB[NWB][2][P * DQN_OBS_F4];
    const int f4 = r.f4;  // float4s per observation (2 R <= DQN_OBS_F4: host check)
    float4(*ob)[P * DQN_OBS_F4] = OB[threadIdx.x >> 6];
    for (int64_t gi = wave; gi < groups; gi += nwaves) {
        const int64_t env0 = gi * P;
        // the env held in registers across the launch's steps (as k_rollout_slice): loaded and
        // observed once, its history counters and scalars stored after the last step
        const int64_t env = env0 + s;
        const bool live = s < P && env < e.B;
        const int64_t j1 = (env0 + P < e.B ? env0 + P : e.B) * f4 - env0 * f4;  // the group's float4s
        SEnv<1> v;
        if (live) {
            slice_load<16, 1>(e, env, l16, v);
            slice_observe<1>(e, v);
        }
        for (int j = lane; j < j1; j += 64) ob[0][j] = r.obs[env0 * f4 + j];
        for (int i = 0; i < nsteps; ++i) {
            const bool explore = (exm >> i) & 1u;
            const int64_t ps = (pos + i) % r.slots;
            float4* cur = ob[i & 1];
            float4* nxt = ob[(i + 1) & 1];
            // the greedy actions of the group's envs (lane s holds env0 + s's; :134-142)
            int32_t act = -1;
            if (!explore) {
                float h0[P][2], m0[2];
                float xr0[2];
                ds_group_obs<1, P, 2>(d, env0, col, grp, R, h0, m0, xr0, reinterpret_cast<const float*>(cur));
                act = ds_group_actor<1, P, 2, true>(d, W, lane, env0, col, grp, R, h0, m0, xs);
            }
            const int32_t ag = __shfl(act, s < P ? s : 0);
            // the env step: lanes 16 s .. 16 s + 15 step env env0 + s (k_step_slice<16, 1>'s body,
            // the observed values kept in registers: a step changes the selected endpoint's)
            int a = 0;
            float rw = 0.f;
            bool dn = false;
            double ret = 0.0;  // the finished episode's return (its ep_stats row's first column)
            if (live) {
                a = explore ? random_action(e, env, v.acc3, v.s.step) : ag;  // (exploring: :128-131)
                if (explore && l16 == 0) d.actions[env] = a;
                const SPrep pr = slice_prep<16, 1>(e, v, a);
                const double tot0 = v.total;
                const double reward = slice_apply<16, 1, false, false>(e, env, l16, v, pr, dn);
                rw = (float)reward;
                ret = e.auto_reset ? tot0 + reward : 0.0;  // (slice_apply's v.total += reward)
                if (l16 == 0) {
                    e.reward[env] = rw;
                    if (e.rew64) e.rew64[env] = reward;
                    e.done[env] = (uint8_t)dn;
                }
                slice_obs_rows<16, 1>(e, l16, v, [&](int q, float4 o) { nxt[s * f4 + q] = o; });
            }
            // the group's replay rows (lb_replay_add's) and obs <- next obs, from LDS (the
            // wave's LDS writes and reads complete in order)
            for (int j = lane; j < j1; j += 64) {
                const float4 o = cur[j], nx = nxt[j];
                const int64_t g = env0 * f4 + j;
                r.rb_obs[ps * n4 + g] = o;
                r.rb_next_obs[ps * n4 + g] = nx;
                r.obs[g] = nx;
                st_stream(reinterpret_cast<float4*>(e.obs) + g, nx);
            }
            if (live && l16 == 0) {  // (the lane that wrote the env's reward, done and stats row)
                r.rb_actions[ps * e.B + env] = a;
                r.rb_rewards[ps * e.B + env] = rw;
                r.rb_dones[ps * e.B + env] = dn ? 1.f : 0.f;
                if (r.ep_sum && dn) {
                    r.ep_sum[env] += e.auto_reset ? ret : e.ep_stats[env * LB_ST_K];
                    r.ep_cnt[env] += 1.0;
                }
            }
        }
        if (live) {
            if (l16 < e.E) e.edyn[eidx(e, env, l16)] = v.ed[0];
            if (l16 == 0) slice_store_scalars<1>(e, env, v);
        }
    }
    if (sync) {  // the last block to finish writes the device words (every block has read them)
        __shared__ int last;
        __syncthreads();
        if (threadIdx.x == 0) {
            __threadfence();
            last = atomicInc(reinterpret_cast<unsigned*>(sync), gridDim.x - 1u) == gridDim.x - 1u;
        }
        __syncthreads();
        if (last && threadIdx.x == 0) {
            *d.ex.explore_out = (int32_t)((exm >> (nsteps - 1)) & 1u);
            *d.ex.vstep_out = t + nsteps;
            *r.pos_out = (pos + nsteps) % r.slots;
        }
    }
}

}  // namespace lbk
