#!/usr/bin/env python3
"""Per-wave step timeline of one lb_rollout launch (diagnostic build with -DLB_TIMELINE:
exp/liblbk8s_timeline.so).  Each wave's lane 0 stamps s_memrealtime (100 MHz) before its
first step, at every step start and after its last step; this prints the block generations'
start/end, and the mean duration of each step index across waves.

    python tools/timeline.py --lib exp/liblbk8s_timeline.so --steps 20
"""
import argparse
import ctypes as C
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "gym-loadbalancing_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default="exp/liblbk8s_timeline.so")
    ap.add_argument("--envs", type=int, default=1 << 20)
    ap.add_argument("--steps", type=int, default=20)
    args = ap.parse_args()
    import numpy as np
    import torch

    from lbk8s import LBVecEnv, _native
    _native.LIB_PATH = os.path.abspath(args.lib)
    L = _native.lib()
    L.lbx_set_timeline.argtypes = [C.c_void_p]
    B, K = args.envs, args.steps
    env = LBVecEnv(B, seed=0, as_tensors=True)
    R, EL = env.cfg.obs_rows, env.cfg.episode_length
    T = 100
    obs = torch.empty((T, B, R, 8), dtype=torch.float32, device="cuda")
    rew = torch.empty((T, B), dtype=torch.float32, device="cuda")
    done = torch.empty((T, B), dtype=torch.uint8, device="cuda")
    env.reset()
    gid = torch.arange(B, device="cuda")
    for r in range(1, EL):
        env.step_device(None, obs_out=obs[0], reward_out=rew[0], done_out=done[0])
        env.reset_masked((gid % EL) == r)
    waves = (B + 63) // 64
    tl = torch.zeros((waves, K + 2), dtype=torch.int64, device="cuda")
    for i in range(3):
        if i == 2:
            assert L.lbx_set_timeline(tl.data_ptr()) == 0
        env.rollout("random", K, obs_out=obs[0], reward_out=rew[0], done_out=done[0])
        torch.cuda.synchronize()
    a = tl.cpu().numpy().astype(np.float64) / 100.0  # us
    a -= a[a > 0].min()
    start, end = a[:, 0], a[:, K + 1]
    steps = np.diff(a[:, 1:K + 2], axis=1)  # duration of step k per wave
    prolog = a[:, 1] - a[:, 0]
    order = np.argsort(start)
    res = {"K": K, "launch_us": float(end.max()), "waves": int(waves),
           "prologue_us_mean": float(prolog.mean()),
           "step_us_mean_by_index": [round(float(x), 2) for x in steps.mean(axis=0)],
           "start_quantiles_us": [round(float(np.quantile(start, q)), 1) for q in (0, .25, .5, .75, 1)],
           "end_quantiles_us": [round(float(np.quantile(end, q)), 1) for q in (0, .25, .5, .75, 1)],
           "wave_life_us_mean": float((end - start).mean())}
    # generations: waves sorted by start, in groups of the resident count
    gens = []
    for g0 in range(0, waves, 4096):
        idx = order[g0:g0 + 4096]
        sd = steps[idx].mean(axis=0)
        pick = sorted(set([0, 1, 2, 4, 8, K // 2, K - 2, K - 1]) & set(range(K)))
        gens.append({"start": round(float(start[idx].min()), 1), "start_p50": round(float(np.median(start[idx])), 1),
                     "end_p50": round(float(np.median(end[idx])), 1), "end": round(float(end[idx].max()), 1),
                     "step_us_by_index": {int(i): round(float(sd[i]), 2) for i in pick},
                     "prologue_us": round(float(prolog[idx].mean()), 2)})
    res["generations"] = gens
    # resident waves over time (20 us bins): the launch's ramp and drain
    edges = np.arange(0.0, float(end.max()) + 20.0, 20.0)
    res["active_waves_20us"] = [int(((start < e + 20.0) & (end > e)).sum()) for e in edges]
    print(json.dumps(res))


if __name__ == "__main__":
    main()
