#!/usr/bin/env python3
"""Interleaved in-process A/B of lb_rollout kernel variants on bench.py's workload.

    python tools/roll_variants.py [--envs N] [--steps K ...] [--variants 0,3] [--reps 3]

Variants are selected with the experiment switch lbx_set_rollout_variant, which only a
build with -DLB_EXPERIMENTS exports (0 the product dispatch, k_rollout_lean; 1
k_rollout_img; 3 the round-2 k_rollout_tpe); the product library runs variant 0 only.  The env is staggered as in bench.py (1/L of the envs finish every
step); each measurement is ONE HIP-event pair around `launches` back-to-back K-step launches
into the obs ring.  Prints one JSON line per (rep, K, variant).
"""
import argparse
import ctypes as C
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "gym-loadbalancing_amd")]


def _kernel_name(env, K):
    try:
        return env.rollout_kernel(K)
    except AttributeError:  # a diagnostic library from before lb_rollout_kernel
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=1 << 20)
    ap.add_argument("--steps", default="100,20")
    ap.add_argument("--variants", default="3,0")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--launches", type=int, default=3)
    ap.add_argument("--config", default="default")
    ap.add_argument("--touch", action="store_true", help="write the whole ring once before timing")
    ap.add_argument("--lib", default=None, help="another build of liblbk8s.so (an A/B across builds)")
    ap.add_argument("--no-obs", action="store_true", help="launch without the obs output (compute + small outputs)")
    ap.add_argument("--slot0", action="store_true", help="every timed launch writes from ring slot 0")
    ap.add_argument("--graph", action="store_true", help="issue the timed launches as one captured HIP graph")
    ap.add_argument("--stats-before", action="store_true",
                    help="as bench.py: an env.stats() reduction + host sync right before the timed window")
    ap.add_argument("--lockstep", action="store_true",
                    help="no staggering: every env restarts before each measurement (no episode ends "
                         "inside warm-up + timed launches when (launches + 1) * K < L)")
    args = ap.parse_args()
    import torch

    import bench
    from lbk8s import LBVecEnv, _native
    if args.lib:
        _native.LIB_PATH = os.path.abspath(args.lib)
    L = _native.lib()
    fn = getattr(L, "lbx_set_rollout_variant", None)
    if fn is not None and type(fn).__name__ != "_Missing":
        L.lbx_set_rollout_variant.argtypes = [C.c_int]
        set_variant = L.lbx_set_rollout_variant
    else:
        def set_variant(v):
            if v != 0:
                raise SystemExit(f"{_native.LIB_PATH} has no experiment switch: variant 0 only")
    staggers = [None]
    dev = torch.device("cuda", 0)
    B = args.envs
    env = LBVecEnv(B, device=dev, seed=0, as_tensors=True, **bench.CONFIGS[args.config])
    R, EL = env.cfg.obs_rows, env.cfg.episode_length
    T = 100
    obs = torch.empty((T, B, R, 8), dtype=torch.float32, device=dev)
    rew = torch.empty((T, B), dtype=torch.float32, device=dev)
    done = torch.empty((T, B), dtype=torch.uint8, device=dev)
    if args.touch:
        obs.zero_()
        rew.zero_()
        done.zero_()
    env.reset()
    gid = torch.arange(B, device=dev)
    for r in range(1, 1 if args.lockstep else EL):
        env.step_device(None, obs_out=obs[0], reward_out=rew[0], done_out=done[0])
        env.reset_masked((gid % EL) == r)
    stream = torch.cuda.current_stream(dev)
    for rep in range(args.reps):
        for K in [int(x) for x in args.steps.split(",")]:
            for var, stg in [(v, g) for v in [int(x) for x in args.variants.split(",")] for g in staggers]:
                set_variant(var)
                if args.lockstep:
                    env.reset()
                env.rollout("random", K, obs_out=obs[0], reward_out=rew[0], done_out=done[0])  # warm
                torch.cuda.synchronize()
                def launches():
                    for i in range(args.launches):
                        s = 0 if args.slot0 else (i * K) % max(1, T - K + 1)
                        env.rollout("random", K, obs_out=None if args.no_obs else obs[s], reward_out=rew[s],
                                    done_out=done[s])
                g = None
                if args.graph:
                    g = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(g):
                        launches()
                    env.rollout("random", K, obs_out=obs[0], reward_out=rew[0], done_out=done[0])  # warm again
                if args.stats_before:
                    env.stats()[:, 0].sum().item()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                if g is not None:
                    g.replay()
                else:
                    launches()
                e1.record(stream)
                torch.cuda.synchronize()
                us_launch = e0.elapsed_time(e1) * 1e3 / args.launches
                us = us_launch / max(K, 1)
                print(json.dumps({"rep": rep, "K": K, "variant": var, "stagger": stg, "lockstep": args.lockstep,
                                  "lib": os.path.basename(_native.LIB_PATH),
                                  "kernel": _kernel_name(env, K),
                                  "envs": B, "us_per_launch": round(us_launch, 2), "us_per_step": round(us, 2),
                                  "env_steps_per_s": B * K / us_launch * 1e6}), flush=True)
    set_variant(0)
    assert env.status() == 0


if __name__ == "__main__":
    main()
