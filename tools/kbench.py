#!/usr/bin/env python3
"""Kernel micro-bench: lb_step time vs batch size and scenario (one process, HIP events).

    python tools/kbench.py [--configs default,cfg1,e64_multi] [--sizes 16,18,20,22]
    python tools/kbench.py --config2          # BASELINE config 2: 4096 envs, random policy
Prints one JSON line per (config, B): ms per step, env-steps/s, algorithmic GB/s.

--config2: 4096 default envs driven by the env's own Philox random policy (lb_policy +
lb_step per vector step), 1,000 warm-up + 10,000 timed vector steps, launched eagerly and
as HIP graphs of 100 vector steps each (at this size a step is a few microseconds of GPU
time, below the cost of launching it from the host), as graphs of lb_step with the
random policy fused into the step kernel (actions == NULL: one launch per vector step),
and as lb_rollout (100 vector steps per launch, the state in registers between steps,
each step's obs / reward / done into its own ring slot).
--config1: run_baselines.py's workload (2000 episodes x 100 steps, E=6, N=48, Z=12, naive)
for each greedy policy, one lb_rollout launch per policy (lbk8s.run_baselines).
--rollout: lb_rollout with the random policy at large batches (K = ring steps per launch).
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "gym-loadbalancing_amd")]

from bench import CONFIGS, algorithmic_bytes  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="default,cfg1,e64_multi")
    ap.add_argument("--sizes", default="16,18,20,22")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--ring", type=int, default=16)
    ap.add_argument("--config2", action="store_true")
    ap.add_argument("--config1", action="store_true")
    ap.add_argument("--rollout", action="store_true")
    ap.add_argument("--lib", default=None, help="another build of liblbk8s.so (A/B)")
    ap.add_argument("--geometry", default="auto", help="--rollout: state layout (auto / tpe / slice)")
    args = ap.parse_args()
    if args.lib:
        from lbk8s import _native
        _native.LIB_PATH = os.path.abspath(args.lib)
    import torch

    from lbk8s import LBVecEnv
    dev = torch.device("cuda", 0)
    if args.config2:
        return config2(torch, LBVecEnv, dev)
    if args.config1:
        return config1(torch)
    if args.rollout:
        return rollout(torch, LBVecEnv, dev, args)
    for name in args.configs.split(","):
        for lg in (int(x) for x in args.sizes.split(",")):
            B = 1 << lg
            if name == "e64_multi" and lg > 20:
                continue
            env = LBVecEnv(B, device=dev, seed=0, as_tensors=True, **CONFIGS[name])
            R = env.cfg.obs_rows
            T = args.ring
            ring = torch.empty((T, B, R, 8), dtype=torch.float32, device=dev)
            rew = torch.empty((T, B), dtype=torch.float32, device=dev)
            dn = torch.empty((T, B), dtype=torch.uint8, device=dev)
            acts = torch.randint(0, env.action_space.n, (16, B), dtype=torch.int32, device=dev)
            env.reset()
            for i in range(20):
                env.step_device(acts[i % 16], obs_out=ring[i % T], reward_out=rew[i % T], done_out=dn[i % T])
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            s.record()
            for i in range(args.steps):
                env.step_device(acts[i % 16], obs_out=ring[i % T], reward_out=rew[i % T], done_out=dn[i % T])
            e.record()
            torch.cuda.synchronize()
            ms = s.elapsed_time(e) / args.steps
            b = algorithmic_bytes(env.cfg)
            print(json.dumps(dict(config=name, envs=B, ms_per_step=round(ms, 5),
                                  env_steps_per_s=B / ms * 1e3, alg_GBps=b * B / ms / 1e6,
                                  bytes_per_env_step=b)), flush=True)
            del env, ring, rew, dn, acts
            torch.cuda.empty_cache()


def config2(torch, LBVecEnv, dev, B=4096, warmup=1000, steps=10000, per_graph=100):
    env = LBVecEnv(B, device=dev, seed=0, as_tensors=True)
    R, T = env.cfg.obs_rows, 100
    ring = torch.empty((T, B, R, 8), dtype=torch.float32, device=dev)
    rew = torch.empty((T, B), dtype=torch.float32, device=dev)
    dn = torch.empty((T, B), dtype=torch.uint8, device=dev)
    act = torch.empty(B, dtype=torch.int32, device=dev)
    env.reset()

    def vector_step(i):
        env.policy("random", out=act)
        env.step_device(act, obs_out=ring[i % T], reward_out=rew[i % T], done_out=dn[i % T])

    def timed(fn, n):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        s.record()
        fn(n)
        e.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e)

    for i in range(warmup):
        vector_step(i)
    eager_ms = timed(lambda n: [vector_step(i) for i in range(n)], steps)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for i in range(per_graph):
            vector_step(i)
    g.replay()
    graph_ms = timed(lambda n: [g.replay() for _ in range(n // per_graph)], steps)
    assert env.status() == 0
    # the random policy fused into the step kernel (lb_step with actions == NULL)
    def fused_step(i):
        env.step_device(None, obs_out=ring[i % T], reward_out=rew[i % T], done_out=dn[i % T])

    g2 = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g2):
        for i in range(per_graph):
            fused_step(i)
    g2.replay()
    fused_ms = timed(lambda n: [g2.replay() for _ in range(n // per_graph)], steps)
    assert env.status() == 0
    # K = per_graph vector steps per lb_rollout launch
    def roll(n):
        for _ in range(n // per_graph):
            env.rollout("random", per_graph, obs_out=ring, reward_out=rew, done_out=dn)

    roll(per_graph)
    roll_ms = timed(roll, steps)
    assert env.status() == 0
    for mode, ms in (("eager", eager_ms), ("hip_graph", graph_ms), ("hip_graph_fused_policy", fused_ms),
                     ("lb_rollout_k100", roll_ms)):
        print(json.dumps(dict(config="config2 default, random policy", envs=B, mode=mode, vector_steps=steps,
                              ms_per_step=round(ms / steps, 5), env_steps_per_s=B * steps / ms * 1e3)), flush=True)


def config1(torch):
    from lbk8s.run_baselines import POLICIES, run_baselines
    run_baselines("topo", 2000)  # warm-up (module load, LUTs)
    for kind in POLICIES:
        best = None
        for _ in range(5):
            res = run_baselines(kind, 2000)
            best = res if best is None or res["wall_s"] < best["wall_s"] else best
        print(json.dumps(dict(config="config1 run_baselines (E=6, N=48, Z=12, naive)", policy=kind, episodes=2000,
                              steps_per_episode=100, launch_ms=round(best["wall_s"] * 1e3, 4),
                              env_steps_per_s=best["env_steps_per_s"],
                              mean_return=float(best["returns"].mean()))), flush=True)


def rollout(torch, LBVecEnv, dev, args):
    for name in args.configs.split(","):
        for lg in (int(x) for x in args.sizes.split(",")):
            B = 1 << lg
            if name == "e64_multi" and lg > 20:
                continue
            env = LBVecEnv(B, device=dev, seed=0, as_tensors=True, geometry=args.geometry, **CONFIGS[name])
            R, T = env.cfg.obs_rows, args.ring
            ring = torch.empty((T, B, R, 8), dtype=torch.float32, device=dev)
            rew = torch.empty((T, B), dtype=torch.float32, device=dev)
            dn = torch.empty((T, B), dtype=torch.uint8, device=dev)
            env.reset()
            env.rollout("random", T, obs_out=ring, reward_out=rew, done_out=dn)
            n = max(1, args.steps // T)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            s.record()
            for _ in range(n):
                env.rollout("random", T, obs_out=ring, reward_out=rew, done_out=dn)
            e.record()
            torch.cuda.synchronize()
            ms = s.elapsed_time(e) / (n * T)
            # per env-step: obs + reward + done written every step; the state read and
            # written once per launch (the lb_step figure less obs/reward/done, over K)
            b_step = algorithmic_bytes(env.cfg, reads_actions=False)
            out_b = 32 * R + 5
            b = out_b + (b_step - out_b) / T
            print(json.dumps(dict(config=name, envs=B, mode=f"lb_rollout_random_k{T}", geometry=args.geometry, ms_per_step=round(ms, 5),
                                  env_steps_per_s=B / ms * 1e3, alg_GBps=b * B / ms / 1e6,
                                  bytes_per_env_step=round(b, 1))), flush=True)
            del env, ring, rew, dn
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
