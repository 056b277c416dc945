#!/usr/bin/env python3
"""Workload for the rocprofv3 PMC passes: bench.py's timed step (2^20 default envs, the
env's random policy drawn in the kernel, obs / reward / done ring of 16, episodes staggered
so 1/episode_length of the envs end and auto-reset every step), 16 lb_step launches after
the stagger setup (PMC_MODE=rollout: 8 lb_rollout launches of PMC_K (default 100) steps into a
100-deep ring -- bench.py's launch shape for its default window, PMC_K=20 for the driver's
--steps 20 window), then 3 torch copies of 1 GiB (known bytes: calibrates FETCH_SIZE /
WRITE_SIZE)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "gym-loadbalancing_amd")]

import torch  # noqa: E402

from lbk8s import LBVecEnv  # noqa: E402


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "default"
    if os.environ.get("PMC_LIB"):  # A/B: another build of liblbk8s.so
        from lbk8s import _native
        _native.LIB_PATH = os.path.abspath(os.environ["PMC_LIB"])
    from bench import CONFIGS
    B = int(os.environ.get("PMC_ENVS", 1 << 20))
    env = LBVecEnv(B, seed=0, as_tensors=True, **CONFIGS[cfg])
    rollout = os.environ.get("PMC_MODE") == "rollout"
    R, T = env.cfg.obs_rows, (100 if rollout else 16)  # bench.py's ring; a rollout launch fills it
    ring = torch.empty((T, B, R, 8), dtype=torch.float32, device="cuda")
    rew = torch.empty((T, B), dtype=torch.float32, device="cuda")
    done = torch.empty((T, B), dtype=torch.uint8, device="cuda")
    L = env.cfg.episode_length
    env.reset()
    gid = torch.arange(B, device="cuda")
    for r in range(1, L):  # bench.py's stagger
        env.step_device(None, obs_out=ring[0], reward_out=rew[0], done_out=done[0])
        env.reset_masked((gid % L) == r)
    torch.cuda.synchronize()
    if rollout:
        K = int(os.environ.get("PMC_K", T))
        for i in range(8):
            s = (i * K) % (T - K + 1)
            env.rollout("random", K, obs_out=ring[s], reward_out=rew[s], done_out=done[s])
    else:
        for i in range(16):
            env.step_device(None, obs_out=ring[i % T], reward_out=rew[i % T], done_out=done[i % T])
    torch.cuda.synchronize()
    x = torch.empty(1 << 28, dtype=torch.float32, device="cuda").uniform_()
    y = torch.empty_like(x)
    for _ in range(3):
        y.copy_(x)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
