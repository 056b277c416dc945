#!/usr/bin/env python3
"""Workload for the rocprofv3 PMC passes: 10 lb_step launches at 2^20 default envs (obs ring
of 16), then 3 torch copies of 1 GiB (known bytes: calibrates FETCH_SIZE / WRITE_SIZE)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "gym-loadbalancing_amd")]

import torch  # noqa: E402

from lbk8s import LBVecEnv  # noqa: E402


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "default"
    from bench import CONFIGS
    B = int(os.environ.get("PMC_ENVS", 1 << 20))
    env = LBVecEnv(B, seed=0, as_tensors=True, **CONFIGS[cfg])
    R, T = env.cfg.obs_rows, 16
    ring = torch.empty((T, B, R, 8), dtype=torch.float32, device="cuda")
    acts = torch.randint(0, env.action_space.n, (16, B), dtype=torch.int32, device="cuda")
    env.reset()
    for i in range(15):
        env.step_device(acts[i], obs_out=ring[i % T])
    torch.cuda.synchronize()
    x = torch.empty(1 << 28, dtype=torch.float32, device="cuda").uniform_()
    y = torch.empty_like(x)
    for _ in range(3):
        y.copy_(x)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
