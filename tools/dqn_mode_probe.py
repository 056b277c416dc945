#!/usr/bin/env python3
"""DQN device loop vs host loop at config 5's setting (tools/rl_bench.py --algo dqn: 4096
default-scenario envs, 2 replay slots per env, learning_starts 100, a 300-step warm-up
learn() then a 2000-step learn()), for several learner seeds: the last flushed mean episode
return (rl_bench's ep_return), the greedy policy's mean return on 256 fresh scenarios, and
its action histogram (the reject action is the last).

    python tools/dqn_mode_probe.py [--seeds 1,2,3]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "gym-loadbalancing_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", default="1,2,3")
    ap.add_argument("--envs", type=int, default=4096)
    args = ap.parse_args()
    import torch

    from bench import CONFIGS
    from lbk8s import LBVecEnv
    from lbk8s.dqn import DQN_DeepSets
    for seed in [int(s) for s in args.seeds.split(",")]:
        for device_rng in (True, False):
            env = LBVecEnv(args.envs, seed=0, as_tensors=True, monitor=not device_rng, monitor_file=None,
                           **CONFIGS["default"])
            dqn = DQN_DeepSets(env, seed=seed, learning_starts=100, device_rng=device_rng)
            dqn.learn(300)
            dqn.learn(2000)
            last = dqn.episode_returns[-1] if dqn.episode_returns else None
            ev = LBVecEnv(256, seed=12345, as_tensors=True, **CONFIGS["default"])
            obs = ev.reset()
            ret = torch.zeros(256, dtype=torch.float64, device="cuda")
            hist = torch.zeros(ev.action_space.n, dtype=torch.int64, device="cuda")
            for _ in range(ev.cfg.episode_length):
                a = dqn.predict(obs).to(torch.int32)
                hist += torch.bincount(a.to(torch.int64), minlength=ev.action_space.n)
                obs, r, _, _ = ev.step(a)
                ret += r.to(torch.float64)
            print(json.dumps({"seed": seed, "device_loop": device_rng, "ep_return_last": last,
                              "greedy_mean": float(ret.mean()), "greedy_actions": hist.tolist(),
                              "train_steps": dqn.train_steps}), flush=True)
            env.close()


if __name__ == "__main__":
    main()
