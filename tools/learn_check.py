#!/usr/bin/env python3
"""tests/test_gpu_learners.py::test_*_run_py_setup_beats_uniform_random's measurement, printed
(greedy and uniform-random mean returns on 256 fresh scenarios) for a build:
    python tools/learn_check.py [--lib exp/x.so] [--algo dqn|ppo] [--host-loop] [--seed S] [--steps N]"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "gym-loadbalancing_amd"), os.path.join(REPO, "tests")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=None)
    ap.add_argument("--algo", default="dqn")
    ap.add_argument("--host-loop", action="store_true")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20000)
    a = ap.parse_args()
    import torch  # noqa: F401  (before the library: one HIP runtime)
    from lbk8s import _native
    if a.lib:
        _native.LIB_PATH = os.path.abspath(a.lib)
    from lbk8s import LBVecEnv, cli
    from test_gpu_learners import _greedy_vs_uniform
    if a.algo == "dqn":
        from lbk8s.dqn import DQN_DeepSets
        if a.host_loop:
            env = cli.get_env("loadbalancer", False, 6, 4, 24, "multi", num_envs=8, seed=0, monitor_file=None)
        else:
            env = LBVecEnv(8, seed=0, as_tensors=True, **cli.env_kwargs(False, 6, 4, 24, "multi"))
        model = DQN_DeepSets(env, num_steps=100, n_minibatches=8, seed=a.seed, device_rng=not a.host_loop)
    else:
        from lbk8s.ppo import PPO_DeepSets
        env = cli.get_env("loadbalancer", False, 6, 4, 24, "multi", num_envs=8, seed=0, monitor_file=None)
        model = PPO_DeepSets(env, num_steps=100, n_minibatches=8, ent_coef=0.001, seed=a.seed)
    model.learn(total_timesteps=a.steps)
    g, u = _greedy_vs_uniform(model.predict)
    print(json.dumps({"lib": os.path.basename(a.lib or "liblbk8s.so"), "algo": a.algo, "host_loop": a.host_loop,
                      "seed": a.seed, "steps": a.steps, "greedy": g, "uniform": u, "margin": g - u}))


if __name__ == "__main__":
    main()
