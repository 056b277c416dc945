#!/usr/bin/env python3
"""Learning curves of the deep-sets learners at run.py's training setup, and their greedy
policies against the uniform-random policy on the same scenario.

run.py's defaults (run.py:23-45, 164-216): loadbalancer env, 6 endpoints, 4 zones, 24 nodes,
no rejection, multi reward (latency weight 1, cpu 0, gini 0), 8 parallel envs,
total_steps 200,000; get_model (run.py:54-72): PPO T=100, 8 minibatches, ent_coef 0.001;
DQN num_steps 100, 8 minibatches (learning_starts 10,000, the DQN default).  The learners'
own loops are the reference's: DQN's learn() runs total_steps VECTOR steps
(dqn_deepset.py:122), PPO's total_steps // (8 x 100) updates (ppo_deepset.py:147).

    python tools/learn_curves.py --alg dqn [--total-steps 200000] [--host-rng] --out curve.json

Prints a progress line per 1000 learner steps (the VecMonitor-style mean return of the
episodes finished since the last line), then one JSON line: the curve, the wall time, and
greedy / uniform-random mean episode returns over --eval-episodes fresh episodes (Philox seed
--eval-seed, the same scenarios for both policies).
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "gym-loadbalancing_amd")]


def eval_policy(act_fn, kw, episodes, seed, device):
    """Mean return of `episodes` episodes played side by side (one env each) from reset."""
    import torch

    from lbk8s import LBVecEnv
    env = LBVecEnv(episodes, device=device, seed=seed, as_tensors=True, **kw)
    obs = env.reset()
    ret = torch.zeros(episodes, dtype=torch.float64, device=device)
    for _ in range(env.cfg.episode_length):
        a = act_fn(env, obs)
        obs, r, d, _ = env.step(a)
        ret += r.to(torch.float64)
    return float(ret.mean().item()), float(ret.std().item())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--alg", choices=("dqn", "ppo"), default="dqn")
    ap.add_argument("--total-steps", type=int, default=200000)
    ap.add_argument("--learning-starts", type=int, default=None, help="DQN (default: the learner's 10,000)")
    ap.add_argument("--host-rng", action="store_true",
                    help="DQN: the host loop (explore draws with random.random(), the CLI's monitored env); "
                         "default: the device loop (lb_dqn_act draws, an env without monitor)")
    ap.add_argument("--seed", type=int, default=0, help="Philox seed of the training envs")
    ap.add_argument("--eval-episodes", type=int, default=256)
    ap.add_argument("--eval-seed", type=int, default=12345)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    import torch

    from lbk8s import cli
    dev = "cuda"
    kw = cli.env_kwargs(False, 6, 4, 24, "multi")
    device_loop = args.alg == "dqn" and not args.host_rng
    if device_loop:  # DQN's device loop (explore draws on the device) runs on an env without monitor
        from lbk8s import LBVecEnv
        env = LBVecEnv(8, device=dev, seed=args.seed, as_tensors=True, **kw)
    else:  # the CLI's env (run.py's VecMonitor wrapper): DQN's host loop
        env = cli.get_env("loadbalancer", False, 6, 4, 24, "multi", num_envs=8, device=dev, seed=args.seed,
                          monitor_file=None)
    curve = []
    t0 = time.time()

    def log(d):
        d = {k: (float(v) if isinstance(v, (int, float)) and v is not None else v) for k, v in d.items()}
        d["wall_s"] = round(time.time() - t0, 2)
        curve.append(d)
        print(json.dumps(d), flush=True)

    if args.alg == "dqn":
        from lbk8s.dqn import DQN_DeepSets
        extra = {} if args.learning_starts is None else dict(learning_starts=args.learning_starts)
        model = DQN_DeepSets(env, num_steps=100, n_minibatches=8, seed=1, log_fn=log,
                             device_rng=not args.host_rng, **extra)
    else:
        from lbk8s.ppo import PPO_DeepSets
        model = PPO_DeepSets(env, num_steps=100, n_minibatches=8, ent_coef=0.001, seed=2, log_fn=log)
    model.learn(total_timesteps=args.total_steps)
    torch.cuda.synchronize()
    wall = time.time() - t0
    env.close()

    def greedy(e, obs):
        return model.predict(obs).to(torch.int32)

    def uniform(e, obs):
        return e.policy("random")

    g_mean, g_std = eval_policy(greedy, kw, args.eval_episodes, args.eval_seed, dev)
    r_mean, r_std = eval_policy(uniform, kw, args.eval_episodes, args.eval_seed, dev)
    out = {"alg": args.alg + ("_deepsets"), "device_rng": (not args.host_rng) if args.alg == "dqn" else None,
           "total_steps": args.total_steps, "num_envs": 8, "scenario": kw, "wall_s": round(wall, 1),
           "episode_returns": [float(x) for x in model.episode_returns],
           "eval": {"episodes": args.eval_episodes, "seed": args.eval_seed, "greedy_mean": g_mean, "greedy_std": g_std,
                    "uniform_random_mean": r_mean, "uniform_random_std": r_std},
           "curve": curve}
    if args.out:
        with open(args.out, "w") as f:
            json.dump(out, f)
    print(json.dumps({k: v for k, v in out.items() if k not in ("curve", "episode_returns")}), flush=True)


if __name__ == "__main__":
    main()
