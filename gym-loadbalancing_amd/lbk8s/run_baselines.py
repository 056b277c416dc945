"""run_baselines.py equivalent (BASELINE config 1): greedy heuristics over many episodes.

    python -m lbk8s.run_baselines --policy topo --n_episodes 2000

The reference (/root/reference/run_baselines.py:28-78) plays `n_episodes` episodes of one
greedy policy (envs/baselines.py: topology / zone-cpu / endpoint-cpu greedy) one after
another on ONE env (E=6, N=48, Z=12, rejection, naive reward, latency weight 1), adding
up each episode's return.  Here the episodes run side by side, one env per episode, and
the whole 100-step episode is ONE launch (lb_rollout): the policy is evaluated inside the
step kernel on the env state it holds in registers, and the per-step rewards land in a
(steps, episodes) device buffer.  Episode i is the scenario of global env id
`env_id_offset + i` (Philox); the per-step semantics (draws aside) are pinned by the
reference's greedy-policy fixtures (tests/golden/greedy_*.npz through lb_policy, and
lb_rollout == lb_policy + lb_step, tests/test_gpu_api.py).
"""
import argparse
import csv
import json
import os
import time

import numpy as np
import torch

from .info import CSV_FIELDS, INFO_KEYS, ST_RETURN, csv_rows, info_matrix
from .vec_env import LBVecEnv

# run_baselines.py:16-56
CFG1 = dict(num_nodes=48, num_zones=12, num_endpoints=6, rejection_allowed=True, arrival_rate_r=100,
            call_duration_r=1, episode_length=100, reward_function="naive", latency_weight=1.0, cpu_weight=0.0,
            gini_weight=0.0)
POLICIES = ("topo", "zone_cpu", "endpoint_cpu")


@torch.no_grad()
def run_baselines(policy="topo", n_episodes=2000, device="cuda", seed=42, env_id_offset=0, **env_kwargs):
    """n_episodes greedy episodes -> dict: "returns" (float64, the reference's return_),
    "rewards" (steps, episodes) float32, the 12 numeric info keys of each episode's last
    step, "wall_s" of the rollout launch, "env_steps_per_s", and the per-episode CSV rows the
    reference's env appends at every episode end (loadbalancer_k8s_env.py:488-510):
    "csv_results" (its file_results_name file) and "csv_no_cost_updated" (no_cost_updated.csv),
    episode i of the batch numbered i + 1 as the reference's sequential episode_count.
    execution_time (the reference's per-episode wall clock) is the launch's wall time per
    episode here (unpinned)."""
    if policy not in POLICIES:
        raise ValueError(f"unrecognized policy {policy!r} (one of {POLICIES})")
    kw = dict(CFG1)
    kw.update(env_kwargs)
    # one episode per env, no auto-reset (the reference resets explicitly per episode); the
    # slice layout so the whole episode is one launch at any episode count
    env = LBVecEnv(n_episodes, device=device, seed=seed, env_id_offset=env_id_offset, auto_reset=False,
                   as_tensors=True, geometry="slice", **kw)
    env.reset()
    L = env.cfg.episode_length
    rewards = torch.empty((L, n_episodes), dtype=torch.float32, device=env.device)
    actions = torch.empty((L, n_episodes), dtype=torch.int32, device=env.device)
    torch.cuda.synchronize(env.device)
    t0 = time.perf_counter()
    env.rollout(policy, L, reward_out=rewards, actions_out=actions)
    torch.cuda.synchronize(env.device)
    wall = time.perf_counter() - t0
    st = env.stats().cpu().numpy()
    assert env.status() == 0
    info = info_matrix(st, rewards[-1].cpu().numpy(), actions[-1].cpu().numpy())
    out = {"returns": st[:, ST_RETURN].copy(), "rewards": rewards.cpu().numpy(), "wall_s": wall,
           "env_steps_per_s": n_episodes * L / wall, "csv_results": [], "csv_no_cost_updated": []}
    for i in range(n_episodes):
        res, upd = csv_rows(st[i], i + 1, wall / n_episodes)
        out["csv_results"].append(res)
        out["csv_no_cost_updated"].append(upd)
    for j, k in enumerate(INFO_KEYS[:12]):
        out[k] = info[:, j]
    return out


def baseline_file_name(index, policy, num_endpoints):
    """run_baselines.py:50-56: file_results_name of the i-th endpoint count's env."""
    return str(index) + "_" + policy + "_baselines_num_endpoints_" + str(num_endpoints)


def write_csvs(res, file_results_name, directory="."):
    """Append the rows as the reference's save_to_csv does (utils.py:99-127: mode 'a+', no
    header) to <file_results_name>.csv and no_cost_updated.csv."""
    for name, key in ((file_results_name + ".csv", "csv_results"), ("no_cost_updated.csv", "csv_no_cost_updated")):
        with open(os.path.join(directory, name), "a+", newline="") as f:
            w = csv.DictWriter(f, fieldnames=list(CSV_FIELDS))
            for row in res[key]:
                w.writerow(row)


def main(argv=None):
    ap = argparse.ArgumentParser(description="greedy baselines (run_baselines.py)")
    ap.add_argument("--policy", default="topo", choices=POLICIES)
    ap.add_argument("--n_episodes", type=int, default=2000)
    ap.add_argument("--num_endpoints", type=int, default=6)
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--device", default="cuda")
    ap.add_argument("--index", type=int, default=0, help="i of the results file name (run_baselines.py:50)")
    ap.add_argument("--results-dir", default=".")
    ap.add_argument("--no-csv", action="store_true")
    args = ap.parse_args(argv)
    res = run_baselines(args.policy, args.n_episodes, args.device, args.seed, num_endpoints=args.num_endpoints)
    if not args.no_csv:
        write_csvs(res, baseline_file_name(args.index, args.policy, args.num_endpoints), args.results_dir)
    summary = {"policy": args.policy, "n_episodes": args.n_episodes, "mean_return": float(np.mean(res["returns"])),
               "env_steps_per_s": res["env_steps_per_s"], "wall_s": res["wall_s"]}
    for k in INFO_KEYS[2:12]:
        summary["mean_" + k] = float(np.mean(res[k]))
    print(json.dumps(summary))
    return res


if __name__ == "__main__":
    main()
