"""Evaluation of trained deep-sets agents: run_test_deepset.py.

The reference (/root/reference/run_test_deepset.py:44-98) loads a PPO or DQN checkpoint
(`agent.load(path)`: a torch state_dict, ppo_deepset.py:296-300, dqn_deepset.py:227-231)
and plays `n_episodes` episodes on ONE env, one after the other, with deterministic
masked argmax actions (`agent.predict(obs, action_mask)`), while VecMonitor writes the
per-episode return and the info keywords.

Two forms:
* run_test: the episodes run side by side: `n_episodes` envs on the device, one vector
  step per time step: logits (PPO actor) or Q values (DQN) from the fused forward kernel,
  masked argmax, the fused env step.  Auto-reset is off, so every env plays exactly one
  episode (episode_length steps).  Episode i is the scenario of global env id
  `env_id_offset + i` (Philox), so any single episode can be replayed alone.
* run_sequential: the reference loop as written — ONE env, episodes one after another,
  DummyVecEnv's auto-reset on done followed by the loop's own reset() (so the auto-reset's
  scenario is drawn and discarded), VecMonitor's float32 episode return.  Pinned by
  fixtures recorded from the reference env + the reference networks
  (tests/golden/gen_golden_eval.py) replayed in trace mode.
"""
import csv
import time

import numpy as np
import torch

from . import fused
from .deepsets import HUGE_NEG, DeepSetAgent, DQNDeepSetAgent
from .info import INFO_KEYS, ST_LENGTH, ST_RETURN, info_matrix
from .vec_env import LBVecEnv

# run_test_deepset.py:19-57 (its env_kwargs' n_nodes is unused: NUM_NODES / NUM_ZONES win)
TEST_ENV = dict(num_nodes=48, num_zones=12, num_endpoints=6, rejection_allowed=True, arrival_rate_r=100,
                call_duration_r=1, episode_length=100, reward_function="multi", latency_weight=1.0,
                cpu_weight=0.0, gini_weight=0.0)


def load_agent(path, alg, in_channels=8, device="cuda"):
    """A reference checkpoint (torch state_dict) -> DeepSetAgent ("ppo") or DQNDeepSetAgent ("dqn")."""
    agent = (DeepSetAgent if alg == "ppo" else DQNDeepSetAgent)(in_channels).to(device)
    agent.load_state_dict(torch.load(path, map_location=device, weights_only=True))
    agent.eval()
    return agent


@torch.no_grad()
def greedy_actions(agent, obs, masks):
    """agent.predict(obs, masks) of ppo_deepset.py:289-294 / dqn_deepset.py: argmax of the
    masked logits (Categorical(logits).mode) or Q values; first index on ties."""
    if isinstance(agent, DeepSetAgent):
        scores, _ = fused.deepsets_forward(agent, obs)
    else:
        scores = fused.q_forward(agent, obs)
    scores = torch.where(masks, scores, torch.full((), HUGE_NEG, device=scores.device))
    return torch.argmax(scores, dim=1).to(torch.int32)


@torch.no_grad()
def run_test(agent, n_episodes=2000, seed=42, env_id_offset=0, device="cuda", monitor_path=None, **env_kwargs):
    """Play n_episodes greedy episodes in parallel -> dict of per-episode numpy arrays:
    "r" return, "l" length, the 12 numeric info keys of the final step, and "wall_s"."""
    kw = dict(TEST_ENV)
    kw.update(env_kwargs)
    env = LBVecEnv(n_episodes, device=device, seed=seed, env_id_offset=env_id_offset, auto_reset=False,
                   as_tensors=True, **kw)
    obs = env.reset()
    masks = env.action_masks()
    t0 = time.time()
    for _ in range(env.cfg.episode_length):
        obs, _, _, _ = env.step(greedy_actions(agent, obs, masks))
    st = env.stats().cpu().numpy()
    wall = time.time() - t0
    info = info_matrix(st, env.rewards.cpu().numpy(), env.actions.cpu().numpy())
    out = {"r": st[:, ST_RETURN].copy(), "l": st[:, ST_LENGTH].astype(np.int64), "wall_s": wall}
    for j, k in enumerate(INFO_KEYS[:12]):
        out[k] = info[:, j]
    if monitor_path is not None:
        write_monitor_csv(monitor_path, out, INFO_KEYS[:12])
    return out


@torch.no_grad()
def run_sequential(agent, n_episodes, env, draws=None, monitor_path=None, info_keywords=INFO_KEYS):
    """run_test_deepset.py:83-98 on a one-env LBVecEnv (auto_reset on, as DummyVecEnv):

        for episode: obs = envs.reset(); mask = env_method("action_masks")
                     while not done: obs, r, dones, info = envs.step(agent.predict(obs, mask))

    draws: None (Philox) or, for an env in trace mode, an object whose next_reset() /
    next_step() return the reference's draws for the next reset() / step() in call order
    (the step that ends an episode also consumes the auto-reset's).  Returns per-step
    "actions" / "rewards" / "dones" and per-episode "r" (VecMonitor's float32 return), "l",
    "total_reward" (float64) and the final info's keys."""
    if env.num_envs != 1 or not env.auto_reset:
        raise ValueError("run_sequential plays one env with auto-reset (DummyVecEnv of one env)")
    L = env.cfg.episode_length
    out = {k: [] for k in ("actions", "rewards", "dones", "r", "l", "total_reward")}
    for k in info_keywords:
        out[k] = []
    for _ in range(n_episodes):
        obs = env.reset(trace=draws.next_reset() if draws is not None else None)
        obs = torch.as_tensor(obs, device=env.device)
        masks = env.action_masks()
        done, ret32, length = False, np.float32(0.0), 0
        while not done:
            a = greedy_actions(agent, obs, masks)
            st = draws.next_step() if draws is not None else None
            rt = draws.next_reset() if (draws is not None and length + 1 == L) else None
            obs, rew, dones, infos = env.step(a, trace=st, reset_trace=rt)
            obs = torch.as_tensor(obs, device=env.device)
            r = float(np.asarray(rew.cpu() if isinstance(rew, torch.Tensor) else rew)[0])
            done = bool(np.asarray(dones.cpu() if isinstance(dones, torch.Tensor) else dones)[0])
            ret32 = np.float32(ret32 + np.float32(r))
            length += 1
            out["actions"].append(int(a[0]))
            out["rewards"].append(r)
            out["dones"].append(done)
            if done:
                info = infos[0]
                out["r"].append(float(ret32))
                out["l"].append(length)
                out["total_reward"].append(float(env._host_ep_stats()[0, ST_RETURN]))
                for k in info_keywords:
                    out[k].append(info[k])
    res = {k: np.asarray(v) for k, v in out.items()}
    if monitor_path is not None:
        res["wall_s"] = 0.0
        write_monitor_csv(monitor_path, res, info_keywords)
    return res


def write_monitor_csv(path, res, info_keywords):
    """VecMonitor's file layout: a '#' JSON header line, then r, l, t and the info keywords."""
    with open(path, "w", newline="") as f:
        f.write('#{"t_start": %.6f}\n' % time.time())
        w = csv.writer(f)
        w.writerow(["r", "l", "t"] + list(info_keywords))
        for i in range(len(res["r"])):
            w.writerow([round(float(res["r"][i]), 6), int(res["l"][i]), round(res["wall_s"], 6)]
                       + [res[k][i] for k in info_keywords])
