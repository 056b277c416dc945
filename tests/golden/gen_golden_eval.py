#!/usr/bin/env python3
"""Golden fixtures for the evaluation loop of run_test_deepset.py.

Run here only (imports /root/reference through the gym stand-in):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_golden_eval.py

The reference loop (/root/reference/run_test_deepset.py:58-98) plays n_episodes greedy
episodes one after another on ONE env inside DummyVecEnv + VecMonitor:

    obs = envs.reset(); mask = envs.env_method("action_masks")
    while not done: action = agent.predict(obs, mask); obs, r, dones, info = envs.step(action)

DummyVecEnv resets the env itself when an episode ends, and the loop then calls reset()
again, so every episode after the first starts from the SECOND reset after the previous
one (the auto-reset's draws are consumed and discarded).  This script drives the
reference env (its own seed-42 generator, :128-129) exactly that way, with the
reference's own networks (envs/deep_sets_agent_original.py DeepSetAgent for PPO,
envs/deep_sets_agent_dqn.py DQNDeepSetAgent for DQN) initialised by torch.manual_seed(42)
(the PPO_DeepSets constructor seeds 42 before building it; the DQN fixture uses seed 7 so
that its network differs from the PPO actor; no trained checkpoint ships with the
reference), and agent.predict's deterministic masked mode.

Recorded per fixture: the weights (data), the env's draws in call order (resets and
steps), every action / reward / done, and VecMonitor's per-episode values (return
accumulated in float32 as VecMonitor does, length, the final info).
Writes tests/golden/eval_{ppo,dqn}.npz.
"""
import importlib
import json
import os
import sys

import numpy as np
import torch

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
REF = os.environ.get("LBK8S_REFERENCE", "/root/reference")
sys.path.insert(0, HERE)
from gen_golden import INFO_KEYS, Recorder, parse_reset, parse_step  # noqa: E402

# run_test_deepset.py:19-57 (NUM_NODES / NUM_ZONES / weights; n_nodes of env_kwargs is unused)
TEST_ENV = dict(num_nodes=48, num_zones=12, num_endpoints=6, rejection_allowed=True, arrival_rate_r=100,
                call_duration_r=1, episode_length=100, reward_function="multi", latency_weight=1.0,
                cpu_weight=0.0, gini_weight=0.0)


class _Space:
    def __init__(self, shape, n=None):
        self.shape, self.n = shape, n


class _Envs:
    def __init__(self, R, A):
        self.observation_space = _Space((R, 8))
        self.action_space = _Space((), A)


def run(mod, agent_mod, alg, n_episodes, tmpdir):
    cwd = os.getcwd()
    os.chdir(tmpdir)
    try:
        env = mod.LoadBalancerK8sEnv(file_results_name="eval", **TEST_ENV)
        rec = Recorder(env.np_random)
        env.np_random = rec
        E, Z, N = env.num_endpoints, env.num_zones, env.num_nodes
        R, A = env.observation_space.shape[0], env.action_space.n
        # PPO_DeepSets / DQN_DeepSets(seed=42) seed torch with 42 before building the net; the
        # two nets' equivariant stacks would then be equal, so the DQN fixture takes seed 7
        torch.manual_seed(42 if alg == "ppo" else 7)
        if alg == "ppo":
            agent = agent_mod.DeepSetAgent(_Envs(R, A))
            head = agent.actor
        else:
            agent = agent_mod.DQNDeepSetAgent(_Envs(R, A))
            head = agent.q_network
        calls, actions, rewards, dones, ep, margins = [], [], [], [], [], []
        t0 = float(env.current_time)

        def reset():
            obs = env.reset()
            calls.append(("reset", parse_reset(rec.take(), E, Z, N)))
            return np.asarray(obs, dtype=np.float32)

        for _ in range(n_episodes):
            obs = reset()                                      # envs.reset()
            mask = np.asarray(env.action_masks(), dtype=bool)  # env_method("action_masks")
            done, ret32, length = False, np.float32(0.0), 0
            while not done:
                with torch.no_grad():  # agent.predict(obs, mask): deterministic masked mode
                    logits = head(torch.as_tensor(obs[None], dtype=torch.float32))
                    logits = torch.where(torch.as_tensor(mask[None]), logits, torch.tensor(-1e8))
                    a = int(torch.distributions.Categorical(logits=logits).mode[0])
                    top2 = torch.topk(logits[0], 2).values
                    margins.append(float(top2[0] - top2[1]))  # gap to the runner-up (tie risk)
                obs, r, done, info = env.step(a)
                calls.append(("step", parse_step(rec.take())))
                actions.append(a)
                rewards.append(float(r))
                dones.append(bool(done))
                ret32 = np.float32(ret32 + np.float32(r))    # VecMonitor: float32 episode_returns
                length += 1
                obs = np.asarray(obs, dtype=np.float32)
                if done:
                    ep.append([float(ret32), length, float(env.total_reward)] + [float(info[k]) for k in INFO_KEYS])
                    reset()                                    # DummyVecEnv's auto-reset
                mask = np.asarray(env.action_masks(), dtype=bool)
    finally:
        os.chdir(cwd)
    d = dict(t0=np.float64(t0), config_json=np.array(json.dumps(TEST_ENV)), alg=np.array(alg),
             actions=np.array(actions, np.int64), rewards=np.array(rewards), dones=np.array(dones),
             margins=np.array(margins),
             episodes=np.array(ep), episode_cols=np.array(json.dumps(["r_monitor", "l", "total_reward"] + INFO_KEYS)),
             call_kind=np.array([0 if k == "reset" else 1 for k, _ in calls], np.int8))
    resets = [c for k, c in calls if k == "reset"]
    steps = [c for k, c in calls if k == "step"]
    for key in ["lat0", "topo", "ntype", "nzone", "ncpu", "enode"]:
        d["reset_" + key] = np.stack([r[key] for r in resets])
    d["reset_req_x"] = np.array([[r["req"][0], r["req"][1]] for r in resets])
    d["reset_req_i"] = np.array([[r["req"][2], r["req"][3]] for r in resets], np.int64)
    d["step_x"] = np.array([[s[0], s[1]] for s in steps])
    d["step_i"] = np.array([[s[2], s[3]] for s in steps], np.int64)
    for k, v in agent.state_dict().items():
        d["agent__" + k.replace(".", "__")] = v.detach().numpy().copy()
    return d


def main():
    if not os.path.isdir(os.path.join(REF, "envs")):
        print(f"reference not found at {REF}; nothing to do")
        return 0
    import tempfile
    sys.path.insert(0, os.path.join(HERE, "gym_standin"))
    sys.path.insert(0, REF)
    mod = importlib.import_module("envs.loadbalancer_k8s_env")
    torch.set_num_threads(4)
    for alg, module, n in (("ppo", "envs.deep_sets_agent_original", 5), ("dqn", "envs.deep_sets_agent_dqn", 3)):
        with tempfile.TemporaryDirectory() as tmp:
            d = run(mod, importlib.import_module(module), alg, n, tmp)
        path = os.path.join(HERE, f"eval_{alg}.npz")
        np.savez_compressed(path, **d)
        print(alg, "episodes", len(d["episodes"]), "returns", d["episodes"][:, 0], os.path.getsize(path), "B")
    return 0


if __name__ == "__main__":
    sys.exit(main())
