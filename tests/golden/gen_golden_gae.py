#!/usr/bin/env python3
"""Golden fixture for PPO's rollout storage and GAE, made by the reference's own learn().

Run here only (imports /root/reference through stand-ins; nothing of the reference is stored):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_golden_gae.py

/root/reference/envs/ppo_deepset.py imports four names it uses only for type hints and
logging: stable_baselines3's DummyVecEnv / SubprocVecEnv (annotations), safe_mean (a print)
and torch.utils.tensorboard's SummaryWriter (scalars).  Neither package is installed, so
this script registers from-scratch stand-ins for those modules (a no-op writer, a plain
mean) in sys.modules before the import -- as tests/golden/gym_standin does for gym.

It then runs the reference's PPO_DeepSets.learn() (ppo_deepset.py:145-267) for ONE update
on a small vector env made of reference LoadBalancerK8sEnv instances (the SB3 VecEnv
contract: auto-reset on done, obs returned as the post-reset obs), and records, at the line
after the GAE loop (ppo_deepset.py:192-205), the storage the loop filled -- rewards, values,
dones (dones[t] = the done flag that came back from step t-1, :162-176) -- with next_value,
next_done, the advantages and returns, and the raw per-step done flags the env returned.
Writes tests/golden/nn_gae.npz.
"""
import importlib
import os
import sys
import tempfile
import types

import numpy as np
import torch

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
REF = os.environ.get("LBK8S_REFERENCE", "/root/reference")

# the scenario: multi reward (float rewards), short episodes of different lengths per env
# (5, 6, 7, 8 steps) so dones fall inside the rollout at different steps
ENV_KW = dict(num_nodes=24, num_zones=4, num_endpoints=6, rejection_allowed=True, reward_function="multi",
              latency_weight=1.0, cpu_weight=0.0, gini_weight=0.0)
EPISODE_LENGTHS = (5, 6, 7, 8)
NUM_ENVS, NUM_STEPS, SEED = 4, 24, 2


def install_standins():
    """sys.modules stand-ins for the logging / typing-only imports of ppo_deepset.py:15-19."""
    class SummaryWriter:  # torch.utils.tensorboard: every call is a no-op
        def __init__(self, *a, **k):
            pass

        def __getattr__(self, name):
            return lambda *a, **k: None

    def safe_mean(arr):  # stable_baselines3.common.utils.safe_mean
        return float("nan") if len(arr) == 0 else float(np.mean(arr))

    class _VecEnvName:  # DummyVecEnv / SubprocVecEnv appear only in annotations
        pass

    mods = {
        "stable_baselines3": {},
        "stable_baselines3.common": {},
        "stable_baselines3.common.vec_env": {},
        "stable_baselines3.common.vec_env.dummy_vec_env": {"DummyVecEnv": _VecEnvName},
        "stable_baselines3.common.vec_env.subproc_vec_env": {"SubprocVecEnv": _VecEnvName},
        "stable_baselines3.common.utils": {"safe_mean": safe_mean},
        "torch.utils.tensorboard": {"SummaryWriter": SummaryWriter},
    }
    for name, attrs in mods.items():
        m = types.ModuleType(name)
        m.__dict__.update(attrs)
        sys.modules[name] = m


class RefVecEnv:
    """The SB3 VecEnv contract over reference env instances: step() auto-resets a finished env
    and returns its post-reset obs (the terminal obs goes to info)."""

    def __init__(self, mod, n):
        self.envs = [mod.LoadBalancerK8sEnv(file_results_name=f"gae{i}", episode_length=EPISODE_LENGTHS[i], **ENV_KW)
                     for i in range(n)]
        self.num_envs = n
        self.observation_space = self.envs[0].observation_space
        self.action_space = self.envs[0].action_space
        self.raw_dones = []

    def reset(self):
        return np.stack([e.reset() for e in self.envs])

    def step(self, actions):
        obs, rews, dones, infos = [], [], [], []
        for e, a in zip(self.envs, actions):
            o, r, d, info = e.step(int(a))
            if d:
                info = dict(info, terminal_observation=o)
                o = e.reset()
            obs.append(o)
            rews.append(r)
            dones.append(d)
            infos.append(info)
        self.raw_dones.append(np.array(dones, bool))
        return np.stack(obs), np.array(rews, dtype=np.float64), np.array(dones), infos

    def env_method(self, name):
        return [getattr(e, name)() for e in self.envs]


def main():
    if not os.path.isdir(os.path.join(REF, "envs")):
        print(f"reference not found at {REF}; nothing to do")
        return 0
    install_standins()
    sys.path.insert(0, os.path.join(HERE, "gym_standin"))
    sys.path.insert(0, REF)
    envmod = importlib.import_module("envs.loadbalancer_k8s_env")
    ppo_ref = importlib.import_module("envs.ppo_deepset")
    torch.set_num_threads(4)
    captured = {}

    def tracer(frame, event, arg):
        # capture learn()'s storage and GAE result at the first line after the GAE loop
        if frame.f_code.co_name != "learn" or "ppo_deepset" not in frame.f_code.co_filename:
            return None

        def local(fr, ev, a):
            if ev == "line" and not captured and "returns" in fr.f_locals:
                self = fr.f_locals["self"]
                captured.update(
                    rewards=self.rewards.clone(), values=self.values.clone(), dones=self.dones.clone(),
                    actions=self.actions.clone(), logprobs=self.logprobs.clone(),
                    next_value=fr.f_locals["next_value"].clone(), next_done=fr.f_locals["next_done"].clone(),
                    advantages=fr.f_locals["advantages"].clone(), returns=fr.f_locals["returns"].clone(),
                    gamma=self.gamma, gae_lambda=self.gae_lambda)
            return local
        return local

    cwd = os.getcwd()
    with tempfile.TemporaryDirectory() as tmp:
        os.chdir(tmp)
        try:
            venv = RefVecEnv(envmod, NUM_ENVS)
            algo = ppo_ref.PPO_DeepSets(venv, num_steps=NUM_STEPS, num_envs=NUM_ENVS, n_minibatches=2,
                                        update_epochs=1, seed=SEED, device="cpu", tensorboard_log=tmp)
            sys.settrace(tracer)
            try:
                algo.learn(total_timesteps=NUM_STEPS * NUM_ENVS)  # num_updates = 1
            finally:
                sys.settrace(None)
        finally:
            os.chdir(cwd)
    assert captured, "the GAE line was not reached"
    d = {k: (v.numpy() if torch.is_tensor(v) else np.float64(v)) for k, v in captured.items()}
    d["raw_dones"] = np.stack(venv.raw_dones)
    d["config"] = np.array(repr(dict(ENV_KW, episode_lengths=EPISODE_LENGTHS, num_envs=NUM_ENVS,
                                     num_steps=NUM_STEPS, seed=SEED)))
    path = os.path.join(HERE, "nn_gae.npz")
    np.savez_compressed(path, **d)
    print("dones per step", d["raw_dones"].sum(1), "adv[0]", d["advantages"][0], os.path.getsize(path), "B")
    return 0


if __name__ == "__main__":
    sys.exit(main())
