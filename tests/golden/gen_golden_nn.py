#!/usr/bin/env python3
"""Golden fixtures for the deep-sets networks and the PPO / DQN update math.

Run here only (imports /root/reference through the gym stand-in):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_golden_nn.py

* Networks: the reference's own `DeepSetAgent` (envs/deep_sets_agent_original.py:109-145)
  and `DQNDeepSetAgent` (envs/deep_sets_agent_dqn.py:10-42), torch.manual_seed(2)
  initialisation, evaluated on real observations taken from the env fixtures
  (E = 6, 8, 64) with random masks -> logits, values, log-probs, entropy, masked argmax.
* PPO: one minibatch update of ppo_deepset.py:216-267 (clipped policy loss, clipped value
  loss, entropy bonus, normalised advantages, clip_grad_norm 0.5, Adam(2.5e-4, eps 1e-5))
  on a fixed batch; the loss is restated here from those lines because ppo_deepset.py
  itself needs stable_baselines3 / tensorboard (absent).  Gradients and the updated
  parameters are recorded.
* DQN: one train step of dqn_deepset.py:180-205 (target-network max, TD target,
  gather, MSE, Adam(2.5e-4)) on a fixed batch, same treatment.
Writes tests/golden/nn_*.npz (+ MANIFEST_nn.json).
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


class _Space:
    def __init__(self, shape, n=None):
        self.shape, self.n = shape, n


class _Envs:  # what DeepSetAgent reads from its `envs` argument
    def __init__(self, R, A):
        self.observation_space = _Space((R, 8))
        self.action_space = _Space((), A)


def real_obs(name, n):
    d = np.load(os.path.join(HERE, name + ".npz"))
    obs = d["obs"].reshape(-1, *d["obs"].shape[2:]).astype(np.float32)
    idx = np.random.default_rng(0).choice(len(obs), size=n, replace=False)
    return obs[idx]


def sd_arrays(module, prefix):
    return {prefix + k.replace(".", "__"): v.detach().numpy().copy() for k, v in module.state_dict().items()}


def gen_forward(ds, dqn_mod, name, fixture):
    obs = torch.from_numpy(real_obs(fixture, 64))
    B, R, _ = obs.shape
    torch.manual_seed(2)
    agent = ds.DeepSetAgent(_Envs(R, R))
    torch.manual_seed(3)
    qnet = dqn_mod.DQNDeepSetAgent(_Envs(R, R))
    g = torch.Generator().manual_seed(4)
    masks = torch.rand((B, R), generator=g) > 0.25
    masks[:, 0] = True
    actions = torch.randint(0, R, (B,), generator=g)
    with torch.no_grad():
        logits = agent.actor(obs)
        value = agent.critic(obs)
        _, logp, ent, v2 = agent.get_action_and_value(obs, actions)
        _, logp_m, ent_m, _ = agent.get_action_and_value(obs, actions, masks)
        mode_m = agent.get_action(obs, masks, deterministic=True)
        q = qnet(obs)
        q_mode_m = qnet.get_action(obs, masks, deterministic=True)
    out = dict(obs=obs.numpy(), masks=masks.numpy(), actions=actions.numpy(), logits=logits.numpy(),
               value=value.numpy(), logprob=logp.numpy(), entropy=ent.numpy(), value2=v2.numpy(),
               logprob_masked=logp_m.numpy(), entropy_masked=ent_m.numpy(), mode_masked=mode_m.numpy(),
               q=q.numpy(), q_mode_masked=q_mode_m.numpy())
    out.update(sd_arrays(agent, "agent__"))
    out.update(sd_arrays(qnet, "qnet__"))
    np.savez_compressed(os.path.join(HERE, f"nn_forward_{name}.npz"), **out)
    return dict(B=B, R=R)


def ppo_minibatch_loss(agent, mb, clip_coef=0.2, ent_coef=0.001, vf_coef=0.5, norm_adv=True, clip_vloss=True):
    """Restatement of ppo_deepset.py:227-263 for one minibatch."""
    _, newlogprob, entropy, newvalue = agent.get_action_and_value(mb["obs"], mb["actions"].long(), mb["masks"])
    logratio = newlogprob - mb["logprobs"]
    ratio = logratio.exp()
    adv = mb["advantages"]
    if norm_adv:
        adv = (adv - adv.mean()) / (adv.std() + 1e-8)
    pg_loss = torch.max(-adv * ratio, -adv * torch.clamp(ratio, 1 - clip_coef, 1 + clip_coef)).mean()
    newvalue = newvalue.view(-1)
    if clip_vloss:
        v_unclipped = (newvalue - mb["returns"]) ** 2
        v_clipped = mb["values"] + torch.clamp(newvalue - mb["values"], -clip_coef, clip_coef)
        v_loss = 0.5 * torch.max(v_unclipped, (v_clipped - mb["returns"]) ** 2).mean()
    else:
        v_loss = 0.5 * ((newvalue - mb["returns"]) ** 2).mean()
    entropy_loss = entropy.mean()
    loss = pg_loss - ent_coef * entropy_loss + v_loss * vf_coef
    approx_kl = ((ratio - 1) - logratio).mean()
    return loss, pg_loss, v_loss, entropy_loss, approx_kl


def gen_ppo(ds, fixture="default_naive", n=100, out_name="nn_ppo_update.npz", random_masks=False):
    """One PPO minibatch update.  The E = 64 variant (config 4's geometry, R = 65, 256 sets,
    ~10% of the actions masked out, the taken action always valid) pins the fused training
    kernels and the loss head at the shape the config-4 learner runs."""
    obs = torch.from_numpy(real_obs(fixture, n))
    B, R, _ = obs.shape
    torch.manual_seed(2)
    agent = ds.DeepSetAgent(_Envs(R, R))
    init = sd_arrays(agent, "init__")
    g = torch.Generator().manual_seed(7)
    with torch.no_grad():
        actions, logprobs, _, values = agent.get_action_and_value(obs)
    masks = torch.ones((B, R), dtype=torch.bool)
    if random_masks:
        masks = torch.rand((B, R), generator=g) > 0.1
        masks[torch.arange(B), actions] = True
    advantages = torch.randn(B, generator=g)
    returns = values.view(-1) + torch.randn(B, generator=g) * 0.5
    mb = dict(obs=obs, actions=actions.float(), logprobs=logprobs + 0.05 * torch.randn(B, generator=g),
              masks=masks, advantages=advantages, returns=returns, values=values.view(-1))
    opt = torch.optim.Adam(agent.parameters(), lr=2.5e-4, eps=1e-5)
    loss, pg, vl, ent, kl = ppo_minibatch_loss(agent, mb)
    opt.zero_grad()
    loss.backward()
    grads = {"grad__" + k.replace(".", "__"): p.grad.detach().numpy().copy() for k, p in agent.named_parameters()}
    gnorm = torch.nn.utils.clip_grad_norm_(agent.parameters(), 0.5)
    opt.step()
    out = {k: (v.numpy() if isinstance(v, torch.Tensor) else v) for k, v in mb.items()}
    out.update(init)
    out.update(grads)
    out.update(sd_arrays(agent, "after__"))
    out.update(loss=loss.item(), pg_loss=pg.item(), v_loss=vl.item(), entropy_loss=ent.item(),
               approx_kl=kl.item(), grad_norm=gnorm.item(), ent_coef=0.001, clip_coef=0.2, vf_coef=0.5)
    np.savez_compressed(os.path.join(HERE, out_name), **out)


def gen_dqn(dqn_mod):
    obs_all = torch.from_numpy(real_obs("default_naive", 256))
    obs, next_obs = obs_all[:128], obs_all[128:]
    B, R, _ = obs.shape
    torch.manual_seed(3)
    q = dqn_mod.DQNDeepSetAgent(_Envs(R, R))
    torch.manual_seed(5)
    target = dqn_mod.DQNDeepSetAgent(_Envs(R, R))
    init = sd_arrays(q, "init__")
    tinit = sd_arrays(target, "target__")
    g = torch.Generator().manual_seed(8)
    actions = torch.randint(0, R, (B, 1), generator=g)
    rewards = torch.randint(0, 2, (B, 1), generator=g).float() * 2 - 1
    dones = (torch.rand((B, 1), generator=g) < 0.1).float()
    gamma = 0.99
    # dqn_deepset.py:180-205
    with torch.no_grad():
        target_max, _ = target(next_obs).max(dim=1)
        td_target = rewards.flatten() + gamma * target_max * (1 - dones.flatten())
    old_val = q(obs).gather(1, actions).squeeze()
    loss = torch.nn.functional.mse_loss(td_target, old_val)
    opt = torch.optim.Adam(q.parameters(), lr=2.5e-4)
    opt.zero_grad()
    loss.backward()
    grads = {"grad__" + k.replace(".", "__"): p.grad.detach().numpy().copy() for k, p in q.named_parameters()}
    opt.step()
    out = dict(obs=obs.numpy(), next_obs=next_obs.numpy(), actions=actions.numpy(), rewards=rewards.numpy(),
               dones=dones.numpy(), td_target=td_target.numpy(), old_val=old_val.detach().numpy(),
               loss=loss.item(), gamma=gamma)
    out.update(init)
    out.update(tinit)
    out.update(grads)
    out.update(sd_arrays(q, "after__"))
    np.savez_compressed(os.path.join(HERE, "nn_dqn_update.npz"), **out)


def main():
    if not os.path.isdir(os.path.join(REF, "envs")):
        print(f"reference not found at {REF}; nothing to do")
        return 0
    sys.path.insert(0, os.path.join(HERE, "gym_standin"))
    sys.path.insert(0, REF)
    ds = importlib.import_module("envs.deep_sets_agent_original")
    dqn_mod = importlib.import_module("envs.deep_sets_agent_dqn")
    torch.set_num_threads(4)
    man = {}
    for name, fx in (("e6", "cfg1_multi"), ("e8", "default_naive"), ("e64", "e64_multi")):
        man[name] = gen_forward(ds, dqn_mod, name, fx)
    gen_ppo(ds)
    gen_ppo(ds, "e64_multi", 256, "nn_ppo_update_e64.npz", random_masks=True)
    gen_dqn(dqn_mod)
    man["torch"] = torch.__version__
    with open(os.path.join(HERE, "MANIFEST_nn.json"), "w") as f:
        json.dump(man, f, indent=1)
    for f in sorted(os.listdir(HERE)):
        if f.startswith("nn_"):
            print(f, os.path.getsize(os.path.join(HERE, f)))
    return 0


if __name__ == "__main__":
    sys.exit(main())
