"""A14/A16: the fused deep-sets training step (lb_ds_train_forward / lb_ds_train_backward,
csrc/lbk8s_ds_train.h; host side lbk8s/fused_train.py).

Oracle: torch autograd through the same modules (the reference's EquivariantLayer /
EquivariantDeepSet / InvariantDeepSet, envs/deep_sets_agent_original.py:56-106) in
float64 on the CPU, with the same parameters and inputs.  The loss is a fixed random
linear functional of logits and value, so every parameter — the actor's last Gamma
included — has a real gradient.
Inputs are multiples of 1/4 and weights multiples of 1/32, so layer 1 and every
positive pre-activation of layer 2 are exact in float32: the set-wise argmaxes cannot
flip between the f32 kernel and the f64 oracle on a near-tie (with unquantised inputs,
torch's own f32 autograd flips one now and then, e.g. R = 65 with tied rows).
Tolerance (f32 kernel vs f64 autograd; gradients are sums over B x R rows): forward
rtol 1e-4 with an absolute floor of 4e-6 x max|expected|; gradients rtol 1e-3 with an
absolute floor of 1e-4 x max|expected| per tensor.
"""
import copy

import numpy as np
import pytest
import torch

from nn_helpers import close

pytestmark = pytest.mark.gpu


def _inputs(B, R, seed, ties=False):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(B, R, 8, generator=g) * torch.linspace(0.5, 3.0, 8) + 0.2
    x = torch.round(x * 4) / 4
    if ties:
        # observation-like structure: request columns equal on every row, integer zone ids,
        # duplicated rows (exact ties in every set-wise max)
        x[:, :, 5:] = x[:, :1, 5:]
        x[:, :, 0] = torch.randint(0, 4, (B, R), generator=g).float()
        if R > 2:
            x[:, 1] = x[:, 0]
    return x


def _agent(seed):
    from lbk8s.deepsets import DeepSetAgent
    torch.manual_seed(seed)
    agent = DeepSetAgent(8)
    with torch.no_grad():  # larger, asymmetric weights than the default init
        for p in agent.parameters():
            p.mul_(1.5).add_(0.01)
            p.copy_(torch.round(p * 32) / 32)
    return agent


def _check(got, exp, what, rtol, rel_floor):
    exp = exp.detach().cpu().double().numpy()
    got = got.detach().cpu().double().numpy()
    close(got, exp, rtol=rtol, atol=rel_floor * float(np.abs(exp).max()) + 1e-12, what=what)


@pytest.mark.parametrize("R,ties", [(1, False), (7, True), (9, False), (9, True), (16, False), (17, True),
                                    (33, False), (65, False), (65, True), (80, False)])
def test_train_step_matches_autograd(R, ties):
    from lbk8s import fused_train
    agent = _agent(200 + R)
    B = 257
    x = _inputs(B, R, seed=R, ties=ties)
    g = torch.Generator().manual_seed(1000 + R)
    wl, wv = torch.randn(B, R, generator=g), torch.randn(B, generator=g)

    ref = copy.deepcopy(agent).double()
    xl, vl = ref.actor(x.double()), ref.critic(x.double())
    ((xl * wl.double()).sum() + (vl * wv.double()).sum()).backward()

    dev = agent.cuda()
    logits, value = fused_train.actor_critic(dev, x.cuda())
    _check(logits, xl, f"logits R={R}", 1e-4, 4e-6)
    _check(value, vl, f"value R={R}", 1e-4, 4e-6)
    ((logits * wl.cuda()).sum() + (value * wv.cuda()).sum()).backward()
    for (name, p), (_, q) in zip(dev.named_parameters(), ref.named_parameters()):
        assert p.grad is not None, name
        _check(p.grad, q.grad, f"grad {name} R={R}", 1e-3, 1e-4)


def test_train_step_actor_only_and_many_sets():
    """The DQN Q network (actor stack only); more sets than resident waves."""
    from lbk8s import fused_train
    from lbk8s.deepsets import DQNDeepSetAgent
    torch.manual_seed(5)
    q = DQNDeepSetAgent(8)
    with torch.no_grad():
        for p in q.parameters():
            p.copy_(torch.round(p * 32) / 32)
    B, R = 20001, 9
    x = _inputs(B, R, seed=3, ties=True)
    w = torch.randn(B, R, generator=torch.Generator().manual_seed(4))
    ref = copy.deepcopy(q).double()
    (ref(x.double()) * w.double()).sum().backward()
    dev = q.cuda()
    out = fused_train.actor_only(dev, dev.q_network.net, x.cuda())
    _check(out, ref(x.double()), "q", 1e-4, 4e-6)
    (out * w.cuda()).sum().backward()
    for (name, p), (_, r) in zip(dev.named_parameters(), ref.named_parameters()):
        _check(p.grad, r.grad, f"grad {name}", 1e-3, 1e-4)


def test_train_forward_caches_follow_updates():
    """Two optimizer steps: the forward image is repacked (parameter versions move)."""
    from lbk8s import fused_train
    agent = _agent(9).cuda()
    ref = copy.deepcopy(agent).cpu().double()
    x = _inputs(64, 65, seed=11)
    opt = torch.optim.SGD(agent.parameters(), lr=1e-3)
    opt_r = torch.optim.SGD(ref.parameters(), lr=1e-3)
    for _ in range(2):
        opt.zero_grad()
        opt_r.zero_grad()
        lg, v = fused_train.actor_critic(agent, x.cuda())
        (lg.square().mean() + v.square().mean()).backward()
        opt.step()
        (ref.actor(x.double()).square().mean() + ref.critic(x.double()).square().mean()).backward()
        opt_r.step()
    for (name, p), (_, q) in zip(agent.named_parameters(), ref.named_parameters()):
        _check(p, q, f"param {name}", 1e-4, 1e-5)
