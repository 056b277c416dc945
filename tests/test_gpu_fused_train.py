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
                                    (33, False), (49, True), (65, False), (65, True), (80, False),
                                    # above 80: the chunked training forward; 257 = E 256 + reject row
                                    (81, False), (129, True), (181, False), (257, True)])
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


def test_train_step_extra_row_many_sets_per_wave():
    """R = 65 (the extra-row training forward, the backward's one-row last tile and its pooled
    term) with 4,500 sets: more sets than the kernels' 2,048 waves, so waves loop over sets and
    reuse their LDS scratch and pooled-term rows; actor and critic against float64 autograd."""
    from lbk8s import fused_train
    agent = _agent(65)
    B, R = 4500, 65
    x = _inputs(B, R, seed=77, ties=True)
    g = torch.Generator().manual_seed(78)
    wl, wv = torch.randn(B, R, generator=g), torch.randn(B, generator=g)
    ref = copy.deepcopy(agent).double()
    xl, vl = ref.actor(x.double()), ref.critic(x.double())
    ((xl * wl.double()).sum() + (vl * wv.double()).sum()).backward()
    dev = agent.cuda()
    logits, value = fused_train.actor_critic(dev, x.cuda())
    _check(logits, xl, "logits", 1e-4, 4e-6)
    _check(value, vl, "value", 1e-4, 4e-6)
    ((logits * wl.cuda()).sum() + (value * wv.cuda()).sum()).backward()
    for (name, p), (_, q) in zip(dev.named_parameters(), ref.named_parameters()):
        _check(p.grad, q.grad, f"grad {name}", 1e-3, 1e-4)


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


@pytest.mark.parametrize("B,R,critic", [(1, 9, True), (128, 9, False), (128, 65, True), (300, 257, False),
                                         (512, 17, True)])
def test_set_grads_kernel_matches_gemm_path(B, R, critic, monkeypatch):
    """lb_ds_set_grads (the small-batch path: one launch) against the chunked GEMMs and
    reductions of _over_sets on the same backward (both f32; rtol 1e-5)."""
    from lbk8s import fused_train
    from lbk8s.deepsets import DQNDeepSetAgent
    x = _inputs(B, R, seed=B + R).cuda()
    w = torch.randn(B, R, generator=torch.Generator().manual_seed(B)).cuda()
    grads = []
    for limit in (fused_train.SET_GRADS_MAX_SETS, 0):
        monkeypatch.setattr(fused_train, "SET_GRADS_MAX_SETS", limit)
        if critic:
            agent = _agent(R).cuda()
            logits, value = fused_train.actor_critic(agent, x)
            ((logits * w).sum() + (value * w[:, 0]).sum()).backward()
        else:
            torch.manual_seed(R)
            agent = DQNDeepSetAgent(8).cuda()
            (fused_train.actor_only(agent, agent.q_network.net, x) * w).sum().backward()
        grads.append([p.grad.clone() for p in agent.parameters()])
    for i, (a, b) in enumerate(zip(*grads)):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6 * float(b.abs().max()) + 1e-12, msg=f"param {i}")


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


@pytest.mark.parametrize("R,masked", [(9, False), (65, True), (80, True), (181, True), (257, False)])
def test_ppo_head_matches_autograd(R, masked):
    """lb_ppo_head (loss terms and d loss / d logits, d loss / d value) against autograd
    through ppo_deepset.py:227-263's ops in float64 (the reference's formulation: masked
    Categorical, clipped ratio, clipped value loss, entropy bonus)."""
    from torch.distributions import Categorical
    from lbk8s import fused_train
    g = torch.Generator().manual_seed(R)
    M = 3001
    logits = torch.randn(M, R, generator=g) * 3
    masks = torch.rand(M, R, generator=g) > 0.2 if masked else torch.ones(M, R, dtype=torch.bool)
    actions = torch.randint(0, R, (M,), generator=g).float()
    masks[torch.arange(M), actions.long()] = True  # the taken action is valid (ratio ~ 1, not exp(1e8))
    value = torch.randn(M, generator=g) * 5
    ret = value + torch.randn(M, generator=g) * 2
    vold = value + torch.randn(M, generator=g) * 0.3      # |v - vold| on both sides of clip
    adv = torch.randn(M, generator=g)
    with torch.no_grad():  # old log-probs around the new ones: ratios in and out of [0.8, 1.2]
        lp = torch.log_softmax(torch.where(masks, logits, torch.full((), -1e8)), 1)
        oldlogp = lp.gather(1, actions.long()[:, None]).squeeze(1) + torch.randn(M, generator=g) * 0.3
    clip, ent_c, vf_c = 0.2, 0.01, 0.5

    L = logits.double().requires_grad_()
    V = value.double().requires_grad_()
    dist = Categorical(logits=torch.where(masks, L, torch.full((), -1e8, dtype=torch.float64)))
    nlp = dist.log_prob(actions.long())
    logratio = nlp - oldlogp.double()
    ratio = logratio.exp()
    A = adv.double()
    pg = torch.max(-A * ratio, -A * torch.clamp(ratio, 1 - clip, 1 + clip)).mean()
    vu = (V - ret.double()) ** 2
    vc = vold.double() + torch.clamp(V - vold.double(), -clip, clip)
    vl = 0.5 * torch.max(vu, (vc - ret.double()) ** 2).mean()
    ent = dist.entropy().mean()
    loss = pg - ent_c * ent + vl * vf_c
    loss.backward()

    Lg = logits.cuda().requires_grad_()
    Vg = value.cuda().requires_grad_()
    gl, st = fused_train.ppo_head(Lg, Vg, masks.cuda(), actions.cuda(), oldlogp.cuda(), adv.cuda(), ret.cuda(),
                                  vold.cuda(), clip, ent_c, vf_c, True)
    gl.backward()
    close(gl, loss.item(), rtol=1e-5, atol=1e-6, what="loss")
    close(st[0], pg.item(), rtol=1e-5, atol=1e-6, what="pg_loss")
    close(0.5 * st[1], vl.item(), rtol=1e-5, atol=1e-6, what="v_loss")
    close(st[2], ent.item(), rtol=1e-5, atol=1e-6, what="entropy")
    kl = ((ratio - 1) - logratio).mean().item()
    close(st[3], kl, rtol=1e-4, atol=1e-6, what="approx_kl")
    cf = ((ratio - 1).abs() > clip).double().mean().item()
    assert abs(float(st[4]) - cf) <= 2.0 / M, "clipfrac"
    _check(Lg.grad, L.grad, "d loss / d logits", 1e-4, 1e-5)
    _check(Vg.grad, V.grad, "d loss / d value", 1e-4, 1e-6)


@pytest.mark.gpu
def test_sums_over_sets_match_torch():
    """lb_ds_over_sets (the PPO minibatch's sums over 51,200 sets: Gamma / Lambda3 / rho weight
    gradients, bias sums) == float64 a^T b, for job shapes of the training step (M, N in {1, 8,
    64}, a NULL = a plain sum; M = 20: a partly filled 4-tile job), strided setvec-like views
    (aligned: float4 operand loads; offset by 10 floats: scalar loads), and set counts that are
    not multiples of the MFMA's 4 sets or the 256-set span; tolerance: f32 sums of S products."""
    from lbk8s import fused_train
    g = torch.Generator(device="cuda").manual_seed(11)
    for S in (51200, 1500, 1023, 5):
        wide = torch.randn((S, 300), generator=g, device="cuda")
        jobs = [(wide[:, 0:64], wide[:, 100:108], -1.0), (wide[:, 64:128], wide[:, 128:192], 1.0),
                (None, wide[:, 200:264], 1.0), (wide[:, 264:265], wide[:, 192:256], -1.0),
                (wide[:, 10:74], wide[:, 290:291], 0.5), (None, wide[:, 299:300], 1.0),
                (wide[:, 0:20], wide[:, 4:68], 2.0), (wide[:, 8:72], wide[:, 30:94], 1.0)]
        outs = fused_train.sums_over_sets(jobs, S, wide.device)
        for (a, b, sc), o in zip(jobs, outs):
            a64 = torch.ones((S, 1), dtype=torch.float64, device="cuda") if a is None else a.double()
            ref = sc * a64.t() @ b.double()
            assert o.shape == ref.shape
            torch.testing.assert_close(o.double(), ref, rtol=1e-4, atol=1e-4 * (S ** 0.5))


@pytest.mark.gpu
@pytest.mark.parametrize("critic", [True, False])
def test_train_backward_sets_equals_two_calls(critic):
    """lb_ds_train_backward_sets (the slot reduction and the set-gradient jobs in one launch,
    the DQN train step's path) == lb_ds_train_backward then lb_ds_set_grads, bit for bit."""
    from lbk8s import _native, fused, fused_train
    agent = _agent(11).cuda()
    B, R = 128, 9
    dev = torch.device("cuda")
    x = _inputs(B, R, seed=5).cuda()
    crit = agent.critic if critic else None
    frag = fused.packed(agent, agent.actor.net, crit)
    logits = torch.empty((B, R), device=dev)
    save_a = torch.empty((2, B, R, 64), device=dev)
    setvec = torch.empty((B, _native.LB_DS_SETVEC_FLOATS), device=dev)
    mean = torch.empty((B, 64), device=dev) if critic else None
    save_c = torch.empty((2, B, R, 64), device=dev) if critic else None
    L, st = _native.lib(), torch.cuda.current_stream().cuda_stream
    _native.check(L.lb_ds_train_forward(frag.data_ptr(), x.data_ptr(), B, R, logits.data_ptr(), fused._ptr(mean),
                                        save_a.data_ptr(), fused._ptr(save_c), setvec.data_ptr(), st))
    bfrag = fused_train._pack_backward(agent.actor.net, crit, dev)
    g = torch.Generator(device="cuda").manual_seed(3)
    dl = torch.randn((B, R), generator=g, device=dev)
    dm = torch.randn((B, 64), generator=g, device=dev) if critic else None
    n = _native.LB_DS_SETGRAD_ACTOR + (_native.LB_DS_SETGRAD_CRITIC if critic else 0)
    out = []
    for merged in (False, True):
        wg = torch.empty((2, _native.LB_DS_WGRAD_FLOATS), device=dev)
        sg = torch.empty(n, device=dev)
        args = (bfrag.data_ptr(), x.data_ptr(), B, R, save_a.data_ptr(), fused._ptr(save_c), dl.data_ptr(),
                fused._ptr(dm), wg.data_ptr(), fused_train._workspace(dev).data_ptr(), setvec.data_ptr())
        if merged:
            _native.check(L.lb_ds_train_backward_sets(*args, sg.data_ptr(), st))
        else:
            _native.check(L.lb_ds_train_backward(*args, st))
            _native.check(L.lb_ds_set_grads(setvec.data_ptr(), dl.data_ptr(), fused._ptr(dm), B, R, sg.data_ptr(), st))
        out.append((wg, sg))
    torch.cuda.synchronize()
    assert torch.equal(out[0][0], out[1][0]) and torch.equal(out[0][1], out[1][1])
