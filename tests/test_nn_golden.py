"""T6: deep-sets networks (A14), the PPO minibatch update (A16) and the DQN train step
(A17) against fixtures produced by the reference's own modules (tests/golden/gen_golden_nn.py).

Runs on the CPU here (torch CPU, same float32 ops as the reference: tolerance rtol 1e-5)
and, marked gpu, on the MI355X (hipBLASLt float32 GEMMs: only the summation order
differs; tolerance rtol 1e-4 / atol 1e-5 on activations, 1e-4 on parameters)."""
import numpy as np
import pytest
import torch

from nn_helpers import close, load_nn, state_dict_from

DEVICES = ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)]
LR = 2.5e-4


def check_adam_step(module, d, gmax, device):
    """Parameters after one Adam step.  The first Adam step moves every entry by
    lr * g / (|g| + eps), i.e. by at most lr; where |g| is at the rounding-noise level
    (the true gradient is ~0) the direction is not reproducible across devices, so those
    entries are only bounded by lr, and the entries with a real gradient must match."""
    for n, p in module.named_parameters():
        key = n.replace(".", "__")
        got = p.detach().cpu().numpy()
        exp, init, g = d["after__" + key], d["init__" + key], np.abs(d["grad__" + key])
        assert np.all(np.abs(got - init) <= LR * 1.001), n
        # (the same threshold on every device: a CPU with another BLAS sums in another
        # order too, and eps=1e-5 makes entries with |g| ~ 1e-6 sensitive to that)
        real = g > 1e-3 * gmax
        np.testing.assert_allclose(got[real], exp[real], rtol=1e-4, atol=2e-6, err_msg="param " + n)


def tol(device):
    return dict(rtol=1e-5, atol=1e-6) if device == "cpu" else dict(rtol=1e-4, atol=2e-5)


def near(got, exp, device, what):
    """tol(device) plus an absolute floor proportional to the output's magnitude: another
    BLAS (another host CPU, or the GPU) sums in another order, and a rounding difference
    scales with the summands (Q values of ~40 cancel to ~0.04 in places)."""
    t = tol(device)
    scale = 1e-6 if device == "cpu" else 4e-6
    close(got, exp, rtol=t["rtol"], atol=t["atol"] + scale * float(np.abs(np.asarray(exp)).max()), what=what)


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("name", ["e6", "e8", "e64"])
def test_deepsets_forward_matches_reference(name, device):
    from lbk8s.deepsets import DeepSetAgent, DQNDeepSetAgent
    d = load_nn(f"nn_forward_{name}")
    obs = torch.from_numpy(d["obs"]).to(device)
    agent = DeepSetAgent(8).to(device)
    agent.load_state_dict(state_dict_from(d, "agent__"))
    q = DQNDeepSetAgent(8).to(device)
    q.load_state_dict(state_dict_from(d, "qnet__"))
    masks = torch.from_numpy(d["masks"]).to(device)
    actions = torch.from_numpy(d["actions"]).to(device)
    t = tol(device)
    with torch.no_grad():
        near(agent.actor(obs), d["logits"], device, "logits")
        near(agent.critic(obs), d["value"], device, "value")
        _, lp, ent, v = agent.get_action_and_value(obs, actions)
        near(lp, d["logprob"], device, "logprob")
        near(ent, d["entropy"], device, "entropy")
        _, lpm, entm, _ = agent.get_action_and_value(obs, actions, masks)
        near(lpm, d["logprob_masked"], device, "logprob masked")
        near(entm, d["entropy_masked"], device, "entropy masked")
        assert (agent.get_action(obs, masks).cpu().numpy() == d["mode_masked"]).all()
        near(q(obs), d["q"], device, "q")
        assert (q.get_action(obs, masks).cpu().numpy() == d["q_mode_masked"]).all()


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("golden", ["nn_ppo_update", "nn_ppo_update_e64"])
def test_ppo_minibatch_update_matches_reference(device, golden):
    """R = 9 (100 sets) and config 4's R = 65 (256 sets, masked actions): on the GPU the
    fused training kernels and the fused loss head run."""
    from lbk8s.deepsets import DeepSetAgent
    from lbk8s.ppo import ppo_loss
    d = load_nn(golden)
    agent = DeepSetAgent(8).to(device)
    agent.load_state_dict(state_dict_from(d, "init__"))
    f = lambda k, dt=torch.float32: torch.from_numpy(np.asarray(d[k])).to(device, dt)  # noqa: E731
    loss, pg, vl, ent, kl, _ = ppo_loss(agent, f("obs"), f("actions"), f("logprobs"), f("masks", torch.bool),
                                        f("advantages"), f("returns"), f("values"), clip_coef=0.2,
                                        ent_coef=0.001, vf_coef=0.5)
    t = tol(device)
    for got, key in ((loss, "loss"), (pg, "pg_loss"), (vl, "v_loss"), (ent, "entropy_loss"), (kl, "approx_kl")):
        close(got, d[key], what=key, **t)
    opt = torch.optim.Adam(agent.parameters(), lr=2.5e-4, eps=1e-5)
    opt.zero_grad()
    loss.backward()
    # gradients: elementwise, with an absolute floor of 1e-5 x the largest gradient.  The
    # actor's last Gamma has a true gradient of 0 (Gamma max(h) adds the same constant to
    # every logit of a set, and the log-softmax is shift-invariant): its entries are the
    # rounding noise of sum_r dlogits, which depends on the host BLAS's summation order, so
    # both sides are only bounded there (1e-4 x the largest gradient; R = 65's noise reaches
    # ~2e-5 of it on some CPUs).
    gmax = max(np.abs(d["grad__" + n.replace(".", "__")]).max() for n, _ in agent.named_parameters())
    for n, p in agent.named_parameters():
        exp = d["grad__" + n.replace(".", "__")]
        if n == "actor.net.4.Gamma.weight":
            assert np.abs(exp).max() <= 1e-4 * gmax
            assert float(p.grad.abs().max()) <= 1e-4 * gmax, n
            continue
        close(p.grad, exp, what="grad " + n, rtol=t["rtol"] * 10, atol=max(t["atol"] * 10, 1e-5 * gmax))
    gn = torch.nn.utils.clip_grad_norm_(agent.parameters(), 0.5)
    close(gn, d["grad_norm"], what="grad norm", **t)
    opt.step()
    check_adam_step(agent, d, gmax, device)


@pytest.mark.parametrize("device", DEVICES)
def test_dqn_train_step_matches_reference(device):
    from lbk8s.deepsets import DQNDeepSetAgent
    from lbk8s.dqn import dqn_loss
    d = load_nn("nn_dqn_update")
    q = DQNDeepSetAgent(8).to(device)
    q.load_state_dict(state_dict_from(d, "init__"))
    tgt = DQNDeepSetAgent(8).to(device)
    tgt.load_state_dict(state_dict_from(d, "target__"))
    f = lambda k, dt=torch.float32: torch.from_numpy(np.asarray(d[k])).to(device, dt)  # noqa: E731
    loss, td, old = dqn_loss(q, tgt, f("obs"), f("actions", torch.long), f("next_obs"), f("rewards"), f("dones"),
                             float(d["gamma"]))
    t = tol(device)
    close(td, d["td_target"], what="td target", **t)
    close(old, d["old_val"], what="old val", **t)
    close(loss, d["loss"], what="loss", **t)
    opt = torch.optim.Adam(q.parameters(), lr=2.5e-4)
    opt.zero_grad()
    loss.backward()
    gmax = max(np.abs(d["grad__" + n.replace(".", "__")]).max() for n, _ in q.named_parameters())
    for n, p in q.named_parameters():
        close(p.grad, d["grad__" + n.replace(".", "__")], what="grad " + n, rtol=t["rtol"] * 10,
              atol=max(t["atol"] * 10, 1e-5 * gmax))
    opt.step()
    check_adam_step(q, d, gmax, device)


def test_state_dict_names_match_reference():
    from lbk8s.deepsets import DeepSetAgent, DQNDeepSetAgent
    d = load_nn("nn_forward_e8")
    assert set(DeepSetAgent(8).state_dict()) == set(state_dict_from(d, "agent__"))
    assert set(DQNDeepSetAgent(8).state_dict()) == set(state_dict_from(d, "qnet__"))
    assert sum(p.numel() for p in DeepSetAgent(8).actor.parameters()) == 9344
    assert sum(p.numel() for p in DeepSetAgent(8).critic.parameters()) == 21633


def test_rollout_sampler_is_the_categorical_distribution():
    """DeepSetAgent.act(uniforms=...) (the PPO rollout's inverse-CDF sampler on pre-drawn
    uniforms, ppo_deepset.py:169's Categorical.sample()): action frequencies follow the
    softmax of the (masked) logits, masked actions (logit -1e8) are never taken, and the
    log-prob is that of the taken action."""
    from lbk8s.deepsets import DeepSetAgent
    torch.manual_seed(0)
    agent = DeepSetAgent(8)
    n = 200_000
    x = torch.rand(1, 9, 8).expand(n, 9, 8).contiguous()
    masks = torch.ones(n, 9, dtype=torch.bool)
    masks[:, 2] = False
    masks[:, 7] = False
    g = torch.Generator().manual_seed(1)
    u = torch.rand(n, generator=g)
    a, lp, _ = agent.act(x, masks, uniforms=u)
    assert not bool(((a == 2) | (a == 7)).any())
    with torch.no_grad():
        p = torch.softmax(torch.where(masks[0], agent.actor(x[:1])[0], torch.tensor(-1e8)), dim=-1)
    freq = torch.bincount(a, minlength=9).double() / n
    assert torch.allclose(freq, p.double(), atol=4e-3), (freq, p)
    torch.testing.assert_close(lp, torch.log(p)[a], rtol=1e-5, atol=1e-6)


def test_gae_matches_direct_recursion():
    from lbk8s.ppo import compute_gae
    g = torch.Generator().manual_seed(0)
    T, B = 7, 5
    r, v = torch.randn(T, B, generator=g), torch.randn(T, B, generator=g)
    dn = (torch.rand(T, B, generator=g) < 0.2).float()
    nv, nd = torch.randn(1, B, generator=g), (torch.rand(B, generator=g) < 0.2).float()
    adv, ret = compute_gae(r, v, dn, nv, nd, 0.95, 0.97)
    for b in range(B):
        last = 0.0
        for t in reversed(range(T)):
            nnt = 1.0 - (nd[b] if t == T - 1 else dn[t + 1, b])
            nval = nv[0, b] if t == T - 1 else v[t + 1, b]
            delta = r[t, b] + 0.95 * nval * nnt - v[t, b]
            last = delta + 0.95 * 0.97 * nnt * last
            assert abs(adv[t, b] - last) < 1e-5
    assert torch.allclose(ret, adv + v)


def _gae_fixture():
    import os
    return np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "nn_gae.npz"))


@pytest.mark.parametrize("device", DEVICES)
def test_gae_matches_reference_learn(device):
    """compute_gae (lbk8s/ppo.py) against the advantages / returns the reference's own
    PPO_DeepSets.learn() computed (ppo_deepset.py:192-205) on the storage its rollout loop
    filled (tests/golden/gen_golden_gae.py: reference envs, multi reward, dones at staggered
    steps).  Same float32 tensor ops in the same order: bit for bit on the CPU, 1e-6 on the
    GPU."""
    from lbk8s.ppo import compute_gae
    d = _gae_fixture()
    t = {k: torch.from_numpy(d[k]).to(device) for k in ("rewards", "values", "dones", "next_value", "next_done")}
    adv, ret = compute_gae(t["rewards"], t["values"], t["dones"], t["next_value"], t["next_done"],
                           float(d["gamma"]), float(d["gae_lambda"]))
    adv, ret = adv.cpu().numpy(), ret.cpu().numpy()
    if device == "cpu":
        assert np.array_equal(adv, d["advantages"]) and np.array_equal(ret, d["returns"])
    else:
        np.testing.assert_allclose(adv, d["advantages"], rtol=1e-6, atol=1e-6)
        np.testing.assert_allclose(ret, d["returns"], rtol=1e-6, atol=1e-6)


def test_ppo_storage_sequencing_matches_reference_learn():
    """learn()'s storage convention (ppo_deepset.py:162-176): dones[t] is the done flag that
    came back from step t - 1 (zeros at t = 0), rewards[t] the reward of step t, next_done the
    flags of the last step.  The reference fixture shows it; PPO_DeepSets._rollout_body (our
    rollout) fills its storage the same way when its env returns the reference's per-step
    rewards and dones."""
    from lbk8s.ppo import PPO_DeepSets
    d = _gae_fixture()
    raw = d["raw_dones"].astype(np.float32)
    T, B = raw.shape
    assert np.array_equal(d["dones"][0], np.zeros(B, np.float32))
    assert np.array_equal(d["dones"][1:], raw[:-1]) and np.array_equal(d["next_done"], raw[-1])

    class _Space:
        def __init__(self, shape, n=None):
            self.shape, self.n = shape, n

    class StubEnv:  # returns the reference's step outputs in order
        num_envs, device = B, torch.device("cpu")
        observation_space, action_space = _Space((7, 8)), _Space((), 7)
        ep_stats = torch.zeros((B, 16), dtype=torch.float64)

        def __init__(self):
            self.t = 0

        def step_device(self, act, obs_out, reward_out, done_out):
            obs_out.zero_()
            reward_out.copy_(torch.from_numpy(d["rewards"][self.t]))
            done_out.copy_(torch.from_numpy(d["raw_dones"][self.t].astype(np.uint8)))
            self.t += 1

        def record_episodes(self, *a):
            pass

    algo = PPO_DeepSets(StubEnv(), num_steps=T, n_minibatches=2, update_epochs=1, seed=2, device="cpu",
                        use_graphs=False)
    next_done = algo._rollout_body(torch.zeros(B))
    assert np.array_equal(algo.dones.numpy(), d["dones"])
    assert np.array_equal(algo.rewards.numpy(), d["rewards"])
    assert np.array_equal(next_done.numpy(), d["next_done"])


def test_equivariant_custom_backward_gradcheck():
    """The GPU training path's hand-written backward (_EquivariantFn) against numerical
    gradients, float64 on the CPU; inputs include exact ties in the set-wise max (as the
    tiled request columns of real observations have)."""
    from lbk8s.deepsets import _EquivariantFn
    g = torch.Generator().manual_seed(0)
    x = torch.randn(3, 5, 4, generator=g, dtype=torch.float64)
    x[:, :, 3] = x[:, :1, 3]  # a column equal on every element: ties everywhere
    x.requires_grad_(True)
    lam = torch.randn(6, 4, generator=g, dtype=torch.float64, requires_grad=True)
    gam = torch.randn(6, 4, generator=g, dtype=torch.float64, requires_grad=True)
    # ties make max non-differentiable in x; check x where the max is unique, weights everywhere
    assert torch.autograd.gradcheck(lambda a, b: _EquivariantFn.apply(x, a, b), (lam, gam))
    xu = torch.randn(3, 5, 4, generator=g, dtype=torch.float64, requires_grad=True)
    assert torch.autograd.gradcheck(lambda a, b, c: _EquivariantFn.apply(a, b, c), (xu, lam, gam))
    # with ties, the gradient must equal autograd's through torch.max (first index returned)
    gy = torch.randn(3, 5, 6, generator=g, dtype=torch.float64)
    ref_x = x.detach().clone().requires_grad_(True)
    pooled, _ = torch.max(ref_x, dim=1, keepdim=True)
    (torch.nn.functional.linear(ref_x, lam) - torch.nn.functional.linear(pooled, gam)).backward(gy)
    got_x = x.detach().clone().requires_grad_(True)
    _EquivariantFn.apply(got_x, lam, gam).backward(gy)
    torch.testing.assert_close(got_x.grad, ref_x.grad, rtol=1e-12, atol=1e-12)


def test_splitk_weight_grad_remainder():
    from lbk8s.deepsets import splitk_weight_grad
    g = torch.Generator().manual_seed(1)
    a = torch.randn(11, 9, 6, generator=g, dtype=torch.float64)
    b = torch.randn(11, 9, 4, generator=g, dtype=torch.float64)
    ref = a.reshape(-1, 6).t() @ b.reshape(-1, 4)
    for rows in (7, 16, 99, 1000):
        torch.testing.assert_close(splitk_weight_grad(a, b, rows), ref, rtol=1e-12, atol=1e-12)
