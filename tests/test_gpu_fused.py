"""A14: the fused deep-sets forward kernel (lb_ds_forward, csrc/lbk8s_deepsets.h).

* against the reference modules' own outputs (nn_forward_{e6,e8,e64}.npz, produced by
  envs/deep_sets_agent_original.py / deep_sets_agent_dqn.py on real observations);
* against the torch modules on the same device for every set size 1..80 (all five
  set-tile variants, ragged last tiles) with asymmetric random inputs;
* the weight image follows optimizer steps (cache invalidation by parameter version).
Tolerance: f32 MFMA products are exact, only the summation order differs from the
torch GEMMs: rtol 1e-4, and an absolute floor of 2e-5 + 4e-6 x max|expected| (a rounding
difference scales with the summands: Q values of ~40 cancel to ~0.04 in places).
"""
import numpy as np
import pytest
import torch

from nn_helpers import close, load_nn, state_dict_from

pytestmark = pytest.mark.gpu


def near(got, exp, what):
    exp = exp.detach().cpu().numpy() if isinstance(exp, torch.Tensor) else np.asarray(exp)
    close(got, exp, rtol=1e-4, atol=2e-5 + 4e-6 * float(np.abs(exp).max()), what=what)


@pytest.mark.parametrize("name", ["e6", "e8", "e64"])
def test_fused_forward_matches_reference(name):
    from lbk8s import fused
    from lbk8s.deepsets import DeepSetAgent, DQNDeepSetAgent
    d = load_nn(f"nn_forward_{name}")
    obs = torch.from_numpy(d["obs"]).cuda()
    agent = DeepSetAgent(8).cuda()
    agent.load_state_dict(state_dict_from(d, "agent__"))
    q = DQNDeepSetAgent(8).cuda()
    q.load_state_dict(state_dict_from(d, "qnet__"))
    logits, value = fused.deepsets_forward(agent, obs, require=True)
    near(logits, d["logits"], what="logits")
    near(value, d["value"], what="value")
    near(fused.q_forward(q, obs, require=True), d["q"], what="q")
    masks = torch.from_numpy(d["masks"]).cuda()
    qm = torch.where(masks, fused.q_forward(q, obs, require=True), torch.full((), -1e8, device="cuda"))
    assert (qm.argmax(1).cpu().numpy() == d["q_mode_masked"]).all()


@pytest.mark.parametrize("R", [1, 2, 7, 9, 15, 16, 17, 31, 32, 33, 48, 49, 64, 65, 79, 80, 81, 128, 129, 181, 257])
def test_fused_forward_all_set_sizes(R):
    from lbk8s import fused
    from lbk8s.deepsets import DeepSetAgent
    torch.manual_seed(100 + R)
    agent = DeepSetAgent(8).cuda()
    with torch.no_grad():  # larger, asymmetric weights than the default init
        for p in agent.parameters():
            p.mul_(1.5).add_(0.01)
    B = 300
    x = torch.randn(B, R, 8, device="cuda") * torch.linspace(0.5, 3.0, 8, device="cuda") + 0.2
    logits, value = fused.deepsets_forward(agent, x, require=True)
    with torch.no_grad():
        near(logits, agent.actor(x), what=f"logits R={R}")
        near(value, agent.critic(x), what=f"value R={R}")
    assert logits.shape == (B, R) and value.shape == (B,)


def test_fused_forward_large_batch_and_tail():
    """More envs than resident waves (grid-stride loop) and an odd batch."""
    from lbk8s import fused
    from lbk8s.deepsets import DeepSetAgent
    torch.manual_seed(7)
    agent = DeepSetAgent(8).cuda()
    x = torch.randn(70001, 9, 8, device="cuda")
    logits, value = fused.deepsets_forward(agent, x, require=True)
    with torch.no_grad():
        near(logits, agent.actor(x), what="logits")
        near(value, agent.critic(x), what="value")


@pytest.mark.parametrize("R", [9, 20])
@pytest.mark.parametrize("B", [1, 255, 256, 257, 1023, 1025, 2047, 4095, 4097, 8193])
def test_fused_forward_batch_sizes_around_the_grid(R, B):
    """Batch sizes around the launch's choices: P envs per wave (4 / 2 / 1 for R <= 16,
    fewer when the groups would not cover every SIMD), the grid (one block per CU up to the
    CU count, waves numbered wave-major), partial last groups."""
    from lbk8s import fused
    from lbk8s.deepsets import DeepSetAgent
    torch.manual_seed(11 * B + R)
    agent = DeepSetAgent(8).cuda()
    x = torch.randn(B, R, 8, device="cuda") * 1.5
    logits, value = fused.deepsets_forward(agent, x, require=True)
    with torch.no_grad():
        near(logits, agent.actor(x), what=f"logits B={B} R={R}")
        near(value, agent.critic(x), what=f"value B={B} R={R}")


def test_fused_weights_follow_optimizer_steps():
    from lbk8s import fused
    from lbk8s.deepsets import DeepSetAgent
    torch.manual_seed(3)
    agent = DeepSetAgent(8).cuda()
    x = torch.randn(64, 9, 8, device="cuda")
    l0, v0 = fused.deepsets_forward(agent, x, require=True)
    opt = torch.optim.Adam(agent.parameters(), lr=1e-2)
    loss = agent.actor(x).square().mean() + agent.critic(x).square().mean()
    opt.zero_grad()
    loss.backward()
    opt.step()
    l1, v1 = fused.deepsets_forward(agent, x, require=True)
    assert not torch.allclose(l0, l1)
    with torch.no_grad():
        near(l1, agent.actor(x), what="logits after step")
        near(v1, agent.critic(x), what="value after step")
    agent.load_state_dict({k: v.clone() for k, v in agent.state_dict().items()})  # copy_ bumps versions
    near(fused.deepsets_forward(agent, x, require=True)[0], l1.cpu().numpy(), what="after reload")


def test_fused_rejects_uncovered_inputs():
    from lbk8s import fused
    from lbk8s.deepsets import DeepSetAgent
    agent = DeepSetAgent(8).cuda()
    x = torch.randn(4, 258, 8, device="cuda")
    with pytest.raises(RuntimeError):
        fused.deepsets_forward(agent, x, require=True)
    logits, value = fused.deepsets_forward(agent, x)  # torch modules on the same device
    assert logits.shape == (4, 258) and value.shape == (4,) and logits.is_cuda
    np.testing.assert_array_equal(np.isfinite(logits.cpu().numpy()), True)


@pytest.mark.parametrize("R", [7, 9, 20, 65, 100, 181])
def test_fused_q_argmax(R):
    """lb_ds_q_argmax: the Q forward with the masked greedy action fused
    (dqn_deepset.py:134-142: argmax of where(mask, q, -1e8), first index on ties)."""
    from lbk8s import fused
    from lbk8s.deepsets import DQNDeepSetAgent
    torch.manual_seed(40 + R)
    q = DQNDeepSetAgent(8).cuda()
    B = 1001
    x = torch.randn(B, R, 8, device="cuda") * 2
    x[5] = x[5, :1]  # every row equal: Q ties on the whole set -> action 0
    masks = torch.rand(B, R, device="cuda") > 0.3
    masks[7] = False  # nothing valid: every entry -1e8 -> action 0
    masks[5] = True
    frag = fused.frag_buffer("cuda")
    act = torch.empty(B, dtype=torch.int32, device="cuda")
    qv = torch.empty(B, R, device="cuda")
    fused.q_argmax_graphable(q, x, masks, act, frag, q_out=qv)
    with torch.no_grad():
        near(qv, q.q_network(x), what=f"q R={R}")
    expect = torch.where(masks, qv, torch.full((), -1e8, device="cuda")).argmax(1)
    assert torch.equal(act.long(), expect)
    assert int(act[5]) == 0 and int(act[7]) == 0
    fused.q_argmax_graphable(q, x, None, act, frag)
    assert torch.equal(act.long(), qv.argmax(1))


def test_replay_add_matches_torch():
    """lb_replay_add == the torch replay add (DeviceReplayBuffer.add_device) + obs <- next_obs
    + per-env finished-episode sums, with the slot word alternating."""
    from lbk8s.dqn import DeviceReplayBuffer
    torch.manual_seed(0)
    B, R, slots = 300, 9, 4
    g = torch.Generator(device="cuda")
    a = DeviceReplayBuffer(slots * B, B, (R, 8), "cuda", g)
    b = DeviceReplayBuffer(slots * B, B, (R, 8), "cuda", g)
    obs_a = torch.randn(B, R, 8, device="cuda")
    obs_b = obs_a.clone()
    es_a = torch.zeros(B, dtype=torch.float64, device="cuda")
    ec_a = torch.zeros_like(es_a)
    es_b, ec_b = es_a.clone(), ec_a.clone()
    for step in range(slots + 2):  # wraps around
        nxt = torch.randn(B, R, 8, device="cuda")
        act = torch.randint(0, R, (B,), dtype=torch.int32, device="cuda")
        rew = torch.randn(B, device="cuda")
        done = (torch.rand(B, device="cuda") < 0.3).to(torch.uint8)
        ep = torch.randn(B, 16, dtype=torch.float64, device="cuda")
        a.add_fused(obs_a, nxt, act, rew, done, ep, es_a, ec_a, step % 2)
        d = done.double()
        es_b += ep[:, 0] * d
        ec_b += d
        b.add_device(obs_b, nxt, act, rew, done.float())
        obs_b.copy_(nxt)
    torch.cuda.synchronize()
    for f in ("obs", "next_obs", "actions", "rewards", "dones"):
        assert torch.equal(getattr(a, f), getattr(b, f)), f
    assert torch.equal(obs_a, obs_b)
    assert torch.equal(ec_a, ec_b) and torch.allclose(es_a, es_b, rtol=0, atol=1e-12)
    assert int(a.pos_pp[(slots + 2) % 2]) == int(b.pos_t) == (slots + 2) % slots
