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


@pytest.mark.parametrize("R", [1, 2, 7, 9, 15, 16, 17, 31, 32, 33, 48, 49, 64, 65, 79, 80])
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
    x = torch.randn(4, 81, 8, device="cuda")
    with pytest.raises(RuntimeError):
        fused.deepsets_forward(agent, x, require=True)
    logits, value = fused.deepsets_forward(agent, x)  # torch modules on the same device
    assert logits.shape == (4, 81) and value.shape == (4,) and logits.is_cuda
    np.testing.assert_array_equal(np.isfinite(logits.cpu().numpy()), True)
