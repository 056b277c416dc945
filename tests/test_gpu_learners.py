"""GPU end-to-end runs of the device-resident learners (A16 PPO, A17 DQN) on LBVecEnv."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu


def test_ppo_learns_end_to_end():
    from lbk8s import LBVecEnv
    from lbk8s.ppo import PPO_DeepSets
    env = LBVecEnv(512, seed=3, as_tensors=True, episode_length=10, reward_function="multi",
                   latency_weight=1.0, cpu_weight=0.0, gini_weight=0.0)
    logs = []
    algo = PPO_DeepSets(env, num_steps=16, n_minibatches=4, update_epochs=2, ent_coef=0.001, seed=2,
                        log_fn=logs.append)
    before = [p.detach().clone() for p in algo.agent.parameters()]
    algo.learn(total_timesteps=512 * 16 * 3)
    assert len(logs) == 3
    for s in logs:
        for k in ("loss", "pg_loss", "v_loss", "entropy", "approx_kl"):
            assert math.isfinite(s[k])
    assert algo.episode_returns and all(math.isfinite(r) for r in algo.episode_returns)
    assert any(not torch.equal(a, b) for a, b in zip(before, algo.agent.parameters()))
    a = algo.predict(env.obs, env.action_masks())
    assert a.shape == (512,) and int(a.max()) < env.action_space.n


def test_dqn_learns_end_to_end():
    from lbk8s import LBVecEnv
    from lbk8s.dqn import DQN_DeepSets
    env = LBVecEnv(64, seed=4, as_tensors=True, episode_length=10)
    algo = DQN_DeepSets(env, buffer_size=64 * 100, batch_size=64, learning_starts=50, train_frequency=5,
                        target_network_frequency=100, seed=1)
    before = [p.detach().clone() for p in algo.q_network.parameters()]
    algo.learn(total_timesteps=300)
    assert algo.train_steps == len([s for s in range(300) if s > 50 and s % 5 == 0])
    assert any(not torch.equal(a, b) for a, b in zip(before, algo.q_network.parameters()))
    # target network was hard-synced at step 100 and 200
    assert algo.rb.full or algo.rb.pos == 300 % algo.rb.size
    assert algo.episode_returns


def test_dqn_graph_train_step_matches_eager():
    """The HIP-graph train step (captured once on fixed sample buffers, replayed) trains as
    the eager one: same samples (the capture draws nothing), same updates; and after the
    hard target syncs the fused forward of the target network sees the synced weights
    (the cached weight image is rebuilt, not the initial one)."""
    from lbk8s import LBVecEnv, fused
    from lbk8s.dqn import DQN_DeepSets
    res = []
    for graph in (False, True):
        env = LBVecEnv(64, seed=4, as_tensors=True, episode_length=10)
        algo = DQN_DeepSets(env, buffer_size=64 * 100, batch_size=64, learning_starts=50, train_frequency=5,
                            target_network_frequency=100, seed=1, train_graph=graph)
        assert algo.train_graph == graph
        algo.learn(total_timesteps=300)
        assert algo.train_steps == len([s for s in range(300) if s > 50 and s % 5 == 0])
        res.append([p.detach().clone() for p in algo.q_network.parameters()])
        x = torch.rand((256, 9, 8), device="cuda")
        with torch.no_grad():
            for net in (algo.q_network, algo.target_network):
                torch.testing.assert_close(fused.q_forward(net, x), net.q_network(x), rtol=1e-4, atol=1e-4)
    for a, b in zip(*res):
        torch.testing.assert_close(b, a, rtol=1e-4, atol=2e-6)


def test_ppo_graph_update_matches_eager():
    """The HIP-graph minibatch step (captured once, replayed) computes the eager update:
    two updates, so the second rollout must see the first update's weights (the fused
    forward's weight image is invalidated after replays the version counters miss)."""
    from lbk8s import LBVecEnv
    from lbk8s.ppo import PPO_DeepSets
    res = []
    for graphs in (False, True):
        env = LBVecEnv(256, seed=5, as_tensors=True, episode_length=10)
        algo = PPO_DeepSets(env, num_steps=8, n_minibatches=4, update_epochs=2, seed=2, use_graphs=graphs)
        assert algo.use_graphs == graphs
        algo.learn(total_timesteps=256 * 8 * 2)
        res.append([p.detach().clone() for p in algo.agent.parameters()])
    for a, b in zip(*res):
        torch.testing.assert_close(b, a, rtol=1e-4, atol=2e-6)


def test_ppo_config4_end_to_end_graph_step_matches_reference():
    """Config 4 end to end: PPO_DeepSets on 512 E=64 multi-reward envs (R = 65), T = 8,
    graphs on: a rollout + update runs, then the captured minibatch step (fused forward,
    fused loss head, fused backward, clip_grad_norm, Adam) is replayed on the reference's
    own R = 65 minibatch (tests/golden/nn_ppo_update_e64.npz, ppo_deepset.py:216-267 through
    envs/deep_sets_agent_original.py) from the reference's initial weights: gradients,
    their clipped norm and the Adam step must match."""
    import numpy as np

    from lbk8s import LBVecEnv
    from lbk8s.ppo import PPO_DeepSets
    from nn_helpers import close, load_nn, state_dict_from
    from test_nn_golden import check_adam_step
    d = load_nn("nn_ppo_update_e64")
    S = d["obs"].shape[0]  # 256 sets = one minibatch of 512 envs x 8 steps / 16
    env = LBVecEnv(512, seed=9, as_tensors=True, num_endpoints=64, reward_function="multi",
                   latency_weight=1.0, cpu_weight=0.0, gini_weight=0.0)
    logs = []
    algo = PPO_DeepSets(env, num_steps=8, n_minibatches=16, update_epochs=1, ent_coef=float(d["ent_coef"]), seed=2,
                        log_fn=logs.append)
    assert algo.use_graphs and algo.minibatch_size == S and env.observation_space.shape == (65, 8)
    algo.learn(total_timesteps=512 * 8)
    assert len(logs) == 1 and all(math.isfinite(logs[0][k]) for k in ("loss", "pg_loss", "v_loss", "entropy"))
    assert algo._mb_graphs is not None
    # the reference's minibatch and initial weights into the captured step's buffers
    with torch.no_grad():
        algo.agent.load_state_dict(state_dict_from(d, "init__"))
        for st in algo.optimizer.state.values():
            for v in st.values():
                if isinstance(v, torch.Tensor):
                    v.zero_()
        names = ("obs", "actions", "logprobs", "masks", "advantages", "returns", "values")
        for buf, k in zip(algo._static, names):
            buf.copy_(torch.from_numpy(np.asarray(d[k])).to(buf.device, buf.dtype))
    from lbk8s import fused
    fused.invalidate(algo.agent)
    algo._replay()
    torch.cuda.synchronize()
    loss = algo._static_out[0]
    close(loss, d["loss"], rtol=1e-4, atol=2e-5, what="loss")
    gmax = max(np.abs(d["grad__" + n.replace(".", "__")]).max() for n, _ in algo.agent.named_parameters())
    gn = float(d["grad_norm"])
    scale = min(1.0, 0.5 / (gn + 1e-6))  # clip_grad_norm_ already scaled the replayed gradients
    for n, p in algo.agent.named_parameters():
        close(p.grad / scale, d["grad__" + n.replace(".", "__")], what="grad " + n, rtol=1e-3,
              atol=max(2e-4, 1e-5 * gmax))
    check_adam_step(algo.agent, d, gmax, "cuda")
