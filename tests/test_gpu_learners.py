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
