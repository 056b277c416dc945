"""Rank body of tests/test_gpu_dist.py (launched by torch.distributed.run, 2 ranks).

Both ranks may share one GPU (LBK8S_DIST_BACKEND=gloo).  For use_graphs in (False, True):
a fresh LBVecEnv shard (global env ids rank*B ...) and PPO_DeepSets, two updates (argv[2]
== "dqn": DQN_DeepSets, 150 vector steps with a train step every 5 and its HIP-graph train
step); the parameters of every rank must agree (averaged gradients, replicated weights) and
the graph path must equal the eager one.  Rank 0 writes a JSON verdict to argv[1].
"""
import json
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gym-loadbalancing_amd"))

from lbk8s import LBVecEnv  # noqa: E402
from lbk8s.dist import init_from_env  # noqa: E402
from lbk8s.dqn import DQN_DeepSets  # noqa: E402
from lbk8s.ppo import PPO_DeepSets  # noqa: E402


def main(out, algo_name="ppo"):
    rank, world, dev = init_from_env("cuda")
    B, T = 128, 8
    res = {}
    for graphs in (False, True):
        env = LBVecEnv(B, device=dev, seed=5, env_id_offset=rank * B, as_tensors=True, episode_length=6,
                       reward_function="multi", latency_weight=1.0, cpu_weight=0.0, gini_weight=0.0)
        if algo_name == "dqn":
            algo = DQN_DeepSets(env, buffer_size=B * 50, batch_size=64, learning_starts=20, train_frequency=5,
                                target_network_frequency=50, seed=2 + rank, train_graph=graphs)
            assert algo._multi and algo.train_graph == graphs
            algo.learn(total_timesteps=150)
            net = algo.q_network
        else:
            algo = PPO_DeepSets(env, num_steps=T, n_minibatches=4, update_epochs=2, seed=2 + rank,
                                use_graphs=graphs)
            assert algo._multi and algo.use_graphs == graphs
            algo.learn(total_timesteps=B * T * 2)
            net = algo.agent
        flat = torch.cat([p.detach().reshape(-1) for p in net.parameters()])
        allp = [torch.zeros_like(flat) for _ in range(world)]
        dist.all_gather(allp, flat)
        res[graphs] = (allp, algo.episode_returns)
    ok = {}
    for graphs, (allp, _) in res.items():
        ok[f"ranks_agree_graphs{int(graphs)}"] = all(torch.equal(allp[0], p) for p in allp[1:])
    e, g = res[False][0][0], res[True][0][0]
    ok["graph_vs_eager_maxdiff"] = float((e - g).abs().max())
    ok["graph_eq_eager"] = bool(torch.allclose(e, g, rtol=1e-4, atol=2e-6))
    ok["returns_eq"] = res[False][1] == res[True][1] or all(
        abs(a - b) < 1e-3 for a, b in zip(res[False][1], res[True][1]))
    ok["world"] = world
    if rank == 0:
        with open(out, "w") as f:
            json.dump(ok, f)
    dist.destroy_process_group()


if __name__ == "__main__":
    main(*sys.argv[1:])
