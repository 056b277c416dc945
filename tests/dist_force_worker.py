"""Body of tests/test_gpu_dist.py::test_rccl_one_rank_multi_path_equals_single_rank (one
process, plain python): a one-rank process group on the backend LBK8S_DIST_BACKEND (nccl =
RCCL), then for PPO (graphs) and DQN (train graph): the learner built with the multi-rank
path forced (LBK8S_FORCE_MULTI=1: parameter broadcast, gradient all_reduce between the
split graphs, episode-return all_reduce) and the learner built on the single-rank path, from
the same seeds; writes the parameter difference, returns and collective timing to argv[1]."""
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gym-loadbalancing_amd"))

from lbk8s import LBVecEnv  # noqa: E402
from lbk8s import dist as lbdist  # noqa: E402
from lbk8s.dqn import DQN_DeepSets  # noqa: E402
from lbk8s.ppo import PPO_DeepSets  # noqa: E402


def train(algo_name, forced):
    os.environ["LBK8S_FORCE_MULTI"] = "1" if forced else "0"
    B, T = 128, 8
    env = LBVecEnv(B, seed=5, as_tensors=True, episode_length=6, reward_function="multi", latency_weight=1.0,
                   cpu_weight=0.0, gini_weight=0.0)
    if algo_name == "dqn":
        algo = DQN_DeepSets(env, buffer_size=B * 50, batch_size=64, learning_starts=20, train_frequency=5,
                            target_network_frequency=50, seed=2, train_graph=True)
        assert algo._multi == forced and algo.train_graph
        algo.learn(total_timesteps=150)
        net = algo.q_network
    else:
        algo = PPO_DeepSets(env, num_steps=T, n_minibatches=4, update_epochs=2, seed=2, use_graphs=True)
        assert algo._multi == forced and algo.use_graphs
        algo.learn(total_timesteps=B * T * 2)
        net = algo.agent
    torch.cuda.synchronize()
    return torch.cat([p.detach().reshape(-1) for p in net.parameters()]), list(algo.episode_returns)


def main(out):
    os.environ["LBK8S_FORCE_MULTI"] = "1"
    rank, world, dev = lbdist.init_from_env("cuda")
    assert dist.is_initialized() and world == 1 and dist.get_world_size() == 1
    res = {"backend": dist.get_backend(), "world": dist.get_world_size()}
    for algo_name in ("ppo", "dqn"):
        pm, rm = train(algo_name, True)
        ps, rs = train(algo_name, False)
        res[algo_name] = {"params": int(pm.numel()), "maxdiff": float((pm - ps).abs().max()),
                          "equal": bool(torch.equal(pm, ps)), "returns_multi": rm, "returns_single": rs}
    # the gradient all_reduce itself: 31k floats (the PPO actor + critic), one rank
    g = torch.randn(31000, device=dev)
    for _ in range(5):
        dist.all_reduce(g)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(100):
        dist.all_reduce(g)
    torch.cuda.synchronize()
    res["all_reduce_31k_f32_us"] = (time.perf_counter() - t0) / 100 * 1e6
    with open(out, "w") as f:
        json.dump(res, f)
    dist.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1])
