"""CPU tests of the host-side logic and of the oracle's RNG (no GPU).

* greedy policies (lbk8s.baselines) against hand-computed expectations incl. the
  mask[:-1] quirk and ties (envs/baselines.py:6-35);
* env sharding arithmetic and the gloo world_size-2 episode-statistics reduction;
* Philox4x32-R round function pinned by the Random123 philox4x32_10 known answers (R = 10);
  the draw map runs R = 7; the fdlibm-style log;
* T3 (statistical) checks of the Philox draw map through the oracle;
* sharding invariance of Philox trajectories (global env ids) through the oracle.
"""
import math
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


class FakeEnv:
    def __init__(self, topo, cap, cpu):
        self.endpoint_topology_latency = np.asarray(topo, float)
        self.endpoint_zone_cpu_capacity = np.asarray(cap, float)
        self.endpoint_cpu_usage_percentage = np.asarray(cpu, float)


def test_greedy_policies_semantics():
    from lbk8s import baselines as b
    env = FakeEnv([5, 1, 1, 7], [4, 9, 9, 2], [50.5, 50.5, 10.0, 3.0])
    mask_rej = np.ones(5, bool)  # rejection: last entry is the reject action
    assert b.topology_greedy_policy(env, mask_rej) == 1       # first of the tied minima
    assert b.zone_cpu_greedy_policy(env, mask_rej) == 1       # first of the tied maxima
    assert b.endpoint_cpu_greedy_policy(env, mask_rej) == 3
    mask_norej = np.ones(4, bool)  # no rejection: mask[:-1] drops endpoint 3 (reference quirk)
    assert b.endpoint_cpu_greedy_policy(env, mask_norej) == 2
    assert b.topology_greedy_policy(env, np.array([True])) == 0  # nothing feasible -> last index
    partial = np.array([True, False, False, True, True])
    assert b.topology_greedy_policy(env, partial) == 0


def test_shard_partitions_env_ids():
    from lbk8s.dist import shard
    for total in (1, 7, 1 << 20, 1000003):
        for world in (1, 2, 3, 8):
            parts = [shard(total, r, world) for r in range(world)]
            assert parts[0][0] == 0
            for (o1, n1), (o2, _) in zip(parts, parts[1:]):
                assert o1 + n1 == o2
            assert sum(n for _, n in parts) == total
            assert max(n for _, n in parts) - min(n for _, n in parts) <= 1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _gloo_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from lbk8s.dist import reduce_episode_stats
    st = torch.zeros((4, 16), dtype=torch.float64)
    st[:, 0] = torch.arange(4) + 10 * rank   # returns
    st[:, 1] = 100
    st[:, 2] = 50 + rank
    dones = torch.tensor([1, 0, 1, rank], dtype=torch.uint8)
    v = reduce_episode_stats(st, dones)
    q.put((rank, v.tolist()))
    dist.destroy_process_group()


def test_gloo_world2_episode_stats_reduce():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gloo_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    # rank0 done rows 0,2 -> returns 0+2; rank1 rows 0,2,3 -> 10+12+13
    expect = [5.0, 37.0, 500.0, 2 * 50 + 3 * 51]
    assert out[0] == expect and out[1] == expect


def test_philox_known_answers(oracle_mod):
    # Random123 kat_vectors, philox4x32_10
    kat = [
        ((0, 0, 0, 0), (0, 0), (0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8)),
        ((0xffffffff,) * 4, (0xffffffff, 0xffffffff), (0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd)),
        ((0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344), (0xa4093822, 0x299f31d0),
         (0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1)),
    ]
    for ctr, key, out in kat:
        assert tuple(int(x) for x in oracle_mod.philox(ctr, key, rounds=10)) == out
    # the draw map IS Philox4x32-10 (the production round count): the known answers pin the
    # map the kernels use (device == oracle bit for bit in the Philox-mode parity tests)
    assert oracle_mod.philox_rounds() == 10
    for ctr, key, out in kat:
        assert tuple(int(x) for x in oracle_mod.philox(ctr, key)) == out


def test_fd_log_accuracy(oracle_mod):
    rng = np.random.default_rng(0)
    xs = np.concatenate([rng.random(20000), 1 - rng.random(2000) * 1e-9, [1.0, 0.5, 2.0 ** -53]])
    xs = xs[xs > 0]
    worst = 0.0
    for x in xs:
        got, ref = oracle_mod.fd_log(float(x)), math.log(float(x))
        if ref != 0:
            worst = max(worst, abs(got - ref) / math.ulp(ref))
    assert oracle_mod.fd_log(1.0) == 0.0
    assert worst <= 1.0


def test_philox_draw_map_statistics(oracle_mod):
    """T3: dt ~ Exp(call_duration), thresholds uniform over the 7 endpoints, request zones
    and random actions uniform, initial latency U(1,100) (Philox mode, 2^16 envs)."""
    B = 1 << 16
    o = oracle_mod.OracleBatch({}, B, trace=False, seed=99)
    o.init()
    o.reset()
    dts, thr, rz, acts = [], [], [], []
    for _ in range(4):
        a = o.policy_random()
        acts.append(a)
        o.step(a)
        dts.append(o.field("dt"))
        thr.append(o.field("req_thr"))
        rz.append(o.field("req_zone"))
    dt = np.concatenate(dts)
    assert abs(dt.mean() - 1.0) < 0.01 and abs(dt.var() - 1.0) < 0.03  # Exp(1): mean 1, var 1
    vals, cnt = np.unique(np.concatenate(thr), return_counts=True)
    assert set(vals) == {150, 200, 250, 375, 400, 450, 500}
    exp = len(np.concatenate(thr)) / 7
    assert ((cnt - exp) ** 2 / exp).sum() < 30  # chi2, 6 dof
    av, ac = np.unique(np.concatenate(acts), return_counts=True)
    assert list(av) == list(range(9))
    exp = len(np.concatenate(acts)) / 9
    assert ((ac - exp) ** 2 / exp).sum() < 35  # chi2, 8 dof
    assert set(np.unique(np.concatenate(rz))) <= {0, 1, 2, 3}
    o2 = oracle_mod.OracleBatch({}, B, trace=False, seed=5)
    o2.init()
    o2.reset()
    lat = o2.field("ep_lat")
    assert lat.min() >= 1.0 and lat.max() < 100.0 and abs(lat.mean() - 50.5) < 0.2


def test_sharding_invariance_oracle(oracle_mod):
    """Trajectories key on the global env id: 1 shard of B == 2 shards of B/2."""
    B = 512
    cfg = dict(num_endpoints=6, reward_function="multi")
    full = oracle_mod.OracleBatch(cfg, B, seed=3)
    parts = [oracle_mod.OracleBatch(cfg, B // 2, seed=3, env_id_offset=o) for o in (0, B // 2)]
    for o in [full] + parts:
        o.init()
    obs = full.reset()
    np.testing.assert_array_equal(obs, np.concatenate([p.reset() for p in parts]))
    for _ in range(230):
        a = full.policy_random()
        np.testing.assert_array_equal(a, np.concatenate([p.policy_random() for p in parts]))
        o1, r1, d1, _, _ = full.step(a)
        outs = [p.step(a[i * (B // 2):(i + 1) * (B // 2)]) for i, p in enumerate(parts)]
        np.testing.assert_array_equal(o1, np.concatenate([x[0] for x in outs]))
        np.testing.assert_array_equal(r1, np.concatenate([x[1] for x in outs]))


def _allreduce_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from lbk8s.deepsets import DQNDeepSetAgent, allreduce_gradients
    torch.manual_seed(0)
    net = DQNDeepSetAgent(8)
    x = torch.full((3, 9, 8), float(rank + 1))
    net(x).sum().backward()
    allreduce_gradients(net)
    q.put((rank, torch.cat([p.grad.reshape(-1) for p in net.parameters()]).numpy()))
    dist.destroy_process_group()


def test_gloo_world2_gradient_allreduce():
    """The learners' one-bucket gradient average over 2 ranks equals the mean of the
    per-rank gradients (identical replicas afterwards)."""
    from lbk8s.deepsets import DQNDeepSetAgent
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_allreduce_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    expect = []
    for r in range(2):
        torch.manual_seed(0)
        net = DQNDeepSetAgent(8)
        net(torch.full((3, 9, 8), float(r + 1))).sum().backward()
        expect.append(torch.cat([p.grad.reshape(-1) for p in net.parameters()]).numpy())
    mean = (expect[0] + expect[1]) / 2
    np.testing.assert_allclose(out[0], mean, rtol=1e-6, atol=1e-7)
    np.testing.assert_array_equal(out[0], out[1])


def test_bench_launcher_creates_ranks():
    """bench.py --gpus 2 (no torchrun environment) launches 2 ranks itself; --plan-only runs
    the sharding + episode-statistics reduction path on gloo without a GPU."""
    import json
    import subprocess
    import sys
    from conftest import REPO
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    out = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--plan-only",
                          "--envs", "1000001"], capture_output=True, text=True, env=env, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    line = json.loads([ln for ln in out.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["world"] == 2
    shards = sorted(tuple(x) for x in line["shards"])
    assert [r for r, _, _ in shards] == [0, 1]
    assert shards[0][1:] == (0, 500001) and shards[1][1:] == (500001, 500000)
    n = 1000001
    # every env "finished" with return = its global id: the reduction sees all of them
    assert line["reduced"] == [float(n), float(n * (n - 1) // 2), 100.0 * n, 0.0]
    # a world size that disagrees with --gpus is an error, never a silent 1-GPU run
    env2 = dict(env, WORLD_SIZE="1")
    bad = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "3", "--plan-only"],
                         capture_output=True, text=True, env=dict(env2, WORLD_SIZE="2"), timeout=120)
    assert bad.returncode != 0 and "WORLD_SIZE" in (bad.stdout + bad.stderr)


def _mean_return_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from lbk8s.dist import mean_episode_return
    s = torch.tensor([10.0 * (rank + 1)], dtype=torch.float64)
    n = torch.tensor([float(rank + 1)], dtype=torch.float64)
    q.put((rank, mean_episode_return(s, n)))
    dist.destroy_process_group()


def test_gloo_world2_mean_episode_return():
    """The learners' logged return is the mean over every rank's finished episodes."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_mean_return_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert res[0] == res[1] == ((10.0 + 20.0) / 3.0, 3.0)
