"""GPU tests of the drop-in surfaces and full-size properties (through the C ABI).

* single-env LoadBalancerK8sEnv + host greedy policies == C oracle (run_baselines loop);
* LBVecEnv SB3 surface: infos (13 keys, terminal_observation, VecMonitor episode),
  env_method / get_attr / step_async / as_tensors;
* T4 sharding invariance on the device (1 shard == 2 shards with env id offsets);
* 2^20-env properties: value ranges, done cadence, episode-statistics invariants,
  determinism, status word.
"""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_single_env_greedy_matches_oracle(oracle_mod, tmp_path):
    from lbk8s import LoadBalancerK8sEnv
    from lbk8s.baselines import POLICIES
    cfg = dict(num_endpoints=6, num_nodes=48, num_zones=12, reward_function="naive",
               latency_weight=1.0, cpu_weight=0.0, gini_weight=0.0, episode_length=30)
    cwd = os.getcwd()
    os.chdir(tmp_path)
    try:
        for kind, pol in POLICIES.items():
            env = LoadBalancerK8sEnv(seed=42, file_results_name=f"res_{kind}", **cfg)
            orc = oracle_mod.OracleBatch(cfg, 1, trace=False, auto_reset=False, seed=42)
            orc.init()
            for ep in range(3):
                obs = env.reset()
                np.testing.assert_array_equal(obs, orc.reset()[0])
                done, ret = False, 0.0
                while not done:
                    a = pol(env, env.action_masks())
                    assert a == int(orc.policy_greedy(kind)[0])
                    obs, r, done, info = env.step(a)
                    o2, r2, d2, _, _ = orc.step(np.array([a], np.int32))
                    np.testing.assert_array_equal(obs, o2[0])
                    assert r == r2[0] and done == d2[0]
                    ret += r
                assert ret == cfg["episode_length"]  # greedy never rejects (masks all True)
                assert info["ep_accepted_requests"] == cfg["episode_length"]
            rows = open(f"res_{kind}.csv").read().strip().splitlines()
            assert len(rows) == 3 and rows[0].startswith("1,")
            assert len(open("no_cost_updated.csv").read().strip().splitlines()) >= 3
    finally:
        os.chdir(cwd)


def test_vecenv_sb3_surface():
    from lbk8s import INFO_KEYS, LBVecEnv
    B = 16
    env = LBVecEnv(B, seed=1, monitor=True, info_keywords=("gini", "avg_cost"), episode_length=5,
                   reward_function="multi")
    assert env.num_envs == B and env.observation_space.shape == (9, 8) and env.action_space.n == 9
    masks = np.array(env.env_method("action_masks"))
    assert masks.shape == (B, 9) and masks.all()
    with pytest.raises(TypeError):
        env.step(np.zeros(B, np.int32))  # before reset: reference raises TypeError
    obs = env.reset()
    assert obs.shape == (B, 9, 8) and obs.dtype == np.float32
    for s in range(5):
        env.step_async(np.full(B, s % 9, np.int32))
        obs, rew, done, infos = env.step_wait()
        assert len(infos) == B
        info = infos[3]
        for k in INFO_KEYS:
            assert k in info
        if s < 4:
            assert not done.any() and "episode" not in info
    assert done.all()
    for i, info in enumerate(infos):
        assert info["terminal_observation"].shape == (9, 8)
        ep = info["episode"]
        assert ep["l"] == 5 and "gini" in ep and "avg_cost" in ep
        assert abs(ep["r"] - float(np.float32(ep["r"]))) < 1e-3
    # the post-reset obs differs from the terminal one (new scenario)
    assert not np.array_equal(obs[0], infos[0]["terminal_observation"])
    topo = env.get_attr("endpoint_topology_latency")
    assert len(topo) == B and topo[0].shape == (8,)
    assert env.get_attr("num_endpoints", indices=[0, 1]) == [8, 8]
    tenv = LBVecEnv(B, seed=1, as_tensors=True)
    o = tenv.reset()
    assert isinstance(o, torch.Tensor) and o.is_cuda
    o, r, d, _ = tenv.step(torch.zeros(B, dtype=torch.int64, device="cuda"))
    assert r.is_cuda and d.dtype == torch.bool


@pytest.mark.parametrize("sizes", [(2048, 2048), (65536, 100)])
def test_sharding_invariance_device(sizes):
    """Shards see their global env ids' trajectories.  (65536, 100): the whole batch runs
    the 256-thread-block step kernel with a ragged tail, the shards the 64-thread one."""
    from lbk8s import LBVecEnv
    B = sum(sizes)
    offs = [sum(sizes[:i]) for i in range(len(sizes))]
    cfg = dict(num_endpoints=8, reward_function="fairness")
    full = LBVecEnv(B, seed=11, as_tensors=True, **cfg)
    parts = [LBVecEnv(n, seed=11, env_id_offset=o, as_tensors=True, **cfg) for n, o in zip(sizes, offs)]
    a0 = full.reset().clone()
    torch.testing.assert_close(a0, torch.cat([p.reset().clone() for p in parts]), rtol=0, atol=0)
    gen = torch.Generator(device="cuda")
    gen.manual_seed(0)
    for s in range(150):
        a = torch.randint(0, 9, (B,), dtype=torch.int32, device="cuda", generator=gen)
        o1, r1, d1, _ = full.step(a)
        outs = [p.step(a[o:o + n]) for n, o, p in zip(sizes, offs, parts)]
        assert torch.equal(o1, torch.cat([x[0] for x in outs]))
        assert torch.equal(r1, torch.cat([x[1] for x in outs]))
        assert torch.equal(d1, torch.cat([x[2] for x in outs]))


def test_full_size_properties():
    from lbk8s import LBVecEnv
    from lbk8s.info import ST_ACC, ST_GINI, ST_INTER, ST_INTRA, ST_LENGTH, ST_RETURN
    B = 1 << 20
    env = LBVecEnv(B, seed=2024, as_tensors=True)
    obs = env.reset()
    gen = torch.Generator(device="cuda")
    gen.manual_seed(1)
    thresholds = torch.tensor([150., 200., 250., 375., 400., 450., 500.], device="cuda")
    for s in range(1, 201):
        a = torch.randint(0, 9, (B,), dtype=torch.int32, device="cuda", generator=gen)
        obs, rew, done, _ = env.step(a)
        if s % 50 == 0 or s % 100 == 0:
            ep = obs[:, :8]
            assert ep[..., 0].min() >= 0 and ep[..., 0].max() <= 3
            assert ep[..., 1].min() >= 2 and ep[..., 1].max() <= 8 * 24
            assert ep[..., 2].min() >= 1 and ep[..., 2].max() <= 100
            assert ep[..., 3].min() >= 1 and ep[..., 3].max() <= 499
            assert ep[..., 4].min() >= 1 and ep[..., 4].max() <= 500
            assert torch.isin(obs[:, 0, 6], thresholds).all()
            assert (obs[:, :, 7] > 0).all() and (obs[:, 8, :5] == -1).all()
            assert ((rew == 1) | (rew == -1)).all()
        assert bool(done.all()) == (s % 100 == 0) and bool(done.any()) == (s % 100 == 0)
        if s % 100 == 0:
            st = env.ep_stats
            assert (st[:, ST_LENGTH] == 100).all()
            assert (st[:, ST_INTRA] + st[:, ST_INTER] == st[:, ST_ACC]).all()
            assert torch.allclose(st[:, ST_RETURN], 2 * st[:, ST_ACC] - 100)  # naive: +1 / -1
            assert (st[:, ST_GINI] >= 0).all() and (st[:, ST_GINI] < 1).all()
            frac = (st[:, ST_ACC] / 100).mean().item()
            assert abs(frac - 8 / 9) < 0.002  # uniform random actions accept 8 of 9
    assert env.status() == 0
    # determinism: an identically seeded env reproduces the stream
    env2 = LBVecEnv(B, seed=2024, as_tensors=True)
    env2.reset()
    gen.manual_seed(1)
    for s in range(1, 201):
        a = torch.randint(0, 9, (B,), dtype=torch.int32, device="cuda", generator=gen)
        o2, _, _, _ = env2.step(a)
    assert torch.equal(o2, obs)


@pytest.mark.parametrize("B,kw", [(4096, {}), (1 << 18, {}), (3000, dict(num_endpoints=64, reward_function="multi")),
                                  (40000, dict(num_endpoints=20))])
def test_fused_random_policy_step(B, kw):
    """lb_step with actions == NULL (the env's Philox random policy drawn inside the step
    kernel) == lb_policy(random) then lb_step, bit for bit, across auto-resets; covers the
    thread-per-env kernel (stored and recomputed scenario) and both slice shapes."""
    from lbk8s import LBVecEnv
    envs = [LBVecEnv(B, seed=11, as_tensors=True, episode_length=7, **kw) for _ in range(2)]
    for e in envs:
        e.reset()
    act = torch.empty(B, dtype=torch.int32, device="cuda")
    for _ in range(16):
        envs[0].policy("random", out=act)
        envs[0].step_device(act)
        envs[1].step_device(None)
        for f in ("obs", "rewards", "dones"):
            assert torch.equal(getattr(envs[0], f), getattr(envs[1], f)), f
    assert torch.equal(envs[0].stats(), envs[1].stats())
    assert envs[1].status() == 0


@pytest.mark.parametrize("B", [2048, 1 << 18])
def test_seed_applies_at_next_reset(oracle_mod, B):
    """seed() mid-episode changes nothing until the next reset(); from there every env runs
    on the new key (the oracle re-keyed at the same point).  B = 2^18 takes the step that
    redraws the episode's scenario from the key."""
    from lbk8s import LBVecEnv
    L = 8
    env = LBVecEnv(B, seed=5, as_tensors=True, episode_length=L)
    orc = oracle_mod.OracleBatch(dict(episode_length=L), B, trace=False, seed=5)
    orc.init()
    assert torch.equal(env.reset().cpu(), torch.from_numpy(orc.reset()))

    def steps(n):
        for _ in range(n):
            a = orc.policy_random()
            o1, r1, d1, _ = env.step(torch.from_numpy(a).cuda())
            o2, r2, d2, _, _ = orc.step(a)
            np.testing.assert_array_equal(o1.cpu().numpy(), o2)
            np.testing.assert_array_equal(r1.cpu().numpy(), r2)
            np.testing.assert_array_equal(d1.cpu().numpy(), d2)

    steps(3)
    env.seed(987654321)          # mid-episode: pending
    steps(L + 2)                 # an auto-reset in between still uses the old key
    orc.set_seed(987654321)
    np.testing.assert_array_equal(env.reset().cpu().numpy(), orc.reset())
    steps(L + 2)
    assert env.status() == 0


def test_masked_reset_matches_oracle(oracle_mod):
    """reset_masked (the bench's episode staggering) == the oracle's masked reset."""
    from lbk8s import LBVecEnv
    B, L = 4096, 10
    env = LBVecEnv(B, seed=3, as_tensors=True, episode_length=L)
    orc = oracle_mod.OracleBatch(dict(episode_length=L), B, trace=False, seed=3)
    orc.init()
    env.reset()
    orc.reset()
    gid = np.arange(B)
    for r in range(1, L):
        a = orc.policy_random()
        env.step(torch.from_numpy(a).cuda())
        orc.step(a)
        mask = (gid % L) == r
        env.reset_masked(torch.from_numpy(mask).cuda())
        o2 = orc.reset(mask=mask)
        np.testing.assert_array_equal(env.obs.cpu().numpy()[mask], o2[mask])
    steps = env.field("current_step").cpu().numpy()
    np.testing.assert_array_equal(steps, (L - 1 - gid % L) % L)
    for k in range(3):  # every step ends the episodes of one residue class
        a = orc.policy_random()
        o1, r1, d1, _ = env.step(torch.from_numpy(a).cuda())
        o2, r2, d2, _, _ = orc.step(a)
        np.testing.assert_array_equal(o1.cpu().numpy(), o2)
        np.testing.assert_array_equal(d1.cpu().numpy(), (gid % L) == k)


def test_vecmonitor_file_during_training(tmp_path):
    """LBVecEnv(monitor_file=...) writes VecMonitor's CSV (run.py:122) from the drop-in
    step and from a device learner's step_device loop."""
    import csv as _csv
    import json as _json

    from lbk8s import INFO_KEYS, LBVecEnv
    from lbk8s.ppo import PPO_DeepSets
    f = str(tmp_path / "vec_loadbalancer_k8s_gym_results")
    env = LBVecEnv(32, seed=1, monitor_file=f, info_keywords=INFO_KEYS, episode_length=5, reward_function="multi")
    env.reset()
    for s in range(10):
        env.step(np.full(32, s % 9, np.int32))
    env.close()
    lines = open(f + ".monitor.csv").read().splitlines()
    assert lines[0].startswith("#") and "t_start" in _json.loads(lines[0][1:])
    rows = list(_csv.DictReader(lines[1:]))
    assert len(rows) == 64 and list(rows[0])[:3] == ["r", "l", "t"]
    assert all(int(r["l"]) == 5 for r in rows)
    assert set(INFO_KEYS) <= set(rows[0])
    g = str(tmp_path / "ppo_run")
    env = LBVecEnv(64, seed=2, as_tensors=True, monitor_file=g, info_keywords=INFO_KEYS, episode_length=10,
                   reward_function="multi", latency_weight=1.0, cpu_weight=0.0, gini_weight=0.0)
    algo = PPO_DeepSets(env, num_steps=20, n_minibatches=2, update_epochs=1, seed=2)
    algo.learn(total_timesteps=64 * 20 * 2)
    env.close()
    rows = list(_csv.DictReader(open(g + ".monitor.csv").read().splitlines()[1:]))
    assert len(rows) == 64 * 4  # 2 updates x 20 steps / episode length 10
    rets = np.array([float(r["r"]) for r in rows])
    assert abs(rets.mean() - np.mean(algo.episode_returns)) < 1e-3 * max(1.0, abs(rets.mean()))


@pytest.mark.parametrize("B,kw,geometry", [
    (4096, {}, "auto"),                                                        # config 2 shape
    (2000, dict(num_endpoints=6, num_nodes=48, num_zones=12, reward_function="multi"), "auto"),
    (3000, dict(num_endpoints=64, reward_function="multi"), "auto"),
    (40000, dict(num_endpoints=20, reward_function="fairness"), "auto"),       # 4-envs-per-wave slice
    (40000, {}, "slice"),
    (40000, dict(num_endpoints=6), "tpe"),                                     # k_rollout_tpe (L < K), 64-thread blocks
    (70000, {}, "tpe"),                                                        # k_rollout_tpe (L < K), 256-thread blocks
    (40000, dict(num_nodes=100), "tpe"),                                       # N > 64: K policy + step launches
    (70000, dict(auto_reset=False), "tpe"),      # k_rollout_tpe without auto-reset, envs stepped past L
])
@pytest.mark.parametrize("kind", ["random", "topo", "zone_cpu", "endpoint_cpu"])
def test_rollout_equals_policy_plus_step(B, kw, geometry, kind):
    """lb_rollout (K steps in one launch, the policy evaluated on the state in registers)
    == K x (lb_policy + lb_step), bit for bit, across auto-resets."""
    from lbk8s import LBVecEnv
    K, L = 13, 5
    a_env = LBVecEnv(B, seed=21, as_tensors=True, episode_length=L, geometry=geometry, **kw)
    b_env = LBVecEnv(B, seed=21, as_tensors=True, episode_length=L, geometry=geometry, **kw)
    a_env.reset()
    b_env.reset()
    R = a_env.cfg.obs_rows
    obs = torch.empty((K, B, R, 8), device="cuda")
    rew = torch.empty((K, B), device="cuda")
    dn = torch.empty((K, B), dtype=torch.uint8, device="cuda")
    act = torch.empty((K, B), dtype=torch.int32, device="cuda")
    a_env.rollout(kind, K, obs_out=obs, reward_out=rew, done_out=dn, actions_out=act)
    for k in range(K):
        ak = b_env.policy(kind)
        assert torch.equal(act[k], ak), k
        b_env.step_device(ak)
        assert torch.equal(obs[k], b_env.obs), k
        assert torch.equal(rew[k], b_env.rewards), k
        assert torch.equal(dn[k], b_env.dones), k
    assert torch.equal(a_env.stats(), b_env.stats())
    assert torch.equal(a_env.terminal_obs, b_env.terminal_obs)
    for f in ("endpoint_latency", "endpoint_cpu_usage_percentage", "avg_load_served"):
        assert torch.equal(a_env.field(f), b_env.field(f)), f
    # the env goes on from where the rollout left it
    a_env.step_device(act[0])
    b_env.step_device(act[0])
    assert torch.equal(a_env.obs, b_env.obs)
    assert a_env.status() == 0


@pytest.mark.parametrize("B,kw", [(40000, dict(num_endpoints=6, reward_function="multi")), (70000, {}),
                                  (131072, dict(reward_function="latency"))])
@pytest.mark.parametrize("kind", ["random", "endpoint_cpu"])
@pytest.mark.parametrize("K,L", [(23, 9), (16, 20), (20, 20)])
def test_rollout_tpe_staggered_equals_policy_plus_step(B, kw, kind, K, L):
    """lb_rollout with staggered episodes (1/L of the envs finish at every step, the
    bench's steady state): == K x (lb_policy + lb_step), bit for bit, including the terminal
    obs and the episode-stats rows.  L < K: k_rollout_tpe (envs can finish twice in a launch:
    in-loop block-list resets); L >= K: next episodes drawn into records before the first step
    (L == K: every env ends exactly once per launch) by k_rollout_img, or k_rollout_lean at
    131,072 default envs -- the kernel lb_rollout_kernel names, asserted below."""
    from lbk8s import LBVecEnv
    envs = [LBVecEnv(B, seed=5, as_tensors=True, episode_length=L, geometry="tpe", **kw) for _ in range(2)]
    gid = torch.arange(B, device="cuda")
    for e in envs:
        e.reset()
        for r in range(1, L):
            e.step_device(None)
            e.reset_masked((gid % L) == r)
    a_env, b_env = envs
    lean = B % 64 == 0 and B > 65536 and kw.get("num_endpoints", 8) in (6, 8)
    assert a_env.rollout_kernel(K) == ("k_rollout_tpe" if L < K else ("k_rollout_lean_split" if K <= 32 else "k_rollout_lean") if lean
                                          else "k_rollout_img")
    R = a_env.cfg.obs_rows
    obs = torch.empty((K, B, R, 8), device="cuda")
    rew = torch.empty((K, B), device="cuda")
    dn = torch.empty((K, B), dtype=torch.uint8, device="cuda")
    act = torch.empty((K, B), dtype=torch.int32, device="cuda")
    a_env.rollout(kind, K, obs_out=obs, reward_out=rew, done_out=dn, actions_out=act)
    for k in range(K):
        ak = b_env.policy(kind)
        assert torch.equal(act[k], ak), k
        b_env.step_device(ak)
        assert torch.equal(obs[k], b_env.obs), k
        assert torch.equal(rew[k], b_env.rewards), k
        assert torch.equal(dn[k], b_env.dones), k
        assert 0 < int(dn[k].sum()) < B
    assert torch.equal(a_env.stats(), b_env.stats())
    assert torch.equal(a_env.terminal_obs, b_env.terminal_obs)
    assert torch.equal(a_env.ep_stats, b_env.ep_stats)
    for f in ("endpoint_latency", "endpoint_cpu_usage_percentage", "avg_load_served", "current_time"):
        assert torch.equal(a_env.field(f), b_env.field(f)), f
    a_env.step_device(None)
    b_env.step_device(None)
    assert torch.equal(a_env.obs, b_env.obs)
    assert a_env.status() == 0


def test_run_baselines_greedy_matches_oracle(oracle_mod, tmp_path):
    """Config 1 driver (run_baselines.py): one launch per 100-step episode batch; every
    episode's return and final accumulators equal the oracle's greedy episodes, and so do the
    per-episode CSV rows the reference's env appends (loadbalancer_k8s_env.py:488-510), as
    written to <i>_<policy>_baselines_num_endpoints_<e>.csv and no_cost_updated.csv."""
    import csv

    from lbk8s.info import CSV_FIELDS, ST_RETURN, csv_rows
    from lbk8s.run_baselines import CFG1, baseline_file_name, run_baselines, write_csvs
    n = 512
    for kind in ("topo", "zone_cpu", "endpoint_cpu"):
        res = run_baselines(kind, n, seed=42)
        orc = oracle_mod.OracleBatch(CFG1, n, trace=False, auto_reset=False, seed=42)
        orc.init()
        orc.reset()
        for s in range(CFG1["episode_length"]):
            _, r, _, _, _ = orc.step(orc.policy_greedy(kind))
            np.testing.assert_array_equal(res["rewards"][s], r)
        st = orc.stats()
        np.testing.assert_array_equal(res["returns"], st[:, ST_RETURN])
        assert (res["returns"] == 100).all()  # greedy never rejects (masks all True), naive +1
        name = baseline_file_name(0, kind, 6)
        write_csvs(res, name, str(tmp_path))
        for fname, col in ((name + ".csv", 0), ("no_cost_updated.csv", 1)):
            with open(tmp_path / fname) as f:
                rows = list(csv.DictReader(f, fieldnames=list(CSV_FIELDS)))
            rows = rows[-n:]  # no_cost_updated.csv is shared by the three policies (append)
            assert len(rows) == n
            for i in (0, 1, n // 2, n - 1):
                exp = csv_rows(st[i], i + 1)[col]
                got = rows[i]
                for k in CSV_FIELDS[:-1]:  # (execution_time is wall clock)
                    assert float(got[k]) == float(exp[k]), (fname, i, k)


@pytest.mark.parametrize("B,E", [(512, 8), (300, 64)])  # thread-per-env and slice step kernels
def test_vecmonitor_return_rounds_once(oracle_mod, B, E):
    """SB3 VecMonitor (run.py:114-122) keeps float32 episode_returns and adds the float64
    rewards SubprocVecEnv hands it (the env's Python floats), so numpy rounds each sum once:
    ret32 = float32(float64(ret32) + r64).  The monitor's `r` (infos[i]["episode"]["r"]) is
    checked against that restatement driven by the C oracle's float64 rewards, on a
    multi-reward scenario where rounding twice (float32(ret32 + float32(r64))) differs."""
    from lbk8s import LBVecEnv
    L = 25
    cfg = dict(num_endpoints=E, episode_length=L, reward_function="multi")
    env = LBVecEnv(B, seed=31, monitor=True, **cfg)
    orc = oracle_mod.OracleBatch(cfg, B, trace=False, seed=31)
    orc.init()
    np.testing.assert_array_equal(env.reset(), orc.reset())
    ret = np.zeros(B, np.float32)   # VecMonitor.episode_returns
    ret2 = np.zeros(B, np.float32)  # the same sums rounded twice
    rng = np.random.default_rng(5)
    episodes = differ = 0
    for s in range(3 * L):
        a = rng.integers(0, E + 1, size=B).astype(np.int32)
        _, r, d, infos = env.step(a)
        _, r2, d2, _, _ = orc.step(a)
        r64 = orc.last_reward64()
        np.testing.assert_array_equal(r, r2)
        np.testing.assert_array_equal(r, r64.astype(np.float32))
        ret += r64  # numpy: float32 array += float64 array -> computed in float64, cast once
        ret2 += r64.astype(np.float32)
        for i in np.flatnonzero(d):
            assert infos[i]["episode"]["r"] == float(ret[i]), (s, i)
            episodes += 1
            differ += int(ret[i] != ret2[i])
        ret[d] = 0
        ret2[d] = 0
    assert episodes == 3 * B
    assert differ > 0  # the scenario does tell one rounding from two
