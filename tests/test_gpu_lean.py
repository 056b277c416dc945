"""k_rollout_lean (lbk8s_lean.h): the headline rollout kernel, bench.py's launch at 2^20 envs.

Every test here first asserts that lb_rollout picks k_rollout_lean for the case (host-side
lb_rollout_kernel), then checks one launch of K vector steps against K single steps of the
already-verified step kernel (lb_policy + lb_step, themselves == the C oracle in
test_gpu_parity.py), bit for bit: obs, reward, done, actions, terminal obs, episode-stats
rows, the accumulators and the env fields afterwards, and the env going on from there.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

CFG1 = dict(num_endpoints=6, num_nodes=48, num_zones=12)


def _staggered_pair(B, L, kw, stagger=True, seed=5):
    from lbk8s import LBVecEnv
    envs = [LBVecEnv(B, seed=seed, as_tensors=True, episode_length=L, **kw) for _ in range(2)]
    gid = torch.arange(B, device="cuda")
    for e in envs:
        e.reset()
        if stagger:  # bench.py's stagger: envs with id % L == r restart after step r
            for r in range(1, L):
                e.step_device(None)
                e.reset_masked((gid % L) == r)
    return envs


def _compare_after(a_env, b_env, B):
    assert torch.equal(a_env.stats(), b_env.stats())
    assert torch.equal(a_env.terminal_obs, b_env.terminal_obs)
    assert torch.equal(a_env.ep_stats, b_env.ep_stats)
    for f in ("endpoint_latency", "endpoint_cpu_usage_percentage", "avg_load_served", "current_time"):
        assert torch.equal(a_env.field(f), b_env.field(f)), f
    # the env goes on from where the launch left it, across its next episode boundary
    for _ in range(a_env.cfg.episode_length + 1):
        a_env.step_device(None)
        b_env.step_device(None)
        assert torch.equal(a_env.obs, b_env.obs)
        assert torch.equal(a_env.rewards, b_env.rewards)
    assert a_env.status() == 0 and b_env.status() == 0


@pytest.mark.parametrize("B,kw", [
    (65600, {}),                                           # partial last block (one live wave)
    (131072, dict(reward_function="latency")),
    (65536 + 192, dict(CFG1, reward_function="naive")),    # config 1's shape, three live waves
    (131072, dict(CFG1, reward_function="multi", latency_weight=1.0, cpu_weight=0.0, gini_weight=0.0)),
    (98304, dict(reward_function="multi", latency_weight=0.4, cpu_weight=0.3, gini_weight=0.3)),
    (98304, dict(num_nodes=28, num_zones=5, reward_function="fairness")),
    (65536 + 320, dict(num_endpoints=6, reward_function="multi")),  # E = 6, N = 24: one node-zone word
])
@pytest.mark.parametrize("kind", ["random", "topo", "zone_cpu", "endpoint_cpu"])
@pytest.mark.parametrize("K,L", [(20, 20), (13, 20), (7, 9), (40, 40)])  # (40: the single-wave layout)
def test_lean_staggered_equals_policy_plus_step(B, kw, kind, K, L):
    """Staggered episodes (1/L of the envs end at every step; some waves have more enders
    in a step than the prefetch covers, so both restart paths run), actions written."""
    a_env, b_env = _staggered_pair(B, L, kw)
    assert a_env.rollout_kernel(K).startswith("k_rollout_lean")
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
    _compare_after(a_env, b_env, B)


@pytest.mark.parametrize("kw", [{}, dict(CFG1, reward_function="multi")])
@pytest.mark.parametrize("kind", ["random", "endpoint_cpu"])
def test_lean_lockstep_equals_policy_plus_step(kw, kind):
    """Every env ends at the same step (no stagger, L == K): every wave restarts all 64 envs
    in one step, in groups, the first from the prefetched records and the rest loaded there;
    no actions_out (the kernel variant that writes none)."""
    B, K = 131072, 20
    a_env, b_env = _staggered_pair(B, K, kw, stagger=False)
    assert a_env.rollout_kernel(K).startswith("k_rollout_lean")
    R = a_env.cfg.obs_rows
    obs = torch.empty((K, B, R, 8), device="cuda")
    rew = torch.empty((K, B), device="cuda")
    dn = torch.empty((K, B), dtype=torch.uint8, device="cuda")
    for rep in range(2):  # the second launch starts on the episodes the first one restarted
        a_env.rollout(kind, K, obs_out=obs, reward_out=rew, done_out=dn)
        for k in range(K):
            b_env.step_device(b_env.policy(kind))
            assert torch.equal(obs[k], b_env.obs), (rep, k)
            assert torch.equal(rew[k], b_env.rewards), (rep, k)
            assert torch.equal(dn[k], b_env.dones), (rep, k)
        assert int(dn[K - 1].sum()) == B
    _compare_after(a_env, b_env, B)


def test_lean_headline_size_equals_single_steps():
    """The headline launch at its headline size: 2^20 default envs, staggered, K = 20 (the
    driver's bench shape), three launches, == 20 x step_device(None) per launch, bit for bit
    -- obs, reward, done, terminal obs, episode-stats rows, the state afterwards."""
    B, K, L = 1 << 20, 20, 100
    a_env, b_env = _staggered_pair(B, L, {}, seed=11)
    assert a_env.rollout_kernel(K).startswith("k_rollout_lean")
    R = a_env.cfg.obs_rows
    obs = torch.empty((K, B, R, 8), device="cuda")
    rew = torch.empty((K, B), device="cuda")
    dn = torch.empty((K, B), dtype=torch.uint8, device="cuda")
    for launch in range(3):
        a_env.rollout("random", K, obs_out=obs, reward_out=rew, done_out=dn)
        for k in range(K):
            b_env.step_device(None)
            assert torch.equal(obs[k], b_env.obs), (launch, k)
            assert torch.equal(rew[k], b_env.rewards), (launch, k)
            assert torch.equal(dn[k], b_env.dones), (launch, k)
            assert int(dn[k].sum()) > 0
        assert torch.equal(a_env.terminal_obs, b_env.terminal_obs), launch
        assert torch.equal(a_env.ep_stats, b_env.ep_stats), launch
    _compare_after(a_env, b_env, B)


def test_lean_not_chosen_outside_its_shapes():
    """k_rollout_lean runs only where it was built for: E = 8 (R = 9, N <= 32) or E = 6
    (R = 7, N <= 64), B a multiple of 64 above 65,536, episodes at least K long, every output."""
    from lbk8s import LBVecEnv
    assert LBVecEnv(131072 + 32, seed=1, as_tensors=True).rollout_kernel(20) == "k_rollout_img"
    assert LBVecEnv(65536, seed=1, as_tensors=True).rollout_kernel(20) == "k_rollout_img"
    assert LBVecEnv(131072, seed=1, as_tensors=True, num_endpoints=7).rollout_kernel(20) == "k_rollout_img"
    assert LBVecEnv(131072, seed=1, as_tensors=True, episode_length=10).rollout_kernel(20) == "k_rollout_tpe"
    env = LBVecEnv(131072, seed=1, as_tensors=True)
    assert env.rollout_kernel(20, outputs_all=False) == "k_rollout_img"
    assert env.rollout_kernel(20) == "k_rollout_lean_split"


def test_rollout_past_4gib_takes_64bit_kernel():
    """Above 4 GiB of state the 32-bit-offset kernels (k_rollout_lean / k_rollout_img) are not
    used: lb_rollout takes k_rollout_tpe (64-bit indexing), and its launch at such a B
    equals K x step_device, bit for bit (12,000,000 default envs: a 4.56 GB state blob)."""
    from lbk8s import LBVecEnv, _native
    B, K, L = 12_000_000, 3, 3
    a_env = LBVecEnv(B, seed=9, as_tensors=True, episode_length=L)
    assert a_env.state.numel() > (1 << 32)
    assert a_env.rollout_kernel(K) == "k_rollout_tpe"
    R = a_env.cfg.obs_rows
    obs = torch.empty((K, B, R, 8), device="cuda")
    rew = torch.empty((K, B), device="cuda")
    dn = torch.empty((K, B), dtype=torch.uint8, device="cuda")
    a_env.reset()
    a_env.rollout("random", K, obs_out=obs, reward_out=rew, done_out=dn)
    a_stats, a_term = a_env.stats(), a_env.terminal_obs.clone()
    del a_env
    b_env = LBVecEnv(B, seed=9, as_tensors=True, episode_length=L)
    b_env.reset()
    for k in range(K):
        b_env.step_device(None)
        assert torch.equal(obs[k], b_env.obs), k
        assert torch.equal(rew[k], b_env.rewards), k
        assert torch.equal(dn[k], b_env.dones), k
    assert int(dn[K - 1].sum()) == B
    assert torch.equal(a_stats, b_env.stats())
    assert torch.equal(a_term, b_env.terminal_obs)
    assert b_env.status() == 0


def test_lean_shard_equals_slice_of_whole():
    """A rank's shard (env_id_offset = n) runs the same trajectories as envs n .. 2n - 1 of
    one 2n-env batch: k_rollout_lean keys every draw (steps and the records of the next
    episodes) on the global env id, so bench.py --gpus N measures the same work at any N."""
    from lbk8s import LBVecEnv
    n, K, L = 131072, 20, 20
    whole = LBVecEnv(2 * n, seed=3, as_tensors=True, episode_length=L)
    shard = LBVecEnv(n, seed=3, env_id_offset=n, as_tensors=True, episode_length=L)
    assert whole.rollout_kernel(K) == "k_rollout_lean_split" and shard.rollout_kernel(K) == "k_rollout_lean_split"
    outs = []
    for e, B in ((whole, 2 * n), (shard, n)):
        e.reset()
        R = e.cfg.obs_rows
        o = torch.empty((K, B, R, 8), device="cuda")
        r = torch.empty((K, B), device="cuda")
        d = torch.empty((K, B), dtype=torch.uint8, device="cuda")
        for _ in range(2):  # the second launch starts on the episodes the first restarted
            e.rollout("random", K, obs_out=o, reward_out=r, done_out=d)
        outs.append((o, r, d, e.stats(), e.terminal_obs))
    (o1, r1, d1, s1, t1), (o2, r2, d2, s2, t2) = outs
    assert torch.equal(o1[:, n:], o2) and torch.equal(r1[:, n:], r2) and torch.equal(d1[:, n:], d2)
    assert torch.equal(s1[n:], s2) and torch.equal(t1[n:], t2)
    assert int(d2.sum()) == n  # every env ended once per launch (L == K, no stagger)
