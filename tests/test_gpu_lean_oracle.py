"""k_rollout_lean (the headline kernel) pinned DIRECTLY to the C oracle.

test_gpu_lean.py checks k_rollout_lean against K x (lb_policy + lb_step), i.e. HIP against
HIP.  Here the other side is oracle.OracleBatch (oracle/lbk8s_oracle.c, itself bit-exact to
the reference-run fixtures in test_oracle_golden.py), stepping one vector step at a time
with its own policies (envs/baselines.py:6-35 restated, and the Philox random action):
every obs, reward, done, action, terminal obs and episode-statistics row of the launch,
and the env's fields and accumulators afterwards, bit for bit.

The envs are staggered as bench.py does (env i restarts after step i mod L), so 1/L of the
envs end at every step of the launch and the in-launch restarts from the next-episode
records run in every wave; two launches, so the second starts on episodes the first one
restarted.  Reference: envs/loadbalancer_k8s_env.py:403-513 (step, done, reset through the
VecEnv's auto-reset), envs/baselines.py:6-35.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

CFGS = {
    "default": {},
    "cfg1_multi": dict(num_endpoints=6, num_nodes=48, num_zones=12, reward_function="multi"),
    "fair_n28_z5": dict(num_nodes=28, num_zones=5, reward_function="fairness"),
    "e6_n24_latency": dict(num_endpoints=6, reward_function="latency"),  # one node-zone word
}
ORC_KIND = {"topo": "topo", "zone_cpu": "zone_cpu", "endpoint_cpu": "endpoint_cpu"}


def _orc_policy(orc, kind):
    return orc.policy_random() if kind == "random" else orc.policy_greedy(ORC_KIND[kind])


# K <= 32: the split layout (an env wave and a copy wave per block, k_rollout_lean_split);
# K = 40: the single-wave layout (lbk8s.hip: LEAN_SPLIT_MAX_K)
@pytest.mark.parametrize("B,cfg,K", [(131072, c, 20) for c in CFGS] + [(65600, "default", 20), (65600, "cfg1_multi", 20),
                                                                      (65600, "default", 40), (65600, "cfg1_multi", 40)])
@pytest.mark.parametrize("kind", ["random", "topo", "zone_cpu", "endpoint_cpu"])
def test_lean_rollout_equals_oracle(oracle_mod, B, cfg, K, kind):
    from lbk8s import LBVecEnv
    L = K
    seed = 1000 + B % 977
    kw = dict(CFGS[cfg], episode_length=L)
    env = LBVecEnv(B, seed=seed, as_tensors=True, **kw)
    orc = oracle_mod.OracleBatch(kw, B, trace=False, seed=seed)
    orc.init()
    assert env.rollout_kernel(K).startswith("k_rollout_lean")
    np.testing.assert_array_equal(env.reset().cpu().numpy(), orc.reset())
    gid = np.arange(B)
    for r in range(1, L):  # bench.py's stagger, both sides under their own random policy
        a = env.policy("random")
        np.testing.assert_array_equal(a.cpu().numpy(), orc.policy_random())
        env.step_device(a)
        orc.step(a.cpu().numpy())
        m = ((gid % L) == r).astype(np.uint8)
        env.reset_masked(torch.from_numpy(m))
        orc.reset(mask=m)
    R = env.cfg.obs_rows
    obs = torch.empty((K, B, R, 8), device="cuda")
    rew = torch.empty((K, B), device="cuda")
    dn = torch.empty((K, B), dtype=torch.uint8, device="cuda")
    act = torch.empty((K, B), dtype=torch.int32, device="cuda")
    for launch in range(2):
        env.rollout(kind, K, obs_out=obs, reward_out=rew, done_out=dn, actions_out=act)
        o, rw, d, ac = obs.cpu().numpy(), rew.cpu().numpy(), dn.cpu().numpy().astype(bool), act.cpu().numpy()
        term = np.zeros((B, R, 8), np.float32)
        rows = np.zeros((B, 16), np.float64)
        ended = np.zeros(B, bool)
        for k in range(K):
            a2 = _orc_policy(orc, kind)
            np.testing.assert_array_equal(ac[k], a2, err_msg=f"action launch {launch} step {k}")
            o2, r2, d2, t2, st2 = orc.step(a2)
            assert 0 < d2.sum() < B
            np.testing.assert_array_equal(rw[k], r2, err_msg=f"reward launch {launch} step {k}")
            np.testing.assert_array_equal(d[k], d2, err_msg=f"done launch {launch} step {k}")
            np.testing.assert_array_equal(o[k], o2, err_msg=f"obs launch {launch} step {k}")
            term[d2] = t2[d2]
            rows[d2] = st2[d2]
            ended |= d2
        assert ended.all()  # L == K: every env ended once in the launch
        np.testing.assert_array_equal(env.terminal_obs.cpu().numpy(), term)
        np.testing.assert_array_equal(env.ep_stats.cpu().numpy(), rows)
    np.testing.assert_array_equal(env.stats().cpu().numpy(), orc.stats())
    for f, g in (("endpoint_latency", "ep_lat"), ("endpoint_cpu_usage_percentage", "ep_cpu"),
                 ("avg_load_served", "loads"), ("current_time", "t")):
        np.testing.assert_array_equal(env.field(f).cpu().numpy(), orc.field(g), err_msg=f)
    assert env.status() == 0
