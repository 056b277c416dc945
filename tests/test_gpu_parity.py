"""T2 (kernel-trace parity) and T3 (Philox self-consistency) on a real MI355X.

T2: the HIP step/reset kernels in trace-injection mode, driven by the reference's own
numpy draws recorded in tests/golden/*.npz, reproduce the reference bit-exactly:
obs (float32 cast), reward (float32 cast), done, float64 latency/CPU state, loads,
current_time, counters and the per-episode accumulators.  All through the C ABI
(liblbk8s.so) via the drop-in LBVecEnv.

T3: in Philox mode the kernels and the C oracle (same draw map, restated
independently) produce identical trajectories, at batch sizes the oracle finishes in
seconds.  Tolerance everywhere: bit-exact (integers, and floats because both sides
do the reference's float64 IEEE arithmetic without FMA contraction).
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN, golden_names
from golden_driver import load, replay

pytestmark = pytest.mark.gpu

FIELD_MAP = dict(ep_lat="endpoint_latency", ep_cpu="endpoint_cpu_usage_percentage",
                 ep_topo="endpoint_topology_latency", ep_cap="endpoint_zone_cpu_capacity",
                 ep_zone="endpoint_zone", ep_node="endpoint_node", loads="avg_load_served",
                 t="current_time", step="current_step", req_zone="request_zone",
                 req_thr="request_threshold")


class GpuBackend:
    def __init__(self, cfg, B, geometry="auto"):
        self.cfg, self.B, self.geometry = cfg, B, geometry
        self.env = None

    def init(self, t0):
        from lbk8s import LBVecEnv
        self.env = LBVecEnv(self.B, trace=True, t0=t0, geometry=self.geometry, **self.cfg)

    def reset(self, ra):
        return self.env.reset(trace=ra)

    def step(self, actions, sa, ra):
        obs, rew, done, _ = self.env.step(actions, trace=sa, reset_trace=ra)
        return (obs, rew, done, self.env.terminal_obs.cpu().numpy(),
                self.env.ep_stats.cpu().numpy())

    def stats(self):
        return self.env.stats().cpu().numpy()

    def fields(self):
        return {k: self.env.field(v).cpu().numpy() for k, v in FIELD_MAP.items()}


def pin_geometry(geometry, cfg):
    """Below 32,768 envs E <= 8 runs the slice kernels; "tpe" pins the thread-per-env
    kernels (lb_config.geometry) so both stay covered."""
    if geometry == "tpe" and cfg.get("num_endpoints", 8) > 8:
        pytest.skip("thread-per-env kernels take E <= 8")


@pytest.mark.parametrize("geometry", ["auto", "tpe"])
@pytest.mark.parametrize("name", golden_names())
def test_kernel_trace_parity_with_reference(name, geometry):
    d = load(os.path.join(GOLDEN, name + ".npz"))
    pin_geometry(geometry, dict(d["config"]))
    be = GpuBackend(d["config"], d["actions"].shape[0], geometry)
    policy = None
    if name.startswith("greedy_"):
        kind = name[len("greedy_"):].replace("_e64", "")
        policy = lambda b: b.env.policy(kind).cpu().numpy()  # noqa: E731
    c = replay(d, be, policy=policy)
    assert c["steps"] == d["actions"].shape[1]
    assert be.env.status() == 0


PHILOX_CFGS = {
    "default": dict(),
    "cfg1_multi": dict(num_endpoints=6, num_nodes=48, num_zones=12, reward_function="multi",
                       latency_weight=1.0, cpu_weight=0.0, gini_weight=0.0),
    "e64_multi": dict(num_endpoints=64, reward_function="multi"),
    "e100_fair_norej": dict(num_endpoints=100, reward_function="fairness", rejection_allowed=False),
    "e3_latency_short": dict(num_endpoints=3, reward_function="latency", episode_length=9),
    "e13_n70": dict(num_endpoints=13, num_nodes=70, num_zones=7, reward_function="multi"),
    # E in (100, 256]: the reference's own sweep lists 128 / 150 / 180 (run_baselines.py:32);
    # 512 envs run the one-env-per-wave slice shape, W = 64 with EPL = 2 (E = 128) or 4 (E > 128)
    "e128_multi": dict(num_endpoints=128, reward_function="multi"),
    "e150_fair_norej": dict(num_endpoints=150, reward_function="fairness", rejection_allowed=False),
    "e180_multi_n64": dict(num_endpoints=180, num_nodes=64, num_zones=6, reward_function="multi",
                           latency_weight=0.5, cpu_weight=0.3, gini_weight=0.2),
    "e256_latency_n200": dict(num_endpoints=256, num_nodes=200, num_zones=9, reward_function="latency"),
}


@pytest.mark.parametrize("geometry", ["auto", "tpe"])
@pytest.mark.parametrize("name", sorted(PHILOX_CFGS))
def test_philox_mode_matches_oracle(oracle_mod, name, geometry):
    """Same seed, same env ids, same actions -> identical trajectories (GPU vs C oracle)."""
    from lbk8s import LBVecEnv
    cfg = PHILOX_CFGS[name]
    pin_geometry(geometry, cfg)
    B = 2048 if cfg.get("num_endpoints", 8) <= 16 else 512
    seed, off = 12345, 7_000_000_000  # env ids above 2^32 exercise the counter's high word
    env = LBVecEnv(B, seed=seed, env_id_offset=off, geometry=geometry, **cfg)
    orc = oracle_mod.OracleBatch(cfg, B, trace=False, seed=seed, env_id_offset=off)
    orc.init()
    np.testing.assert_array_equal(env.reset(), orc.reset())
    rng = np.random.default_rng(0)
    A = env.action_space.n
    E = env.cfg.num_endpoints
    L = env.cfg.episode_length
    for s in range(2 * L + 17):
        if s % 3 == 0:
            a = env.policy("random").cpu().numpy()
            np.testing.assert_array_equal(a, orc.policy_random())
        else:
            a = rng.integers(-E - 1, A + 2, size=B).astype(np.int32)  # incl. negative / invalid
        o1, r1, d1, _ = env.step(a)
        o2, r2, d2, t2, st2 = orc.step(a)
        np.testing.assert_array_equal(r1, r2, err_msg=f"reward step {s}")
        np.testing.assert_array_equal(d1, d2, err_msg=f"done step {s}")
        np.testing.assert_array_equal(o1, o2, err_msg=f"obs step {s}")
        if d1.any():
            np.testing.assert_array_equal(env.terminal_obs.cpu().numpy()[d1], t2[d1])
            st1 = env.ep_stats.cpu().numpy()[d1]
            st2 = st2[d1]
            # every column bit-exact, incl. the exact sums' remainders and D (include/lbk8s.h)
            np.testing.assert_array_equal(st1, st2)
    for f in ("endpoint_latency", "endpoint_cpu_usage_percentage", "avg_load_served"):
        key = {"endpoint_latency": "ep_lat", "endpoint_cpu_usage_percentage": "ep_cpu",
               "avg_load_served": "loads"}[f]
        np.testing.assert_array_equal(env.field(f).cpu().numpy(), orc.field(key))
    np.testing.assert_array_equal(env.field("current_time").cpu().numpy(), orc.field("t"))
    # actions < -E were issued above: the status word must say so
    assert env.status() & 1


# Many envs take other kernel variants: from 32,768 envs (E > 8) the 4-envs-per-wave
# slice shape (W = 16 or 32 lanes per env, 2 or 4 endpoints per lane), from 262,144 envs
# (E <= 8) the thread-per-env step that redraws the scenario instead of loading it.  Same
# check as above at sizes that select them, with short episodes so auto-resets run.
MANY_CFGS = {
    "e64_multi_l10": dict(num_endpoints=64, reward_function="multi", episode_length=10),
    "e20_latency_l10": dict(num_endpoints=20, reward_function="latency", episode_length=10),
    "e100_fair_norej_l10": dict(num_endpoints=100, reward_function="fairness", rejection_allowed=False,
                                episode_length=10),
    "default_l10": dict(episode_length=10),
    "cfg1_multi_l7": dict(num_endpoints=6, num_nodes=48, num_zones=12, reward_function="multi",
                          latency_weight=0.5, cpu_weight=0.3, gini_weight=0.2, episode_length=7),
    "e5_fair_norej_l10": dict(num_endpoints=5, num_nodes=70, reward_function="fairness",
                              rejection_allowed=False, episode_length=10),
    # E in (100, 256] at 32,768 envs: W = 32 / EPL = 4 (E = 128) and W = 64 / EPL = 4 (E > 128)
    "e128_fair_l10": dict(num_endpoints=128, reward_function="fairness", episode_length=10),
    "e150_multi_norej_l10": dict(num_endpoints=150, reward_function="multi", rejection_allowed=False,
                                 episode_length=10),
    "e180_latency_n48_l10": dict(num_endpoints=180, num_nodes=48, num_zones=5, reward_function="latency",
                                 episode_length=10),
    "e256_multi_l10": dict(num_endpoints=256, reward_function="multi", latency_weight=1.0, cpu_weight=0.0,
                           gini_weight=0.0, episode_length=10),
}


@pytest.mark.parametrize("name", sorted(MANY_CFGS))
def test_philox_many_envs_matches_oracle(oracle_mod, name):
    from lbk8s import LBVecEnv
    cfg = MANY_CFGS[name]
    B = 32768 if cfg.get("num_endpoints", 8) > 8 else 262144
    seed = 99
    env = LBVecEnv(B, seed=seed, **cfg)
    orc = oracle_mod.OracleBatch(cfg, B, trace=False, seed=seed)
    orc.init()
    np.testing.assert_array_equal(env.reset(), orc.reset())
    rng = np.random.default_rng(1)
    A = env.action_space.n
    E = env.cfg.num_endpoints
    for s in range(2 * env.cfg.episode_length + 3):
        a = rng.integers(-E, A, size=B).astype(np.int32)
        o1, r1, d1, _ = env.step(a)
        o2, r2, d2, t2, _ = orc.step(a)
        np.testing.assert_array_equal(r1, r2, err_msg=f"reward step {s}")
        np.testing.assert_array_equal(d1, d2, err_msg=f"done step {s}")
        np.testing.assert_array_equal(o1, o2, err_msg=f"obs step {s}")
        if d1.any():
            np.testing.assert_array_equal(env.terminal_obs.cpu().numpy()[d1], t2[d1])
    np.testing.assert_array_equal(env.field("avg_load_served").cpu().numpy(), orc.field("loads"))
    assert env.status() == 0


@pytest.mark.gpu
def test_config2_rollout_matches_oracle(oracle_mod):
    """BASELINE config 2 at its size: 4096 default envs under the env's own random policy,
    run as lb_rollout launches of 50 vector steps (the config-2 fast path), == the C oracle
    stepping one vector step at a time with its random policy, bit for bit, across the
    auto-resets of 2.5 episodes."""
    import torch

    from lbk8s import LBVecEnv
    B, K, seed = 4096, 50, 2024
    env = LBVecEnv(B, seed=seed, as_tensors=True)
    orc = oracle_mod.OracleBatch({}, B, trace=False, seed=seed)
    orc.init()
    np.testing.assert_array_equal(env.reset().cpu().numpy(), orc.reset())
    R = env.cfg.obs_rows
    obs = torch.empty((K, B, R, 8), dtype=torch.float32, device="cuda")
    rew = torch.empty((K, B), dtype=torch.float32, device="cuda")
    done = torch.empty((K, B), dtype=torch.uint8, device="cuda")
    for launch in range(5):
        env.rollout("random", K, obs_out=obs, reward_out=rew, done_out=done)
        o, r, d = obs.cpu().numpy(), rew.cpu().numpy(), done.cpu().numpy().astype(bool)
        for k in range(K):
            o2, r2, d2, _, _ = orc.step(orc.policy_random())
            s = launch * K + k
            np.testing.assert_array_equal(r[k], r2, err_msg=f"reward step {s}")
            np.testing.assert_array_equal(d[k], d2, err_msg=f"done step {s}")
            np.testing.assert_array_equal(o[k], o2, err_msg=f"obs step {s}")
    assert env.status() == 0


@pytest.mark.gpu
@pytest.mark.parametrize("B,K,kw", [
    (40000, 20, {}), (70000, 20, {}), (70000, 7, {}),
    (70000, 20, dict(num_endpoints=3, num_nodes=30, num_zones=5, reward_function="fairness",
                     rejection_allowed=False)),
    (40000, 20, dict(num_endpoints=6, num_nodes=48, num_zones=12, reward_function="multi")),
])
def test_rollout_tpe_staggered_matches_oracle(oracle_mod, B, K, kw):
    """lb_rollout with the env's random policy (K vector steps per launch, staggered episodes,
    next episodes drawn into records before the first step since L >= K: k_rollout_img here,
    as lb_rollout_kernel reports; k_rollout_lean is tested at its shapes in test_gpu_lean.py)
    against the C oracle stepping one vector step at a time, bit for bit: obs,
    reward, done, terminal obs, and the state after the launches.  64-thread blocks (40,000
    envs, geometry pinned to tpe) and 256-thread blocks with a partial last block (70,000);
    the default scenario, E = 3 without rejection (fairness reward), config 1's E = 6, N = 48,
    Z = 12 (multi reward)."""
    import torch

    from lbk8s import LBVecEnv
    L, seed = 20, 99
    cfg = dict(episode_length=L, **kw)
    env = LBVecEnv(B, seed=seed, as_tensors=True, geometry="tpe", **cfg)
    assert env.rollout_kernel(K) == "k_rollout_img"
    orc = oracle_mod.OracleBatch(cfg, B, trace=False, seed=seed)
    orc.init()
    np.testing.assert_array_equal(env.reset().cpu().numpy(), orc.reset())
    gid = np.arange(B)
    for r in range(1, L):  # bench.py's stagger
        env.step_device(None)
        orc.step(orc.policy_random())
        m = (gid % L) == r
        env.reset_masked(torch.from_numpy(m.astype(np.uint8)).cuda())
        orc.reset(mask=m.astype(np.uint8))
    R = env.cfg.obs_rows
    obs = torch.empty((K, B, R, 8), dtype=torch.float32, device="cuda")
    rew = torch.empty((K, B), dtype=torch.float32, device="cuda")
    done = torch.empty((K, B), dtype=torch.uint8, device="cuda")
    for launch in range(3):
        env.rollout("random", K, obs_out=obs, reward_out=rew, done_out=done)
        o, rw, d = obs.cpu().numpy(), rew.cpu().numpy(), done.cpu().numpy().astype(bool)
        for k in range(K):
            o2, r2, d2, t2, _ = orc.step(orc.policy_random())
            st = launch * K + k
            assert 0 < d[k].sum() < B
            np.testing.assert_array_equal(rw[k], r2, err_msg=f"reward step {st}")
            np.testing.assert_array_equal(d[k], d2, err_msg=f"done step {st}")
            np.testing.assert_array_equal(o[k], o2, err_msg=f"obs step {st}")
        last = d[K - 1]
        np.testing.assert_array_equal(env.terminal_obs.cpu().numpy()[last], t2[last])
    np.testing.assert_array_equal(env.field("avg_load_served").cpu().numpy(), orc.field("loads"))
    np.testing.assert_array_equal(env.field("current_time").cpu().numpy(), orc.field("t"))
    np.testing.assert_array_equal(env.field("endpoint_latency").cpu().numpy(), orc.field("ep_lat"))
    assert env.status() == 0


@pytest.mark.gpu
@pytest.mark.parametrize("B", [4096, 131072, (1 << 19) + 4096])
def test_staggered_auto_reset_matches_oracle(oracle_mod, B):
    """Auto-reset with staggered episodes (1/L of the envs end every step, as in bench.py):
    the finishing envs' reset() inside k_step_tpe (a block's list, 8 lanes per env, after
    one LDS-only barrier) with 64-thread blocks (4096), 256-thread blocks with the stored
    scenario (131,072) and with the recomputed one (2^19 + 4096).  Kernels == C oracle bit
    for bit: obs, reward, done, terminal obs, times, latencies, loads."""
    import torch

    from lbk8s import LBVecEnv
    L, seed = 10, 4242
    cfg = dict(episode_length=L)
    env = LBVecEnv(B, seed=seed, **cfg)
    orc = oracle_mod.OracleBatch(cfg, B, trace=False, seed=seed)
    orc.init()
    np.testing.assert_array_equal(env.reset(), orc.reset())
    rng = np.random.default_rng(7)
    A, E = env.action_space.n, env.cfg.num_endpoints
    gid = np.arange(B)
    for r in range(1, L):  # bench.py's stagger: envs with id % L == r restart after step r
        a = rng.integers(-E, A, size=B).astype(np.int32)
        env.step(a)
        orc.step(a)
        m = (gid % L) == r
        env.reset_masked(torch.from_numpy(m.astype(np.uint8)))
        orc.reset(mask=m.astype(np.uint8))
    for s in range(2 * L + 3):
        a = rng.integers(-E, A, size=B).astype(np.int32)
        o1, r1, d1, _ = env.step(a)
        o2, r2, d2, t2, _ = orc.step(a)
        assert 0 < d1.sum() < B
        np.testing.assert_array_equal(r1, r2, err_msg=f"reward step {s}")
        np.testing.assert_array_equal(d1, d2, err_msg=f"done step {s}")
        np.testing.assert_array_equal(o1, o2, err_msg=f"obs step {s}")
        np.testing.assert_array_equal(env.terminal_obs.cpu().numpy()[d1], t2[d1])
    np.testing.assert_array_equal(env.field("avg_load_served").cpu().numpy(), orc.field("loads"))
    np.testing.assert_array_equal(env.field("current_time").cpu().numpy(), orc.field("t"))
    np.testing.assert_array_equal(env.field("endpoint_latency").cpu().numpy(), orc.field("ep_lat"))
    assert env.status() == 0
