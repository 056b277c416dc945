"""lb_dqn_step (csrc/lbk8s_dqn.h): one DQN vector step in one launch at config 5's shape ==
lb_dqn_act + lb_step + lb_replay_add, bit for bit: the actions, the next observations, rewards,
dones, terminal observations and episode-statistics rows, the replay rows, obs <- next obs,
the finished-episode sums, the device step / slot words, and the env state afterwards --
over enough steps that both the explore and the greedy branch run and episodes end.
Reference: envs/dqn_deepset.py:122-174 (the vector step the three launches restate).
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _setup(B, kw, seed):
    from lbk8s import LBVecEnv, _native, fused
    from lbk8s.dqn import DQN_DeepSets, DeviceReplayBuffer
    env = LBVecEnv(B, seed=seed, as_tensors=True, **kw)
    env.reset()
    algo = DQN_DeepSets(env, seed=3)
    frag = fused.frag_buffer(env.device)
    fused.pack_q_into(algo.q_network, frag)
    R = env.cfg.obs_rows
    rb = DeviceReplayBuffer(16 * B, B, (R, 8), env.device, None)  # 16 slots
    st = dict(
        obs=env.obs.clone(), next_obs=torch.empty_like(env.obs), act=torch.empty(B, dtype=torch.int32, device="cuda"),
        rew=torch.empty(B, device="cuda"), done=torch.empty(B, dtype=torch.uint8, device="cuda"),
        ep_sum=torch.zeros(B, dtype=torch.float64, device="cuda"), ep_cnt=torch.zeros(B, dtype=torch.float64, device="cuda"),
        vpp=torch.zeros(2, dtype=torch.int64, device="cuda"), flag=torch.zeros(1, dtype=torch.int32, device="cuda"))
    return env, frag, rb, st, _native


def _ex(_native, st, parity, eps_start):
    b = st["vpp"].data_ptr()
    # eps from eps_start down to 0.05 over 40 steps: early steps mostly explore, later greedy
    return _native.LBDQNExploreC(eps_start, -(eps_start - 0.05) / 40.0, 0.05, 77, b + 8 * parity,
                                 b + 8 * (1 - parity), st["flag"].data_ptr())


@pytest.mark.parametrize("B,kw", [(4096, {}), (4096 + 8, dict(reward_function="multi", episode_length=9)),
                                  (8192, dict(num_endpoints=6, reward_function="fairness", episode_length=7)),
                                  (8, dict(num_endpoints=6, reward_function="multi", episode_length=7))])
def test_dqn_step_equals_three_launches(B, kw):
    """(8 envs: run.py's own DQN setup, far fewer envs than the chip's SIMDs: the one-launch
    path is a property of the env's shape, not of the device's CU count.)"""
    kw = dict(dict(episode_length=7), **kw)
    a_env, frag, a_rb, a, nat = _setup(B, kw, seed=5)
    b_env, _, b_rb, b, _ = _setup(B, kw, seed=5)
    # the path under test is the one-launch step (else lb_dqn_step would compare its fallback,
    # the three launches, with themselves)
    assert a_env.dqn_steps_supported(a_env.cfg.obs_rows)
    masks = torch.ones((B, a_env.cfg.obs_rows), dtype=torch.uint8, device="cuda")
    explored = greedy = 0
    for t in range(40):
        parity = t & 1
        ex_a, ex_b = _ex(nat, a, parity, 0.9), _ex(nat, b, parity, 0.9)
        pa, pb = a_rb.pos_pp.data_ptr(), b_rb.pos_pp.data_ptr()
        a_env.dqn_step(frag, a["obs"], masks, ex_a, a["act"], a["next_obs"], a["rew"], a["done"], a_rb,
                       pa + 8 * parity, pa + 8 * (1 - parity), a["ep_sum"], a["ep_cnt"])
        # the three launches
        b_env.dqn_act(frag, b["obs"], masks, ex_b, b["act"])
        b_env.step_device(b["act"], obs_out=b["next_obs"], reward_out=b["rew"], done_out=b["done"])
        b_rb.add_fused(b["obs"], b["next_obs"], b["act"], b["rew"], b["done"], b_env.ep_stats, b["ep_sum"], b["ep_cnt"],
                       parity)
        f = int(a["flag"].item())
        assert f == int(b["flag"].item()), t
        explored += f
        greedy += 1 - f
        for k in ("act", "next_obs", "rew", "done", "obs", "ep_sum", "ep_cnt", "vpp"):
            assert torch.equal(a[k], b[k]), (t, k)
        assert torch.equal(a_rb.pos_pp, b_rb.pos_pp), t
        assert torch.equal(a_env.terminal_obs, b_env.terminal_obs), t
        assert torch.equal(a_env.ep_stats, b_env.ep_stats), t
    for name in ("obs", "next_obs", "actions", "rewards", "dones"):
        assert torch.equal(getattr(a_rb, name), getattr(b_rb, name)), name
    assert torch.equal(a_env.stats(), b_env.stats())
    for f in ("endpoint_latency", "endpoint_cpu_usage_percentage", "avg_load_served", "current_time"):
        assert torch.equal(a_env.field(f), b_env.field(f)), f
    assert explored > 0 and greedy > 0
    assert int(a["ep_cnt"].sum().item()) > 0  # episodes ended inside the window


@pytest.mark.parametrize("B,kw,n", [(4096, {}, 10), (4096 + 8, dict(reward_function="multi", episode_length=9), 7),
                                    (8192, dict(num_endpoints=6, reward_function="fairness"), 2)])
def test_dqn_steps_equals_single_steps(B, kw, n):
    """lb_dqn_steps(n) (n vector steps in one launch, the device words in place for even n)
    == n x lb_dqn_step with the ping-pong words, bit for bit, over launches that cross the
    explore / greedy boundary and episode ends."""
    kw = dict(dict(episode_length=7), **kw)
    a_env, frag, a_rb, a, nat = _setup(B, kw, seed=9)
    b_env, _, b_rb, b, _ = _setup(B, kw, seed=9)
    assert a_env.dqn_steps_supported(a_env.cfg.obs_rows)
    masks = torch.ones((B, a_env.cfg.obs_rows), dtype=torch.uint8, device="cuda")
    sync = torch.zeros(1, dtype=torch.int32, device="cuda")
    pa, pb = a_rb.pos_pp.data_ptr(), b_rb.pos_pp.data_ptr()
    va = a["vpp"].data_ptr()
    parity = 0
    flags = set()
    for _ in range(48 // n):
        end = parity ^ (n & 1)
        ex_a = nat.LBDQNExploreC(0.9, -(0.9 - 0.05) / 40.0, 0.05, 77, va + 8 * parity, va + 8 * end, a["flag"].data_ptr())
        a_env.dqn_steps(n, frag, a["obs"], masks, ex_a, a["act"], a["next_obs"], a["rew"], a["done"], a_rb,
                        pa + 8 * parity, pa + 8 * end, a["ep_sum"], a["ep_cnt"], sync)
        for i in range(n):
            q = parity ^ (i & 1)
            b_env.dqn_step(frag, b["obs"], masks, _ex(nat, b, q, 0.9), b["act"], b["next_obs"], b["rew"], b["done"],
                           b_rb, pb + 8 * q, pb + 8 * (1 - q), b["ep_sum"], b["ep_cnt"])
        parity = end
        flags.add(int(b["flag"].item()))
        assert int(a["flag"].item()) == int(b["flag"].item())
        assert int(sync.item()) == 0
        assert int(a["vpp"][parity].item()) == int(b["vpp"][parity].item())
        assert int(a_rb.pos_pp[parity].item()) == int(b_rb.pos_pp[parity].item())
        for k in ("act", "next_obs", "rew", "done", "obs", "ep_sum", "ep_cnt"):
            assert torch.equal(a[k], b[k]), k
        assert torch.equal(a_env.terminal_obs, b_env.terminal_obs)
        assert torch.equal(a_env.ep_stats, b_env.ep_stats)
    for name in ("obs", "next_obs", "actions", "rewards", "dones"):
        assert torch.equal(getattr(a_rb, name), getattr(b_rb, name)), name
    assert torch.equal(a_env.stats(), b_env.stats())
    assert int(a["ep_cnt"].sum().item()) > 0
