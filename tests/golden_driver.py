"""Replay a golden fixture (tests/golden/*.npz, produced by the reference) through a backend.

A backend exposes (with B = number of env instances in the fixture):
    init(t0)                                   # __init__'s surviving current_time
    reset(reset_trace_arrays) -> obs (B,R,8) f32
    step(actions, step_trace_arrays, reset_trace_arrays_or_None)
        -> obs, reward(f32), done(bool), terminal_obs, stats (B,16) f64 at done
    stats() -> (B,16) f64 accumulators after the last step
    fields() -> dict of state views (ep_lat, ep_cpu, loads, t, ...), float64
Both the C oracle and the GPU VecEnv implement it, so the same comparisons pin both.
"""
import json

import numpy as np


def load(path):
    d = dict(np.load(path))
    d["config"] = json.loads(str(d["config_json"]))
    return d


def reset_arrays(d, k):
    return dict(lat0=d["reset_lat0"][:, k], topo=d["reset_topo"][:, k], ntype=d["reset_ntype"][:, k],
                nzone=d["reset_nzone"][:, k], ncpu=d["reset_ncpu"][:, k], enode=d["reset_enode"][:, k],
                x1=d["reset_req_x"][:, k, 0], x2=d["reset_req_x"][:, k, 1],
                r=d["reset_req_i"][:, k, 0], n=d["reset_req_i"][:, k, 1])


def step_arrays(d, s):
    return dict(x1=d["step_x"][:, s, 0], x2=d["step_x"][:, s, 1], r=d["step_i"][:, s, 0],
                n=d["step_i"][:, s, 1])


def _eq(name, got, exp, where):
    got = np.asarray(got)
    exp = np.asarray(exp)
    if not np.array_equal(got, exp):
        bad = np.argwhere(got != exp)
        i = tuple(bad[0])
        raise AssertionError(f"{name} mismatch at {where} index {i}: got {got[i]!r} expected {exp[i]!r} "
                             f"({len(bad)} mismatches)")


def replay(d, backend, check_state=True, n_steps=None, policy=None):
    """Drive `backend` with the fixture's actions + draws; assert bit-exact outputs.

    policy: optional callable(backend) -> actions; then the backend's own choice must
    equal the recorded action (greedy-policy fixtures).
    Returns a dict of counters (compared values) for reporting.
    """
    B, S = d["actions"].shape
    S = S if n_steps is None else min(S, n_steps)
    from lbk8s.info import ST_ACC, ST_INTER, ST_INTRA, ST_LENGTH, ST_RETURN, ST_SUM_COST, \
        ST_SUM_TOPO, step_info
    backend.init(d["t0"])
    obs = backend.reset(reset_arrays(d, 0))
    _eq("reset obs", obs, d["reset_obs"][:, 0].astype(np.float32), "reset 0")
    k = 1
    counts = dict(steps=0, obs_values=0, info_exact=0, info_total=0)
    reset_at = list(d["reset_at"])
    for s in range(S):
        actions = d["actions"][:, s]
        if policy is not None:
            chosen = policy(backend)
            _eq("policy action", chosen, actions, f"step {s}")
        rt = reset_arrays(d, k) if (k < len(reset_at) and reset_at[k] == s + 1) else None
        obs, rew, done, term, st = backend.step(actions, step_arrays(d, s), rt)
        where = f"step {s}"
        _eq("reward", rew, d["reward"][:, s].astype(np.float32), where)
        _eq("done", np.asarray(done, bool), d["done"][:, s], where)
        exp_obs = d["obs"][:, s].astype(np.float32)
        if rt is not None:
            _eq("terminal obs", term, exp_obs, where)
            _eq("post-reset obs", obs, d["reset_obs"][:, k].astype(np.float32), where)
            stats = st
            k += 1
        else:
            _eq("obs", obs, exp_obs, where)
            stats = backend.stats()
        # info: every key exactly the reference's float("{:.2f}") (exact-rational means)
        info = d["info"][:, s]
        for b in range(B):
            got = step_info(stats[b], float(d["reward"][b, s]), int(actions[b]))
            expv = dict(zip(["reward_step", "action", "reward", "ep_block_prob",
                             "ep_accepted_requests", "avg_endpoint_latency", "avg_topology_latency",
                             "avg_cost", "avg_cpu_endpoint_selected", "ep_intra_zone_percentage",
                             "ep_inter_zone_percentage", "gini"], info[b, :12]))
            for key, ev in expv.items():
                counts["info_total"] += 1
                if got[key] != ev:
                    raise AssertionError(f"info[{key}] {got[key]} != {ev} at {where} env {b}")
                counts["info_exact"] += 1
            assert int(stats[b, ST_ACC]) == d["state_counters"][b, s, 1]
            assert int(stats[b, ST_INTRA]) == d["state_counters"][b, s, 2]
            assert int(stats[b, ST_INTER]) == d["state_counters"][b, s, 3]
            assert int(stats[b, ST_LENGTH]) == d["state_counters"][b, s, 0]
            _ = (ST_RETURN, ST_SUM_COST, ST_SUM_TOPO)
        if check_state and rt is None:
            f = backend.fields()
            exp = dict(ep_lat=d["state_ep_lat"][:, s], ep_cpu=d["state_ep_cpu"][:, s],
                       ep_topo=d["state_ep_topo"][:, s], ep_cap=d["state_ep_cap"][:, s],
                       ep_zone=d["state_ep_zone"][:, s], ep_node=d["state_ep_node"][:, s],
                       loads=d["state_loads"][:, s], t=d["state_t"][:, s], dt=d["state_dt"][:, s],
                       step=d["state_counters"][:, s, 0], req_zone=d["state_req"][:, s, 0],
                       req_thr=d["state_req"][:, s, 1])
            for key, val in f.items():
                _eq(key, val, exp[key], where)
        counts["steps"] += 1
        counts["obs_values"] += exp_obs.size
    return counts
