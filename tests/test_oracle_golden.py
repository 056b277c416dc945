"""T1: the C oracle (oracle/lbk8s_oracle.c) equals the reference on every golden fixture.

The fixtures were produced by running the reference env itself
(tests/golden/gen_golden.py); this pins the oracle before it is trusted as the
GPU checker.  Bit-exact: obs (float32 cast of the reference's float64), reward,
done, float64 state (latency, CPU, topology latency, loads, time), counters.
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN, golden_names
from golden_driver import load, replay


class OracleBackend:
    def __init__(self, oracle_mod, cfg, B):
        self.m = oracle_mod
        self.o = oracle_mod.OracleBatch(cfg, B, trace=True, auto_reset=True)

    def init(self, t0):
        self.o.init(t0)

    def reset(self, ra):
        return self.o.reset(trace=self.m.ResetTrace(**ra))

    def step(self, actions, sa, ra):
        rt = self.m.ResetTrace(**ra) if ra is not None else None
        return self.o.step(actions, self.m.StepTrace(**sa), rt)

    def stats(self):
        return self.o.stats()

    def fields(self):
        return {k: self.o.field(k) for k in ("ep_lat", "ep_cpu", "ep_topo", "loads", "t", "dt",
                                             "req_zone", "req_thr")}


@pytest.mark.parametrize("name", golden_names())
def test_oracle_matches_reference(oracle_mod, name):
    d = load(os.path.join(GOLDEN, name + ".npz"))
    be = OracleBackend(oracle_mod, d["config"], d["actions"].shape[0])
    policy = None
    if name.startswith("greedy_"):
        kind = name[len("greedy_"):].replace("_e64", "")
        policy = lambda b: b.o.policy_greedy(kind)  # noqa: E731
    c = replay(d, be, policy=policy)
    assert c["steps"] == d["actions"].shape[1]
    assert c["info_exact"] == c["info_total"]


def test_oracle_csv_rows_match_reference(oracle_mod):
    from lbk8s.info import csv_rows
    d = load(os.path.join(GOLDEN, "edge_actions_multi.npz"))
    B, S = d["actions"].shape
    be = OracleBackend(oracle_mod, d["config"], B)
    be.init(d["t0"])
    from golden_driver import reset_arrays, step_arrays
    be.reset(reset_arrays(d, 0))
    k, ep = 1, 0
    for s in range(S):
        rt = reset_arrays(d, k) if (k < len(d["reset_at"]) and d["reset_at"][k] == s + 1) else None
        _, _, done, _, st = be.step(d["actions"][:, s], step_arrays(d, s), rt)
        if rt is not None:
            for b in range(B):
                res, upd = csv_rows(st[b], ep + 1)
                exp_r, exp_u = d["csv_results"][b, ep], d["csv_no_cost_updated"][b, ep]
                got_r = np.array(list(res.values())[:-1])
                got_u = np.array(list(upd.values())[:-1])
                np.testing.assert_array_equal(got_r, exp_r[:-1])
                np.testing.assert_array_equal(got_u, exp_u[:-1])
            k += 1
            ep += 1
    assert ep == d["csv_results"].shape[1]
