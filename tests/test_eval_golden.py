"""The evaluation loop of run_test_deepset.py against fixtures
recorded from the reference env + the reference networks (tests/golden/gen_golden_eval.py):
ONE env, sequential greedy episodes, DummyVecEnv's auto-reset then the loop's reset().

* CPU: the C oracle env (trace mode) + the framework's deep-sets modules on torch CPU,
  driven by the same loop, reproduce every action, reward and VecMonitor return;
* GPU: lbk8s.evaluate.run_sequential (LBVecEnv in trace mode + the fused forward kernel).
Actions and dones exact, rewards bit-exact as float32, VecMonitor's float32 return exact,
the float64 episode return exact; info means within one 2-dp unit (statistics.mean).
"""
import json
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from nn_helpers import state_dict_from


def load_eval(alg):
    d = dict(np.load(os.path.join(GOLDEN, f"eval_{alg}.npz")))
    d["config"] = json.loads(str(d["config_json"]))
    d["cols"] = json.loads(str(d["episode_cols"]))
    return d


class Draws:
    """The fixture's reference draws in call order (resets and steps)."""

    def __init__(self, d, batched=False):
        self.d, self.r, self.s, self.batched = d, 0, 0, batched

    def next_reset(self):
        d, k = self.d, self.r
        self.r += 1
        a = dict(lat0=d["reset_lat0"][k], topo=d["reset_topo"][k], ntype=d["reset_ntype"][k],
                 nzone=d["reset_nzone"][k], ncpu=d["reset_ncpu"][k], enode=d["reset_enode"][k],
                 x1=d["reset_req_x"][k, 0], x2=d["reset_req_x"][k, 1], r=d["reset_req_i"][k, 0],
                 n=d["reset_req_i"][k, 1])
        return {k: np.asarray(v)[None] for k, v in a.items()}

    def next_step(self):
        d, k = self.d, self.s
        self.s += 1
        a = dict(x1=d["step_x"][k, 0], x2=d["step_x"][k, 1], r=d["step_i"][k, 0], n=d["step_i"][k, 1])
        return {k: np.asarray(v)[None] for k, v in a.items()}


def agent_for(d, device):
    from lbk8s.deepsets import DeepSetAgent, DQNDeepSetAgent
    agent = (DeepSetAgent if str(d["alg"]) == "ppo" else DQNDeepSetAgent)(8).to(device)
    agent.load_state_dict(state_dict_from(d, "agent__"))
    return agent.eval()


def check_episodes(d, res):
    n = len(d["episodes"])
    ep = d["episodes"]
    np.testing.assert_array_equal(res["actions"], d["actions"])
    np.testing.assert_array_equal(np.asarray(res["rewards"], np.float32), d["rewards"].astype(np.float32))
    np.testing.assert_array_equal(res["dones"], d["dones"])
    np.testing.assert_array_equal(np.asarray(res["r"], np.float32), ep[:, 0].astype(np.float32))
    np.testing.assert_array_equal(res["l"], ep[:, 1])
    np.testing.assert_array_equal(res["total_reward"], ep[:, 2])
    cols = d["cols"]
    for key in ("reward_step", "action", "reward", "ep_block_prob", "ep_accepted_requests",
                "avg_endpoint_latency", "avg_topology_latency", "avg_cost", "avg_cpu_endpoint_selected",
                "ep_intra_zone_percentage", "ep_inter_zone_percentage", "gini"):
        np.testing.assert_array_equal(res[key], ep[:, cols.index(key)], err_msg=key)
    assert len(res["r"]) == n


@pytest.mark.parametrize("alg", ["ppo", "dqn"])
def test_eval_loop_oracle_cpu(oracle_mod, alg):
    """The fixture's loop semantics on the CPU: oracle env + torch CPU networks."""
    from lbk8s.deepsets import DeepSetAgent, masked_logits
    from lbk8s.info import ST_RETURN, step_info
    d = load_eval(alg)
    cfg = d["config"]
    agent = agent_for(d, "cpu")
    head = agent.actor if isinstance(agent, DeepSetAgent) else agent.q_network
    orc = oracle_mod.OracleBatch(cfg, 1, trace=True, auto_reset=True)
    orc.init(np.array([d["t0"]]))
    draws = Draws(d)
    L = cfg["episode_length"]
    res = {k: [] for k in ("actions", "rewards", "dones", "r", "l", "total_reward")}
    info_res = {}
    for _ in range(len(d["episodes"])):
        obs = orc.reset(trace=oracle_mod.ResetTrace(**_rt(draws.next_reset())))
        done, ret32, length = False, np.float32(0), 0
        while not done:
            with torch.no_grad():
                lg = masked_logits(head(torch.from_numpy(obs)), torch.ones((1, obs.shape[1]), dtype=torch.bool))
                a = int(torch.argmax(lg[0]))
            st = draws.next_step()
            rt = draws.next_reset() if length + 1 == L else None
            obs, r, dn, _, stats = orc.step(np.array([a], np.int32), oracle_mod.StepTrace(**_st(st)),
                                            oracle_mod.ResetTrace(**_rt(rt)) if rt is not None else None)
            done = bool(dn[0])
            ret32 = np.float32(ret32 + np.float32(r[0]))
            length += 1
            res["actions"].append(a)
            res["rewards"].append(float(r[0]))
            res["dones"].append(done)
            if done:
                res["r"].append(float(ret32))
                res["l"].append(length)
                res["total_reward"].append(float(stats[0, ST_RETURN]))
                for k, v in step_info(stats[0], float(r[0]), a).items():
                    info_res.setdefault(k, []).append(v)
    res = {k: np.asarray(v) for k, v in res.items()}
    res.update({k: np.asarray(v) for k, v in info_res.items()})
    check_episodes(d, res)


def _rt(a):
    return dict(lat0=a["lat0"], topo=a["topo"], ntype=a["ntype"], nzone=a["nzone"], ncpu=a["ncpu"],
                enode=a["enode"], x1=a["x1"], x2=a["x2"], r=a["r"], n=a["n"])


def _st(a):
    return dict(x1=a["x1"], x2=a["x2"], r=a["r"], n=a["n"])


@pytest.mark.gpu
@pytest.mark.parametrize("alg", ["ppo", "dqn"])
def test_eval_run_sequential_gpu(alg, tmp_path):
    """lbk8s.evaluate.run_sequential: LBVecEnv (trace mode) + the fused greedy forward."""
    from lbk8s import LBVecEnv
    from lbk8s.evaluate import run_sequential
    d = load_eval(alg)
    env = LBVecEnv(1, trace=True, t0=np.array([d["t0"]]), as_tensors=True, **d["config"])
    res = run_sequential(agent_for(d, "cuda"), len(d["episodes"]), env, draws=Draws(d),
                         monitor_path=str(tmp_path / "m.monitor.csv"))
    check_episodes(d, res)
    rows = open(tmp_path / "m.monitor.csv").read().splitlines()
    assert rows[0].startswith("#") and len(rows) == 2 + len(d["episodes"])
