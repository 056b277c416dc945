#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ by RUNNING THE REFERENCE ENV.

Run here only (the reference never travels to the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_golden.py

What it does (SURVEY.md §8(c) "Procedure"):
  * imports /root/reference/envs/loadbalancer_k8s_env.py through the from-scratch
    `gym` stand-in in tests/golden/gym_standin (gym is not installed);
  * after __init__ (which seeds Generator(PCG64(SeedSequence(42))) —
    loadbalancer_k8s_env.py:128-129) swaps `env.np_random` for a recording proxy.
    Env instance 0 keeps the seed-42 stream; instances b>=1 wrap
    Generator(PCG64(1000+b)) so the batch carries distinct traces (every
    reference env is otherwise seeded 42 and identical);
  * drives the env like an SB3 VecEnv worker (reset, step, reset-on-done) with
    random / edge / greedy actions and records, per call:
      - the RNG draws the call consumed (the injected trace for the GPU kernel),
      - obs (float64), reward, done, the 13-key info, integer + float state,
      - the per-episode CSV rows written by utils.save_to_csv (cwd = tmp dir).
  * writes tests/golden/<scenario>.npz (compressed) + tests/golden/MANIFEST.json.

Fixtures are data (inputs + expected outputs); no reference source is stored.
"""
import csv
import importlib
import json
import os
import sys
import tempfile

import numpy as np

sys.dont_write_bytecode = True  # never write .pyc into /root/reference

HERE = os.path.dirname(os.path.abspath(__file__))
REF = os.environ.get("LBK8S_REFERENCE", "/root/reference")

INFO_KEYS = ["reward_step", "action", "reward", "ep_block_prob", "ep_accepted_requests",
             "avg_endpoint_latency", "avg_topology_latency", "avg_cost",
             "avg_cpu_endpoint_selected", "ep_intra_zone_percentage",
             "ep_inter_zone_percentage", "gini", "executionTime"]
CSV_KEYS = ["episode", "reward", "ep_block_prob", "ep_accepted_requests",
            "avg_endpoint_latency", "avg_topology_latency", "avg_cost",
            "avg_cpu_endpoint_selected", "ep_intra_zone_percentage",
            "ep_inter_zone_percentage", "gini", "execution_time"]

# name -> (constructor kwargs, n_env_instances, n_steps, action mode)
SCENARIOS = {
    "default_naive": (dict(), 4, 300, "random"),
    "cfg1_multi": (dict(num_endpoints=6, num_nodes=48, num_zones=12, reward_function="multi",
                        latency_weight=1.0, cpu_weight=0.0, gini_weight=0.0), 4, 300, "random"),
    "norej_multi": (dict(num_endpoints=6, rejection_allowed=False, reward_function="multi"),
                    4, 300, "random"),
    "e64_multi": (dict(num_endpoints=64, reward_function="multi", latency_weight=1.0,
                       cpu_weight=0.0, gini_weight=0.0), 2, 200, "random"),
    "latency": (dict(reward_function="latency"), 4, 300, "random"),
    "fairness_n30z5": (dict(num_nodes=30, num_zones=5, reward_function="fairness"), 4, 300, "random"),
    "edge_actions_multi": (dict(reward_function="multi"), 4, 300, "edge"),
    "short_ep_e3": (dict(num_endpoints=3, episode_length=7, reward_function="multi"), 4, 70, "random"),
    "e1_latency": (dict(num_endpoints=1, reward_function="latency"), 2, 120, "random"),
    "greedy_topo": (dict(num_endpoints=6, num_nodes=48, num_zones=12, reward_function="naive",
                         latency_weight=1.0, cpu_weight=0.0, gini_weight=0.0), 4, 300, "topo"),
    "greedy_zone_cpu": (dict(num_endpoints=6, num_nodes=48, num_zones=12, reward_function="naive",
                             latency_weight=1.0, cpu_weight=0.0, gini_weight=0.0), 4, 300, "zone_cpu"),
    "greedy_endpoint_cpu": (dict(num_endpoints=6, num_nodes=48, num_zones=12, reward_function="naive",
                                 latency_weight=1.0, cpu_weight=0.0, gini_weight=0.0), 4, 300,
                            "endpoint_cpu"),
    "greedy_endpoint_cpu_e64": (dict(num_endpoints=64, reward_function="naive"), 2, 200, "endpoint_cpu"),
}


class Recorder:
    """Proxy over a numpy Generator that logs every draw (copies arrays: the env
    aliases the uniform(size=E) result as endpoint_latency and mutates it,
    loadbalancer_k8s_env.py:328)."""

    def __init__(self, gen):
        self.gen = gen
        self.log = []

    def uniform(self, low=0.0, high=1.0, size=None):
        v = self.gen.uniform(low, high, size)
        self.log.append(("uniform", np.array(v, dtype=np.float64, copy=True)))
        return v

    def integers(self, low, high=None, size=None):
        v = self.gen.integers(low, high, size)
        self.log.append(("integers", (int(low), int(high)), int(v)))
        return v

    def exponential(self, scale=1.0, size=None):
        v = self.gen.exponential(scale, size)
        self.log.append(("exponential", float(v)))
        return v

    def take(self):
        out, self.log = self.log, []
        return out


def _req(log, i):
    (k1, x1), (k2, x2), (k3, _, r), (k4, _, n) = log[i:i + 4]
    assert (k1, k2, k3, k4) == ("exponential", "exponential", "integers", "integers"), log[i:i + 4]
    return x1, x2, r, n


def parse_step(log):
    assert len(log) == 4, [x[0] for x in log]
    return _req(log, 0)


def parse_reset(log, E, Z, N):
    i = 0
    assert log[i][0] == "uniform"
    lat0 = log[i][1]
    i += 1
    topo = [log[i + k][2] for k in range(Z * (Z - 1))]
    i += Z * (Z - 1)
    ntype, nzone = [], []
    for _ in range(N):
        ntype.append(log[i][2])
        nzone.append(log[i + 1][2])
        i += 2
    ncpu = [log[i + k][2] for k in range(N)]
    i += N
    enode = [log[i + k][2] for k in range(E)]
    i += E
    req = _req(log, i)
    i += 4
    assert i == len(log), (i, len(log))
    return dict(lat0=lat0, topo=np.array(topo), ntype=np.array(ntype), nzone=np.array(nzone),
                ncpu=np.array(ncpu), enode=np.array(enode), req=req)


def snapshot(env):
    Z = env.num_zones
    return dict(
        ep_node=np.asarray(env.endpoint_node, dtype=np.int64).copy(),
        ep_zone=np.asarray(env.endpoint_zone, dtype=np.int64).copy(),
        ep_cap=np.asarray(env.endpoint_zone_cpu_capacity, dtype=np.float64).copy(),
        ep_cpu=np.asarray(env.endpoint_cpu_usage_percentage, dtype=np.float64).copy(),
        ep_lat=np.asarray(env.endpoint_latency, dtype=np.float64).copy(),
        ep_topo=np.asarray(env.endpoint_topology_latency, dtype=np.float64).copy(),
        node_cpu=np.asarray(env.node_cpu_usage_percentage, dtype=np.float64).copy(),
        loads=np.asarray(env.avg_load_served, dtype=np.float64).copy(),
        topo=np.asarray(env.topology_latency_matrix, dtype=np.float64).reshape(Z, Z).copy(),
        counters=np.array([env.current_step, env.ep_accepted_requests, env.intra_zone_requests,
                           env.inter_zone_requests, int(bool(env.penalty))], dtype=np.int64),
        t=np.float64(env.current_time), dt=np.float64(env.dt),
        total_reward=np.float64(env.total_reward),
        req=np.array([int(env.endpoint_request.input_zone), int(env.endpoint_request.latency_threshold),
                      int(env.endpoint_request.input_node)], dtype=np.int64),
    )


def run_instance(mod, baselines, kw, b, n_steps, mode, tmpdir):
    # utils.save_to_csv writes into the cwd (loadbalancer_k8s_env.py:488-510): isolate it
    tmpdir = tempfile.mkdtemp(dir=tmpdir)
    cwd = os.getcwd()
    os.chdir(tmpdir)
    try:
        return _run_instance(mod, baselines, kw, b, n_steps, mode, tmpdir)
    finally:
        os.chdir(cwd)


def _run_instance(mod, baselines, kw, b, n_steps, mode, tmpdir):
    env = mod.LoadBalancerK8sEnv(file_results_name=os.path.join(tmpdir, f"res{b}"), **kw)
    if b > 0:
        env.np_random = np.random.Generator(np.random.PCG64(1000 + b))
    rec = Recorder(env.np_random)
    env.np_random = rec
    E, Z, N = env.num_endpoints, env.num_zones, env.num_nodes
    A = env.action_space.n
    arng = np.random.default_rng(1234 + b)
    out = dict(t0=np.float64(env.current_time), resets=[], reset_obs=[], reset_state=[],
               reset_at=[], steps=[])

    def do_reset(step_idx):
        obs = env.reset()
        out["resets"].append(parse_reset(rec.take(), E, Z, N))
        out["reset_obs"].append(np.asarray(obs, dtype=np.float64).copy())
        out["reset_state"].append(snapshot(env))
        out["reset_at"].append(step_idx)

    do_reset(0)
    for s in range(n_steps):
        mask = env.action_masks()
        if mode == "random":
            a = int(arng.integers(0, A))
        elif mode == "edge":
            u = arng.random()
            if u < 0.08:
                a = -int(arng.integers(1, E + 1))      # negative: Python wrap
            elif u < 0.14:
                a = E + 1 + int(arng.integers(0, 3))  # unrecognised: stale penalty
            elif u < 0.30:
                a = E                                  # reject
            else:
                a = int(arng.integers(0, E))
        elif mode == "topo":
            a = int(baselines.topology_greedy_policy(env, mask))
        elif mode == "zone_cpu":
            a = int(baselines.zone_cpu_greedy_policy(env, mask))
        elif mode == "endpoint_cpu":
            a = int(baselines.endpoint_cpu_greedy_policy(env, mask))
        else:
            raise ValueError(mode)
        obs, reward, done, info = env.step(a)
        x1, x2, r, n = parse_step(rec.take())
        st = snapshot(env)
        out["steps"].append(dict(action=a, x1=x1, x2=x2, r=r, n=n,
                                 obs=np.asarray(obs, dtype=np.float64).copy(),
                                 reward=float(reward), done=bool(done),
                                 info=np.array([float(info[k]) for k in INFO_KEYS]), state=st))
        if done:
            do_reset(s + 1)

    def read_csv(path):
        if not os.path.exists(path):
            return np.zeros((0, len(CSV_KEYS)))
        with open(path) as f:
            rows = [[float(x) for x in row] for row in csv.reader(f) if row]
        return np.array(rows, dtype=np.float64).reshape(-1, len(CSV_KEYS))

    out["csv_results"] = read_csv(os.path.join(tmpdir, f"res{b}.csv"))
    ncu = os.path.join(tmpdir, "no_cost_updated.csv")
    out["csv_no_cost_updated"] = read_csv(ncu)
    return env, out


def pack(name, kw, outs, env):
    B = len(outs)
    E, Z, N = env.num_endpoints, env.num_zones, env.num_nodes
    d = {}
    cfg = dict(num_endpoints=E, rejection_allowed=bool(env.rejection_allowed), num_zones=Z,
               num_nodes=N, arrival_rate_r=float(env.arrival_rate_r),
               call_duration_r=float(env.call_duration_r), episode_length=int(env.episode_length),
               reward_function=env.reward_function, latency_weight=float(env.latency_weight),
               cpu_weight=float(env.cpu_weight), gini_weight=float(env.gini_weight))
    d["config_json"] = np.array(json.dumps(cfg))
    d["t0"] = np.array([o["t0"] for o in outs])
    d["reset_at"] = np.array(outs[0]["reset_at"], dtype=np.int64)
    for o in outs:
        assert o["reset_at"] == outs[0]["reset_at"]
    for key in ["lat0", "topo", "ntype", "nzone", "ncpu", "enode"]:
        d["reset_" + key] = np.stack([np.stack([r[key] for r in o["resets"]]) for o in outs])
    d["reset_req_x"] = np.array([[[r["req"][0], r["req"][1]] for r in o["resets"]] for o in outs])
    d["reset_req_i"] = np.array([[[r["req"][2], r["req"][3]] for r in o["resets"]] for o in outs],
                                dtype=np.int64)
    d["reset_obs"] = np.stack([np.stack(o["reset_obs"]) for o in outs])
    for key in outs[0]["reset_state"][0]:
        d["reset_state_" + key] = np.stack([np.stack([s[key] for s in o["reset_state"]]) for o in outs])
    d["actions"] = np.array([[s["action"] for s in o["steps"]] for o in outs], dtype=np.int64)
    d["step_x"] = np.array([[[s["x1"], s["x2"]] for s in o["steps"]] for o in outs])
    d["step_i"] = np.array([[[s["r"], s["n"]] for s in o["steps"]] for o in outs], dtype=np.int64)
    d["obs"] = np.stack([np.stack([s["obs"] for s in o["steps"]]) for o in outs])
    d["reward"] = np.array([[s["reward"] for s in o["steps"]] for o in outs])
    d["done"] = np.array([[s["done"] for s in o["steps"]] for o in outs])
    d["info"] = np.stack([np.stack([s["info"] for s in o["steps"]]) for o in outs])
    for key in outs[0]["steps"][0]["state"]:
        d["state_" + key] = np.stack([np.stack([s["state"][key] for s in o["steps"]]) for o in outs])
    n_ep = min(len(o["csv_results"]) for o in outs)
    d["csv_results"] = np.stack([o["csv_results"][:n_ep] for o in outs])
    d["csv_no_cost_updated"] = np.stack([o["csv_no_cost_updated"][:n_ep] for o in outs])
    return d


def main():
    if not os.path.isdir(os.path.join(REF, "envs")):
        print(f"reference not found at {REF}; nothing to do")
        return 0
    sys.path.insert(0, os.path.join(HERE, "gym_standin"))
    sys.path.insert(0, REF)
    mod = importlib.import_module("envs.loadbalancer_k8s_env")
    baselines = importlib.import_module("envs.baselines")
    only = set(sys.argv[1:])
    manifest = {}
    with tempfile.TemporaryDirectory() as tmp:
        for name, (kw, B, S, mode) in SCENARIOS.items():
            if only and name not in only:
                continue
            outs, env = [], None
            for b in range(B):
                env, o = run_instance(mod, baselines, kw, b, S, mode, tmp)
                outs.append(o)
            d = pack(name, kw, outs, env)
            path = os.path.join(HERE, name + ".npz")
            np.savez_compressed(path, **d)
            manifest[name] = dict(kwargs=kw, envs=B, steps=S, actions=mode,
                                  bytes=os.path.getsize(path))
            print(f"{name}: B={B} S={S} resets={len(d['reset_at'])} -> {os.path.getsize(path)} B")
    if not only:
        with open(os.path.join(HERE, "MANIFEST.json"), "w") as f:
            json.dump(dict(reference="jpedro1992/gym-loadbalancing @ 2024-08-07 (/root/reference)",
                           generator="tests/golden/gen_golden.py", numpy=np.__version__,
                           scenarios=manifest), f, indent=1, sort_keys=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
