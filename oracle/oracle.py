"""ctypes front-end of the C oracle (oracle/lbk8s_oracle.c) — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this.
The product package (gym-loadbalancing_amd/lbk8s) never does.
"""
import ctypes as C
import os
import subprocess
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "liblbk8s_oracle.so")

REWARD_IDS = {"naive": 0, "latency": 1, "fairness": 2, "multi": 3}
ST_K = 16
FIELDS = dict(ep_lat=0, ep_cpu=1, ep_topo=2, ep_cap=3, ep_zone=4, ep_node=5, loads=6, t=7,
              step=8, req_zone=9, req_thr=10, dt=11, node_cpu=12)


class _Cfg(C.Structure):
    _fields_ = [("num_endpoints", C.c_int32), ("num_zones", C.c_int32), ("num_nodes", C.c_int32),
                ("episode_length", C.c_int32), ("reward_fn", C.c_int32),
                ("rejection_allowed", C.c_int32), ("auto_reset", C.c_int32), ("rng_mode", C.c_int32),
                ("arrival_rate", C.c_double), ("call_duration", C.c_double),
                ("latency_weight", C.c_double), ("cpu_weight", C.c_double),
                ("gini_weight", C.c_double), ("seed", C.c_uint64), ("env_id_offset", C.c_int64)]


class _StepTrace(C.Structure):
    _fields_ = [("x1", C.c_void_p), ("x2", C.c_void_p), ("r", C.c_void_p), ("n", C.c_void_p)]


class _ResetTrace(C.Structure):
    _fields_ = [("lat0", C.c_void_p), ("topo", C.c_void_p), ("ntype", C.c_void_p),
                ("nzone", C.c_void_p), ("ncpu", C.c_void_p), ("enode", C.c_void_p),
                ("x1", C.c_void_p), ("x2", C.c_void_p), ("r", C.c_void_p), ("n", C.c_void_p)]


_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        L.orc_create.restype = C.c_void_p
        L.orc_create.argtypes = [C.POINTER(_Cfg), C.c_int64]
        L.orc_destroy.argtypes = [C.c_void_p]
        L.orc_init.argtypes = [C.c_void_p, C.c_void_p]
        L.orc_reset.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.POINTER(_ResetTrace)]
        L.orc_step.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                               C.c_void_p, C.c_void_p, C.POINTER(_StepTrace), C.POINTER(_ResetTrace)]
        L.orc_get_stats.argtypes = [C.c_void_p, C.c_void_p]
        L.orc_last_reward64.argtypes = [C.c_void_p, C.c_void_p]
        L.orc_policy_greedy.argtypes = [C.c_void_p, C.c_int, C.c_void_p]
        L.orc_policy_random.argtypes = [C.c_void_p, C.c_void_p]
        L.orc_get_field.argtypes = [C.c_void_p, C.c_int, C.c_void_p]
        L.orc_num_threads.restype = C.c_int
        L.orc_philox_r.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_int32, C.c_void_p]
        L.orc_philox_rounds.restype = C.c_int32
        L.orc_log.restype = C.c_double
        L.orc_log.argtypes = [C.c_double]
        L.orc_set_seed.argtypes = [C.c_void_p, C.c_uint64]
        L.orc_dqn_explore.restype = C.c_int32
        L.orc_dqn_explore.argtypes = [C.c_uint64, C.c_double, C.c_double, C.c_double, C.c_int64]
        L.orc_replay_sample.argtypes = [C.c_uint64, C.c_int64, C.c_int64, C.c_int64, C.c_int32, C.c_void_p,
                                        C.c_void_p]
        _lib = L
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def _c(a, dt):
    return np.ascontiguousarray(a, dtype=dt)


class ResetTrace:
    """One reset call's draws for all B envs (arrays with leading B)."""

    def __init__(self, lat0, topo, ntype, nzone, ncpu, enode, x1, x2, r, n):
        self.arrays = [_c(lat0, np.float64), _c(topo, np.int32), _c(ntype, np.int32),
                       _c(nzone, np.int32), _c(ncpu, np.int32), _c(enode, np.int32),
                       _c(x1, np.float64), _c(x2, np.float64), _c(r, np.int32), _c(n, np.int32)]

    def c(self):
        return _ResetTrace(*[_p(a) for a in self.arrays])


class StepTrace:
    def __init__(self, x1, x2, r, n):
        self.arrays = [_c(x1, np.float64), _c(x2, np.float64), _c(r, np.int32), _c(n, np.int32)]

    def c(self):
        return _StepTrace(*[_p(a) for a in self.arrays])


class OracleBatch:
    """B independent reference envs, batched (trace- or Philox-driven)."""

    def __init__(self, cfg, num_envs, trace=False, auto_reset=True, seed=0, env_id_offset=0):
        self.cfg = dict(cfg)
        self.B = int(num_envs)
        self.E = int(cfg.get("num_endpoints", 8))
        self.rej = bool(cfg.get("rejection_allowed", True))
        self.R = self.E + (1 if self.rej else 0)
        self.N = int(cfg.get("num_nodes", 24))
        c = _Cfg(self.E, int(cfg.get("num_zones", 4)), self.N, int(cfg.get("episode_length", 100)),
                 REWARD_IDS[cfg.get("reward_function", "naive")], int(self.rej), int(auto_reset),
                 int(trace), float(cfg.get("arrival_rate_r", 100)), float(cfg.get("call_duration_r", 1)),
                 float(cfg.get("latency_weight", 0.7)), float(cfg.get("cpu_weight", 0.1)),
                 float(cfg.get("gini_weight", 0.2)), int(seed) & (2**64 - 1), int(env_id_offset))
        self._cfg = c
        self.h = lib().orc_create(C.byref(c), self.B)

    def __del__(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib.orc_destroy(self.h)
            self.h = None

    def init(self, t0=None):
        t0 = None if t0 is None else _c(t0, np.float64)
        lib().orc_init(self.h, _p(t0))

    def reset(self, mask=None, trace=None):
        obs = np.zeros((self.B, self.R, 8), np.float32)
        mask = None if mask is None else _c(mask, np.uint8)
        tr = C.byref(trace.c()) if trace is not None else None
        lib().orc_reset(self.h, _p(mask), _p(obs), tr)
        return obs

    def step(self, actions, step_trace=None, reset_trace=None):
        a = _c(actions, np.int32)
        obs = np.zeros((self.B, self.R, 8), np.float32)
        term = np.zeros((self.B, self.R, 8), np.float32)
        rew = np.zeros(self.B, np.float32)
        done = np.zeros(self.B, np.uint8)
        st = np.zeros((self.B, ST_K), np.float64)
        s_tr = C.byref(step_trace.c()) if step_trace is not None else None
        r_tr = C.byref(reset_trace.c()) if reset_trace is not None else None
        lib().orc_step(self.h, _p(a), _p(obs), _p(rew), _p(done), _p(term), _p(st), s_tr, r_tr)
        return obs, rew, done.astype(bool), term, st

    def stats(self):
        st = np.zeros((self.B, ST_K), np.float64)
        lib().orc_get_stats(self.h, _p(st))
        return st

    def last_reward64(self):
        """(B,) float64: each env's reward of the last step() before the float32 cast."""
        out = np.zeros(self.B, np.float64)
        lib().orc_last_reward64(self.h, _p(out))
        return out

    def field(self, name):
        n = {"t": 1, "step": 1, "req_zone": 1, "req_thr": 1, "dt": 1}.get(name)
        size = self.B if n else (self.B * self.N if name == "node_cpu" else self.B * self.E)
        out = np.zeros(size, np.float64)
        lib().orc_get_field(self.h, FIELDS[name], _p(out))
        return out if n else out.reshape(self.B, -1)

    def policy_greedy(self, kind):
        out = np.zeros(self.B, np.int32)
        lib().orc_policy_greedy(self.h, {"topo": 0, "zone_cpu": 1, "endpoint_cpu": 2}[kind], _p(out))
        return out

    def policy_random(self):
        out = np.zeros(self.B, np.int32)
        lib().orc_policy_random(self.h, _p(out))
        return out

    def set_seed(self, seed):
        lib().orc_set_seed(self.h, int(seed) & (2**64 - 1))


def _subproc_worker(conn, cfg, wid):
    """One SubprocVecEnv-style worker: a single oracle env, one Pipe round trip per step."""
    os.environ["OMP_NUM_THREADS"] = "1"
    orc = OracleBatch(cfg, 1, trace=False, seed=0, env_id_offset=wid)
    orc.init()
    conn.send(orc.reset())
    while True:
        a = conn.recv()
        if a is None:
            break
        obs, rew, done, _, _ = orc.step(np.asarray([a], np.int32))
        conn.send((obs, rew, done))
    conn.close()


def subproc_vecenv_rate(cfg, workers, seconds=5.0):
    """env-steps/s of the reference's process pattern (run.py:114-122: SubprocVecEnv, one
    env per worker process, actions out and (obs, reward, done) back over a Pipe every
    vector step), with the oracle's single env in each worker instead of the Python env."""
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    pipes, procs = [], []
    for w in range(workers):
        a, b = ctx.Pipe()
        p = ctx.Process(target=_subproc_worker, args=(b, dict(cfg), w), daemon=True)
        p.start()
        pipes.append(a)
        procs.append(p)
    try:
        for c in pipes:
            c.recv()
        A = int(cfg.get("num_endpoints", 8)) + (1 if cfg.get("rejection_allowed", True) else 0)
        rng = np.random.default_rng(0)
        steps = 0
        t0 = time.perf_counter()
        while True:
            acts = rng.integers(0, A, size=workers)
            for c, a in zip(pipes, acts):
                c.send(int(a))
            _ = np.stack([c.recv()[0] for c in pipes])
            steps += 1
            el = time.perf_counter() - t0
            if el >= seconds:
                break
    finally:
        for c in pipes:
            c.send(None)
        for p in procs:
            p.join(timeout=10)
    return dict(value=workers * steps / el, unit="env-steps/s", workers=workers, kind="port",
                sample=f"SubprocVecEnv pattern: {workers} worker processes x 1 oracle env, Pipe per "
                       f"vector step, {steps} vector steps ({el:.1f} s)")


def philox(ctr, key, rounds=None):
    """Philox4x32-R block; rounds None = the draw map's round count (philox_rounds())."""
    out = np.zeros(4, np.uint32)
    c = np.asarray(ctr, np.uint32)
    r = philox_rounds() if rounds is None else int(rounds)
    lib().orc_philox_r(_p(c), int(key[0]), int(key[1]), r, _p(out))
    return out


def philox_rounds():
    return int(lib().orc_philox_rounds())


def fd_log(x):
    return lib().orc_log(float(x))


def num_threads():
    return lib().orc_num_threads()


def dqn_explore(seed, start_e, slope, end_e, t):
    """The DQN's explore decision at vector step t (lb_dqn_act's draw)."""
    return int(lib().orc_dqn_explore(int(seed), float(start_e), float(slope), float(end_e), int(t)))


def replay_sample(seed, t, upper, n_envs, batch):
    """(slot, env) int64 arrays of lb_replay_sample's draws at counter t."""
    slot = np.zeros(batch, np.int64)
    env = np.zeros(batch, np.int64)
    lib().orc_replay_sample(int(seed), int(t), int(upper), int(n_envs), int(batch), _p(slot), _p(env))
    return slot, env


# ---- golden fixture helpers ---------------------------------------------------------------

def golden_reset_trace(d, k):
    """Reset call k of a golden fixture as a ResetTrace (all B instances)."""
    return ResetTrace(d["reset_lat0"][:, k], d["reset_topo"][:, k], d["reset_ntype"][:, k],
                      d["reset_nzone"][:, k], d["reset_ncpu"][:, k], d["reset_enode"][:, k],
                      d["reset_req_x"][:, k, 0], d["reset_req_x"][:, k, 1],
                      d["reset_req_i"][:, k, 0], d["reset_req_i"][:, k, 1])


def golden_step_trace(d, s):
    return StepTrace(d["step_x"][:, s, 0], d["step_x"][:, s, 1], d["step_i"][:, s, 0],
                     d["step_i"][:, s, 1])
