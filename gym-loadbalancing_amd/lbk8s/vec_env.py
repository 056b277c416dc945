"""LBVecEnv — drop-in SB3-style VecEnv over the HIP kernels.

Replaces `SubprocVecEnv([lambda: LoadBalancerK8sEnv(...)] * 8)` + `VecMonitor` of
run.py:95-127 for the callers envs/ppo_deepset.py:145-189 and envs/dqn_deepset.py:116-156:

    reset() -> obs (B, R, 8) float32
    step(actions) -> (obs, rewards (B,) float32, dones (B,) bool, infos: sequence of dicts)
    step_async / step_wait, env_method("action_masks"), get_attr, num_envs,
    observation_space, action_space, close(), seed()

Semantics (SB3 VecEnv, documented there, not pinned by the reference's tests):
auto-reset on done; infos[i]["terminal_observation"] holds the pre-reset obs; with
monitor=True infos[i]["episode"] = {"r", "l", "t"} plus the info_keywords copied from
the final info, like VecMonitor, and with monitor_file=name every finished episode is
appended to name.monitor.csv in VecMonitor's layout (run.py:122 wraps the training envs
in VecMonitor(env, "vec_loadbalancer_k8s_gym_results", info_keywords)).  `infos` is
lazy: a dict is built only when indexed (per-env Python dicts for 10^6 envs would cost
more than the step itself).  seed(s) is applied at the next reset() (SB3's convention;
the reference's own env.seed raises TypeError, loadbalancer_k8s_env.py:128,569).

Every buffer is a torch tensor on the HIP device; calls are asynchronous on torch's
current stream.  With as_tensors=True the step returns those device tensors (zero
copy); otherwise numpy copies (the reference callers wrap them in torch.Tensor()).
"""
import ctypes as C
import csv
import json
import os
import time

import numpy as np

from . import _native
from .config import LBConfig
from .info import ST_ACC, ST_EPISODE, ST_LENGTH, ST_RETURN, csv_rows, step_info

# trace array name -> (dtype, per-env length key)
_TRACE_SPEC = {
    "t0": ("f8", None), "step_x1": ("f8", None), "step_x2": ("f8", None), "step_r": ("i4", None),
    "step_n": ("i4", None), "reset_lat0": ("f8", "E"), "reset_topo": ("i4", "ZZ"),
    "reset_ntype": ("i4", "N"), "reset_nzone": ("i4", "N"), "reset_ncpu": ("i4", "N"),
    "reset_enode": ("i4", "E"), "reset_x1": ("f8", None), "reset_x2": ("f8", None),
    "reset_r": ("i4", None), "reset_n": ("i4", None),
}


class LazyInfos:
    """Sequence of per-env info dicts, materialised on access."""

    def __init__(self, env, rewards, actions, dones, monitor_t):
        self._env, self._r, self._a, self._d = env, rewards, actions, dones
        self._t = monitor_t
        self._stats = None
        self._cache = {}

    def __len__(self):
        return self._env.num_envs

    def __iter__(self):
        for i in range(len(self)):
            yield self[i]

    def _host(self):
        if not isinstance(self._r, np.ndarray):
            self._r = self._r.cpu().numpy()
            self._a = self._a.cpu().numpy()
            self._d = self._d.cpu().numpy().astype(bool)

    def __getitem__(self, i):
        if isinstance(i, slice):
            return [self[k] for k in range(*i.indices(len(self)))]
        i = int(i)
        if i < 0:
            i += len(self)
        if i in self._cache:
            return self._cache[i]
        self._host()
        env = self._env
        if self._d[i] and env.auto_reset:  # ep_stats rows are written by the auto-reset
            st = env._host_ep_stats()[i]
        else:
            if self._stats is None:
                self._stats = env.stats().cpu().numpy()
            st = self._stats[i]
        info = step_info(st, float(self._r[i]), int(self._a[i]))
        if self._d[i] and env.auto_reset:
            info["terminal_observation"] = env._host_terminal_obs()[i]
            if env.monitor:  # (VecMonitor: the float32 running return)
                ep = {"r": float(env._host_ep_r32()[i]), "l": int(st[ST_LENGTH]),
                      "t": round(time.time() - env._t_start, 6)}
                for k in env.info_keywords:
                    ep[k] = info[k]
                info["episode"] = ep
        self._cache[i] = info
        return info


class _MonitorWriter:
    """VecMonitor's results file (SB3 ResultsWriter): a '#' JSON header line, then one row
    per finished episode: r, l, t (seconds since t_start) and the info keywords."""

    def __init__(self, filename, t_start, info_keywords):
        if not filename.endswith("monitor.csv"):
            filename = os.path.join(filename, "monitor.csv") if os.path.isdir(filename) else filename + ".monitor.csv"
        self.path = filename
        self.t_start = t_start
        self.keys = tuple(info_keywords)
        self.f = open(filename, "w", newline="")
        self.f.write("#" + json.dumps({"t_start": t_start, "env_id": "None"}) + "\n")
        self.w = csv.writer(self.f)
        self.w.writerow(["r", "l", "t"] + list(self.keys))
        self.f.flush()

    def write(self, rows, t):
        """rows: episode-log rows (lb_episode_log layout); t: host time of each row's step.
        'r' is VecMonitor's float32 running return."""
        for row, tt in zip(rows, t):
            info = step_info(row[:_native.LB_ST_K], float(row[_native.LB_EPLOG_REWARD]),
                             int(row[_native.LB_EPLOG_ACTION]))
            # VecMonitor writes its float32 running return as it stands (str of the float32,
            # no rounding; only the time is rounded to 6 places)
            r32 = np.float32(row[_native.LB_EPLOG_RET32])
            self.w.writerow([r32, int(row[ST_LENGTH]), round(tt - self.t_start, 6)]
                            + [info[k] for k in self.keys])
        self.f.flush()

    def close(self):
        self.f.close()


class LBVecEnv:
    """B vectorized LoadBalancerK8sEnv instances resident on one HIP device."""

    def __init__(self, num_envs, device=None, seed=0, env_id_offset=0, trace=False, t0=None,
                 auto_reset=True, as_tensors=False, monitor=False, info_keywords=(),
                 save_csv=False, monitor_file=None, geometry="auto", **env_kwargs):
        import torch
        self.torch = torch
        self.cfg = LBConfig(**env_kwargs)
        self.num_envs = int(num_envs)
        if self.num_envs < 1:
            raise ValueError("num_envs must be >= 1")
        self.device = torch.device(device if device is not None else "cuda")
        if self.device.type != "cuda":
            raise RuntimeError("LBVecEnv runs on a HIP device (there is no CPU fallback)")
        self.trace_mode = bool(trace)
        self.auto_reset = bool(auto_reset)
        self.as_tensors = bool(as_tensors)
        self.monitor = bool(monitor) or monitor_file is not None
        self.info_keywords = tuple(info_keywords)
        self.geometry = geometry
        self.save_csv = bool(save_csv)
        self.env_id_offset = int(env_id_offset)
        self.observation_space = self.cfg.observation_space()
        self.action_space = self.cfg.action_space()
        self._c = self.cfg.to_c(seed, env_id_offset, auto_reset, trace, geometry)
        self._pending_seed = None
        self._L = _native.lib()
        nbytes = C.c_uint64()
        _native.check(self._L.lb_state_bytes(C.byref(self._c), self.num_envs, C.byref(nbytes)))
        B, R = self.num_envs, self.cfg.obs_rows
        dev = self.device
        self.state = torch.zeros(int(nbytes.value), dtype=torch.uint8, device=dev)
        self.obs = torch.zeros((B, R, 8), dtype=torch.float32, device=dev)
        self.terminal_obs = torch.zeros((B, R, 8), dtype=torch.float32, device=dev)
        self.rewards = torch.zeros(B, dtype=torch.float32, device=dev)
        self.dones = torch.zeros(B, dtype=torch.uint8, device=dev)
        self.ep_stats = torch.zeros((B, _native.LB_ST_K), dtype=torch.float64, device=dev)
        self.actions = torch.zeros(B, dtype=torch.int32, device=dev)
        self._flags = torch.zeros(1, dtype=torch.int32, device=dev)
        self._trace_bufs = {}
        self._trace = _native.LBTraceC()
        self._pending = None
        self._reset_called = False
        self._episode_count = 0
        self._t_start = time.time()
        self._host_cache = {}
        self._monitor = _MonitorWriter(monitor_file, self._t_start, self.info_keywords) if monitor_file else None
        # the float64 rewards of the last lb_step, inside the state blob (lb_reward64): VecMonitor
        # adds them to its float32 returns with one rounding (lb_episode_log)
        ptr = C.c_void_p()
        _native.check(self._L.lb_reward64(self._ptr(self.state), C.byref(self._c), B, C.byref(ptr)))
        self._rew64 = ptr
        if self.monitor:  # VecMonitor: float32 running returns and the device episode log
            self._ret32 = torch.zeros(B, dtype=torch.float32, device=dev)
            self._ep_r32 = torch.zeros(B, dtype=torch.float32, device=dev)
            # an env finishes at most once per episode_length steps, so flushing every
            # min(64, L) steps never holds more than B rows
            self._log = torch.empty((B, _native.LB_EPLOG_W), dtype=torch.float64, device=dev)
            self._log_count = torch.zeros(1, dtype=torch.int32, device=dev)
            self._log_every = max(1, min(64, self.cfg.episode_length))
            self._log_times = []
        if self.trace_mode:
            if t0 is None:
                raise ValueError("trace mode needs t0 (current_time after __init__) per env")
            self._set_trace({"t0": t0})
        _native.check(self._L.lb_init(self._ptr(self.state), C.byref(self._c), B,
                                      C.byref(self._trace) if self.trace_mode else None, self._stream()))

    # ---- plumbing ---------------------------------------------------------------------------
    def _stream(self):
        return C.c_void_p(self.torch.cuda.current_stream(self.device).cuda_stream)

    @staticmethod
    def _ptr(t):
        return C.c_void_p(t.data_ptr()) if t is not None else None

    def _set_trace(self, arrays):
        """Validate and upload injected draws (trace mode); keeps device copies alive."""
        cfg, B = self.cfg, self.num_envs
        sizes = {None: 1, "E": cfg.num_endpoints, "N": cfg.num_nodes,
                 "ZZ": cfg.num_zones * (cfg.num_zones - 1)}
        for name, arr in arrays.items():
            dt, per = _TRACE_SPEC[name]
            a = np.ascontiguousarray(np.asarray(arr).reshape(B, -1), dtype=dt)
            if a.shape[1] != sizes[per]:
                raise ValueError(f"trace {name}: expected {sizes[per]} values per env, got {a.shape[1]}")
            self._validate_trace(name, a)
            t = self.torch.from_numpy(a.reshape(-1)).to(self.device)
            self._trace_bufs[name] = t
            setattr(self._trace, name, t.data_ptr())

    def _validate_trace(self, name, a):
        # the kernels index tables with these values: reject what the reference's numpy
        # generator could never have produced
        cfg = self.cfg
        lim = {"reset_nzone": (0, 3), "reset_ntype": (0, 4), "reset_ncpu": (0, 127),
               "reset_enode": (0, min(23, cfg.num_nodes - 1)), "reset_topo": (0, 511),
               "step_r": (0, 6), "reset_r": (0, 6), "step_n": (0, cfg.num_nodes - 1),
               "reset_n": (0, cfg.num_nodes - 1)}
        if name in lim:
            lo, hi = lim[name]
            if a.size and (a.min() < lo or a.max() > hi):
                raise ValueError(f"trace {name} outside [{lo}, {hi}]")
        if name == "reset_lat0" and a.size and (a.min() < 0 or a.max() >= 501):
            raise ValueError("trace reset_lat0 outside [0, 501)")

    def _host_ep_stats(self):
        if "ep_stats" not in self._host_cache:
            self._host_cache["ep_stats"] = self.ep_stats.cpu().numpy()
        return self._host_cache["ep_stats"]

    def _host_ep_r32(self):
        if "r32" not in self._host_cache:
            self._host_cache["r32"] = self._ep_r32.cpu().numpy()
        return self._host_cache["r32"]

    def _host_terminal_obs(self):
        if "term" not in self._host_cache:
            self._host_cache["term"] = self.terminal_obs.cpu().numpy()
        return self._host_cache["term"]

    def _out(self, t):
        return t if self.as_tensors else t.cpu().numpy()

    # ---- VecEnv API -----------------------------------------------------------------------------
    def reset(self, trace=None):
        """reset() of every env (loadbalancer_k8s_env.py:290-400) -> obs (B, R, 8) float32."""
        if self._pending_seed is not None:  # seed() takes effect here, for every env at once
            self._c.seed = self._pending_seed
            self._pending_seed = None
        if self.trace_mode:
            if trace is None:
                raise ValueError("trace mode: reset() needs the reset draws")
            self._set_trace({"reset_" + k: v for k, v in trace.items()})
        _native.check(self._L.lb_reset(self._ptr(self.state), C.byref(self._c), self.num_envs, None,
                                       self._ptr(self.obs),
                                       C.byref(self._trace) if self.trace_mode else None, self._stream()))
        self._reset_called = True
        return self._out(self.obs)

    def step_async(self, actions, trace=None, reset_trace=None):
        self._pending = (actions, trace, reset_trace)

    def step_wait(self):
        if self._pending is None:
            raise RuntimeError("step_wait() without step_async()")
        actions, trace, reset_trace = self._pending
        self._pending = None
        return self._step(actions, trace, reset_trace)

    def step(self, actions, trace=None, reset_trace=None):
        return self._step(actions, trace, reset_trace)

    def _step(self, actions, trace, reset_trace):
        torch = self.torch
        if not self._reset_called:
            # the reference raises TypeError here (node_type is a float array until reset)
            raise TypeError("step() called before reset()")
        if isinstance(actions, torch.Tensor):
            a = actions.reshape(-1).to(device=self.device, dtype=torch.int32)
        else:
            a = torch.from_numpy(np.ascontiguousarray(np.asarray(actions).reshape(-1), np.int32)).to(self.device)
        if a.numel() != self.num_envs:
            raise ValueError(f"expected {self.num_envs} actions, got {a.numel()}")
        self.actions.copy_(a)
        if self.trace_mode:
            if trace is None:
                raise ValueError("trace mode: step() needs the step draws")
            self._set_trace({"step_" + k: v for k, v in trace.items()})
            if reset_trace is not None:
                self._set_trace({"reset_" + k: v for k, v in reset_trace.items()})
        _native.check(self._L.lb_step(
            self._ptr(self.state), C.byref(self._c), self.num_envs, self._ptr(self.actions),
            self._ptr(self.obs), self._ptr(self.rewards), self._ptr(self.dones),
            self._ptr(self.terminal_obs), self._ptr(self.ep_stats),
            C.byref(self._trace) if self.trace_mode else None, self._stream()))
        self._host_cache = {}
        dones_b = self.dones.bool()
        infos = LazyInfos(self, self.rewards, self.actions, self.dones, self._t_start)
        if self.save_csv:
            self._write_csv()
        if self.monitor:
            self.record_episodes()
            self.flush_monitor()
        if self.as_tensors:
            return self.obs, self.rewards, dones_b, infos
        obs = self.obs.cpu().numpy()
        rew = self.rewards.cpu().numpy()
        dn = dones_b.cpu().numpy()
        infos._r, infos._a, infos._d = rew, self.actions.cpu().numpy(), dn
        return obs, rew, dn, infos

    def _write_csv(self):
        dn = self.dones.cpu().numpy().astype(bool)
        if not dn.any():
            return
        st = self._host_ep_stats()
        with open(self.cfg.file_results_name + ".csv", "a+", newline="") as f1, \
                open("no_cost_updated.csv", "a+", newline="") as f2:
            w1 = csv.DictWriter(f1, fieldnames=list(csv_rows(st[0], 0)[0].keys()))
            w2 = csv.DictWriter(f2, fieldnames=list(csv_rows(st[0], 0)[1].keys()))
            for i in np.flatnonzero(dn):
                self._episode_count += 1
                r1, r2 = csv_rows(st[i], int(st[i, ST_EPISODE]))
                w1.writerow(r1)
                w2.writerow(r2)

    def env_method(self, method_name, *args, indices=None, **kwargs):
        idx = self._indices(indices)
        if method_name == "action_masks":
            # loadbalancer_k8s_env.py:808-821: every action is always valid
            return [np.ones(self.cfg.num_actions, dtype=bool) for _ in idx]
        raise AttributeError(f"LBVecEnv has no env method {method_name!r}")

    def action_masks(self):
        """(B, A) bool device tensor, all True (the batched form of env_method('action_masks'))."""
        return self.torch.ones((self.num_envs, self.cfg.num_actions), dtype=self.torch.bool,
                               device=self.device)

    def get_attr(self, attr_name, indices=None):
        idx = self._indices(indices)
        if attr_name in _native.LB_FIELD:
            vals = self.field(attr_name).cpu().numpy()
            return [vals[i] for i in idx]
        v = getattr(self.cfg, attr_name)
        return [v for _ in idx]

    def set_attr(self, attr_name, value, indices=None):
        raise AttributeError("LBVecEnv attributes are device state; set them through reset()")

    def _indices(self, indices):
        if indices is None:
            return range(self.num_envs)
        if isinstance(indices, int):
            return [indices]
        return indices

    def seed(self, seed=None):
        """Re-key the Philox stream at the next reset() (SB3 VecEnv convention).

        Until then every env keeps its current key, auto-resets included: an episode never
        mixes two keys (the step may redraw the current episode's scenario from the key)."""
        self._pending_seed = int(seed or 0) & (2**64 - 1)
        return [seed] * self.num_envs

    def close(self):
        if self._monitor is not None:
            self.flush_monitor()
            self._monitor.close()
        self.state = None

    # ---- VecMonitor file ------------------------------------------------------------------------
    def record_episodes(self, dones=None, rewards=None, actions=None):
        """VecMonitor bookkeeping of the last vector step, on the device: the float32 running
        returns and, for the finished envs only, their rows appended to the episode log
        (lb_episode_log; nothing per env crosses to the host).  The device learners call this
        after every step_device with the buffers they passed it; the drop-in step() does it
        itself.  The host reads the log at flush_monitor (every min(64, L) steps)."""
        if not self.monitor:
            return
        d = self.dones if dones is None else dones
        r = self.rewards if rewards is None else rewards
        a = self.actions if actions is None else actions
        _native.check(self._L.lb_episode_log(
            self.num_envs, self._ptr(d), self._ptr(self.ep_stats), self._ptr(r), self._rew64, self._ptr(a),
            self._ptr(self._ret32), self._ptr(self._ep_r32), len(self._log_times), self._ptr(self._log),
            self.num_envs, self._ptr(self._log_count), self._stream()))
        self._log_times.append(time.time())
        if len(self._log_times) >= self._log_every:
            self.flush_monitor()

    def flush_monitor(self):
        """Write the logged episodes (one host sync): in step order, env order within a step."""
        if not self.monitor or not self._log_times:
            return
        n = int(self._log_count.item())
        if n > self.num_envs:
            raise RuntimeError(f"episode log overflow ({n} rows > {self.num_envs})")
        rows = self._log[:n].cpu().numpy() if n else np.zeros((0, _native.LB_EPLOG_W))
        order = np.lexsort((rows[:, _native.LB_EPLOG_ENV], rows[:, _native.LB_EPLOG_TAG]))
        rows = rows[order]
        if self._monitor is not None and n:
            t = [self._log_times[int(g)] for g in rows[:, _native.LB_EPLOG_TAG]]
            self._monitor.write(rows, t)
        self._log_count.zero_()
        self._log_times = []

    def reset_masked(self, mask):
        """reset() of the envs where mask (B,) is nonzero; the others keep their episode."""
        m = mask.to(device=self.device, dtype=self.torch.uint8).contiguous()
        _native.check(self._L.lb_reset(self._ptr(self.state), C.byref(self._c), self.num_envs, self._ptr(m),
                                       self._ptr(self.obs), None, self._stream()))

    # ---- framework extras (device-resident) -----------------------------------------------------
    def step_device(self, actions, obs_out=None, terminal_obs_out=None, reward_out=None,
                    done_out=None, ep_stats_out=None):
        """Launch one fused step on device tensors; no host sync, no infos.

        actions: (B,) int32 device tensor, or None: every env takes its uniform random action
        drawn inside the step kernel (the value policy("random") would return; Philox mode).
        obs_out / reward_out / done_out default to the env's own buffers; pass slices of a
        rollout ring to write there directly.
        """
        if not self._reset_called:
            raise TypeError("step() called before reset()")
        _native.check(self._L.lb_step(
            self._ptr(self.state), C.byref(self._c), self.num_envs, self._ptr(actions),
            self._ptr(obs_out if obs_out is not None else self.obs),
            self._ptr(reward_out if reward_out is not None else self.rewards),
            self._ptr(done_out if done_out is not None else self.dones),
            self._ptr(terminal_obs_out if terminal_obs_out is not None else self.terminal_obs),
            self._ptr(ep_stats_out if ep_stats_out is not None else self.ep_stats),
            C.byref(self._trace) if self.trace_mode else None, self._stream()))

    def rollout(self, kind, steps, obs_out=None, reward_out=None, done_out=None, actions_out=None,
                terminal_obs_out=None, ep_stats_out=None):
        """`steps` vector steps under an on-device policy ("topo" / "zone_cpu" /
        "endpoint_cpu" / "random") in one launch (lb_rollout): the same trajectory as
        `steps` x (policy(kind), step_device(actions)).  Step k's outputs go to slot k of
        obs_out (K, B, R, 8), reward_out (K, B), done_out (K, B) uint8, actions_out (K, B)
        int32 (each None = not written)."""
        if not self._reset_called:
            raise TypeError("step() called before reset()")
        if self.trace_mode:
            raise RuntimeError("rollout() draws from Philox; trace mode steps one call at a time")
        _native.check(self._L.lb_rollout(
            self._ptr(self.state), C.byref(self._c), self.num_envs, _native.LB_POLICY[kind], int(steps),
            self._ptr(obs_out), self._ptr(reward_out), self._ptr(done_out), self._ptr(actions_out),
            self._ptr(terminal_obs_out if terminal_obs_out is not None else self.terminal_obs),
            self._ptr(ep_stats_out if ep_stats_out is not None else self.ep_stats), self._stream()))

    def rollout_kernel(self, steps, outputs_all=True):
        """The kernel lb_rollout launches for `steps` vector steps with every output given
        (outputs_all) or not (lb_rollout_kernel; host only)."""
        k = C.c_int32(-1)
        _native.check(self._L.lb_rollout_kernel(C.byref(self._c), self.num_envs, int(steps), int(bool(outputs_all)),
                                                C.byref(k)))
        return _native.LB_ROLLOUT[k.value]

    def policy(self, kind, out=None):
        """Batched envs/baselines.py greedy policy or uniform random -> (B,) int32 device tensor."""
        out = out if out is not None else self.torch.empty(self.num_envs, dtype=self.torch.int32,
                                                           device=self.device)
        _native.check(self._L.lb_policy(self._ptr(self.state), C.byref(self._c), self.num_envs,
                                        _native.LB_POLICY[kind], self._ptr(out), self._stream()))
        return out

    def dqn_act(self, frag, obs, masks, ex, out):
        """lb_dqn_act: the DQN's explore decision for this vector step drawn on the device (ex:
        _native.LBDQNExploreC) and the actions into out -- every env's random action when
        exploring, else the greedy action of the Q network packed in frag."""
        R = obs.shape[1]
        _native.check(self._L.lb_dqn_act(frag.data_ptr(), obs.data_ptr(), self.num_envs, R, self._ptr(masks),
                                         self._ptr(self.state), C.byref(self._c), C.byref(ex), self._ptr(out),
                                         self._stream()))
        return out

    def dqn_step(self, frag, obs, masks, ex, actions, next_obs, reward, done, rb, pos_in, pos_out, ep_sum, ep_cnt):
        """lb_dqn_step: one DQN vector step -- dqn_act, step_device(actions, next_obs, reward, done)
        and the replay write (lb_replay_add into rb at the device slot *pos_in, obs <- next_obs,
        finished-episode sums) -- in one launch where the shape allows it (config 5's 4096 envs),
        else as those three launches; bit for bit the same either way."""
        self._dqn_guard()
        R = obs.shape[1]
        _native.check(self._L.lb_dqn_step(
            frag.data_ptr(), obs.data_ptr(), self.num_envs, R, self._ptr(masks), self._ptr(self.state),
            C.byref(self._c), C.byref(ex), self._ptr(actions), self._ptr(next_obs), self._ptr(reward), self._ptr(done),
            self._ptr(self.terminal_obs), self._ptr(self.ep_stats), rb.size, pos_in, pos_out, rb.obs.data_ptr(),
            rb.next_obs.data_ptr(), rb.actions.data_ptr(), rb.rewards.data_ptr(), rb.dones.data_ptr(),
            self._ptr(ep_sum), self._ptr(ep_cnt), self._stream()))
        return actions

    def _dqn_guard(self):
        """step_device's checks for the DQN step entry points (they step the env too).  A launch
        captured into a HIP graph does not run: the learner captures its period graphs before
        its reset(), and the replays follow the reset."""
        if not self._reset_called and not self.torch.cuda.is_current_stream_capturing():
            raise TypeError("step() called before reset()")
        if self.trace_mode:
            raise RuntimeError("the DQN step draws its exploration and actions from Philox; trace mode steps "
                               "one call at a time (dqn_act + step)")

    def dqn_steps_supported(self, R):
        """Whether lb_dqn_steps (several DQN vector steps in one launch) covers this env with
        R-row observations."""
        return bool(self._L.lb_dqn_steps_supported(C.byref(self._c), self.num_envs, R))

    def dqn_steps(self, n, frag, obs, masks, ex, actions, next_obs, reward, done, rb, pos_in, pos_out, ep_sum, ep_cnt,
                  sync):
        """lb_dqn_steps: n DQN vector steps (dqn_step n times, the explore draw, replay slot and
        step counter advancing per step) in one launch; pos_in / pos_out and the explore
        struct's step words may coincide.  sync: a device int32 tensor holding 0."""
        self._dqn_guard()
        R = obs.shape[1]
        _native.check(self._L.lb_dqn_steps(
            frag.data_ptr(), obs.data_ptr(), self.num_envs, R, self._ptr(masks), self._ptr(self.state),
            C.byref(self._c), C.byref(ex), self._ptr(actions), self._ptr(next_obs), self._ptr(reward), self._ptr(done),
            self._ptr(self.terminal_obs), self._ptr(self.ep_stats), rb.size, pos_in, pos_out, rb.obs.data_ptr(),
            rb.next_obs.data_ptr(), rb.actions.data_ptr(), rb.rewards.data_ptr(), rb.dones.data_ptr(),
            self._ptr(ep_sum), self._ptr(ep_cnt), int(n), sync.data_ptr(), self._stream()))
        return actions

    def field(self, name):
        """Env attribute as a float64 device tensor: (B, E) or (B,)."""
        shape = (self.num_envs,) if name in _native.PER_ENV_FIELDS else (self.num_envs, self.cfg.num_endpoints)
        out = self.torch.empty(shape, dtype=self.torch.float64, device=self.device)
        _native.check(self._L.lb_get_field(self._ptr(self.state), C.byref(self._c), self.num_envs,
                                           _native.LB_FIELD[name], self._ptr(out), self._stream()))
        return out

    def stats(self):
        """Current per-env accumulators (B, 16) float64 (info.py ST_* layout)."""
        out = self.torch.empty((self.num_envs, _native.LB_ST_K), dtype=self.torch.float64,
                               device=self.device)
        _native.check(self._L.lb_get_stats(self._ptr(self.state), C.byref(self._c), self.num_envs,
                                           self._ptr(out), self._stream()))
        return out

    def status(self):
        _native.check(self._L.lb_status(self._ptr(self.state), C.byref(self._c), self.num_envs,
                                        self._ptr(self._flags), self._stream()))
        return int(self._flags.item())

    def accepted_fraction(self):
        st = self.stats()
        return (st[:, ST_ACC] / st[:, ST_LENGTH].clamp(min=1)).mean().item()

    def __repr__(self):
        return f"LBVecEnv(num_envs={self.num_envs}, {self.cfg})"
