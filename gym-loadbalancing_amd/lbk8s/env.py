"""LoadBalancerK8sEnv — the reference's single-env Gym contract on a one-env device batch.

Mirrors /root/reference/envs/loadbalancer_k8s_env.py:82-821 for scripts that drive one
env directly (run_baselines.py:37-78): same constructor keywords, reset() -> obs,
step(action) -> (obs, reward, done, info), action_masks(), and the public attributes the
greedy policies read (baselines.py:13,24,35).  No auto-reset: like the reference, the
caller resets after done.  At episode end the two CSV rows of :488-510 are appended to
`<file_results_name>.csv` and `no_cost_updated.csv` in the working directory (as the
reference does) unless save_csv=False.

Observations are float32 (the Box dtype of :139-148; the reference returns float64
arrays that every consumer casts).  For throughput use LBVecEnv.
"""
import csv
import time

import numpy as np

from .info import ST_EPISODE, csv_rows, step_info
from .vec_env import LBVecEnv

_ATTRS = ("endpoint_latency", "endpoint_cpu_usage_percentage", "endpoint_topology_latency",
          "endpoint_zone_cpu_capacity", "endpoint_zone", "endpoint_node", "avg_load_served")


class LoadBalancerK8sEnv:
    metadata = {"render.modes": ["human", "ansi", "array"]}

    def __init__(self, num_endpoints=8, rejection_allowed=True, num_zones=4, num_nodes=24,
                 arrival_rate_r=100, call_duration_r=1, episode_length=100, reward_function="naive",
                 file_results_name="loadbalancer_k8s_gym_results", latency_weight=0.7, cpu_weight=0.1,
                 gini_weight=0.2, device=None, seed=42, save_csv=True, trace=False, t0=None):
        self._vec = LBVecEnv(1, device=device, seed=seed, auto_reset=False, trace=trace, t0=t0,
                             num_endpoints=num_endpoints, rejection_allowed=rejection_allowed,
                             num_zones=num_zones, num_nodes=num_nodes, arrival_rate_r=arrival_rate_r,
                             call_duration_r=call_duration_r, episode_length=episode_length,
                             reward_function=reward_function, file_results_name=file_results_name,
                             latency_weight=latency_weight, cpu_weight=cpu_weight, gini_weight=gini_weight)
        cfg = self._vec.cfg
        self.name = "loadbalancer_k8s_gym"
        self.num_endpoints, self.num_zones, self.num_nodes = num_endpoints, num_zones, num_nodes
        self.rejection_allowed = rejection_allowed
        self.arrival_rate_r, self.call_duration_r = arrival_rate_r, call_duration_r
        self.episode_length, self.reward_function = episode_length, reward_function
        self.latency_weight, self.cpu_weight, self.gini_weight = latency_weight, cpu_weight, gini_weight
        self.num_actions = cfg.num_actions
        self.observation_space = self._vec.observation_space
        self.action_space = self._vec.action_space
        self.file_results = file_results_name + ".csv"
        self.save_csv = save_csv
        self.execution_time = 0.0
        self._time_start = 0.0
        self.info = {}

    # ---- Gym contract ------------------------------------------------------------------
    def reset(self, trace=None):
        obs = self._vec.reset(trace=trace)
        return obs[0]

    def step(self, action, trace=None):
        if int(self.current_step) == 1:
            self._time_start = time.time()  # :404-405
        obs, rew, done, _ = self._vec.step(np.array([action], dtype=np.int32), trace=trace)
        st = self._vec.stats().cpu().numpy()[0]
        d = bool(done[0])
        reward = float(rew[0])
        self.info = step_info(st, reward, action, self.execution_time)
        if d:
            self.execution_time = time.time() - self._time_start
            if self.save_csv:
                self._save_csv(st)
        return obs[0], reward, d, self.info

    def action_masks(self):
        return np.ones(self.num_actions, dtype=bool)  # :808-821

    def seed(self, seed=None):
        return self._vec.seed(seed)

    def render(self, mode="human", close=False):
        return None

    def close(self):
        self._vec.close()

    def _save_csv(self, st):
        res, upd = csv_rows(st, int(st[ST_EPISODE]), self.execution_time)
        for path, row in ((self.file_results, res), ("no_cost_updated.csv", upd)):
            with open(path, "a+", newline="") as f:
                csv.DictWriter(f, fieldnames=list(row.keys())).writerow(row)

    # ---- attributes read by envs/baselines.py and friends -------------------------------------
    def __getattr__(self, name):
        if name in _ATTRS:
            return self._vec.field(name).cpu().numpy()[0]
        if name in ("current_step", "current_time"):
            v = self._vec.field(name).cpu().numpy()[0]
            return int(v) if name == "current_step" else float(v)
        raise AttributeError(name)
