"""LBConfig — the LoadBalancerK8sEnv constructor arguments (loadbalancer_k8s_env.py:86-97).

Same names and defaults (:42-79).  Validation follows the reference's failure modes:
num_nodes < 24 / num_zones < 4 raise IndexError there (hard-coded draw ranges at
:205, :242, :354, :380) and are rejected here with IndexError; an unknown reward
function makes the reference's step() raise TypeError (`total_reward += None`,
:416, :566-567) and is rejected here with TypeError at construction.
"""
from dataclasses import asdict, dataclass

from . import _native
from .spaces import Box, Discrete


@dataclass(frozen=True)
class LBConfig:
    num_endpoints: int = 8
    rejection_allowed: bool = True
    num_zones: int = 4
    num_nodes: int = 24
    arrival_rate_r: float = 100
    call_duration_r: float = 1
    episode_length: int = 100
    reward_function: str = "naive"
    file_results_name: str = "loadbalancer_k8s_gym_results"
    latency_weight: float = 0.7
    cpu_weight: float = 0.1
    gini_weight: float = 0.2

    def __post_init__(self):
        if self.reward_function not in _native.LB_REWARD:
            raise TypeError(f"unrecognized reward function {self.reward_function!r} "
                            "(the reference's step() would add None to total_reward)")
        if self.num_zones < 4:
            raise IndexError("num_zones < 4: the reference draws zone ids in [0,4) "
                             "(loadbalancer_k8s_env.py:354)")
        if self.num_nodes < 24:
            raise IndexError("num_nodes < 24: the reference draws endpoint hosts in [0,24) "
                             "(loadbalancer_k8s_env.py:380)")
        if not 1 <= self.num_endpoints <= 256:
            raise ValueError("num_endpoints must be in [1, 256]")
        if self.num_nodes > 256:
            raise ValueError("num_nodes must be <= 256")
        if not 1 <= self.episode_length <= 1023:
            raise ValueError("episode_length must be in [1, 1023]")

    @property
    def num_actions(self):
        return self.num_endpoints + (1 if self.rejection_allowed else 0)

    @property
    def obs_rows(self):
        return self.num_actions

    def observation_space(self):
        return Box(low=1, high=500, shape=(self.obs_rows, 8))

    def action_space(self):
        return Discrete(self.num_actions)

    def to_c(self, seed=0, env_id_offset=0, auto_reset=True, trace=False, geometry="auto"):
        return _native.LBConfigC(
            self.num_endpoints, self.num_zones, self.num_nodes, self.episode_length,
            _native.LB_REWARD[self.reward_function], int(bool(self.rejection_allowed)),
            int(bool(auto_reset)), _native.LB_RNG_TRACE if trace else _native.LB_RNG_PHILOX,
            float(self.arrival_rate_r), float(self.call_duration_r), float(self.latency_weight),
            float(self.cpu_weight), float(self.gini_weight), int(seed) & (2**64 - 1),
            int(env_id_offset), _native.LB_GEOMETRY[geometry], 0)

    def as_dict(self):
        return asdict(self)
