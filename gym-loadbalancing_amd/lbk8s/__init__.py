"""lbk8s — MI355X-native vectorized LoadBalancerK8sEnv (gym-loadbalancing hot path).

Host side in Python over a C-ABI HIP library (liblbk8s.so, include/lbk8s.h).
Importing the package never touches the GPU; the native library is loaded on
first use and its absence raises (there is no CPU fallback).
"""
from .info import INFO_KEYS, step_info, csv_rows  # noqa: F401

__all__ = ["INFO_KEYS", "step_info", "csv_rows", "LBConfig", "LBVecEnv", "LoadBalancerK8sEnv"]


def __getattr__(name):
    if name == "LBConfig":
        from .config import LBConfig
        return LBConfig
    if name == "LBVecEnv":
        from .vec_env import LBVecEnv
        return LBVecEnv
    if name == "LoadBalancerK8sEnv":
        from .env import LoadBalancerK8sEnv
        return LoadBalancerK8sEnv
    raise AttributeError(name)
