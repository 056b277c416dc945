"""Observation / action space descriptors (gym is not a dependency).

Same shape/dtype/n as the reference's gym.spaces (loadbalancer_k8s_env.py:138-174):
Box(low=1, high=500, shape=(E[+1], 8), float32) and Discrete(E[+1]).
"""
import numpy as np


class Box:
    def __init__(self, low, high, shape, dtype=np.float32):
        self.low, self.high = low, high
        self.shape = tuple(shape)
        self.dtype = np.dtype(dtype)

    def __repr__(self):
        return f"Box({self.low}, {self.high}, {self.shape}, {self.dtype})"


class Discrete:
    def __init__(self, n):
        self.n = int(n)
        self.shape = ()
        self.dtype = np.dtype(np.int64)

    def sample(self, rng=None):
        rng = rng or np.random.default_rng()
        return int(rng.integers(0, self.n))

    def __repr__(self):
        return f"Discrete({self.n})"
