"""Minimal from-scratch `gym` stand-in used ONLY by tests/golden/gen_golden.py.

gym is not installed in this container. The reference env
(/root/reference/envs/loadbalancer_k8s_env.py:9-12,100,129,139-174) needs only:
  * gym.Env with a lazily-created `np_random` property (+ setter),
  * gym.spaces.Box / gym.spaces.Discrete,
  * gym.utils.seeding.np_random(seed) -> (Generator(PCG64(SeedSequence(seed))), entropy).
This file provides exactly that and nothing else. It is never imported by the
product package or by the GPU tests.
"""
import numpy as np

from . import spaces, utils, vector  # noqa: F401


class Env:
    metadata = {}
    _np_random = None

    @property
    def np_random(self):
        if self._np_random is None:
            self._np_random, _ = utils.seeding.np_random(None)
        return self._np_random

    @np_random.setter
    def np_random(self, value):
        self._np_random = value

    def reset(self):
        raise NotImplementedError

    def step(self, action):
        raise NotImplementedError
