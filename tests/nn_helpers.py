"""Shared helpers for the deep-sets / PPO / DQN golden tests."""
import os

import numpy as np
import torch

from conftest import GOLDEN


def load_nn(name):
    return dict(np.load(os.path.join(GOLDEN, name + ".npz")))


def state_dict_from(d, prefix):
    return {k[len(prefix):].replace("__", "."): torch.from_numpy(np.asarray(v))
            for k, v in d.items() if k.startswith(prefix)}


def close(got, exp, rtol=1e-5, atol=1e-6, what=""):
    got = got.detach().cpu().numpy() if isinstance(got, torch.Tensor) else np.asarray(got)
    np.testing.assert_allclose(got, np.asarray(exp), rtol=rtol, atol=atol, err_msg=what)
