import numpy as np


def np_random(seed=None):
    seq = np.random.SeedSequence(seed)
    return np.random.Generator(np.random.PCG64(seq)), seq.entropy
