"""Deterministic fake PRNG keys (test shim; inference does not depend on RNG)."""
import numpy as _np


def PRNGKey(seed):  # noqa: N802
    return _np.array([0, seed], dtype=_np.uint32)


def split(key, num=2):
    return _np.stack([_np.array([i, 7], dtype=_np.uint32) for i in range(num)])


def fold_in(key, data):
    return key
