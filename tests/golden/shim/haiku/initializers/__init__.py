"""Initializers (shapes only matter: fixtures feed their own parameters; test shim)."""
import numpy as np

Initializer = object
_RNG = np.random.default_rng(1234)


class Constant:
    def __init__(self, constant):
        self.constant = constant

    def __call__(self, shape, dtype):
        return np.full(shape, self.constant, dtype=np.float64)


class TruncatedNormal:
    def __init__(self, stddev=1.0, mean=0.0):
        self.stddev, self.mean = stddev, mean

    def __call__(self, shape, dtype):
        return np.clip(_RNG.standard_normal(shape), -2, 2) * self.stddev + self.mean


class VarianceScaling:
    def __init__(self, scale=1.0, mode="fan_in", distribution="truncated_normal", fan_in_axes=None):
        self.scale, self.mode = scale, mode

    def __call__(self, shape, dtype):
        fan_in = int(np.prod(shape[:-1])) if len(shape) > 1 else shape[0]
        return np.clip(_RNG.standard_normal(shape), -2, 2) * np.sqrt(self.scale / max(1, fan_in))


class Orthogonal(VarianceScaling):
    pass
