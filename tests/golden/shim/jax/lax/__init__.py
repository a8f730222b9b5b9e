"""`jax.lax` subset in NumPy (test shim)."""
import numpy as _np


def rsqrt(x):
    return 1.0 / _np.sqrt(x)


def convert_element_type(x, dtype):
    return _np.asarray(x, dtype=dtype) if not isinstance(x, float) else _np.asarray(x).astype(dtype)


def stop_gradient(x):
    return x


def pmean(x, axis_name=None):
    return x


def index_in_dim(x, index, axis=0, keepdims=True):
    r = _np.take(x, index, axis=axis)
    return _np.expand_dims(r, axis) if keepdims else r


dynamic_index_in_dim = index_in_dim
