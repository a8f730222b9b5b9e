"""`jax.numpy` → NumPy (test shim). With PST_SHIM_F64=1, float32 is promoted to float64."""
import os as _os
import numpy as _np
from numpy import *  # noqa: F401,F403

ndarray = _np.ndarray
_F64 = _os.environ.get("PST_SHIM_F64", "0") == "1"
if _F64:
    float32 = _np.float64  # noqa: F811
    bfloat16 = _np.float64
    float16 = _np.float64
else:
    bfloat16 = _np.float32


def asarray(x, dtype=None):
    a = _np.asarray(x, dtype=dtype)
    if _F64 and a.dtype == _np.float32:
        a = a.astype(_np.float64)
    return a


def array(x, dtype=None, **k):
    return asarray(x, dtype=dtype)

linalg = _np.linalg


def einsum(*operands, precision=None, **kw):
    return _np.einsum(*operands, **kw)


def dot(a, b, precision=None):
    return _np.dot(a, b)
