"""NumPy stand-in for the subset of `jax` the reference's tokenize path uses (test shim)."""
import functools as _ft
import numpy as _np

from . import numpy, nn, lax, tree_util, random, ops  # noqa: F401
from .tree_util import tree_map  # noqa: F401


class _Config:
    def update(self, *a, **k):
        pass


config = _Config()


class Device:
    platform = "cpu"


def devices(*a, **k):
    return [Device()]


local_devices = devices


def local_device_count(*a, **k):
    return 1


def process_index():
    return 0


def device_put(x, *a, **k):
    return x


def block_until_ready(x):
    return x


def jit(f=None, **kw):
    return f if f is not None else (lambda g: g)


def _is_scalar_key(a):
    return isinstance(a, (int, float, _np.integer, _np.floating)) or (
        isinstance(a, _np.ndarray) and a.ndim == 0)


def vmap(fun, in_axes=0, out_axes=0, **_):
    """Loop-based vmap over leading axis. Results for repeated scalar inputs are cached,
    which keeps the reference's per-edge positional-encoding vmaps tractable."""

    @_ft.wraps(fun)
    def mapped(*args, **kwargs):
        axes = in_axes if isinstance(in_axes, (tuple, list)) else (in_axes,) * len(args)
        n = None
        for a, ax in list(zip(args, axes)) + [(v, 0) for v in kwargs.values()]:
            if ax is not None:
                leaves = tree_util.tree_leaves(a)
                n = _np.shape(leaves[0])[ax]
                break
        cache = {}
        outs = []
        for i in range(n):
            a_i = [tree_util.tree_map(lambda x: _np.take(x, i, axis=ax), a) if ax is not None else a
                   for a, ax in zip(args, axes)]
            k_i = {k: tree_util.tree_map(lambda x: _np.take(x, i, axis=0), v) for k, v in kwargs.items()}
            key = None
            if all(_is_scalar_key(x) for x in list(a_i) + list(k_i.values())):
                key = tuple(float(x) for x in a_i) + tuple((k, float(v)) for k, v in k_i.items())
            if key is not None and key in cache:
                outs.append(cache[key])
                continue
            o = fun(*a_i, **k_i)
            if key is not None:
                cache[key] = o
            outs.append(o)
        return tree_util.tree_map(lambda *xs: _np.stack([_np.asarray(x) for x in xs], axis=out_axes), *outs)

    return mapped


def pmap(fun, *a, **k):
    return fun


class util:  # noqa: N801
    @staticmethod
    def wraps(fun, docstr=None, **kw):
        return _ft.wraps(fun)
