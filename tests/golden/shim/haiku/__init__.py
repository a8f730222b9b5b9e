"""NumPy stand-in for the subset of dm-haiku 0.0.10 the reference's tokenize path uses.

Test shim only. Implements module naming ("parent/~/child" for modules built in __init__,
"parent/child" for modules built in a method, `_N` suffixes for repeats within one call,
counters reset per method call so re-calling a module re-uses its parameters), parameter
creation/lookup through custom creators/getters, transform(init/apply), scan, vmap, and the
layers hk.Linear / hk.nets.MLP / hk.LayerNorm / hk.Sequential with their published maths.
"""
import contextlib
import functools
import re
import types

import numpy as np

import jax
import jax.numpy as jnp


# ----------------------------------------------------------------------------- state
class _Frame:
    def __init__(self, module, method):
        self.module, self.method, self.counts = module, method, {}


class _State:
    def __init__(self):
        self.mode = None
        self.params = {}
        self.rng = np.random.default_rng(0)
        self.frames = [_Frame(None, None)]
        self.getters = []
        self.creators = []
        self.created = []  # (module_name, param_name, shape) in creation order


_S = _State()


def _camel_to_snake(value):
    value = re.sub(r"((?<=[a-z0-9])[A-Z]|(?!^)[A-Z](?=[a-z]))", r"_\1", value)
    return value.lower()


def _current_parent_frame(module):
    for f in reversed(_S.frames):
        if f.module is not module:
            return f
    return _S.frames[0]


def transparent(fn):
    fn._hk_transparent = True
    return fn


def _wrap_method(name, fn):
    if getattr(fn, "_hk_transparent", False) or getattr(fn, "_hk_wrapped", False):
        return fn

    @functools.wraps(fn)
    def wrapped(self, *a, **k):
        _S.frames.append(_Frame(self, name))
        try:
            return fn(self, *a, **k)
        finally:
            _S.frames.pop()

    wrapped._hk_wrapped = True
    return wrapped


class Module:
    def __init_subclass__(cls, **kw):
        super().__init_subclass__(**kw)
        for attr, val in list(vars(cls).items()):
            if attr.startswith("__") and attr not in ("__init__", "__call__"):
                continue
            if callable(val) and not isinstance(val, (staticmethod, classmethod, type)):
                setattr(cls, attr, _wrap_method(attr, val))

    def __init__(self, name=None):
        if name is None:
            name = _camel_to_snake(type(self).__name__)
        frame = _current_parent_frame(self)
        parent = frame.module
        if parent is None:
            base = name
        else:
            sep = "/~/" if frame.method == "__init__" else "/"
            base = parent.module_name + sep + name
        cnt = frame.counts.get(base, 0)
        frame.counts[base] = cnt + 1
        self.module_name = base if cnt == 0 else f"{base}_{cnt}"
        self.name = self.module_name.split("/")[-1]


class _Context:
    def __init__(self, module_name, name, shape, dtype):
        self.module_name, self.name = module_name, name
        self.full_name = module_name + "/" + name
        self.original_shape, self.original_dtype = tuple(shape), dtype


def _current_module():
    for f in reversed(_S.frames):
        if f.module is not None:
            return f.module
    return None


def get_parameter(name, shape, dtype=np.float32, init=None):
    mod = _current_module()
    mname = mod.module_name if mod is not None else "~"
    ctx = _Context(mname, name, shape, dtype)
    store = _S.params.setdefault(mname, {})
    if name not in store:
        if _S.mode != "init":
            raise KeyError(f"missing parameter {mname}/{name}")

        def final_creator(shape, dtype, init, context):
            return np.asarray(init(tuple(shape), dtype))

        chain = final_creator
        for c in reversed(_S.creators):
            chain = functools.partial(c, chain) if False else _bind_creator(c, chain)
        value = chain(tuple(shape), dtype, init, ctx)
        store[name] = value
        _S.created.append((mname, name, tuple(np.shape(value))))
    value = store[name]

    def final_getter(v):
        return v

    g = final_getter
    for getter in reversed(_S.getters):
        g = _bind_getter(getter, g, ctx)
    return g(value)


def _bind_creator(c, nxt):
    def f(shape, dtype, init, context):
        return c(lambda s, d, i: nxt(s, d, i, context), shape, dtype, init, context)
    return f


def _bind_getter(getter, nxt, ctx):
    def f(v):
        return getter(nxt, v, ctx)
    return f


def running_init():
    return _S.mode == "init"


def next_rng_key():
    return jax.random.PRNGKey(0)


def maybe_next_rng_key():
    return None


@contextlib.contextmanager
def with_rng(key):
    yield


def remat(f):
    return f


def dropout(key, rate, x):
    return x


def vmap(fun, in_axes=0, out_axes=0, axis_name=None, split_rng=None):
    return jax.vmap(fun, in_axes=in_axes, out_axes=out_axes)


def scan(f, init, xs, length=None, unroll=1):
    leaves = jax.tree_util.tree_leaves(xs)
    n = length if length is not None else np.shape(leaves[0])[0]
    carry, ys = init, []
    for i in range(n):
        x_i = jax.tree_util.tree_map(lambda a: a[i], xs)
        carry, y = f(carry, x_i)
        ys.append(y)
    if all(y is None for y in ys):
        return carry, None
    return carry, jax.tree_util.tree_map(lambda *a: np.stack(a), *ys)


class _Transformed:
    def __init__(self, f):
        self._f = f

    def init(self, rng, *a, **k):
        _reset("init", {})
        self._f(*a, **k)
        params = _S.params
        _reset(None, {})
        return params

    def apply(self, params, rng, *a, **k):
        _reset("apply", params)
        try:
            return self._f(*a, **k)
        finally:
            _reset(None, {})


def _reset(mode, params):
    _S.mode, _S.params = mode, params
    _S.frames = [_Frame(None, None)]
    _S.getters, _S.creators, _S.created = [], [], []


def transform(f, *, apply_rng=True):
    return _Transformed(f)


class Sequential(Module):
    def __init__(self, layers, name=None):
        super().__init__(name=name)
        self.layers = tuple(layers)

    def __call__(self, inputs, *a, **k):
        out = inputs
        for i, layer in enumerate(self.layers):
            out = layer(out, *a, **k) if i == 0 else layer(out)
        return out


class Linear(Module):
    def __init__(self, output_size, with_bias=True, w_init=None, b_init=None, name=None):
        super().__init__(name=name)
        self.output_size, self.with_bias = output_size, with_bias
        self.w_init, self.b_init = w_init, b_init or jnp.zeros

    def __call__(self, inputs, *, precision=None):
        input_size = inputs.shape[-1]
        w_init = self.w_init or initializers.TruncatedNormal(1.0 / np.sqrt(input_size))
        w = get_parameter("w", [input_size, self.output_size], inputs.dtype, init=w_init)
        out = np.dot(inputs, w)
        if self.with_bias:
            b = get_parameter("b", [self.output_size], inputs.dtype, init=self.b_init)
            out = out + np.broadcast_to(b, out.shape)
        return out


class LayerNorm(Module):
    def __init__(self, axis, create_scale, create_offset, eps=1e-5, scale_init=None,
                 offset_init=None, use_fast_variance=False, name=None, *, param_axis=None):
        super().__init__(name=name)
        from haiku._src.layer_norm import to_axes_or_slice
        self.axis = to_axes_or_slice(axis)
        self.eps, self.create_scale, self.create_offset = eps, create_scale, create_offset
        self.scale_init = scale_init or jnp.ones
        self.offset_init = offset_init or jnp.zeros
        self.param_axis = (-1,) if param_axis is None else to_axes_or_slice(param_axis)

    def __call__(self, inputs, scale=None, offset=None):
        from haiku._src.layer_norm import to_abs_axes
        axis = to_abs_axes(self.axis, inputs.ndim)
        mean = np.mean(inputs, axis=axis, keepdims=True)
        variance = np.var(inputs, axis=axis, keepdims=True)
        param_shape = inputs.shape[-1:]
        if self.create_scale:
            scale = get_parameter("scale", param_shape, inputs.dtype, init=self.scale_init)
        elif scale is None:
            scale = np.array(1.0, dtype=inputs.dtype)
        if self.create_offset:
            offset = get_parameter("offset", param_shape, inputs.dtype, init=self.offset_init)
        elif offset is None:
            offset = np.array(0.0, dtype=inputs.dtype)
        inv = scale * (1.0 / np.sqrt(variance + np.asarray(self.eps, variance.dtype)))
        return inv * (inputs - mean) + offset


class BatchNorm(Module):
    pass


def _mlp_module():
    class MLP(Module):
        def __init__(self, output_sizes, w_init=None, b_init=None, with_bias=True,
                     activation=None, activate_final=False, name=None):
            super().__init__(name=name)
            self.activation, self.activate_final = activation, activate_final
            self.layers = [Linear(o, with_bias=with_bias, w_init=w_init, b_init=b_init,
                                  name="linear_%d" % i) for i, o in enumerate(output_sizes)]

        def __call__(self, inputs, dropout_rate=None, rng=None):
            out = inputs
            n = len(self.layers)
            for i, layer in enumerate(self.layers):
                out = layer(out)
                if i < n - 1 or self.activate_final:
                    out = self.activation(out)
            return out

    return types.SimpleNamespace(MLP=MLP)


nets = _mlp_module()

from . import initializers  # noqa: E402
from . import experimental  # noqa: E402
from . import mixed_precision  # noqa: E402

Params = dict
