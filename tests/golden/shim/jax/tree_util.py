"""Minimal pytree utilities (test shim)."""
import dataclasses

_REGISTRY = {}


def register_pytree_node(cls, flatten, unflatten):
    _REGISTRY[cls] = (flatten, unflatten)


def _children(x):
    if isinstance(x, (list, tuple)) and not hasattr(x, "_fields"):
        return list(x), ("seq", type(x))
    if hasattr(x, "_fields"):  # namedtuple
        return list(x), ("nt", type(x))
    if isinstance(x, dict):
        keys = sorted(x.keys())
        return [x[k] for k in keys], ("dict", keys)
    if dataclasses.is_dataclass(x) and not isinstance(x, type):
        names = [f.name for f in dataclasses.fields(x)]
        return [getattr(x, n) for n in names], ("dc", (type(x), names))
    if type(x) in _REGISTRY:
        ch, aux = _REGISTRY[type(x)][0](x)
        return list(ch), ("reg", (type(x), aux))
    return None, None


def _rebuild(spec, ch):
    kind, info = spec
    if kind == "seq":
        return info(ch)
    if kind == "nt":
        return info(*ch)
    if kind == "dict":
        return dict(zip(info, ch))
    if kind == "dc":
        cls, names = info
        return cls(**dict(zip(names, ch)))
    cls, aux = info
    return _REGISTRY[cls][1](aux, ch)


def tree_leaves(x):
    ch, spec = _children(x)
    if ch is None:
        return [] if x is None else [x]
    out = []
    for c in ch:
        out.extend(tree_leaves(c))
    return out


def tree_map(f, tree, *rest):
    ch, spec = _children(tree)
    if ch is None:
        if tree is None:
            return None
        return f(tree, *rest)
    rest_ch = [_children(r)[0] for r in rest]
    new = [tree_map(f, c, *[rc[i] for rc in rest_ch]) for i, c in enumerate(ch)]
    return _rebuild(spec, new)


def tree_flatten(x):
    return tree_leaves(x), x


def tree_unflatten(treedef, leaves):
    it = iter(leaves)
    return tree_map(lambda _: next(it), treedef)
