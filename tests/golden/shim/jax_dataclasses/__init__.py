"""`jax_dataclasses.pytree_dataclass` → plain dataclass (test shim)."""
import dataclasses


def pytree_dataclass(cls=None, **kw):
    if cls is None:
        return lambda c: dataclasses.dataclass(c)
    return dataclasses.dataclass(cls)


Static = object
