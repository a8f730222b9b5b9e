"""custom_getter / custom_creator context managers (test shim)."""
import contextlib


@contextlib.contextmanager
def custom_getter(getter):
    from haiku import _S
    _S.getters.append(getter)
    try:
        yield
    finally:
        _S.getters.pop()


@contextlib.contextmanager
def custom_creator(creator):
    from haiku import _S
    _S.creators.append(creator)
    try:
        yield
    finally:
        _S.creators.pop()
