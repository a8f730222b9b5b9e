"""The C ABI library loads and exports every symbol include/pst.h declares (no GPU needed)."""
import ctypes
import os
import re

import numpy as np
import pytest

from pst_amd import _native
from pst_amd import params as P

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    txt = open(os.path.join(ROOT, "include", "pst.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(pst_[a-z_0-9]+)\s*\(", txt)))


def test_header_declares_the_binding_exports():
    assert sorted(_native.EXPORTS) == _declared()


def test_library_exports_every_declared_symbol():
    L = _native.lib()
    for sym in _declared():
        assert hasattr(L, sym), sym
        assert ctypes.cast(getattr(L, sym), ctypes.c_void_p).value


@pytest.mark.parametrize("D", [5, 6])
def test_param_count_matches_host_spec(D):
    assert _native.lib().pst_param_count(D) == P.param_count(D)
    assert P.param_count(6) == 1573638 and P.param_count(5) == 1573509


def test_create_without_device_fails_loudly():
    if _native.device_count() > 0:
        pytest.skip("a HIP device is visible")
    with pytest.raises(_native.PstError):
        _native.Tokenizer(0, 4096, 1, P.random_blob(6, 0))


def test_create_rejects_bad_blob_before_touching_device():
    with pytest.raises(ValueError):
        _native.Tokenizer(0, 4096, 1, np.zeros(10, np.float32))


def test_error_code_mapping():
    with pytest.raises(NotImplementedError):
        _native.raise_for(_native.PST_E_TOO_LARGE, "x")
    with pytest.raises(NotImplementedError):
        _native.raise_for(_native.PST_E_TOO_SMALL, "x")
    with pytest.raises(ValueError):
        _native.raise_for(_native.PST_E_INVALID, "x")
    with pytest.raises(_native.PstError):
        _native.raise_for(_native.PST_E_HIP, "x")
    _native.raise_for(_native.PST_OK, "")
