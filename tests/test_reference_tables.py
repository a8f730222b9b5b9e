"""Restated tables vs the reference's own module (imported read-only from /root/reference)."""
import pytest

from pst_amd import residue_constants as rc

pytestmark = pytest.mark.reference


def test_residue_tables_match_reference():
    import _refenv
    _refenv.activate(f64=False)
    from structure_tokenizer.data import residue_constants as ref
    assert rc.atom_types == list(ref.atom_types)
    assert rc.restypes == list(ref.restypes)
    assert rc.restype_1to3 == dict(ref.restype_1to3)
    assert rc.restype_3to1 == dict(ref.restype_3to1)
    for k, v in ref.res_atom37_exist.items():
        assert rc.res_atom37_exist[k] == list(v), k
    assert set(rc.res_atom37_exist) == set(ref.res_atom37_exist)
