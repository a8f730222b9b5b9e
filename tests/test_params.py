"""params.npz loader (f2): leaf order, names and shapes of the full Vq3D checkpoint tree."""
import json
import os

import numpy as np
import pytest

from pst_amd import params as P

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def test_full_spec_matches_reference_tree():
    # full_param_names.json: the reference Vq3D initialised under the shim (make_param_names.py)
    ref = json.load(open(os.path.join(GOLD, "full_param_names.json")))
    got = [[m, p, list(sh)] for m, p, sh in P.full_param_spec(ref["codes_dim"])]
    assert got == ref["leaves"]
    assert len(got) == 189


def test_encoder_spec_is_subset_of_full_tree():
    full = {(m, p): sh for m, p, sh in P.full_param_spec(6)}
    for m, p, sh in P.param_spec(6):
        assert full[(m, p)] == sh


@pytest.mark.parametrize("D", [5, 6])
def test_npz_roundtrip_by_leaf_order(tmp_path, D):
    full = P.random_full_params(D, seed=3)
    fn = str(tmp_path / "params.npz")
    names = P.save_params_npz(fn, full)
    assert names == [(m, p) for m, p, _ in P.full_param_spec(D)]
    back = P.load_params_npz(fn)  # codes_dim inferred from the first leaf (down_proj/b)
    assert np.array_equal(P.pack(back, D), P.pack(full, D))


def test_npz_named_and_prefixed(tmp_path):
    full = P.random_full_params(6, seed=4)
    pref = {"forward_vq3_d/" + m: v for m, v in full.items()}
    fn = str(tmp_path / "p.npz")
    P.save_params_npz(fn, pref, named=True)
    back = P.load_params_npz(fn)
    assert set(back) == set(full)
    assert np.array_equal(P.pack(back, 6), P.pack(full, 6))
    raw = P.load_params_npz(fn, convert=False)
    assert all(k.startswith("forward_vq3_d/") for k in raw)


def test_npz_errors(tmp_path):
    full = P.random_full_params(6, seed=5)
    fn = str(tmp_path / "p.npz")
    names = [(m, p) for m in sorted(full) for p in sorted(full[m])]
    np.savez(fn, *[full[m][p] for m, p in names[:-1]])
    with pytest.raises(ValueError, match="leaves"):
        P.load_params_npz(fn)
    bad = dict(full)
    bad["vq3_d/~/structure_encoder/init_node_embed"] = {"w": np.zeros((3, 3), np.float32),
                                                        "b": np.zeros(128, np.float32)}
    P.save_params_npz(fn, bad, named=True)
    with pytest.raises(ValueError, match="shape"):
        P.load_params_npz(fn)


def test_pack_unpack_roundtrip():
    blob = P.random_blob(6, 1)
    assert np.array_equal(P.pack(P.unpack(blob, 6), 6), blob)


def test_params_keys_conversion():
    d = {"forward_vq3_d/vq3_d/down_proj": {"b": 1}, "forward_vq3_d/vq3_d/~/x": {"w": 2}}
    assert P.params_keys_conversion(d) == {"vq3_d/down_proj": {"b": 1}, "vq3_d/~/x": {"w": 2}}
