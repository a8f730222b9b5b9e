"""Decode-path host logic on CPU: masks, token loading, codes, PDB writer, decoder blob."""
import os

import numpy as np
import pytest

from pst_amd import _native
from pst_amd import config as C
from pst_amd import params as P
from pst_amd import runner
from pst_amd.structure_io import atom37_to_pdb


def test_decoder_blob_matches_library_count():
    for D in (5, 6):
        assert _native.lib().pst_decoder_param_count(D) == P.decoder_param_count(D)
        blob = P.pack_decoder(P.random_full_params(D, 1), D)
        assert blob.size == P.decoder_param_count(D)


def test_masks_and_batch(tmp_path):
    f1, f2 = tmp_path / "a_tokens.npy", tmp_path / "b_tokens.npy"
    np.save(f1, np.array([[5, 6, 7]], np.uint32))
    np.save(f2, np.array([[1, 2, 3, 4, 5, 6]], np.uint32))
    tok = runner.load_and_build_batch([str(f1), str(f2)], 5, 4097)
    assert tok.tolist() == [[5, 6, 7, 4097, 4097], [1, 2, 3, 4, 5]]
    tm = runner.build_tokens_mask_from_sequence(tok, 4097)
    assert tm.tolist() == [[1, 1, 1, 0, 0], [1, 1, 1, 1, 1]]
    nm = runner.build_nodes_mask_from_tokens_mask(tm, 2)
    assert nm.sum(-1).tolist() == [6, 10]


def test_token_to_code():
    fn = runner.TokenToCodeFn(C.tokenizer_config(64000, 1))
    lv = np.array(C.LEVELS[64000])
    t = np.array([0, 1, 63999, 32036])
    codes = fn(None, None, t)
    assert np.all(codes[0] == -(lv // 2)) and np.all(codes[2] == lv - 1 - lv // 2)
    assert np.all(codes[3] == 0)  # the padded-token id is the all-zero code


def test_pdb_writer_format_roundtrip():
    from pst_amd.pdb import protein_structure_from_pdb_string
    rng = np.random.default_rng(0)
    pos = np.round(rng.normal(size=(7, 37, 3)) * 10, 3).astype(np.float32)
    mask = np.zeros((7, 37), np.float32)
    mask[:, [0, 1, 2, 4]] = 1
    txt = atom37_to_pdb(pos, mask, np.zeros(7, np.int64))
    lines = txt.splitlines()
    assert lines[0].startswith("MODEL     1") and lines[-1].startswith("END") and all(len(l) == 80 for l in lines)
    assert lines[1][:30] == "ATOM      1  N   ALA A   0    "
    s = protein_structure_from_pdb_string(txt)
    assert s.nb_residues == 7
    assert np.allclose(s.atom37_positions[:, [0, 1, 2, 4]], pos[:, [0, 1, 2, 4]], atol=1e-6)


@pytest.mark.reference
def test_pdb_writer_and_masks_match_reference():
    import _refenv
    _refenv.activate(f64=False)
    from structure_tokenizer.data import protein as ref_protein
    rng = np.random.default_rng(1)
    n = 9
    pos = rng.normal(size=(n, 37, 3)) * 10
    mask = np.zeros((n, 37))
    mask[:, [0, 1, 2, 4]] = 1
    aat = np.concatenate([np.ones((n, 1)), np.zeros((n, 20))], -1)
    prot = ref_protein.Protein.from_atom37_rep(atom37_positions=pos, atom37_gt_exists=mask, atom37_atom_exits=mask,
                                               aatype=aat, chain_id="A")
    assert atom37_to_pdb(pos, mask, np.zeros(n, np.int64)) == ref_protein.to_pdb(prot)
