"""End to end on the GPU: the drop-in CLI (`scripts/tokenize_pdb.py`) and `InferenceRunner`
through libpst, checked against the CPU oracle token for token."""
import os
import sys

import numpy as np
import pytest

from oracle import oracle as O
from pst_amd import config as C
from pst_amd import params as P
from pst_amd import pdb, runner, synthetic

pytestmark = pytest.mark.gpu
SCRIPTS = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                       "protein-structure-tokenizer_amd", "scripts")


@pytest.mark.parametrize("cb,df", [(4096, 1), (64000, 4)])
def test_cli_end_to_end(tmp_path, cb, df):
    sys.path.insert(0, SCRIPTS)
    import tokenize_pdb
    D = len(C.LEVELS[cb])
    pdb_dir = tmp_path / "pdbs"
    pdb_dir.mkdir()
    ss = {f"s{i}": synthetic.synthetic_protein(n, 300 + i) for i, n in enumerate((50, 77, 130, 256, 512))}
    for k, s in ss.items():
        (pdb_dir / f"{k}.pdb").write_text(pdb.to_pdb_string(s))
    mdir = tmp_path / "model"
    mdir.mkdir()
    full = P.random_full_params(D, seed=5)
    P.save_params_npz(str(mdir / "params.npz"), full)
    out = tmp_path / "tokens"
    tokenize_pdb.cli(["--pdb_dir", str(pdb_dir), "--token_save_path", str(out), "--codebook_size", str(cb),
                      "--model_downsampling", str(df), "--batch_size_per_device", "2", "--weights_dir", str(mdir)])
    blob = P.pack(full, D)
    for k, s in ss.items():
        t = np.load(out / f"{k}_tokens.npy")
        want = O.tokenize(blob, C.LEVELS[cb], df, s.atom37_positions, s.atom_flags())["tokens"]
        assert t.dtype == np.uint32 and t.shape == (1, s.nb_residues // df)
        assert np.array_equal(t[0], want), k


def test_tokenize_fn_on_gpu_matches_reference_layout():
    cfg = C.tokenizer_config(4096, 1)
    devs, n = runner.InferenceRunner.prepare_devices("gpu")
    mp = runner.ReplicatedParams(P.random_params(6, 9), devs[:1])
    fn = runner.InferenceRunner.prepare_tokenize_fn(cfg, devs[:1])
    ss = [synthetic.synthetic_protein(m, 17 + m) for m in (51, 199, 64)]
    out = fn(mp, None, runner.batch_collate([1, 3], ss))
    fn.close()
    assert out["tokens"].shape == (1, 3, 512)
    for b, s in enumerate(ss):
        want = O.tokenize(mp.blob, cfg.levels, 1, s.atom37_positions, s.atom_flags())["tokens"]
        assert np.array_equal(out["tokens"][0, b, :s.nb_residues], want)
        assert np.all(out["tokens"][0, b, s.nb_residues:] == runner.pad_token_value(cfg.levels))


def test_tokenize_fn_emit_aux_matches_reference_golden():
    """QuantizerOutput through the runner mirror vs the reference model's own outputs (f64 run
    under the shim, same random weights): tokens exact, aux within f32 tolerance."""
    F = np.load(os.path.join(os.path.dirname(__file__), "golden", "forward_golden_f64.npz"))
    c = "syn51_k4096_df1/"
    from pst_amd.sample import ProteinStructureSample
    pos = F[c + "in_positions"].astype(np.float64)
    fl = F[c + "in_flags"]
    n = pos.shape[0]
    s = ProteinStructureSample(None, n, np.zeros((n, 21)), pos, (fl & 1).astype(bool), ((fl >> 1) & 1).astype(bool), 0.0, 1)
    cfg = C.tokenizer_config(4096, 1)
    mp = runner.ReplicatedParams(P.random_params(6, 1234), [0])
    fn = runner.InferenceRunner.prepare_tokenize_fn(cfg, [0], emit_aux=True)
    out = fn(mp, None, runner.batch_collate([1, 1], [s]))
    fn.close()
    T = int(out["n_tokens"][0, 0])
    assert T == F[c + "tokens"].shape[0]
    assert np.array_equal(out["tokens"][0, 0, :T], F[c + "tokens"])
    np.testing.assert_allclose(out["continuous_embedding"][0, 0, :T], F[c + "bounded"], atol=1e-4)
    np.testing.assert_allclose(out["continuous_embedding_pre_proj"][0, 0, :T], F[c + "pre_proj"], atol=5e-6)
    np.testing.assert_array_equal(out["quantize"][0, 0, :T], F[c + "quantize"])
    np.testing.assert_array_equal(out["straight_through_quantized"], out["quantize"])
    np.testing.assert_allclose(out["distances"][0, 0, :T], F[c + "distances"], rtol=1e-4, atol=1e-3)
    np.testing.assert_allclose(out["soft_proba"][0, 0, :T], F[c + "soft_proba"], rtol=1e-3, atol=1e-5)
    assert abs(out["perplexity"][0] - float(F[c + "perplexity"])) < 1e-4 * float(F[c + "perplexity"])
    assert np.all(out["distances"][0, 0, T:] == 0) and np.all(out["quantize"][0, 0, T:] == 0)
    np.testing.assert_allclose(out["soft_proba"][0, 0, T:].sum(-1), 1.0, rtol=1e-5)


@pytest.mark.parametrize("subset,cb", [("T1024", 4096), ("all", 4096), ("all", 64000)])
def test_cli_casp14(tmp_path, casp14_dir, subset, cb):
    """SURVEY configs 1 (T1024, 391 tokens), 2 (all 31 structures) and 4 (all 31 at codebook
    64 000, df 1) through the drop-in CLI: token files equal to the oracle's and to the
    reference's own float64 forward on the same weights (`forward_ref_wide.npz`)."""
    import shutil
    sys.path.insert(0, SCRIPTS)
    import tokenize_pdb
    pdb_dir = tmp_path / "pdbs"
    pdb_dir.mkdir()
    names = ["T1024"] if subset == "T1024" else sorted(f[:-4] for f in os.listdir(casp14_dir))
    for nm in names:
        shutil.copy(os.path.join(casp14_dir, nm + ".pdb"), pdb_dir / (nm + ".pdb"))
    mdir = tmp_path / "model"
    mdir.mkdir()
    full = P.random_full_params(6, seed=1234)  # encoder half = the reference fixture's weights
    P.save_params_npz(str(mdir / "params.npz"), full)
    out = tmp_path / "tokens"
    tokenize_pdb.cli(["--pdb_dir", str(pdb_dir), "--token_save_path", str(out), "--batch_size_per_device", "8",
                      "--weights_dir", str(mdir), "--codebook_size", str(cb)])
    blob = P.pack(full, 6)
    import refwide
    R = refwide.load()
    F = np.load(os.path.join(os.path.dirname(__file__), "golden", "casp14_atom37.npz"))
    idx = {str(n): i for i, n in enumerate(F["names"])}
    for nm in names:
        i = idx[nm]
        a, b = int(F["offsets"][i]), int(F["offsets"][i + 1])
        want = O.tokenize(blob, C.LEVELS[cb], 1, F["positions"][a:b].astype(np.float64), F["flags"][a:b])["tokens"]
        t = np.load(out / f"{nm}_tokens.npy")
        assert np.array_equal(t[0], want), nm
        assert np.array_equal(t[0], R[f"casp_{nm}_k{cb}_df1/tokens"]), nm
    if subset == "T1024":
        assert np.load(out / "T1024_tokens.npy").shape == (1, 391)


def test_main_reference_keyword_call_selects_64k_df4(tmp_path):
    """the reference's own keyword call of `main` — the model chosen by
    `config_overrides` alone (no config_path) — tokenizes at codebook 64 000 / df 4, token files
    equal to the oracle's; an unknown override raises ValueError instead of a silent default."""
    sys.path.insert(0, SCRIPTS)
    import tokenize_pdb
    cfg = C.tokenizer_config(64000, 4)
    D = len(cfg.levels)
    pdb_dir = tmp_path / "pdbs"
    pdb_dir.mkdir()
    ss = {f"m{i}": synthetic.synthetic_protein(n, 610 + i) for i, n in enumerate((53, 130, 257, 511))}
    for k, s in ss.items():
        (pdb_dir / f"{k}.pdb").write_text(pdb.to_pdb_string(s))
    mdir = tmp_path / "model"
    mdir.mkdir()
    full = P.random_full_params(D, seed=21)
    P.save_params_npz(str(mdir / "params.npz"), full)
    out = tmp_path / "tokens"
    tokenize_pdb.main(pdbs=[str(pdb_dir / f"{k}.pdb") for k in ss], token_save_path=str(out), backend="gpu",
                      batch_size_per_device=2,
                      config_overrides=["model=gnn/ablation_64k_df_4.yaml", "data=ablation_df_4.yaml"],
                      weights_dir=str(mdir))
    blob = P.pack(full, D)
    for k, s in ss.items():
        t = np.load(out / f"{k}_tokens.npy")
        want = O.tokenize(blob, cfg.levels, 4, s.atom37_positions, s.atom_flags())["tokens"]
        assert t.shape == (1, s.nb_residues // 4), k
        assert np.array_equal(t[0], want), k
    with pytest.raises(ValueError):
        tokenize_pdb.main(pdbs=[str(pdb_dir / "m0.pdb")], token_save_path=str(tmp_path / "bad"), backend="gpu",
                          batch_size_per_device=2, config_overrides=["model=gnn/ablation_64k_df_8.yaml"],
                          weights_dir=str(mdir))
    assert not (tmp_path / "bad").exists()


AE_GOLD = os.path.join(os.path.dirname(__file__), "golden", "ae_ref.npz")
# float32 GPU vs the reference's float64 `Vq3D.__call__`: the decoder tolerances of
# test_gpu_decode.py's small cases (atoms 1e-3 Å) and the up_proj of the exact integer codes
AE_TOL_ATOMS, AE_TOL_UP = 1e-3, 1e-5


def _ae_cases():
    if not os.path.exists(AE_GOLD):
        return []
    return sorted({k.split("/")[0] for k in np.load(AE_GOLD).files})


@pytest.mark.parametrize("case", _ae_cases())
def test_prepare_ae_fn_matches_reference(case):
    """`InferenceRunner.prepare_ae_fn` (inference_runner.py:209-222 → Vq3D.__call__) vs the
    reference's own autoencoder pass (`make_ae_golden.py`, float64 under the shim): token ids
    exact, `quantize_post_proj`, and final atoms decoded on the graph's node count (not a
    multiple of df in the df 2 / 4 cases) with the protein's aatype (one UNK residue → zeros)."""
    from pst_amd.sample import sample_from_arrays
    F = np.load(AE_GOLD)
    n, n_node, T, cb, df, D, pseed = (int(v) for v in F[case + "/meta"])
    s = sample_from_arrays(F[case + "/in_positions"].astype(np.float64), F[case + "/in_flags"],
                           F[case + "/in_aatype"].astype(np.int64))
    cfg = C.tokenizer_config(cb, df)
    mp = runner.ReplicatedParams(P.params_keys_conversion(P.random_full_params(D, pseed)), [0])
    fn = runner.InferenceRunner.prepare_ae_fn(cfg, [0])
    st, q = fn(mp, None, runner.batch_collate([1, 1], [s]))
    fn.close()
    assert int(q["n_tokens"][0, 0]) == T
    assert np.array_equal(q["tokens"][0, 0, :T], F[case + "/tokens"])
    e_up = float(np.max(np.abs(q["quantize_post_proj"][0, 0] - F[case + "/quantize_post_proj"])))
    pos = st["final_atom_positions"][0, 0]
    e_atoms = float(np.max(np.abs(pos[:n_node] - F[case + "/final_atom_positions"])))
    print(f"{case}: up_proj {e_up:.2e} atoms {e_atoms:.2e}")
    assert e_up < AE_TOL_UP
    assert e_atoms < AE_TOL_ATOMS
    assert np.array_equal(st["final_atom_mask"][0, 0], F[case + "/final_atom_mask"])
    assert np.all(pos[n_node:] == 0)
    ref_zero = F[case + "/final_atom_positions"] == 0
    assert np.all(pos[:n_node][ref_zero] == 0)  # UNK rows and non-backbone atoms


def test_prepare_ae_fn_equals_tokenize_then_decode():
    """The autoencoder pass is the tokenize path followed by the decode path: at df 1 (node
    count = tokens) its atoms are bitwise the token-file decode's and its tokens the tokenize
    fn's; at df 4 with node counts that are multiples of 4 the same holds."""
    for cb, df, lens in ((4096, 1, (51, 97, 200)), (64000, 4, (52, 96, 200))):
        cfg = C.tokenizer_config(cb, df)
        D = len(cfg.levels)
        mp = runner.ReplicatedParams(P.params_keys_conversion(P.random_full_params(D, 31)), [0])
        ss = [synthetic.synthetic_protein(m, 700 + m) for m in lens]
        batch = runner.batch_collate([1, 3], ss)
        ae = runner.InferenceRunner.prepare_ae_fn(cfg, [0])
        st, q = ae(mp, None, batch)
        ae.close()
        tok_fn = runner.InferenceRunner.prepare_tokenize_fn(cfg, [0], emit_aux=True)
        q2 = tok_fn(mp, None, batch)
        tok_fn.close()
        for k in ("tokens", "n_tokens", "quantize", "continuous_embedding", "distances", "soft_proba"):
            assert np.array_equal(q[k], q2[k]), k
        dec = runner.InferenceRunner.prepare_decode_fn(cfg, [0])
        mask = (np.arange(q["tokens"].shape[-1])[None] < q["n_tokens"].reshape(3, 1)).astype(np.int64)
        d = dec(mp, None, q["tokens"].reshape(1, 3, -1), mask.reshape(1, 3, -1))
        dec.close()
        for b, m in enumerate(lens):
            got = st["final_atom_positions"][0, b, :m]
            want = d["final_atom_positions"][0, b, :m]
            bb = [0, 1, 2, 4]  # backbone atoms bitwise; the others are zeros (signs may differ)
            assert np.array_equal(got[:, bb].view(np.uint32), want[:, bb].view(np.uint32)), (cb, df, b)
            assert np.array_equal(got, want), (cb, df, b)
