"""Host logic on CPU: PDB parser semantics, size gates, batching/collation, the runner's file
layout and the multi-rank sharding. The per-device compute is swapped for the CPU oracle in a
test-only subclass (libpst needs a GPU); everything else is the product code."""
import os

import numpy as np
import pytest

from oracle import oracle as O
from pst_amd import config as C
from pst_amd import params as P
from pst_amd import pdb, runner, synthetic
from pst_amd.sample import ProteinStructureSample

GOLD = os.path.join(os.path.dirname(__file__), "golden")


# ------------------------------------------------------------------------------ PDB parser
def _atom(serial, name, resname, chain, resseq, x, y, z, occ=1.0, altloc=" ", rec="ATOM  ", icode=" "):
    nm = name if len(name) == 4 else " " + name
    return (f"{rec}{serial:5d} {nm:<4s}{altloc}{resname:>3s} {chain}{resseq:4d}{icode}   "
            f"{x:8.3f}{y:8.3f}{z:8.3f}{occ:6.2f}{0.0:6.2f}          {name[0]:>2s}")


def _res(chain, resseq, resname="GLY", base=0.0, **kw):
    return [_atom(1, n, resname, chain, resseq, base + i, 1.0, 2.0, **kw) for i, n in enumerate(("N", "CA", "C", "O"))]


def test_parser_roundtrip_synthetic():
    s = synthetic.synthetic_protein(70, 5)
    r = pdb.protein_structure_from_pdb_string(pdb.to_pdb_string(s))
    assert r.nb_residues == 70
    assert np.array_equal(r.atom37_positions, s.atom37_positions)
    assert np.array_equal(r.atom_flags(), s.atom_flags())
    assert np.array_equal(r.aatype, s.aatype)


def test_parser_multi_model_raises():
    txt = "\n".join(["MODEL        1"] + _res("A", 1) + ["ENDMDL", "MODEL        2"] + _res("A", 1) + ["ENDMDL"])
    with pytest.raises(ValueError, match="single model"):
        pdb.protein_structure_from_pdb_string(txt)


def test_parser_insertion_code_raises():
    txt = "\n".join(_res("A", 1) + _res("A", 1, icode="B"))
    with pytest.raises(ValueError, match="insertion code"):
        pdb.protein_structure_from_pdb_string(txt)


def test_parser_altloc_highest_occupancy_and_unk():
    lines = _res("A", 1, "ALA")
    lines.append(_atom(9, "CB", "ALA", "A", 1, 5.0, 5.0, 5.0, occ=0.3, altloc="A"))
    lines.append(_atom(10, "CB", "ALA", "A", 1, 6.0, 6.0, 6.0, occ=0.7, altloc="B"))
    lines += _res("A", 2, "MSE", base=10.0, rec="HETATM")   # non-standard → UNK
    lines.append(_atom(20, "O", "HOH", "A", 3, 1.0, 1.0, 1.0, rec="HETATM"))  # water: O in atom37
    lines.append(_atom(21, "ZN", "ZN", "A", 4, 1.0, 1.0, 1.0, rec="HETATM"))  # no atom37 atom → skipped
    s = pdb.protein_structure_from_pdb_string("\n".join(lines))
    assert s.nb_residues == 3
    assert np.allclose(s.atom37_positions[0, 3], 6.0)  # CB index 3, altloc B
    assert np.argmax(s.aatype, -1).tolist() == [0, 20, 20]
    assert s.atom37_gt_exists[2].sum() == 1


def test_parser_chain_filter_and_order():
    txt = "\n".join(_res("B", 1) + _res("A", 1, base=5.0) + _res("B", 2, base=9.0))
    s = pdb.protein_structure_from_pdb_string(txt)
    assert s.nb_residues == 3
    # Bio appends a discontinuous chain to the existing one: B1, B2, then A1
    assert s.atom37_positions[:, 1, 0].tolist() == [1.0, 10.0, 6.0]
    sa = pdb.protein_structure_from_pdb_string(txt, chain_id="A")
    assert sa.nb_residues == 1


@pytest.mark.reference
def test_parser_casp14_fixture():
    import glob
    import _refenv
    F = np.load(os.path.join(GOLD, "casp14_atom37.npz"))
    files = sorted(glob.glob(os.path.join(_refenv.REF, "casp14_pdbs", "*.pdb")))
    assert len(files) == len(F["names"]) == 31
    pos = []
    for f in files:
        pos.append(pdb.protein_structure_from_pdb_file(f).atom37_positions)
    assert np.array_equal(np.concatenate(pos), F["positions"].astype(np.float64))


# ------------------------------------------------------------------------------ size gates
def _write(tmp_path, name, s):
    p = tmp_path / name
    p.write_text(pdb.to_pdb_string(s))
    return str(p)


def test_make_graph_size_gates(tmp_path):
    ok = _write(tmp_path, "ok.pdb", synthetic.synthetic_protein(60, 1))
    small = _write(tmp_path, "small.pdb", synthetic.synthetic_protein(49, 1))
    big = _write(tmp_path, "big.pdb", synthetic.synthetic_protein(513, 1))
    kw = dict(num_neighbor=50, downsampling_ratio=1, residue_loc_is_alphac=True, padding_num_residue=512)
    assert runner.make_graph_from_pdb(ok, **kw).nb_residues == 60
    with pytest.raises(NotImplementedError, match="less than 50"):
        runner.make_graph_from_pdb(small, **kw)
    with pytest.raises(NotImplementedError, match="more than 512"):
        runner.make_graph_from_pdb(big, **kw)
    with pytest.raises(NotImplementedError):
        runner.make_graph_from_pdb(ok, **dict(kw, residue_loc_is_alphac=False))


def test_batch_collate_and_shards():
    ss = [synthetic.synthetic_protein(50 + i, i) for i in range(6)]
    b = runner.batch_collate([2, 3], ss)
    assert [s.nb_residues for s in b.shard(1)] == [53, 54, 55]
    with pytest.raises(ValueError):
        runner.batch_collate([4, 2], ss)


def test_pad_token_value():
    assert runner.pad_token_value(C.LEVELS[4096]) == 2730
    assert runner.pad_token_value(C.LEVELS[64000]) == 32036


def test_prepare_devices_rejects_non_gpu_backends():
    for be in ("cpu", "tpu"):
        with pytest.raises(NotImplementedError):
            runner.InferenceRunner.prepare_devices(be)


# ------------------------------------------------------------------------------ configs
@pytest.mark.reference
@pytest.mark.parametrize("cb,df", sorted(C.SHIPPED))
def test_hydra_config_matches_shipped_table(cb, df):
    import _refenv
    cfg = C.load_config("vq3d_inference", overrides=C.overrides_for(cb, df),
                        config_path=os.path.join(_refenv.REF, "config", "structure_tokenizer"))
    got = C.config_from_hydra(cfg)
    want = C.tokenizer_config(cb, df)
    assert got.levels == want.levels and got.downsampling_ratio == df
    assert got.codebook_size == cb and got.weight_dir == want.weight_dir
    assert (got.seq_max_size, got.graph_max_neighbor, got.residue_loc_is_alphac) == (512, 50, True)


# ------------------------------------------------------------------------------ runner
class _OracleCtx:
    """Test stand-in for one libpst context: the CPU oracle behind `tokenize_packed`."""

    def __init__(self, blob, levels, df):
        self.blob, self.levels, self.df = blob, levels, df

    def tokenize_packed(self, pos, flags, off):
        tok, nt = O.tokenize_batch(self.blob, self.levels, self.df, pos, flags, off, n_threads=4)
        full = np.all(flags[:, [0, 1, 2, 4]] & 1, axis=1)  # N, CA, C, O present
        nn = np.array([int(full[off[b]:off[b + 1]].sum()) for b in range(len(off) - 1)], np.int32)
        return tok, nt, nn

    def close(self):
        pass


class OracleTokenizeFn(runner.TokenizeFn):
    def _context(self, model_params, dev):
        return _OracleCtx(model_params.blob, self.cfg.levels, self.cfg.downsampling_ratio)


def _oracle_tokens(blob, cfg, s):
    return O.tokenize(blob, cfg.levels, cfg.downsampling_ratio, s.atom37_positions, s.atom_flags())["tokens"]


@pytest.mark.parametrize("cb,df", [(4096, 1), (64000, 2)])
def test_runner_tokenize_files(tmp_path, cb, df):
    cfg = C.tokenizer_config(cb, df)
    D = len(cfg.levels)
    mdir = tmp_path / "model"
    mdir.mkdir()
    P.save_params_npz(str(mdir / "params.npz"), P.random_full_params(D, seed=11))
    ss = [synthetic.synthetic_protein(n, 40 + i) for i, n in enumerate((55, 64, 81))]
    pdbs = [_write(tmp_path, f"prot{i}.pdb", s) for i, s in enumerate(ss)]
    R = runner.InferenceRunner
    mp = R.load_params(str(mdir), [0, 1])
    fn = OracleTokenizeFn(cfg, [0, 1])
    out = str(tmp_path / "tokens")
    R.tokenize(random_key=None, quantize=fn, model_params=mp, pdbs=pdbs, token_save_path=out,
               num_device=2, data_config=cfg, batch_size_per_device=1)
    assert sorted(os.listdir(out)) == [f"prot{i}_tokens.npy" for i in range(3)]
    blob = P.pack(P.params_keys_conversion(P.random_full_params(D, seed=11)), D)
    for i, s in enumerate(ss):
        t = np.load(os.path.join(out, f"prot{i}_tokens.npy"))
        assert t.dtype == np.uint32 and t.shape == (1, s.nb_residues // df)
        assert np.array_equal(t[0], _oracle_tokens(blob, cfg, s))
    with pytest.raises(FileExistsError):
        R.tokenize(random_key=None, quantize=fn, model_params=mp, pdbs=pdbs, token_save_path=out,
                   num_device=2, data_config=cfg, batch_size_per_device=1)
    fn.close()


def test_tokenize_fn_padding_layout():
    cfg = C.tokenizer_config(4096, 1)
    mp = runner.ReplicatedParams(P.random_params(6, 2), [0])
    ss = [synthetic.synthetic_protein(n, 7 + n) for n in (52, 60)]
    fn = OracleTokenizeFn(cfg, [0])
    out = fn(mp, None, runner.batch_collate([1, 2], ss))
    assert out["tokens"].shape == (1, 2, 512) and out["tokens"].dtype == np.uint32
    assert out["n_tokens"].tolist() == [[52, 60]]
    assert np.all(out["tokens"][0, 0, 52:] == 2730) and np.all(out["tokens"][0, 1, 60:] == 2730)
    fn.close()


def test_shard_for_rank_partitions():
    items = list(range(11))
    parts = [runner.shard_for_rank(items, r, 3) for r in range(3)]
    assert sorted(sum(parts, [])) == items
    assert all(len(set(a) & set(b)) == 0 for i, a in enumerate(parts) for b in parts[i + 1:])
    with pytest.raises(ValueError):
        runner.shard_for_rank(items, 3, 3)


def test_lpt_partition_balances_residues():
    """LPT: heaviest first onto the least-loaded rank; a disjoint cover, input order
    kept inside a shard, and the max load within the LPT bound (4/3 - 1/(3W)) of the optimum."""
    rng = np.random.default_rng(0)
    w = rng.integers(50, 513, 97).tolist()
    for W in (1, 2, 3, 8):
        parts = runner.lpt_partition(w, W)
        assert sorted(sum(parts, [])) == list(range(len(w)))
        assert all(p == sorted(p) for p in parts)
        loads = [sum(w[i] for i in p) for p in parts]
        lower = max(sum(w) / W, max(w))
        assert max(loads) <= (4 / 3 - 1 / (3 * W)) * lower + 1e-9
    # exact small case: 7,6,5,4,3 on 2 ranks -> {7,4,3}=14 / {6,5}=11 greedy
    assert runner.lpt_partition([7, 6, 5, 4, 3], 2) == [[0, 3, 4], [1, 2]]
    items = list("abcde")
    assert runner.shard_for_rank(items, 1, 2, weights=[7, 6, 5, 4, 3]) == ["b", "c"]
    with pytest.raises(ValueError):
        runner.shard_for_rank(items, 0, 2, weights=[1, 2])


# ------------------------------------------------------------------------------ native parser
def _both(txt, chain_id=None):
    from pst_amd import _native
    nat = _native.parse_pdb_strings([txt], chain_id=chain_id, n_threads=1)
    try:
        py = pdb.protein_structure_from_pdb_string(txt, chain_id=chain_id)
    except ValueError as e:
        assert nat.status[0] != 0
        assert nat.errors[0] == str(e)
        return None
    s = nat.sample(0)
    assert s.nb_residues == py.nb_residues
    assert np.array_equal(s.atom37_positions, py.atom37_positions)
    assert np.array_equal(s.atom37_gt_exists, py.atom37_gt_exists)
    assert np.array_equal(s.atom37_atom_exists, py.atom37_atom_exists)
    assert np.array_equal(s.aatype, py.aatype)
    return s


def _edge_texts():
    alt = _res("A", 1, "ALA") + [_atom(9, "CB", "ALA", "A", 1, 5.0, 5.0, 5.0, occ=0.3, altloc="A"),
                                 _atom(10, "CB", "ALA", "A", 1, 6.0, 6.0, 6.0, occ=0.7, altloc="B"),
                                 _atom(11, "CB", "ALA", "A", 1, 7.0, 7.0, 7.0, occ=0.7, altloc="C")]
    het = (_res("A", 1) + _res("A", 2, "MSE", base=10.0, rec="HETATM")
           + [_atom(20, "O", "HOH", "A", 3, 1.0, 1.0, 1.0, rec="HETATM"),
              _atom(21, "ZN", "ZN", "A", 4, 1.0, 1.0, 1.0, rec="HETATM")])
    return {
        "altloc": "\n".join(alt),
        "hetero": "\n".join(het),
        "chains": "\n".join(_res("B", 1) + _res("A", 1, base=5.0) + _res("B", 2, base=9.0)),
        "multimodel": "\n".join(["MODEL        1"] + _res("A", 1) + ["ENDMDL", "MODEL        2"] + _res("A", 1) + ["ENDMDL"]),
        "onemodel": "\n".join(["MODEL        1"] + _res("A", 1) + ["ENDMDL"]),
        "icode": "\n".join(_res("A", 1) + _res("A", 1, icode="B")),
        "crlf": "\r\n".join(_res("A", 1) + _res("A", 2, base=3.0)),
        "empty": "HEADER    nothing\nEND\n",
        "same_key_het_vs_atom": "\n".join(_res("A", 5) + _res("A", 5, "GLY", base=2.0, rec="HETATM")),
        # Bio stops reading coordinates at the first CONECT / "END   " record after the header
        "after_conect": "\n".join(_res("A", 1) + ["CONECT    1    2"] + _res("A", 2, base=3.0, rec="HETATM")),
        "after_padded_end": "\n".join(_res("A", 1) + ["END   "] + _res("A", 2, base=3.0)),
        "after_bare_end": "\n".join(_res("A", 1) + ["END"] + _res("A", 2, base=3.0)),
        "conect_in_header": "\n".join(["CONECT    1    2", "END   "] + _res("A", 1) + _res("A", 2, base=3.0)),
        "record_prefix_only": "\n".join(_res("A", 1) + [l.replace("ATOM  ", "ATOMS ") for l in _res("A", 2, base=3.0)]),
    }


@pytest.mark.parametrize("case,n", [("after_conect", 1), ("after_padded_end", 1), ("after_bare_end", 2),
                                    ("conect_in_header", 2), ("record_prefix_only", 1)])
def test_parser_record_names_and_end_of_coordinates(case, n):
    assert _both(_edge_texts()[case]).nb_residues == n


@pytest.mark.parametrize("case", sorted(_edge_texts()))
def test_native_parser_matches_restatement(case):
    _both(_edge_texts()[case])


def test_native_parser_chain_filter_and_synthetic():
    assert _both(_edge_texts()["chains"], chain_id="A").nb_residues == 1
    for i, n in enumerate((50, 77, 130)):
        s = synthetic.synthetic_protein(n, 60 + i)
        got = _both(pdb.to_pdb_string(s))
        assert np.array_equal(got.atom37_positions, s.atom37_positions)


def test_native_parser_batch_errors_are_per_input(tmp_path):
    from pst_amd import _native
    good = tmp_path / "good.pdb"
    good.write_text(pdb.to_pdb_string(synthetic.synthetic_protein(55, 3)))
    bad = tmp_path / "bad.pdb"
    bad.write_text(_edge_texts()["multimodel"])
    B = _native.parse_pdb_files([str(good), str(bad), str(tmp_path / "missing.pdb"), str(good)], n_threads=3)
    assert B.status.tolist() == [0, -1, -1, 0]
    assert np.diff(B.offsets).tolist() == [55, 0, 0, 55]
    assert "single model" in B.errors[1] and "missing.pdb" in B.errors[2]
    with pytest.raises(ValueError, match="single model"):
        B.sample(1)


@pytest.mark.reference
def test_native_parser_casp14_equals_restatement():
    import glob
    import _refenv
    from pst_amd import _native
    files = sorted(glob.glob(os.path.join(_refenv.REF, "casp14_pdbs", "*.pdb")))
    B = _native.parse_pdb_files(files, n_threads=4)
    F = np.load(os.path.join(GOLD, "casp14_atom37.npz"))
    assert np.array_equal(B.offsets, F["offsets"])
    assert np.array_equal(B.positions, F["positions"].astype(np.float64))
    assert np.array_equal(B.flags, F["flags"])


def test_native_parser_casp14_archive(casp14_dir):
    from pst_amd import _native
    files = sorted(os.path.join(casp14_dir, f) for f in os.listdir(casp14_dir))
    assert len(files) == 31
    B = _native.parse_pdb_files(files, n_threads=4)
    F = np.load(os.path.join(GOLD, "casp14_atom37.npz"))
    assert [os.path.basename(f)[:-4] for f in files] == [str(x) for x in F["names"]]
    assert np.array_equal(B.offsets, F["offsets"])
    assert np.array_equal(B.positions, F["positions"].astype(np.float64))
    assert np.array_equal(B.flags, F["flags"])


def test_make_graph_no_backbone_raises_like_reference(tmp_path):
    s = synthetic.synthetic_protein(60, 2)
    gt = s.atom37_gt_exists.copy()
    gt[:, 4] = False  # every residue lacks O → reference preprocess_sample fails
    p = _write(tmp_path, "noo.pdb", s._replace(atom37_gt_exists=gt))
    with pytest.raises(ValueError, match="need at least one array"):
        runner.make_graph_from_pdb(p, num_neighbor=50, downsampling_ratio=1, residue_loc_is_alphac=True,
                                   padding_num_residue=512)


def test_npy_writer_bytes_equal_np_save(tmp_path):
    """runner.save_npy_files (the CLI's token writer) writes exactly np.save's bytes."""
    import io
    from pst_amd.runner import npy_bytes, save_npy_files
    arrs = [np.arange(391, dtype=np.uint32).reshape(1, -1), np.zeros((1, 0), np.uint32),
            np.arange(5, dtype=np.float64), np.ones((3, 4, 5), np.float32)]
    for a in arrs:
        b = io.BytesIO()
        np.save(b, a)
        assert b.getvalue() == npy_bytes(a), a.shape
    paths = [str(tmp_path / f"t{i}") for i in range(len(arrs))] + [str(tmp_path / "t0")]
    save_npy_files(paths, arrs + [arrs[0] + 1], threads=4)
    assert np.array_equal(np.load(str(tmp_path / "t0.npy")), arrs[0] + 1)
    for i in range(1, len(arrs)):
        assert np.array_equal(np.load(paths[i] + ".npy"), arrs[i])


def _big_variants():
    """Texts well above the native parser's 48 KB scan chunk, with the record sequences that
    matter placed deep inside (so they fall in later chunks or straddle chunk boundaries)."""
    lines = pdb.to_pdb_string(synthetic.synthetic_protein(400, 11)).splitlines()[:-1]  # drop END
    n = len(lines)
    k = (2 * n) // 3
    bad = lines[k][:30] + "   x.abc" + lines[k][38:]
    alt = [_atom(90000 + i, "CB", "ALA", "A", 1, 1.0 * i, 2.0, 3.0, occ=o, altloc=a)
           for i, (o, a) in enumerate(((0.2, "A"), (0.6, "B"), (0.9, " "), (0.7, "C")))]
    return {
        "plain": "\n".join(lines + ["END"]),
        "conect_late": "\n".join(lines[:k] + ["CONECT    1    2"] + lines[k:]),
        "malformed_after_conect": "\n".join(lines[:k] + ["CONECT    1    2", bad] + lines[k:]),
        "malformed_late": "\n".join(lines[:k] + [bad] + lines[k:]),
        "second_model_late": "\n".join(["MODEL        1"] + lines[:k] + ["ENDMDL", "MODEL        2"] + lines[k:]),
        "altloc_late": "\n".join(lines[:k] + alt + lines[k:]),
        "crlf": "\r\n".join(lines),
    }


@pytest.mark.parametrize("case", sorted(_big_variants()))
def test_native_parser_multichunk_matches_restatement(case):
    """The native parser scans big files in parallel line-aligned chunks and replays the records
    in order: every text above splits into >= 3 chunks and must read as the restatement does."""
    txt = _big_variants()[case]
    assert len(txt) > 2 * 48 * 1024  # >= 3 chunks
    if case == "malformed_late":  # both raise ValueError; the messages differ by design
        from pst_amd import _native
        with pytest.raises(ValueError):
            pdb.protein_structure_from_pdb_string(txt)
        nat = _native.parse_pdb_strings([txt], n_threads=4)
        assert nat.status[0] != 0 and nat.errors[0].startswith("malformed ATOM/HETATM record")
        return
    _both(txt)


def test_parse_float32_copy_is_exact():
    """pst_pdb_batch_copy_f32: the parser's coordinates are float32 values (Bio's atom.coord),
    so the float32 copy-out equals the float64 one exactly; flags, aatype and offsets equal."""
    import tarfile
    import tempfile
    from pst_amd._native import parse_pdb_files
    arc = os.path.join(os.path.dirname(__file__), "golden", "casp14_pdbs.tar.gz")
    with tempfile.TemporaryDirectory() as d:
        with tarfile.open(arc) as tf:
            tf.extractall(d, members=[m for m in tf.getmembers() if m.isfile() and m.name.endswith(".pdb")])
        files = sorted(os.path.join(d, "casp14_pdbs", f) for f in os.listdir(os.path.join(d, "casp14_pdbs")))
        a = parse_pdb_files(files, n_threads=4)
        b = parse_pdb_files(files, n_threads=4, float32=True)
    assert b.positions.dtype == np.float32
    assert np.array_equal(b.positions.astype(np.float64), a.positions)
    for k in ("flags", "aatype", "offsets", "status"):
        assert np.array_equal(getattr(a, k), getattr(b, k)), k
