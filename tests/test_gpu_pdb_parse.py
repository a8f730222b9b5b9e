"""The GPU PDB parse of pst_tokenize_pdb_files (pst_pdb_gpu.hip) against the native host parser
(pst_pdb.cpp, itself record-equal to pst_amd/pdb.py): the atom37 rows it writes into the
tokenizer's inputs must be the host parser's bit for bit, file for file, and so must the tokens;
files outside the GPU fast path must go to the host parser (with its results and its errors)."""
import os
import tarfile

import numpy as np
import pytest

from pst_amd import params as P

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def casp(tmp_path_factory):
    d = tmp_path_factory.mktemp("casp")
    with tarfile.open(os.path.join(GOLD, "casp14_pdbs.tar.gz")) as tf:
        tf.extractall(d, members=[m for m in tf.getmembers() if m.isfile() and m.name.endswith(".pdb")])
    return sorted(str(p) for p in (d / "casp14_pdbs").glob("*.pdb"))


@pytest.fixture(scope="module")
def tk():
    from pst_amd._native import Tokenizer
    t = Tokenizer(0, 4096, 1, P.random_blob(6, 1234))
    yield t
    t.close()


def _host(paths):
    from pst_amd._native import parse_pdb_files
    return parse_pdb_files(paths, n_threads=8, float32=True)


def _check_equal(tk, paths, host_files):
    tok, nt, nn, off = tk.tokenize_pdb_files(paths)
    assert tk.pdb_files_host_parsed() == host_files
    B = _host(paths)
    assert np.array_equal(off, B.offsets)
    R = int(off[-1])
    pos = tk.debug_fetch(13, R)
    fl = tk.debug_fetch(14, R)
    assert np.array_equal(pos.view(np.uint32), B.positions.view(np.uint32))
    assert np.array_equal(fl, B.flags)
    tok2, nt2, nn2 = tk.tokenize_packed(B.positions, B.flags, B.offsets)
    assert np.array_equal(nt, nt2) and np.array_equal(nn, nn2)
    for i in range(len(paths)):
        a = int(off[i])
        assert np.array_equal(tok[a:a + nt[i]], tok2[a:a + nt2[i]]), paths[i]


def test_casp14_files_parsed_on_gpu_equal_host_parser(tk, casp):
    """All 31 CASP14 structures take the GPU path (T1024's header has '\\r' line breaks) and give
    the host parser's rows bit for bit, and the same tokens. Then once more from a token buffer too
    small for the batch: the call reports R, the binding grows its buffer and repeats it."""
    _check_equal(tk, casp, host_files=0)
    tk._pdb_tok = np.empty(16, np.uint32)
    _check_equal(tk, casp, host_files=0)
    assert tk._pdb_tok.size >= 5618


def test_large_files_send_the_call_to_the_host_parser(casp, monkeypatch):
    """A file at or above the GPU path's size bound (1 GB: offsets inside a file are 32-bit on the
    GPU) sends the whole call to the native host parser; PST_PDB_GPU_MAX_FILE lowers the bound so
    the route runs here: every CASP14 file host-parsed, rows and tokens as the host parser's."""
    from pst_amd._native import Tokenizer
    monkeypatch.setenv("PST_PDB_GPU_MAX_FILE", "1000")
    t = Tokenizer(0, 4096, 1, P.random_blob(6, 1234))
    try:
        _check_equal(t, casp, host_files=len(casp))
    finally:
        t.close()


def _lines(path):
    with open(path) as fh:
        return fh.read().split("\n")


def _write(tmp_path, name, lines, nl="\n"):
    p = tmp_path / name
    p.write_bytes(nl.join(lines).encode())
    return str(p)


def test_fast_path_variants_and_host_path_triggers(tk, casp, tmp_path):
    """Files built from CASP14 structures: ones the GPU path must take (CRLF endings, no trailing
    newline, an atom name outside atom37, a duplicated atom record, HETATM water and a ligand after
    the chain's residues, a non-standard residue name, two chains) and ones it must hand to the
    host parser (altloc records, MODEL/ENDMDL, a tab, a chain that reappears, a coordinate not in
    %8.3f form, residue numbers that decrease within a chain); one call for all of them."""
    base = _lines(casp[1])
    atoms = [i for i, l in enumerate(base) if l.startswith("ATOM  ")]
    a0, a1 = atoms[0], atoms[-1]

    def with_line(idx, new):
        out = list(base)
        out[idx] = new
        return out

    first = base[a0]
    files, host = [], 0
    # --- GPU path
    files.append(_write(tmp_path, "crlf.pdb", base, nl="\r\n"))
    files.append(_write(tmp_path, "noeol.pdb", [l for l in base if l]))
    files.append(_write(tmp_path, "hname.pdb", base[:a0 + 1] + [first[:12] + " H  " + first[16:]] + base[a0 + 1:]))
    files.append(_write(tmp_path, "dup.pdb", base[:a0 + 1] + [first[:30] + "  99.000  99.000  99.000" + first[54:]]
                        + base[a0 + 1:]))
    last = base[a1]
    rs = int(last[22:26])
    het = ["HETATM" + last[6:17] + "HOH" + last[20:22] + f"{rs + 5:4d}" + last[26:],
           "HETATM" + last[6:12] + " CA " + last[16:17] + "MSE" + last[20:22] + f"{rs + 6:4d}" + last[26:]]
    files.append(_write(tmp_path, "het.pdb", base[:a1 + 1] + het + base[a1 + 1:]))
    mse = [l[:17] + "MSE" + l[20:] if l.startswith("ATOM  ") and int(l[22:26]) == int(first[22:26]) else l
           for l in base]
    files.append(_write(tmp_path, "mse.pdb", mse))
    chB = [l[:21] + "B" + l[22:] if l.startswith("ATOM  ") and int(l[22:26]) > rs - 20 else l for l in base]
    files.append(_write(tmp_path, "twochains.pdb", chB))
    # --- host path
    alt = [first[:16] + "A" + first[17:54] + "  0.40" + first[60:], first[:16] + "B" + first[17:30] +
           "   1.000   2.000   3.000" + first[54:54] + "  0.60" + first[60:]]
    files.append(_write(tmp_path, "altloc.pdb", base[:a0] + alt + base[a0 + 1:]))
    files.append(_write(tmp_path, "model.pdb", base[:a0] + ["MODEL        1"] + base[a0:a1 + 1] + ["ENDMDL"]
                        + base[a1 + 1:]))
    files.append(_write(tmp_path, "tab.pdb", ["REMARK\tTAB"] + base))
    chABA = [l[:21] + "B" + l[22:] if l.startswith("ATOM  ") and rs - 40 < int(l[22:26]) <= rs - 20 else l
             for l in base]
    files.append(_write(tmp_path, "reappear.pdb", chABA))
    files.append(_write(tmp_path, "coord.pdb", with_line(a0 + 3, base[a0 + 3][:30] + "  1.5e+0" + base[a0 + 3][38:])))
    low = int(first[22:26]) - 5  # the chain's last residue renumbered below its first: not increasing
    files.append(_write(tmp_path, "desc.pdb", [l[:22] + f"{low:4d}" + l[26:] if l.startswith("ATOM  ")
                                               and int(l[22:26]) == rs else l for l in base]))
    host = 6
    # a water numbered below the chain's residues is a residue of its own (het flag "W"): GPU path
    hetlow = ["HETATM" + last[6:17] + "HOH" + last[20:22] + f"{low:4d}" + last[26:]]
    files.append(_write(tmp_path, "hetlow.pdb", base[:a1 + 1] + hetlow + base[a1 + 1:]))
    _check_equal(tk, files + casp[:2], host_files=host)


def test_host_path_errors_are_the_host_parsers(tk, casp, tmp_path):
    """Errors come from the host parser with its messages: two models, an insertion code, a
    missing file (files without coordinates: the test below)."""
    from pst_amd._native import PstError
    base = _lines(casp[2])
    atoms = [i for i, l in enumerate(base) if l.startswith("ATOM  ")]
    two = base[:atoms[0]] + ["MODEL        1"] + base[atoms[0]:atoms[-1] + 1] + ["ENDMDL", "MODEL        2"] + \
        base[atoms[0]:atoms[-1] + 1] + ["ENDMDL"]
    bad = _write(tmp_path, "two.pdb", two)
    with pytest.raises(Exception, match="Only single model PDBs are supported. Found 2 models"):
        tk.tokenize_pdb_files([casp[0], bad])
    ins = [l[:26] + "A" + l[27:] if i == atoms[5] else l for i, l in enumerate(base)]
    bad = _write(tmp_path, "ins.pdb", ins)
    with pytest.raises(Exception, match="insertion code"):
        tk.tokenize_pdb_files([bad])
    with pytest.raises(ValueError, match="cannot open"):
        tk.tokenize_pdb_files([casp[0], str(tmp_path / "missing.pdb")])
    # the context keeps working after the errors
    _check_equal(tk, casp[:3], host_files=0)


@pytest.mark.parametrize("kind", ["empty", "header", "remark_ter", "crlf_header"])
def test_files_without_coordinates_take_the_host_parsers_error(tk, casp, tmp_path, kind):
    """A file with no ATOM / HETATM / MODEL line (empty, header-only, REMARK/TER-only) has no
    coordinate section: the GPU scan hands it to the host parser, whose error is the reference's
    ("Found 0 models", protein_structure_sample.py:166-248 via Bio's empty structure), alone and
    beside GPU-path files; the context stays usable afterwards."""
    base = _lines(casp[0])
    header = [l for l in base[:40] if not l.startswith(("ATOM", "HETATM", "MODEL"))]
    body = {"empty": [], "header": header, "remark_ter": ["REMARK   1 NOTHING HERE", "TER", "END"],
            "crlf_header": header}[kind]
    path = _write(tmp_path, f"{kind}.pdb", body, nl="\r\n" if kind == "crlf_header" else "\n")
    with pytest.raises(ValueError) as host_err:
        _host([path]).sample(0)
    for paths in ([path], [casp[0], path, casp[1]]):
        with pytest.raises(Exception) as gpu_err:
            tk.tokenize_pdb_files(paths)
        assert "Found 0 models" in str(gpu_err.value)
    assert "Found 0 models" in str(host_err.value)
    _check_equal(tk, casp[:3], host_files=0)
