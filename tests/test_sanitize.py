"""Sanitizer builds of the host code: libpst's native PDB parser, host thread pool and
token-file writer under AddressSanitizer + UndefinedBehaviorSanitizer and under ThreadSanitizer
(`make -C protein-structure-tokenizer_amd/csrc asan tsan`, harness
`csrc/sanitize/pdb_harness.cpp`: the CASP14 files plus ~170 malformed / truncated / corrupted
variants of each), and the C oracle under ASan + UBSan (`make -C oracle asan`,
`oracle/sanitize_harness.c`) on a ragged batch whose tokens must equal the normal build's.
CPU only; a sanitizer finding aborts the harness with a non-zero status and its report."""
import os
import shutil
import subprocess
import tarfile

import numpy as np
import pytest

from oracle import oracle as O
from pst_amd import params as P
from pst_amd import synthetic
from pst_amd._native import pack_samples
from pst_amd.config import LEVELS

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "protein-structure-tokenizer_amd", "csrc")
SAN = os.path.join(ROOT, "protein-structure-tokenizer_amd", "pst_amd", "_lib", "san")
ORACLE = os.path.join(ROOT, "oracle")

pytestmark = pytest.mark.skipif(shutil.which("g++") is None or shutil.which("make") is None,
                                reason="needs g++ and make")


@pytest.fixture(scope="module")
def casp14_files(tmp_path_factory):
    d = tmp_path_factory.mktemp("c14")
    with tarfile.open(os.path.join(ROOT, "tests", "golden", "casp14_pdbs.tar.gz")) as tf:
        tf.extractall(d, members=[m for m in tf.getmembers() if m.isfile() and m.name.endswith(".pdb")])
    return sorted(str(p) for p in (d / "casp14_pdbs").iterdir())


def _run(cmd, **kw):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:halt_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1", TSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run(cmd, capture_output=True, text=True, env=env, timeout=600, **kw)
    assert r.returncode == 0, f"{cmd[0]} rc={r.returncode}\n{r.stdout[-3000:]}\n{r.stderr[-6000:]}"
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr
    assert "WARNING: ThreadSanitizer" not in r.stderr
    return r


@pytest.mark.parametrize("kind,n_files", [("asan", 31), ("tsan", 6)])
def test_parser_pool_writer_under_sanitizer(tmp_path, casp14_files, kind, n_files):
    _run(["make", "-s", "-C", CSRC, kind])
    cmd = [os.path.join(SAN, f"pdb_harness_{kind}"), str(tmp_path)] + casp14_files[:n_files]
    if kind == "tsan":
        # TSan refuses to start when the kernel places a mapping outside its shadow layout (high
        # ASLR entropy on some hosts): that is the runtime failing to start, not a finding
        probe = subprocess.run(cmd[:1] + [str(tmp_path / "probe")], capture_output=True, text=True, timeout=60)
        if "ThreadSanitizer: unexpected memory mapping" in probe.stderr:
            pytest.skip("TSan runtime cannot start on this host (unexpected memory mapping)")
    r = _run(cmd)
    assert "0 check failures" in r.stdout, r.stdout


def test_oracle_under_asan_ubsan(tmp_path):
    _run(["make", "-s", "-C", ORACLE, "asan"])
    levels = LEVELS[4096]
    D, df = len(levels), 2
    ss = [synthetic.synthetic_protein(n, 50 + n) for n in (52, 61, 130)]
    pos, flags, off = pack_samples(ss)
    flags = flags.copy()
    flags[70, 0] = 0  # a residue without backbone (dropped by the graph)
    blob = P.random_blob(D, 1234)
    inp, out = tmp_path / "in.bin", tmp_path / "out.bin"
    with open(inp, "wb") as fh:
        fh.write(np.array([D, df, len(ss)], np.int32).tobytes())
        fh.write(np.asarray(levels, np.int32).tobytes())
        fh.write(np.asarray(off, np.int64).tobytes())
        fh.write(np.ascontiguousarray(blob, np.float32).tobytes())
        fh.write(np.ascontiguousarray(pos, np.float64).tobytes())
        fh.write(np.ascontiguousarray(flags, np.uint8).tobytes())
    _run([os.path.join(ORACLE, "_build", "san", "oracle_harness_asan"), str(inp), str(out)])
    R = int(off[-1])
    raw = np.fromfile(out, np.uint8)
    tok = raw[:4 * R].view(np.uint32)
    nt = raw[4 * R:].view(np.int32)
    want_tok, want_nt = O.tokenize_batch(blob, levels, df, pos, flags, off, n_threads=2)
    assert np.array_equal(nt, want_nt)
    for b in range(len(ss)):
        a = int(off[b])
        assert np.array_equal(tok[a:a + nt[b]], want_tok[a:a + nt[b]]), b
