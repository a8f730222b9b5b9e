"""Where the native parse of the 31 CASP14 files spends its time (best of 7):
C call alone (pst_pdb_parse_files), the copy-out (_collect_pdb), both through parse_pdb_files."""
import ctypes
import json
import os
import sys
import tarfile
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "protein-structure-tokenizer_amd"))
from pst_amd import _native  # noqa: E402

out = {}
with tempfile.TemporaryDirectory() as d:
    with tarfile.open(os.path.join(ROOT, "tests", "golden", "casp14_pdbs.tar.gz")) as tf:
        tf.extractall(d, members=[m for m in tf.getmembers() if m.isfile() and m.name.endswith(".pdb")])
    files = sorted(os.path.join(d, "casp14_pdbs", f) for f in os.listdir(os.path.join(d, "casp14_pdbs")))
    L = _native.lib()
    enc = [os.fsencode(p) for p in files]
    arr = (ctypes.c_char_p * len(enc))(*enc)
    texts = [open(f, "rb").read() for f in files]
    tarr = (ctypes.c_char_p * len(texts))(*texts)
    lens = (ctypes.c_size_t * len(texts))(*[len(t) for t in texts])
    for th in (1, 4, 8, 16, 32):
        c_ms, s_ms, cp_ms = [], [], []
        for _ in range(7):
            h = ctypes.c_void_p()
            t0 = time.perf_counter()
            L.pst_pdb_parse_files(arr, len(enc), b"\0", th, ctypes.byref(h))
            t1 = time.perf_counter()
            _native._collect_pdb(h)
            t2 = time.perf_counter()
            h2 = ctypes.c_void_p()
            L.pst_pdb_parse_strings(tarr, lens, len(texts), b"\0", th, ctypes.byref(h2))
            t3 = time.perf_counter()
            L.pst_pdb_batch_free(h2)
            c_ms.append(t1 - t0)
            cp_ms.append(t2 - t1)
            s_ms.append(t3 - t2)
        out[f"{th}t"] = {"parse_files_ms": round(min(c_ms) * 1e3, 3), "collect_ms": round(min(cp_ms) * 1e3, 3),
                         "parse_strings_ms": round(min(s_ms) * 1e3, 3)}
print(json.dumps(out))
