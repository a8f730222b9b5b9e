"""Config 2 through the CLI's host path, piece by piece: native parse of the 31 CASP14 files
(thread counts 1/4/8/16), tokenize from host buffers, token-file writes (1/4/16 threads).
Best of 5 per setting; one JSON line.  python tools/casp14_e2e.py"""
import json
import os
import sys
import tarfile
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "protein-structure-tokenizer_amd"))
import torch  # noqa: E402,F401
from pst_amd import params as P  # noqa: E402
from pst_amd._native import Tokenizer, parse_pdb_files  # noqa: E402
from pst_amd.runner import save_npy_files  # noqa: E402

out = {}
with tempfile.TemporaryDirectory() as d:
    with tarfile.open(os.path.join(ROOT, "tests", "golden", "casp14_pdbs.tar.gz")) as tf:
        tf.extractall(d, members=[m for m in tf.getmembers() if m.isfile() and m.name.endswith(".pdb")])
    files = sorted(os.path.join(d, "casp14_pdbs", f) for f in os.listdir(os.path.join(d, "casp14_pdbs")))
    for th in (1, 4, 8, 16):
        ts = []
        for _ in range(5):
            t0 = time.perf_counter()
            B = parse_pdb_files(files, n_threads=th)
            ts.append(time.perf_counter() - t0)
        out[f"parse_ms_{th}t"] = round(min(ts) * 1e3, 3)
    for th in (8, 16):
        ts = []
        for _ in range(5):
            t0 = time.perf_counter()
            B32 = parse_pdb_files(files, n_threads=th, float32=True)
            ts.append(time.perf_counter() - t0)
        out[f"parse_f32_ms_{th}t"] = round(min(ts) * 1e3, 3)
    tk = Tokenizer(0, 4096, 1, P.random_blob(6, 1234))
    ts = []
    for _ in range(5):
        t0 = time.perf_counter()
        tok, nt, _ = tk.tokenize_packed(B.positions, B.flags, B.offsets)
        ts.append(time.perf_counter() - t0)
    out["tokenize_ms"] = round(min(ts) * 1e3, 3)
    # float32 positions (the CLI's wire format) from pageable vs page-locked host memory
    pin_p = torch.from_numpy(np.ascontiguousarray(B32.positions)).pin_memory().numpy()
    pin_f = torch.from_numpy(np.ascontiguousarray(B32.flags)).pin_memory().numpy()
    for name, (pp, pf) in (("tokenize_f32_pageable_ms", (B32.positions, B32.flags)), ("tokenize_f32_pinned_ms", (pin_p, pin_f))):
        ts = []
        for _ in range(7):
            t0 = time.perf_counter()
            tk.tokenize_packed(pp, pf, B32.offsets)
            ts.append(time.perf_counter() - t0)
        out[name] = round(sorted(ts)[3] * 1e3, 3)
    arrs = [tok[int(B.offsets[i]):int(B.offsets[i]) + nt[i]].reshape(1, -1) for i in range(len(files))]
    for th in (1, 4, 16):
        ts = []
        for rep in range(5):
            od = os.path.join(d, f"o{th}_{rep}")
            os.makedirs(od)
            paths = [os.path.join(od, os.path.basename(f)[:-4] + "_tokens") for f in files]
            t0 = time.perf_counter()
            save_npy_files(paths, arrs, threads=th)
            ts.append(time.perf_counter() - t0)
        out[f"write_ms_{th}t"] = round(min(ts) * 1e3, 3)
    tk.close()
out["residues"] = int(B.offsets[-1])
print(json.dumps(out))
