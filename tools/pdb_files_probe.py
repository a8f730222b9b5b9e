"""pst_tokenize_pdb_files on the 31 CASP14 files (config 2): wall time per call (median of --reps
after warm-up), split into the host phases by timing the same call with the GPU work cut short is
not possible from outside, so run it under `rocprofv3 --kernel-trace --memory-copy-trace` and read
the device timeline with tools/pdb_files_timeline.py. Calls are 5 ms apart so they separate.

    python tools/pdb_files_probe.py [--reps 20]
"""
import argparse
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
from pst_amd._native import Tokenizer  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=20)
a = ap.parse_args()
shm = "/dev/shm" if os.path.isdir("/dev/shm") and os.access("/dev/shm", os.W_OK) else None
with tempfile.TemporaryDirectory(dir=shm) as d:
    with tarfile.open(os.path.join(ROOT, "tests", "golden", "casp14_pdbs.tar.gz")) as tf:
        tf.extractall(d, members=[m for m in tf.getmembers() if m.isfile() and m.name.endswith(".pdb")])
    files = sorted(os.path.join(d, "casp14_pdbs", f) for f in os.listdir(os.path.join(d, "casp14_pdbs")))
    tk = Tokenizer(0, 4096, 1, P.random_blob(6, 1234))
    for _ in range(3):
        tk.tokenize_pdb_files(files, n_threads=16)
    ts, tr = [], []
    for _ in range(a.reps):
        time.sleep(0.005)
        t0 = time.perf_counter()
        tok, nt, nn, off = tk.tokenize_pdb_files(files, n_threads=16)
        ts.append(time.perf_counter() - t0)
    for _ in range(a.reps):  # reading the texts alone (Python, one thread) for scale
        t0 = time.perf_counter()
        for f in files:
            with open(f, "rb") as fh:
                fh.read()
        tr.append(time.perf_counter() - t0)
    R = int(off[-1])
    print(json.dumps({"residues": R, "ms_per_call": round(float(np.median(ts)) * 1e3, 3),
                      "ms_min": round(min(ts) * 1e3, 3), "python_read_ms": round(float(np.median(tr)) * 1e3, 3),
                      "bytes": int(sum(os.path.getsize(f) for f in files))}))
    tk.close()
