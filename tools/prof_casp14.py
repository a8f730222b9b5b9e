"""SURVEY config 2 on the device path: the 31 CASP14 structures (5 618 residues, codebook 4096,
df 1), inputs resident in HBM, tokenized --reps times (small batch → split MPNN schedule).
Prints one JSON line with the per-stage times; run under rocprofv3 for per-kernel numbers.

    python tools/prof_casp14.py [--reps 20]
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
import torch  # noqa: E402

from pst_amd import params as P  # noqa: E402
from pst_amd._native import Tokenizer, parse_pdb_files  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=20)
a = ap.parse_args()
with tempfile.TemporaryDirectory() as d:
    with tarfile.open(os.path.join(ROOT, "tests", "golden", "casp14_pdbs.tar.gz")) as tf:
        tf.extractall(d, members=[m for m in tf.getmembers() if m.isfile() and m.name.endswith(".pdb")])
    files = sorted(os.path.join(d, "casp14_pdbs", f) for f in os.listdir(os.path.join(d, "casp14_pdbs")))
    B = parse_pdb_files(files, n_threads=16)
dev = torch.device("cuda", 0)
d_pos = torch.from_numpy(np.ascontiguousarray(B.positions, np.float64)).to(dev)
d_flags = torch.from_numpy(np.ascontiguousarray(B.flags, np.uint8)).to(dev)
off = np.ascontiguousarray(B.offsets, np.int64)
R = int(off[-1])
d_tok = torch.zeros(R, dtype=torch.int32, device=dev)
d_nt = torch.zeros(len(off) - 1, dtype=torch.int32, device=dev)
d_nn = torch.zeros(len(off) - 1, dtype=torch.int32, device=dev)
tk = Tokenizer(0, 4096, 1, P.random_blob(6, 1234))


def step():
    tk.tokenize_device(d_pos.data_ptr(), d_flags.data_ptr(), off, d_tok.data_ptr(), d_nt.data_ptr(), d_nn.data_ptr())


for _ in range(3):
    step()
tk.sync()
t0 = time.perf_counter()
for _ in range(a.reps):
    step()
tk.sync()
dt = (time.perf_counter() - t0) / a.reps
tk.set_timing(True)
step()
st = tk.stage_ms()
tk.set_timing(False)
print(json.dumps({"workload": "CASP14 31 structures, codebook 4096, df 1, device-resident", "residues": R,
                  "ms_per_call": round(dt * 1e3, 3), "residues_per_s": round(R / dt, 1),
                  "stage_ms": {k: round(v, 3) for k, v in st.items()}}))
tk.close()
