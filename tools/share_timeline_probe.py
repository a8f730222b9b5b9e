"""The N = 8 share of config 3 (128 x 256 residues) through the host-buffer path as bench.py runs it
(float32 positions and flags in torch-pinned memory), calls 5 ms apart so a kernel + memory-copy
trace separates them (tools/pdb_files_timeline.py prints the median call). PST_H2D_DENSE selects the
wire format.   python tools/share_timeline_probe.py [--proteins 128] [--reps 10] [--save tokens.npy]"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "protein-structure-tokenizer_amd"))
import torch  # noqa: E402

from pst_amd import params as P, synthetic  # noqa: E402
from pst_amd._native import Tokenizer, pack_samples  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--proteins", type=int, default=128)
ap.add_argument("--reps", type=int, default=10)
ap.add_argument("--save", default="", help="np.save the tokens of the last call here")
a = ap.parse_args()
pos, flags, off = pack_samples(synthetic.synthetic_batch(a.proteins, 256, seed=1000))
ppos = torch.from_numpy(pos.astype(np.float32)).pin_memory().numpy()
pflags = torch.from_numpy(flags).pin_memory().numpy()
tk = Tokenizer(0, 4096, 1, P.random_blob(6, 1234))
for _ in range(3):
    tk.tokenize_packed(ppos, pflags, off)
ts = []
for _ in range(a.reps):
    time.sleep(0.005)
    t0 = time.perf_counter()
    res = tk.tokenize_packed(ppos, pflags, off)
    ts.append(time.perf_counter() - t0)
if a.save:
    np.save(a.save, res[0])
print(json.dumps({"proteins": a.proteins, "ms_median": round(float(np.median(ts)) * 1e3, 3),
                  "dense": os.environ.get("PST_H2D_DENSE", "policy")}))
tk.close()
