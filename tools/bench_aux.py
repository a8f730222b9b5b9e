"""FSQ aux kernel bench (SURVEY config 4): the 31 CASP14 structures (tests/golden/casp14_atom37.npz),
codebook 64000, df 1; distances + soft_proba [T, 64000] f32 materialised in HBM
(pst_codebook_aux_device). Prints one JSON line: achieved write GB/s vs the HBM roofline.

    python tools/bench_aux.py [--codebook 64000] [--df 1] [--reps 20]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "protein-structure-tokenizer_amd"))
import torch  # noqa: E402

from pst_amd import params as P  # noqa: E402
from pst_amd._native import Tokenizer  # noqa: E402
from pst_amd.config import LEVELS  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from provenance import provenance  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--codebook", type=int, default=64000)
ap.add_argument("--df", type=int, default=1)
ap.add_argument("--reps", type=int, default=20)
args = ap.parse_args()

C = np.load(os.path.join(ROOT, "tests", "golden", "casp14_atom37.npz"))
pos, flags, off = C["positions"].astype(np.float64), C["flags"], C["offsets"].astype(np.int64)
dev = torch.device("cuda", 0)
K = args.codebook
tk = Tokenizer(0, K, args.df, P.random_blob(len(LEVELS[K]), 1234))
d_pos, d_flags = torch.from_numpy(pos).to(dev), torch.from_numpy(flags).to(dev)
R = int(off[-1])
d_tok = torch.zeros(R, dtype=torch.int32, device=dev)
d_nt = torch.zeros(len(off) - 1, dtype=torch.int32, device=dev)
d_nn = torch.zeros(len(off) - 1, dtype=torch.int32, device=dev)
tk.tokenize_device(d_pos.data_ptr(), d_flags.data_ptr(), off, d_tok.data_ptr(), d_nt.data_ptr(), d_nn.data_ptr())
tk.sync()
T = int(d_nt.sum().item())
cap = int(sum((off[b + 1] - off[b]) // args.df for b in range(len(off) - 1)))
dd = torch.empty((cap, K), dtype=torch.float32, device=dev)
dp = torch.empty((cap, K), dtype=torch.float32, device=dev)
da = torch.empty(cap, dtype=torch.int32, device=dev)
dh = torch.empty(K, dtype=torch.int32, device=dev)
ext = torch.cuda.ExternalStream(tk.stream, device=dev)


def run():
    tk.codebook_aux_device(dd.data_ptr(), dp.data_ptr(), da.data_ptr(), dh.data_ptr(), cap)


for _ in range(3):
    run()
tk.sync()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
with torch.cuda.stream(ext):
    e0.record()
for _ in range(args.reps):
    run()
with torch.cuda.stream(ext):
    e1.record()
e1.synchronize()
ms = e0.elapsed_time(e1) / args.reps
# algorithmic bytes per launch: 2 tensors x T x K x 4 B written + T x (argmin 4 B + latents 32 B read)
alg = 2 * T * K * 4 + T * (4 + 32)
gbs = alg / (ms * 1e-3) / 1e9
print(json.dumps({"kernel": "k_fsq_aux (+k_row_start, hist memset)", "workload": f"CASP14 31 structures, {T} tokens, K={K}, df={args.df}",
                  "ms_per_launch": round(ms, 4), "bytes_per_launch": alg, "achieved_GBps": round(gbs, 1),
                  "peak_GBps": 8000.0, "frac": round(gbs / 8000.0, 4), "bound": "hbm (write)",
                  "rows_per_s": round(T / (ms * 1e-3), 1), "provenance": provenance()}))
tk.close()
