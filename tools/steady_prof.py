"""Device-resident tokenize steps back to back (inputs already in HBM, no idle gap between steps),
for a rocprofv3 --kernel-trace --stats summary whose per-launch averages are steady-state figures
(the bench's host-path steps leave the compute stream idle during their copies, and the first
launches after an idle gap run slow: profiles/r03_kernel_trace_spread.txt).

    rocprofv3 --kernel-trace --stats ... -- python tools/steady_prof.py [--proteins 1024] [--reps 10]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "protein-structure-tokenizer_amd")]
import torch  # noqa: E402

from pst_amd import params as P, synthetic  # noqa: E402
from pst_amd._native import Tokenizer, pack_samples  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--proteins", type=int, default=1024)
ap.add_argument("--residues", type=int, default=256)
ap.add_argument("--reps", type=int, default=10)
a = ap.parse_args()
samples = synthetic.synthetic_batch(a.proteins, a.residues, seed=1000)
pos, flags, off = pack_samples(samples)
R = int(off[-1])
tk = Tokenizer(0, 4096, 1, P.random_blob(6, 1234))
d_pos = torch.from_numpy(pos).cuda()
d_fl = torch.from_numpy(flags).cuda()
d_tok = torch.zeros(R, dtype=torch.int32, device="cuda")
d_nt = torch.zeros(len(samples), dtype=torch.int32, device="cuda")
d_nn = torch.zeros(len(samples), dtype=torch.int32, device="cuda")
for _ in range(3 + a.reps):  # warm-up steps, then the steps the summary is read from
    tk.tokenize_device(d_pos.data_ptr(), d_fl.data_ptr(), off, d_tok.data_ptr(), d_nt.data_ptr(), d_nn.data_ptr())
tk.sync()
print("steady-state steps done:", 3 + a.reps, "x", a.proteins, "proteins")
tk.close()
