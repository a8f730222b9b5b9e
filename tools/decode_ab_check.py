"""Decode the same random tokens with the in-tree libpst and with PST_LIB=<variant> (separate
processes) and report whether the atom outputs are bitwise equal. Writes gpurun_out/dec_<tag>.npy.
    python tools/decode_ab_check.py TAG   (run once per library, then: --compare TAG_A TAG_B)"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if sys.argv[1] == "--compare":
    a = np.load(os.path.join(ROOT, "gpurun_out", f"dec_{sys.argv[2]}.npy"))
    b = np.load(os.path.join(ROOT, "gpurun_out", f"dec_{sys.argv[3]}.npy"))
    print("bitwise equal:", np.array_equal(a.view(np.uint32), b.view(np.uint32)), "max diff", float(np.max(np.abs(a - b))))
    sys.exit(0)
sys.path.insert(0, os.path.join(ROOT, "protein-structure-tokenizer_amd"))
import torch  # noqa: E402,F401
from pst_amd import params as P  # noqa: E402
from pst_amd._native import Decoder  # noqa: E402
rng = np.random.default_rng(3)
toks = [rng.integers(0, 4096, n) for n in (256, 131, 64, 200)]
dec = Decoder(0, 4096, 1, P.pack_decoder(P.random_full_params(6, 5), 6))
out = np.concatenate([a.reshape(-1) for a in dec.decode(toks)])
dec.close()
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
np.save(os.path.join(ROOT, "gpurun_out", f"dec_{sys.argv[1]}.npy"), out)
