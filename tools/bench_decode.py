"""Decode-path throughput: B proteins × T tokens (random ids, random-init weights) through
pst_decoder_decode (host token ids in, host atom37 out). Prints one JSON line.

    python tools/bench_decode.py [--proteins 8] [--tokens 256] [--codebook 4096] [--df 1] [--reps 3]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "protein-structure-tokenizer_amd"))
import torch  # noqa: E402,F401  (torch's HIP runtime first)

from pst_amd import params as P  # noqa: E402
from pst_amd._native import Decoder  # noqa: E402
from pst_amd.config import LEVELS  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from provenance import provenance  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--proteins", type=int, default=8)
ap.add_argument("--tokens", type=int, default=256)
ap.add_argument("--codebook", type=int, default=4096)
ap.add_argument("--df", type=int, default=1)
ap.add_argument("--reps", type=int, default=3)
a = ap.parse_args()
D = len(LEVELS[a.codebook])
dec = Decoder(0, a.codebook, a.df, P.pack_decoder(P.random_full_params(D, 5), D))
rng = np.random.default_rng(0)
toks = [rng.integers(0, a.codebook, a.tokens) for _ in range(a.proteins)]
dec.decode(toks[:1])
t0 = time.perf_counter()
for _ in range(a.reps):
    out = dec.decode(toks)
dt = (time.perf_counter() - t0) / a.reps
N = a.tokens * a.df
# stage times (HIP events on the decoder's stream, direct launches) and the dominant kernel's
# roofline: k_pair_fused executes MFMA_PER_PAIR_TILE v_mfma_f32_32x32x2_f32 per 32-pair tile
# (pst_decode.hip k_pair_fused: 13 K=128 tile GEMMs x 256 — out1 x4, out2 x2, right1 x2, seq_linear,
# pt1 x2, pt2 x2 — + 2 bias k-step groups x 4 + the 64-step narrow attention-bias GEMM = 3 400)
MFMA_PER_PAIR_TILE = 13 * 256 + 2 * 4 + 64
# launches per fold iteration (pst_decode.hip decode_group): the 384 -> 1152 IPA input GEMM,
# k_ipa_points, k_ipa_attn, k_ipa_values (+ the local frames, round 6), the 2112 -> 384 output
# projection GEMM, k_fold_tail (+ the backbone update and geometry, round 6); 8 before round 6
FOLD_LAUNCHES_PER_ITERATION = 6
FOLD_ITERATIONS = 8
PEAK_FP32_TFLOPS = 157.3
dec.set_timing(True)
for _ in range(a.reps):
    dec.decode(toks)
st = {k: v / a.reps for k, v in dec.stage_ms().items()}
dec.set_timing(False)
tiles = a.proteins * ((N * N + 31) // 32)  # one group: pairs of each protein, 32-pair tiles
ex = tiles * MFMA_PER_PAIR_TILE * 32 * 32 * 2 * 2 / (st["k_pair_fused"] * 1e-3) / 1e12
print(json.dumps({"path": "decode (tokens -> backbone atom37)", "proteins": a.proteins, "tokens_per_protein": a.tokens,
                  "residues_per_protein": N, "codebook": a.codebook, "df": a.df, "ms_per_batch": round(dt * 1e3, 2),
                  "residues_per_s": round(a.proteins * N / dt, 1), "finite": bool(all(np.isfinite(o).all() for o in out)),
                  "stage_ms": {k: round(v, 3) for k, v in st.items()},
                  "fold": {"iterations": FOLD_ITERATIONS, "launches_per_iteration": FOLD_LAUNCHES_PER_ITERATION,
                           "us_per_launch": round(st["fold"] * 1e3 / (FOLD_ITERATIONS * FOLD_LAUNCHES_PER_ITERATION), 1)}
                  if "fold" in st else None,
                  "roofline": {"kernel": "k_pair_fused (pair chain of the sequence decoder + structure-module pair inputs)",
                               "bound": "mfma", "achieved": round(ex, 2), "peak": PEAK_FP32_TFLOPS, "unit": "TFLOP/s",
                               "frac": round(ex / PEAK_FP32_TFLOPS, 4), "mfma_per_32_pair_tile": MFMA_PER_PAIR_TILE,
                               "launch_ms": round(st["k_pair_fused"], 3),
                               "note": "executed f32 MFMA FLOPs / HIP-event launch time (timed pass without graph replay)"},
                  "provenance": provenance()}))
dec.close()
