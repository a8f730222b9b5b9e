"""Exact-match rate and rounding-margin report of the canonical f32 path vs the
reference's float64 forward on every case of tests/golden/forward_ref_wide.npz. The C oracle runs
the GPU's operation sequence bit for bit (the -m gpu tests check GPU == oracle and GPU == fixture
tokens), so its bounded latents are the GPU's. Writes one JSON document to stdout.

    python tools/refwide_report.py > profiles/r02_exact_match_reference.json
"""
import json
import os
import sys
from concurrent.futures import ThreadPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "protein-structure-tokenizer_amd"), os.path.join(ROOT, "tests", "golden")):
    sys.path.insert(0, p)
import refwide  # noqa: E402
from oracle import oracle as O  # noqa: E402
from pst_amd import params as P  # noqa: E402
from pst_amd.config import LEVELS  # noqa: E402

F = refwide.load()


def run(c):
    n, T, cb, df, D, seed = (int(v) for v in F[c + "/meta"])
    o = O.tokenize(P.random_blob(D, seed), LEVELS[cb], df, F[c + "/in_positions"].astype(np.float64), F[c + "/in_flags"])
    return c, o


with ThreadPoolExecutor(8) as ex:
    outs = dict(ex.map(run, refwide.cases(F)))
doc = {"source": "tests/golden/forward_ref_wide.npz (make_forward_wide.py): reference Vq3D.encode_and_quantize "
                 "in float64 under the shim; ours = oracle/pst_oracle.c = GPU bits", "groups": {}}
for prefix, what in (("casp_", "CASP14 31 structures, codebook 4096 and 64000, df 1 (configs 2, 4)"),
                     ("bench256_", "bench workload proteins 0-7, 256 residues, 4096, df 1 (config 3)"),
                     ("bench512_", "512 residues, 64000, df 4 (config 5)"),
                     ("short_", "< 50 residues after filtering (preprocessing.py:229-260)")):
    for var, label in (("_pe32", "PE argument in float32 as JAX x64-off (the reference's value)"),
                       ("", "PE argument in float64")):
        reps = [refwide.report(F[c + "/bounded" + var], F[c + "/tokens" + var], outs[c]["b"], outs[c]["tokens"])
                for c in refwide.cases(F, prefix)]
        r = refwide.merge(reps)
        r["cases"] = len(reps)
        r["what"] = what
        r["reference_rendering"] = label
        doc["groups"][prefix + (var or "_pe64")] = r
allr = [doc["groups"][k] for k in doc["groups"] if k.endswith("_pe32")]
doc["all_pe32"] = {"tokens": sum(r["tokens"] for r in allr), "identical": sum(r["identical"] for r in allr),
                   "min_margin": min(r["min_margin"] for r in allr),
                   "max_deviation": max(r["max_deviation"] for r in allr),
                   "max_deviation_over_margin": max(r["max_deviation_over_margin"] for r in allr)}
print(json.dumps(doc, indent=1))
