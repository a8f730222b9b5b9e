"""Exact-match rate, rounding-margin report and deviation localisation (SURVEY
§8d) of the canonical f32 path vs the reference's forward on every case of
tests/golden/forward_ref_wide.npz, against each of its three renderings:

  _pe64  float64 throughout;
  _pe32  float64 with the PE argument in float32 as JAX forms it (the reference's PE values);
  _f32   float32 weights / edge features / PE (the shim's float32 mode, mixed: see
         make_forward_wide.py).

"ours" is the C oracle, which runs the GPU's operation sequence bit for bit (the -m gpu tests
check GPU == oracle and GPU == fixture tokens), so its latents are the GPU's. Also reported:
oracle/reference_as_computed.py (the reference's padded, dense computation in PyTorch-CPU
float32 — bench.py's CPU baseline) against the same renderings.

Localisation of the bounded-latent deviation b_ours − b_ref (b = FSQ bound of z, the down_proj
output; quantize.py:175-182): the fixture holds the reference's z of each rendering, so
  bound term   = b_canon(z_ref) − b_ref   (our float32 FSQ bound — XLA's rational tanh, float32
                 shift — applied to the reference's own z: the bound's contribution alone)
  encoder term = b_ours − b_canon(z_ref)  (the same bound applied to our z instead: what the
                 encoder + down_proj deviation |z_ours − z_ref| contributes)
Writes one JSON document to stdout.

    python tools/refwide_report.py > profiles/r03_exact_match_reference.json
"""
import ctypes
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
RENDERINGS = (("_pe32", "float64, PE argument in float32 as JAX x64-off (the reference's PE values)"),
              ("_pe64", "float64 throughout"),
              ("_f32", "float32 weights / edge features / PE, shim float32 mode (mixed precision)"))
GROUPS = (("casp_", "CASP14 31 structures, codebook 4096 and 64000, df 1 (configs 2, 4)"),
          ("bench256_", "bench workload proteins 0-7 and 200, 511, 777, 1023; 256 residues, 4096, df 1 (config 3)"),
          ("bench512_", "512 residues, 64000, df 4 (config 5)"),
          ("short_", "< 50 residues after filtering (preprocessing.py:229-260)"))


def key(c, field, var):
    return f"{c}/{field}" + ("" if var == "_pe64" else var)


def run(c):
    n, T, cb, df, D, seed = (int(v) for v in F[c + "/meta"])
    g = O.graph(F[c + "/in_positions"].astype(np.float64), F[c + "/in_flags"])
    return c, O.encode(P.random_blob(D, seed), LEVELS[cb], df, g)


_tanh = O.lib().pst_oracle_tanh
_tanh.restype = ctypes.c_float
_tanh.argtypes = [ctypes.c_float]


def canon_bound(z, levels):
    """The canonical f32 FSQ bound (pst_oracle.c FSQ block, = k_down's) applied to float32(z)."""
    z = np.asarray(z, np.float64).astype(np.float32)
    out = np.zeros(z.shape, np.float32)
    for d, L in enumerate(levels):
        half_l = np.float32(np.float32(L - 1) * np.float32(0.999)) / np.float32(2.0)
        offset = np.float32(0.5 if L % 2 == 0 else 0.0)
        shift = np.float32(np.tan(np.float64(np.float32(offset / half_l))))
        for t in range(z.shape[0]):
            out[t, d] = np.float32(np.float32(_tanh(float(np.float32(z[t, d] + shift)))) * half_l) - offset
    return out


def localise(cases, outs, var):
    """max |z_ours − z_ref|, the bound term and the encoder term over `cases`."""
    dz = bound = enc = 0.0
    for c in cases:
        if key(c, "z", var) not in F.files:
            return None
        n, T, cb, df, D, seed = (int(v) for v in F[c + "/meta"])
        zref = F[key(c, "z", var)]
        bref = F[key(c, "bounded", var)]
        bc = canon_bound(zref, LEVELS[cb]).astype(np.float64)
        o = outs[c]
        dz = max(dz, float(np.abs(o["z"].astype(np.float64) - zref).max()))
        bound = max(bound, float(np.abs(bc - bref).max()))
        enc = max(enc, float(np.abs(o["b"].astype(np.float64) - bc).max()))
    return {"max_abs_z_deviation": dz, "bound_term_max": bound, "encoder_term_max": enc}


def ref_as_computed(cases):
    """reference_as_computed.py (torch float32) token ids and bounded latents, per case."""
    import torch
    from oracle.reference_as_computed import ReferenceAsComputed, padded_graphs
    torch.set_num_threads(8)
    out = {}
    models = {}
    for c in cases:
        n, T, cb, df, D, seed = (int(v) for v in F[c + "/meta"])
        m = models.get((cb, df, seed))
        if m is None:
            m = models[(cb, df, seed)] = ReferenceAsComputed(P.random_params(D, seed), LEVELS[cb], df)
        o = m.forward(padded_graphs([(F[c + "/in_positions"].astype(np.float64), F[c + "/in_flags"])], df))
        b = o.get("bounded", o.get("continuous_embedding"))
        out[c] = {"tokens": np.asarray(o["tokens"][0, :T]),
                  "b": None if b is None else np.asarray(b[0, :T], np.float64)}
    return out


def main():
    with ThreadPoolExecutor(8) as ex:
        outs = dict(ex.map(run, refwide.cases(F)))
    rac = ref_as_computed(refwide.cases(F)) if "--no-torch" not in sys.argv else {}
    doc = {"source": "tests/golden/forward_ref_wide.npz (make_forward_wide.py): reference Vq3D.encode_and_quantize "
                     "under the shim, three renderings; ours = oracle/pst_oracle.c = GPU bits", "groups": {}}
    for var, label in RENDERINGS:
        for prefix, what in GROUPS:
            cs = refwide.cases(F, prefix)
            reps = [refwide.report(F[key(c, "bounded", var)], F[key(c, "tokens", var)], outs[c]["b"], outs[c]["tokens"])
                    for c in cs]
            r = refwide.merge(reps)
            r.update(cases=len(reps), what=what, reference_rendering=label, localisation=localise(cs, outs, var))
            if rac:
                ok = sum(int(np.sum(rac[c]["tokens"] == F[key(c, "tokens", var)])) for c in cs)
                r["reference_as_computed_torch_f32"] = {"identical": ok, "tokens": r["tokens"]}
            doc["groups"][prefix + var] = r
        allr = [doc["groups"][p + var] for p, _ in GROUPS]
        loc = [r["localisation"] for r in allr if r["localisation"]]
        doc["all" + var] = {
            "tokens": sum(r["tokens"] for r in allr), "identical": sum(r["identical"] for r in allr),
            "min_margin": min(r["min_margin"] for r in allr),
            "max_deviation": max(r["max_deviation"] for r in allr),
            "max_deviation_over_margin": max(r["max_deviation_over_margin"] for r in allr),
            "localisation": {k: max(x[k] for x in loc) for k in loc[0]} if loc else None,
            "reference_as_computed_torch_f32": ({"identical": sum(r["reference_as_computed_torch_f32"]["identical"]
                                                                  for r in allr),
                                                 "tokens": sum(r["tokens"] for r in allr)} if rac else None)}
    # the closest call (config 1's protein): every rendering
    c = "casp_T1024_k4096_df1"
    cc = {}
    for var, _ in RENDERINGS:
        m = refwide.dim_margins(F[key(c, "bounded", var)])
        t, d = np.unravel_index(int(np.argmin(m)), m.shape)
        dev = abs(float(outs[c]["b"][t, d]) - float(F[key(c, "bounded", var)][t, d]))
        zc = canon_bound(F[key(c, "z", var)][t:t + 1], LEVELS[4096])[0, d] if key(c, "z", var) in F.files else None
        cc[var] = {"token": int(t), "dim": int(d), "margin": float(m[t, d]), "our_deviation": dev,
                   "deviation_over_margin": dev / float(m[t, d]),
                   "bound_term": None if zc is None else abs(float(zc) - float(F[key(c, "bounded", var)][t, d])),
                   "identical": bool(outs[c]["tokens"][t] == F[key(c, "tokens", var)][t])}
    doc["closest_call_T1024"] = cc
    print(json.dumps(doc, indent=1))


if __name__ == "__main__":
    main()
