"""Reference-forward fixture for the downsampling configs on real structures (build container only).

The reference CLI takes `--model_downsampling {1,2,4}` x `--codebook_size {4096,64000}`
(scripts/tokenize_pdb.py:81-113) and weights ship for every pair
(config/structure_tokenizer/model/gnn/ablation_{4k,64k}_df_{1,2,4}.yaml). df 1 on CASP14 is pinned
in `forward_ref_wide.npz` (configs 2 and 4); this script runs the REFERENCE's own
`Vq3D.encode_and_quantize` (model.py:453-479) under the import shim on all 31 CASP14 structures at
(4096, df 2), (4096, df 4), (64000, df 2) and (64000, df 4) — 124 cases — in the `_pe32` rendering
of `make_forward_wide.py` (float64 with the sinusoidal PE argument rounded to float32 as JAX forms
it, the reference's own PE values), random weights `params.random_params(D, 1234)`.

df > 1 exercises the reference's local-window cross-attention downsampler and its pooling
(model.py:264-318, modules.py:427-534), which the headline (df 1) does not.

Per case `casp_{name}_k{cb}_df{df}`: `tokens`, `bounded` (float64 FSQ-bounded latents), `margin`
(per-token rounding margin) and `meta` = [n, T, codebook, df, D, seed]. Inputs are not stored
again: they are `casp14_atom37.npz`'s rows of that structure (the reference's casp14_pdbs parsed).

    python tests/golden/make_forward_casp_df.py [--jobs 2] [--only casp_T1024]
"""
import argparse
import os
import sys
import time
from multiprocessing import get_context

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "forward_ref_casp_df.npz")
CONFIGS = [(4096, 2), (4096, 4), (64000, 2), (64000, 4)]


def case_list():
    C = np.load(os.path.join(HERE, "casp14_atom37.npz"))
    return [(f"casp_{nm}_k{cb}_df{df}", ("casp", str(nm)), cb, df)
            for cb, df in CONFIGS for nm in C["names"]]


def run_one(case):
    sys.path.insert(0, HERE)
    import make_forward_wide as M
    t0 = time.time()
    name, out = M.run_case(case, pe32=True)
    _, _, cb, df = case
    T = len(out["tokens_pe32"])
    keep = {
        "tokens": out["tokens_pe32"],
        "bounded": out["bounded_pe32"],
        "margin": out["margin_pe32"],
        "meta": np.array([out["n_nodes"], T, cb, df, out["bounded_pe32"].shape[1], M.PARAM_SEED], np.int64),
    }
    return name, keep, time.time() - t0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--jobs", type=int, default=2)
    ap.add_argument("--only", default="")
    args = ap.parse_args()
    sys.path.insert(0, HERE)
    import _refenv
    if not _refenv.available():
        sys.exit("reference not available")
    sys.path.insert(0, _refenv.PKG)
    old = dict(np.load(OUT)) if os.path.exists(OUT) else {}
    todo = [c for c in case_list() if c[0].startswith(args.only) and f"{c[0]}/tokens" not in old]
    # largest first so the pool's tail is short
    C = np.load(os.path.join(HERE, "casp14_atom37.npz"))
    size = {str(n): int(C["offsets"][i + 1] - C["offsets"][i]) for i, n in enumerate(C["names"])}
    todo.sort(key=lambda c: -size[c[1][1]])
    print(f"{len(todo)} cases to run", flush=True)
    done = 0
    with get_context("spawn").Pool(args.jobs) as pool:
        for name, res, dt in pool.imap_unordered(run_one, todo):
            for k, v in res.items():
                old[f"{name}/{k}"] = v
            done += 1
            print(f"{name}: n={res['meta'][0]} T={res['meta'][1]} min margin={res['margin'].min():.3e} "
                  f"({dt:.0f} s) [{done}/{len(todo)}]", flush=True)
            if done % 8 == 0:  # checkpoint: a killed run resumes where it stopped
                np.savez_compressed(OUT, **old)
    np.savez_compressed(OUT, **old)
    print("wrote", OUT)


if __name__ == "__main__":
    main()
