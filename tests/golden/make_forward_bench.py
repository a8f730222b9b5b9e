"""Reference-forward fixture for the HEADLINE workload (build container only).

This script runs the REFERENCE's own `Vq3D.encode_and_quantize` (model.py:453-479) under the
import shim on proteins of bench.py's workload — the `_pe32` rendering of `make_forward_wide.py`
(float64 with the sinusoidal PE argument rounded to float32 exactly as JAX forms it with x64 off,
i.e. the reference's own PE values) — at codebook 4096, df 1, random weights
`params.random_params(6, 1234)` (the bench's). Round 4 ran every 4th protein of
`synthetic_batch(1024, 256, seed=1000)` (`--stride 4`, 256 proteins); round 5 ran the other 768
(`--stride 1`, ~80 s per protein on one core, ~2.8 h on 6 workers), so every protein of the
headline workload is pinned.

`--config 5` does the same for SURVEY config 5's workload (`bench.py --codebook 64000 --df 4
--residues 512 --proteins 512`: synthetic_batch(512, 512, seed=1000)), every 16th protein (32
proteins, 4 096 tokens), case names `bench512_p{p}`.

Raw output per protein `bench{n_res}_p{p}` (into `--out`, a scratch file outside the fixture):
the reference's token ids, its FSQ-bounded latents (float64), the per-token rounding margin,
`meta` = [n, T, codebook, df, D, seed], the SHA-256 of the float32 inputs and the generator
arguments. `compact_bench.py RAW…` packs them into the committed `forward_ref_bench.npz` (tokens,
margins, and the latents of the tokens within refwide.CLOSE of a boundary). Proteins already in
the committed fixture are skipped. The inputs themselves are not stored: they are regenerated
from `pst_amd.synthetic.synthetic_protein(n_res, 1000 + p)` and must hash to the stored SHA
(`tests/test_fixture_recipes.py`).

Round 6: `--config 5 --stride 1` ran the other 480 proteins of config 5 (all 512 pinned), and
`--full-subset` re-runs the proteins whose every latent the compact fixture keeps
(compact_bench.FULL_EVERY / FULL_PHASE: p % 32 == 0 of the headline workload) so the drift of
tokens that cannot flip is bounded too.

    python tests/golden/make_forward_bench.py --out RAW.npz [--jobs 6] [--stride 1] [--config 3|5] [--full-subset]
    python tests/golden/compact_bench.py RAW.npz [RAW2.npz …]
"""
import argparse
import os
import sys
import time
from multiprocessing import get_context

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "forward_ref_bench.npz")
# SURVEY config -> (proteins, residues, seed of protein 0, codebook, df, default stride)
CONFIGS = {3: (1024, 256, 1000, 4096, 1, 4), 5: (512, 512, 1000, 64000, 4, 16)}
N_PROT, N_RES, SEED0, CODEBOOK, DF, _ = CONFIGS[3]


def set_config(cfg):
    global N_PROT, N_RES, SEED0, CODEBOOK, DF
    N_PROT, N_RES, SEED0, CODEBOOK, DF, _ = CONFIGS[cfg]


def proteins(stride=4):
    return list(range(0, N_PROT, stride))


def case_name(p):
    return f"bench{N_RES}_p{p}"


def run_one(job):
    cfg, p = job
    set_config(cfg)
    sys.path.insert(0, HERE)
    import make_forward_wide as M
    t0 = time.time()
    name, out = M.run_case((case_name(p), ("syn", N_RES, SEED0 + p), CODEBOOK, DF), pe32=True)
    pos, fl, sha = M.load_inputs(("syn", N_RES, SEED0 + p))
    T = len(out["tokens_pe32"])
    keep = {
        "tokens_pe32": out["tokens_pe32"],
        "bounded_pe32": out["bounded_pe32"],
        "margin_pe32": out["margin_pe32"],
        "meta": np.array([out["n_nodes"], T, CODEBOOK, DF, out["bounded_pe32"].shape[1], M.PARAM_SEED], np.int64),
        "input_sha256": np.array(sha),
        "synthetic_args": np.array([N_RES, SEED0 + p], np.int64),
    }
    return p, keep, time.time() - t0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--jobs", type=int, default=7)
    ap.add_argument("--stride", type=int, default=None)
    ap.add_argument("--config", type=int, default=3, choices=sorted(CONFIGS))
    ap.add_argument("--full-subset", action="store_true",
                    help="run only the proteins whose every latent compact_bench.py keeps, even if pinned already")
    ap.add_argument("--from-protein", type=int, default=0,
                    help="only proteins >= this (a second generator process working on the top of the range)")
    ap.add_argument("--out", required=True, help="raw per-protein output (merged into the fixture by compact_bench.py)")
    args = ap.parse_args()
    set_config(args.config)
    stride = args.stride or CONFIGS[args.config][5]
    sys.path.insert(0, HERE)
    import _refenv
    if not _refenv.available():
        sys.exit("reference not available")
    sys.path.insert(0, _refenv.PKG)
    old = dict(np.load(args.out)) if os.path.exists(args.out) else {}
    import refwide
    name = case_name(0).split("_p")[0]
    have = set()
    if os.path.exists(OUT) and f"{name}/proteins" in np.load(OUT).files:
        have = {int(p) for p in refwide.load_bench_sample(name).proteins}
    if args.full_subset:
        import compact_bench as CB
        wl = case_name(0).split("_p")[0]
        todo = [p for p in range(N_PROT) if p % CB.FULL_EVERY[wl] == CB.FULL_PHASE[wl]
                and f"{case_name(p)}/tokens_pe32" not in old]
    else:
        todo = [p for p in proteins(stride) if f"{case_name(p)}/tokens_pe32" not in old and p not in have
                and p >= args.from_protein]
    print(f"{len(todo)} proteins to run", flush=True)
    done = 0
    with get_context("spawn").Pool(args.jobs) as pool:
        for p, res, dt in pool.imap_unordered(run_one, [(args.config, p) for p in todo]):
            for k, v in res.items():
                old[f"{case_name(p)}/{k}"] = v
            done += 1
            print(f"p{p}: T={res['meta'][1]} min margin={res['margin_pe32'].min():.3e} ({dt:.0f} s) "
                  f"[{done}/{len(todo)}]", flush=True)
            if done % 16 == 0:  # checkpoint: a killed run resumes where it stopped
                np.savez_compressed(args.out, **old)
    np.savez_compressed(args.out, **old)
    print("wrote", args.out)


if __name__ == "__main__":
    main()
