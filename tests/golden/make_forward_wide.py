"""Reference-forward fixtures at the benchmarked sizes and configs (build container only).

Runs the REFERENCE's own `Vq3D.encode_and_quantize` (model.py:453-479) under the import shim in
float64 — the same recipe as `make_golden.py forward` — on:

* all 31 CASP14 proteins at codebook 4096 / df 1 (BASELINE config 2) and 64 000 / df 1 (config 4);
* the first 8 proteins of the bench workload, `synthetic_batch(1024, 256, seed=1000)` (config 3);
* the first 2 proteins of `synthetic_batch(·, 512, seed=1000)` at 64 000 / df 4 (config 5);
* `syn56_missing9`: 56 residues, 9 without backbone → 47 kept, the reference's short-protein
  branch (preprocessing.py:229-260), at df 1 and df 2.

Three renderings of the same forward: float64 throughout (the fixture's `tokens`, `bounded`,
`z`, `pre_proj`); `_pe32`, float64 with the PE argument rounded to float32 as JAX forms it with
x64 off (`jax_f32_pe_argument`, the reference's own PE values); `_f32`, the shim in float32 mode
(float32 weights and edge features) with the PE in JAX's float32 dtypes (`jax_f32_pe_values`).
The `_f32` rendering is mixed precision, not XLA's float32: NumPy promotes integer-array × float
products (the FSQ levels, masks built with default-dtype ones) to float64 where JAX x64-off keeps
float32, and NumPy's tanh / reductions are not XLA's. `dtypes_f32` records the output dtypes.

Inputs are never regenerated silently: CASP14 inputs come from `casp14_atom37.npz`, the short
case from `graph_golden.npz`, and synthetic inputs are regenerated and checked against the
SHA-256 stored in the fixture (`tests/test_fixture_recipes.py` repeats that check on CPU), so the
recipe and the data cannot drift apart. Weights: `params.random_params(D, 1234)` (no checkpoint is
available offline), the seed `bench.py` uses.

Per case the fixture keeps the inputs, `meta` = [n, T, codebook, df, D, seed], the reference's
token ids, its FSQ-bounded latents `bounded` (float64) and the per-token rounding margin
`margin` = min_d |b_d − (⌊b_d⌋ + ½)| (distance to the nearest round-half-even boundary), and
— for the codebook-4096 cases — `continuous_embedding_pre_proj` rounded to float32.

    python tests/golden/make_forward_wide.py [--jobs 8] [--only PREFIX]        # float64 (the fixture)
    python tests/golden/make_forward_wide.py --pe32                             # + JAX-f32 PE argument
    python tests/golden/make_forward_wide.py --f32                              # + the all-float32 rendering
"""
import argparse
import hashlib
import os
import sys
from multiprocessing import get_context

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "forward_ref_wide.npz")
K_NEIGHBOR, PAD, PARAM_SEED = 50, 512, 1234


def input_sha(pos32: np.ndarray, flags: np.ndarray) -> str:
    h = hashlib.sha256()
    h.update(np.ascontiguousarray(pos32, dtype=np.float32).tobytes())
    h.update(np.ascontiguousarray(flags, dtype=np.uint8).tobytes())
    return h.hexdigest()


def case_list():
    """(name, source, codebook, df). source: ('casp', name) | ('syn', n_res, seed) | ('graph', key)."""
    C = np.load(os.path.join(HERE, "casp14_atom37.npz"))
    cases = []
    for nm in C["names"]:
        nm = str(nm)
        cases.append((f"casp_{nm}_k4096_df1", ("casp", nm), 4096, 1))
        cases.append((f"casp_{nm}_k64000_df1", ("casp", nm), 64000, 1))
    # the first 8 proteins of the bench (its first pipeline chunk) and 4 from the later chunks
    for p in list(range(8)) + [200, 511, 777, 1023]:
        cases.append((f"bench256_p{p}_k4096_df1", ("syn", 256, 1000 + p), 4096, 1))
    for p in range(2):
        cases.append((f"bench512_p{p}_k64000_df4", ("syn", 512, 1000 + p), 64000, 4))
    cases.append(("short_syn56_missing9_k4096_df1", ("graph", "syn56_missing9_df1"), 4096, 1))
    cases.append(("short_syn56_missing9_k4096_df2", ("graph", "syn56_missing9_df1"), 4096, 2))
    return cases


def load_inputs(src):
    """-> (positions f32 [n,37,3], flags u8 [n,37], aatype indices (CASP14) | sha (synthetic) | None)."""
    if src[0] == "casp":
        C = np.load(os.path.join(HERE, "casp14_atom37.npz"))
        i = [str(x) for x in C["names"]].index(src[1])
        a, b = int(C["offsets"][i]), int(C["offsets"][i + 1])
        return C["positions"][a:b], C["flags"][a:b], C["aatype"][a:b]
    if src[0] == "graph":
        G = np.load(os.path.join(HERE, "graph_golden.npz"))
        return G[src[1] + "/in_positions"], G[src[1] + "/in_flags"], None
    from pst_amd import synthetic
    s = synthetic.synthetic_protein(src[1], src[2])
    pos = s.atom37_positions.astype(np.float32)
    fl = s.atom_flags()
    return pos, fl, input_sha(pos, fl)


def margins(b: np.ndarray) -> np.ndarray:
    """Per token, min over latent dims of the distance to the nearest rounding boundary m + ½."""
    return np.abs(b - (np.floor(b) + 0.5)).min(axis=-1)


def jax_f32_pe_argument(pel):
    """Make the float64 shim evaluate the sinusoidal PE argument (positional_encoding_layer.py:
    62-66) with the dtypes JAX gives it when x64 is off: x (int32) · π and n^(2(k−1)/d) are float32
    (weak-typed Python scalars), so the argument is rounded to float32 exactly as the reference
    computes it on any JAX backend; cos/sin stay float64. Everything else stays float64."""
    import math

    def pe(self, x, n, d, k):
        x = np.asarray(x)
        k = np.asarray(k)
        kf = k.astype(np.float64)
        odd = np.mod(k, 2).astype(np.float64)
        num = np.where(np.mod(k, 2) == 1, 2 * (k - 1), 2 * k).astype(np.float32)
        e = num / np.float32(d)
        pw = np.power(np.float64(n), e.astype(np.float64)).astype(np.float32)  # correctly rounded f32 pow
        arg = (x.astype(np.float32) * np.float32(math.pi)) / pw
        arg = arg.astype(np.float64)
        del kf
        return odd * np.cos(arg) - (odd - 1) * np.sin(arg)

    pel.PositionalEncodingLayer.sinusoidal_positional_encoding = pe


def jax_f32_pe_values(pel):
    """For the float32 rendering (--f32): the sinusoidal PE exactly as `jax_f32_pe_argument` forms
    its argument, with cos / sin evaluated in float32 (correctly rounded) and a float32 result —
    JAX's dtypes with x64 off. (The shim's plain float32 mode would evaluate `x * math.pi` on
    NumPy integer arrays in float64.)"""
    import math

    def pe(self, x, n, d, k):
        x = np.asarray(x)
        k = np.asarray(k)
        odd = np.mod(k, 2).astype(np.float32)
        num = np.where(np.mod(k, 2) == 1, 2 * (k - 1), 2 * k).astype(np.float32)
        e = num / np.float32(d)
        pw = np.power(np.float64(n), e.astype(np.float64)).astype(np.float32)
        arg = (x.astype(np.float32) * np.float32(math.pi)) / pw
        cs = np.cos(arg.astype(np.float64)).astype(np.float32)
        sn = np.sin(arg.astype(np.float64)).astype(np.float32)
        return odd * cs - (odd - np.float32(1)) * sn

    pel.PositionalEncodingLayer.sinusoidal_positional_encoding = pe


def run_case(case, f64=True, pe32=False):
    os.environ["OMP_NUM_THREADS"] = "1"
    os.environ["OPENBLAS_NUM_THREADS"] = "1"
    sys.path.insert(0, HERE)
    import _refenv
    pss = _refenv.activate(f64=f64)
    if pe32:
        from structure_tokenizer.model import positional_encoding_layer
        jax_f32_pe_argument(positional_encoding_layer)
    if not f64:
        from structure_tokenizer.model import positional_encoding_layer
        jax_f32_pe_values(positional_encoding_layer)
    import jax
    import haiku as hk
    from structure_tokenizer.data import preprocessing as ref_pp
    from structure_tokenizer.model.model import Vq3D
    from pst_amd import params as P
    from pst_amd.config import LEVELS, load_config, overrides_for
    from pst_amd.sample import sample_from_arrays

    name, src, cb, df = case
    pos32, flags, extra = load_inputs(src)
    sha = extra if src[0] == "syn" else None
    s = sample_from_arrays(pos32.astype(np.float64), flags, extra if src[0] == "casp" else None)
    cfg = load_config("vq3d_inference", overrides=overrides_for(cb, df),
                      config_path=os.path.join(_refenv.REF, "config", "structure_tokenizer"))
    g = ref_pp.preprocess_sample(sample=_refenv.to_ref_sample(pss, s), num_neighbor=K_NEIGHBOR,
                                 downsampling_ratio=df, residue_loc_is_alphac=True,
                                 padding_num_residue=PAD, crop_index=PAD, noise_level=0.0).graph
    gb = jax.tree_util.tree_map(lambda x: np.asarray(x)[None], g)
    ft = np.float64 if f64 else np.float32
    gb.edge_features = gb.edge_features.astype(np.float32).astype(ft)  # JAX x64-off H2D
    D = len(LEVELS[cb])
    params = {m: {k: v.astype(ft) for k, v in d.items()}
              for m, d in P.random_params(D, PARAM_SEED).items()}

    def fn(graph):
        return Vq3D(config=cfg.model, global_config=cfg.data).encode_and_quantize(
            graph, is_training=False, safe_key=None)

    res = hk.transform(fn).apply(params, None, gb)
    n = int(g.n_node[0])
    T = n // df
    b = np.asarray(res["continuous_embedding"][0, :T], dtype=np.float64)
    # the FSQ input z = down_proj(pre_proj) (model.py:417-419), evaluated from the run's own
    # pre-projection embedding with the same weights (Linear: x @ w + b)
    pre = np.asarray(res["continuous_embedding_pre_proj"][0, :T], dtype=ft)
    dp = params["vq3_d/down_proj"]
    z = (pre @ dp["w"].astype(ft) + dp["b"].astype(ft)).astype(np.float64)
    if not f64:  # the reference forward with float32 weights, inputs and PE (see the module docstring)
        out = {"tokens_f32": np.asarray(res["tokens"][0, :T]).astype(np.uint32), "bounded_f32": b,
               "margin_f32": margins(b), "z_f32": z,
               "dtypes_f32": np.array([str(np.asarray(res["continuous_embedding_pre_proj"]).dtype),
                                       str(np.asarray(res["continuous_embedding"]).dtype)])}
        if cb == 4096:
            out["pre_proj_f32"] = np.asarray(res["continuous_embedding_pre_proj"][0, :T], dtype=np.float32)
        return name, out
    if pe32:
        out = {"tokens_pe32": np.asarray(res["tokens"][0, :T]).astype(np.uint32), "bounded_pe32": b,
               "margin_pe32": margins(b), "z_pe32": z, "n_nodes": n}
        if cb == 4096:
            out["pre_proj_pe32"] = np.asarray(res["continuous_embedding_pre_proj"][0, :T], dtype=np.float32)
        return name, out
    out = {
        "in_positions": pos32, "in_flags": flags,
        "meta": np.array([n, T, cb, df, D, PARAM_SEED], np.int64),
        "tokens": np.asarray(res["tokens"][0, :T]).astype(np.uint32),
        "bounded": b, "margin": margins(b), "z": z,
    }
    if sha is not None:
        out["input_sha256"] = np.array(sha)
        out["synthetic_args"] = np.array([src[1], src[2]], np.int64)
    if cb == 4096:
        out["pre_proj"] = np.asarray(res["continuous_embedding_pre_proj"][0, :T], dtype=np.float32)
    return name, out


def run_case_pe32(case):
    return run_case(case, pe32=True)


def run_case_f32(case):
    return run_case(case, f64=False)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--jobs", type=int, default=8)
    ap.add_argument("--only", default="")
    ap.add_argument("--pe32", action="store_true",
                    help="add the variant whose PE argument is float32 as under JAX (tokens_pe32, "
                         "bounded_pe32, margin_pe32, pre_proj_pe32); see jax_f32_pe_argument")
    ap.add_argument("--f32", action="store_true",
                    help="add the rendering with the whole reference forward in float32 (tokens_f32, "
                         "bounded_f32, margin_f32, z_f32, pre_proj_f32)")
    args = ap.parse_args()
    sys.path.insert(0, HERE)
    import _refenv
    if not _refenv.available():
        sys.exit("reference not available")
    sys.path.insert(0, _refenv.PKG)
    cases = [c for c in case_list() if c[0].startswith(args.only)]
    old = dict(np.load(OUT)) if os.path.exists(OUT) else {}
    # drift guard: a stored synthetic input must equal what the generator makes today
    for name, src, _, _ in cases:
        key = f"{name}/input_sha256"
        if src[0] == "syn" and key in old:
            _, _, sha = load_inputs(src)
            if str(old[key]) != sha:
                sys.exit(f"{name}: synthetic generator no longer reproduces the stored inputs")
    with get_context("spawn").Pool(args.jobs) as pool:
        fn = run_case_pe32 if args.pe32 else run_case_f32 if args.f32 else run_case
        for name, res in pool.imap_unordered(fn, cases):
            for k, v in res.items():
                if k != "n_nodes":  # only make_forward_bench.py keeps it (in its meta)
                    old[f"{name}/{k}"] = v
            if args.f32:
                flips = int(np.sum(res["tokens_f32"] != old[f"{name}/tokens"]))
                print(f"{name}: f32 tokens differing from the all-f64 run = {flips}", flush=True)
                continue
            if args.pe32:
                flips = int(np.sum(res["tokens_pe32"] != old[f"{name}/tokens"]))
                print(f"{name}: pe32 tokens differing from the all-f64 run = {flips}", flush=True)
                continue
            m = res["margin"]
            print(f"{name}: n={res['meta'][0]} T={res['meta'][1]} distinct={len(np.unique(res['tokens']))} "
                  f"min margin={m.min():.3e}", flush=True)
    np.savez_compressed(OUT, **old)
    print("wrote", OUT)


if __name__ == "__main__":
    main()
