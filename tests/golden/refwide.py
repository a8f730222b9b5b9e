"""Access to `forward_ref_wide.npz` (the reference's float64 forward on the benchmarked configs,
made by `make_forward_wide.py`) and the exact-match / rounding-margin report (BASELINE.md §4,
SURVEY §8d "Exact-match report"). Pure NumPy: used by tests/, bench.py and tools/, never by the
product path.

Margin of a token = min over latent dims d of |b_d − (⌊b_d⌋ + ½)|, the distance of the
reference's bounded latent to the nearest round-half-even boundary: a token can only flip if
some implementation's deviation from the float64 latent exceeds it.
"""
import os
from collections import OrderedDict

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
PATH = os.path.join(HERE, "forward_ref_wide.npz")
# the headline workload's exact-match sample (every 8th bench protein, make_forward_bench.py)
BENCH_PATH = os.path.join(HERE, "forward_ref_bench.npz")
# log10 bins of the margin histogram: [0, 1e-7), [1e-7, 1e-6), ..., [1e-1, 0.5]
EDGES = [0.0, 1e-7, 1e-6, 1e-5, 1e-4, 1e-3, 1e-2, 1e-1, 0.5000001]


def load():
    return np.load(PATH)


def load_bench():
    return np.load(BENCH_PATH)


def cases(F, prefix=""):
    return sorted({k.split("/")[0] for k in F.files if k.startswith(prefix)})


def groups(F, prefix=""):
    """(codebook, df) -> [case names] (the ones that can share one ragged batch)."""
    out = OrderedDict()
    for c in cases(F, prefix):
        _, _, cb, df, _, _ = (int(v) for v in F[c + "/meta"])
        out.setdefault((cb, df), []).append(c)
    return out


def dim_margins(b_ref: np.ndarray) -> np.ndarray:
    return np.abs(b_ref - (np.floor(b_ref) + 0.5))


def histogram(m: np.ndarray):
    h, _ = np.histogram(np.asarray(m, np.float64), bins=EDGES)
    return {f"[{lo:.0e},{hi:.0e})": int(c) for lo, hi, c in zip(EDGES[:-1], EDGES[1:], h)}


def report(b_ref, tok_ref, b_ours, tok_ours):
    """Exact-match rate and margin statistics of one implementation vs the reference fixture.

    `explained` = every mismatching token has a dim whose margin is below our deviation there
    (the flip is float rounding noise, not a wrong computation)."""
    b_ref = np.asarray(b_ref, np.float64)
    b_ours = np.asarray(b_ours, np.float64)
    tok_ref = np.asarray(tok_ref)
    tok_ours = np.asarray(tok_ours)
    m = dim_margins(b_ref)
    dev = np.abs(b_ours - b_ref)
    tm = m.min(-1)
    bad = np.nonzero(tok_ref != tok_ours)[0]
    explained = bool(np.all([(dev[i] > m[i]).any() for i in bad])) if len(bad) else True
    return {
        "tokens": int(len(tok_ref)), "identical": int(len(tok_ref) - len(bad)),
        "rate": float(1.0 - len(bad) / max(1, len(tok_ref))),
        "min_margin": float(tm.min()) if len(tm) else None,
        "max_deviation": float(dev.max()) if dev.size else None,
        "max_deviation_over_margin": float((dev / np.maximum(m, 1e-300)).max()) if dev.size else None,
        "margin_histogram_all": histogram(tm),
        "margin_histogram_mismatches": histogram(tm[bad]),
        "mismatch_margins": [float(tm[i]) for i in bad[:32]],
        "mismatches_explained_by_rounding": explained,
    }


def merge(reports):
    """Combine per-case reports into one."""
    out = {"tokens": sum(r["tokens"] for r in reports), "identical": sum(r["identical"] for r in reports)}
    out["rate"] = out["identical"] / max(1, out["tokens"])
    out["min_margin"] = min(r["min_margin"] for r in reports)
    out["max_deviation"] = max(r["max_deviation"] for r in reports)
    out["max_deviation_over_margin"] = max(r["max_deviation_over_margin"] for r in reports)
    for k in ("margin_histogram_all", "margin_histogram_mismatches"):
        out[k] = {b: sum(r[k][b] for r in reports) for b in reports[0][k]}
    out["mismatch_margins"] = sum((r["mismatch_margins"] for r in reports), [])[:32]
    out["mismatches_explained_by_rounding"] = all(r["mismatches_explained_by_rounding"] for r in reports)
    return out


def device_outputs(F, make_tokenizer, prefix=""):
    """Run every fixture case through libpst, one ragged batch per (codebook, df):
    `make_tokenizer(cb, df, D, seed)` -> a `pst_amd._native.Tokenizer`. Returns
    {case: (tokens, bounded, pre_proj)} taken from the C ABI's token and aux outputs."""
    out = {}
    for (cb, df), names in groups(F, prefix).items():
        metas = [tuple(int(v) for v in F[c + "/meta"]) for c in names]
        D, seed = metas[0][4], metas[0][5]
        tk = make_tokenizer(cb, df, D, seed)
        pos = np.concatenate([F[c + "/in_positions"] for c in names]).astype(np.float64)
        flags = np.concatenate([F[c + "/in_flags"] for c in names])
        off = np.zeros(len(names) + 1, np.int64)
        off[1:] = np.cumsum([F[c + "/in_positions"].shape[0] for c in names])
        tok, nt, nn = tk.tokenize_packed(pos, flags, off)
        aux = tk.aux(int(off[-1]))
        for i, c in enumerate(names):
            n, T = metas[i][0], metas[i][1]
            if int(nn[i]) != n or int(nt[i]) != T:
                raise AssertionError(f"{c}: n_nodes/n_tokens {nn[i]}/{nt[i]} vs reference {n}/{T}")
            a = int(off[i])
            out[c] = (tok[a:a + T].copy(), aux["bounded"][a:a + T].copy(), aux["pre_proj"][a:a + T].copy())
    return out
