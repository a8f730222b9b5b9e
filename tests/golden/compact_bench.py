"""Compact form of the headline workload's reference fixture (build container only).

`make_forward_bench.py` writes, per protein p, the reference's token ids, its FSQ-bounded latents
(float64) and per-token margins (`bench{n_res}_p{p}/…`, every token's latent kept: ~12 KB per
256-residue protein). With every protein of the 1 024-protein workload that would be ~16 MB, so
this script packs the raw per-protein results into one record per workload:

    {name}/proteins       int64  [P]     protein ids (synthetic_protein(n_res, seed0 + p))
    {name}/tok_off        int64  [P+1]   token offsets into the concatenated arrays
    {name}/tokens         uint16 [T]     the reference's token ids
    {name}/margin         float32[T]     per token: min over dims |b_d - (floor(b_d) + 1/2)|
    {name}/close          int64  [C]     flat indices of the tokens with margin < refwide.CLOSE
    {name}/close_bounded  float64[C, D]  the reference's bounded latents of those tokens
    {name}/n_nodes        int64  [P]
    {name}/input_sha256   str    [P]     SHA-256 of the float32 inputs the reference ran on
    {name}/meta           int64  [6]     n_res, seed0, codebook, df, D, param seed

Only a token with margin below an implementation's deviation (~1e-5 at most here) can flip, so
the latents of the close tokens carry the flip checks. To bound the latent drift of the tokens that
cannot flip too, every protein of a fixed subset keeps ALL its bounded latents (round 6):

    {name}/full_proteins  int64  [F]     proteins p with p % FULL_EVERY == FULL_PHASE[name]
    {name}/full_tok_off   int64  [F+1]   token offsets into full_bounded
    {name}/full_bounded   float32[Tf, D] the reference's bounded latents of every token of those proteins

Raw inputs are merged into the committed fixture: proteins already there keep their record (their
token ids must agree with a raw re-run), new ones are added in protein order, and a raw re-run of a
subset protein adds its full latents.

    python tests/golden/compact_bench.py RAW.npz [RAW.npz ...]   # -> forward_ref_bench.npz
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import refwide  # noqa: E402

WORKLOADS = {"bench256": (256, 1000, 4096, 1), "bench512": (512, 1000, 64000, 4)}
# the subset whose every latent is kept: 32 proteins of each workload (bench512's every-16th sample,
# made before round 6, kept only the close latents, hence its phase 8)
FULL_EVERY = {"bench256": 32, "bench512": 16}
FULL_PHASE = {"bench256": 0, "bench512": 8}


def compact(raw, name):
    n_res, seed0, cb, df = WORKLOADS[name]
    prots = sorted({int(k.split("/")[0].split("_p")[1]) for k in raw if k.startswith(name + "_p")})
    toks, margins, close, cb_rows, nn, sha, off = [], [], [], [], [], [], [0]
    D = None
    for p in prots:
        c = f"{name}_p{p}"
        meta = raw[c + "/meta"]
        n, T, mcb, mdf, mD, pseed = (int(v) for v in meta)
        assert (mcb, mdf) == (cb, df), c
        assert tuple(int(v) for v in raw[c + "/synthetic_args"]) == (n_res, seed0 + p), c
        D = mD if D is None else D
        b = np.asarray(raw[c + "/bounded_pe32"], np.float64)
        t = np.asarray(raw[c + "/tokens_pe32"])
        m = refwide.dim_margins(b).min(-1)
        assert np.array_equal(m, raw[c + "/margin_pe32"]), c
        assert t.max() < 65536
        m32 = m.astype(np.float32)
        for j in np.nonzero(m32 < refwide.CLOSE)[0]:
            close.append(off[-1] + int(j))
            cb_rows.append(b[j])
        toks.append(t.astype(np.uint16))
        margins.append(m32)
        nn.append(n)
        sha.append(str(raw[c + "/input_sha256"]))
        off.append(off[-1] + T)
    full = [p for p in prots if p % FULL_EVERY[name] == FULL_PHASE[name]]
    fb = [np.asarray(raw[f"{name}_p{p}/bounded_pe32"], np.float32) for p in full]
    foff = np.concatenate([[0], np.cumsum([len(b) for b in fb])]).astype(np.int64)
    return {f"{name}/proteins": np.array(prots, np.int64), f"{name}/tok_off": np.array(off, np.int64),
            f"{name}/full_proteins": np.array(full, np.int64), f"{name}/full_tok_off": foff,
            f"{name}/full_bounded": (np.concatenate(fb) if fb else np.zeros((0, D), np.float32)).reshape(-1, D),
            f"{name}/tokens": np.concatenate(toks), f"{name}/margin": np.concatenate(margins),
            f"{name}/close": np.array(close, np.int64),
            f"{name}/close_bounded": np.array(cb_rows, np.float64).reshape(-1, D),
            f"{name}/n_nodes": np.array(nn, np.int64), f"{name}/input_sha256": np.array(sha),
            f"{name}/meta": np.array([n_res, seed0, cb, df, D, pseed], np.int64)}


def merge(old, new, name):
    """Union of two compact records of one workload (`old` = the committed fixture's keys)."""
    g = lambda R, k: R[f"{name}/{k}"]
    rec = {}  # protein -> (tokens, margin, n_nodes, sha, close_rel, close_bounded, full_bounded or None)
    for R in (old, new):
        if f"{name}/proteins" not in R:
            continue
        prots, off = g(R, "proteins"), g(R, "tok_off")
        close, cbnd = g(R, "close"), g(R, "close_bounded")
        fp = list(g(R, "full_proteins")) if f"{name}/full_proteins" in R else []
        for i, p in enumerate(prots):
            a, b = int(off[i]), int(off[i + 1])
            sel = (close >= a) & (close < b)
            fb = None
            if int(p) in fp:
                j = fp.index(int(p))
                fo = g(R, "full_tok_off")
                fb = g(R, "full_bounded")[int(fo[j]):int(fo[j + 1])]
            item = (g(R, "tokens")[a:b], g(R, "margin")[a:b], int(g(R, "n_nodes")[i]), str(g(R, "input_sha256")[i]),
                    close[sel] - a, cbnd[sel], fb)
            if int(p) in rec:
                prev = rec[int(p)]
                assert np.array_equal(prev[0], item[0]) and prev[3] == item[3], f"{name} p{p}: re-run disagrees"
                item = prev[:6] + (prev[6] if prev[6] is not None else item[6],)
            rec[int(p)] = item
    prots = sorted(rec)
    D = int(g(new if f"{name}/meta" in new else old, "meta")[4])
    off, close, cb_rows, full, fb, foff = [0], [], [], [], [], [0]
    for p in prots:
        t, m, n, sha, cl, cbd, fbd = rec[p]
        close.extend((cl + off[-1]).tolist())
        cb_rows.append(cbd.reshape(-1, D))
        off.append(off[-1] + len(t))
        if fbd is not None and p % FULL_EVERY[name] == FULL_PHASE[name]:
            full.append(p)
            fb.append(np.asarray(fbd, np.float32))
            foff.append(foff[-1] + len(fbd))
    return {f"{name}/proteins": np.array(prots, np.int64), f"{name}/tok_off": np.array(off, np.int64),
            f"{name}/tokens": np.concatenate([rec[p][0] for p in prots]),
            f"{name}/margin": np.concatenate([rec[p][1] for p in prots]),
            f"{name}/close": np.array(close, np.int64),
            f"{name}/close_bounded": np.concatenate(cb_rows).reshape(-1, D),
            f"{name}/full_proteins": np.array(full, np.int64), f"{name}/full_tok_off": np.array(foff, np.int64),
            f"{name}/full_bounded": (np.concatenate(fb) if fb else np.zeros((0, D), np.float32)).reshape(-1, D),
            f"{name}/n_nodes": np.array([rec[p][2] for p in prots], np.int64),
            f"{name}/input_sha256": np.array([rec[p][3] for p in prots]),
            f"{name}/meta": g(new if f"{name}/meta" in new else old, "meta")}


def main():
    raw = {}
    for path in sys.argv[1:]:
        with np.load(path) as F:
            for k in F.files:
                raw.setdefault(k, F[k])
    old = dict(np.load(refwide.BENCH_PATH)) if os.path.exists(refwide.BENCH_PATH) else {}
    out = {k: v for k, v in old.items()}
    for name in WORKLOADS:
        if any(k.startswith(name + "_p") for k in raw):
            out.update(merge(old, compact(raw, name), name))
            print(name, len(out[f"{name}/proteins"]), "proteins,", len(out[f"{name}/tokens"]), "tokens,",
                  len(out[f"{name}/close"]), "close")
    np.savez_compressed(refwide.BENCH_PATH, **out)
    print("wrote", refwide.BENCH_PATH, os.path.getsize(refwide.BENCH_PATH), "bytes")


if __name__ == "__main__":
    main()
