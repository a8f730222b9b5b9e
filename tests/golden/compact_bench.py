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
the latents of the close tokens carry every deviation check the tests make.

    python tests/golden/compact_bench.py RAW.npz [RAW.npz ...]   # -> forward_ref_bench.npz
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import refwide  # noqa: E402

WORKLOADS = {"bench256": (256, 1000, 4096, 1), "bench512": (512, 1000, 64000, 4)}


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
    return {f"{name}/proteins": np.array(prots, np.int64), f"{name}/tok_off": np.array(off, np.int64),
            f"{name}/tokens": np.concatenate(toks), f"{name}/margin": np.concatenate(margins),
            f"{name}/close": np.array(close, np.int64),
            f"{name}/close_bounded": np.array(cb_rows, np.float64).reshape(-1, D),
            f"{name}/n_nodes": np.array(nn, np.int64), f"{name}/input_sha256": np.array(sha),
            f"{name}/meta": np.array([n_res, seed0, cb, df, D, pseed], np.int64)}


def main():
    raw = {}
    for path in sys.argv[1:]:
        with np.load(path) as F:
            for k in F.files:
                raw.setdefault(k, F[k])
    out = {}
    for name in WORKLOADS:
        if any(k.startswith(name + "_p") for k in raw):
            out.update(compact(raw, name))
            print(name, len(out[f"{name}/proteins"]), "proteins,", len(out[f"{name}/tokens"]), "tokens,",
                  len(out[f"{name}/close"]), "close")
    np.savez_compressed(refwide.BENCH_PATH, **out)
    print("wrote", refwide.BENCH_PATH, os.path.getsize(refwide.BENCH_PATH), "bytes")


if __name__ == "__main__":
    main()
