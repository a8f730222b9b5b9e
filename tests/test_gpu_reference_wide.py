"""GPU token ids vs the REFERENCE's own forward on the benchmarked configs (`forward_ref_wide.npz`:
reference `Vq3D.encode_and_quantize`, model.py:453-479, under the shim in three renderings:
float64, float64 with JAX's float32 PE argument, and float32) — all 31 CASP14 proteins at
codebook 4096 and 64 000 (BASELINE configs 2 and 4), 12 proteins of the bench workload (config 3:
0-7 from its first pipeline chunk, 200, 511, 777, 1023 from the later ones), 2 × 512 residues at
64 000 / df 4 (config 5) and the < 50-residue branch. Through the C ABI (pst_tokenize + pst_aux).

Bar: token ids identical; a mismatch is tolerated only where the reference's latent sits closer
to a rounding boundary than our float32 deviation from it at that dim (then it is rounding noise
of float32 vs float64, `refwide.report`), and none has occurred (14 630 of 14 630 equal on the
oracle against each rendering, which the GPU matches bit for bit).
"""
import numpy as np
import pytest

import refwide
from pst_amd import params as P

pytestmark = pytest.mark.gpu
F = refwide.load()
# vs the JAX-float32-PE rendering (see test_oracle_wide.py), measured on the oracle = GPU bits:
# pre-projection ≤ 3.0e-7, bounded ≤ 1.04e-5; vs the all-float64 rendering ≤ 6.1e-6 / 1.5e-4;
# vs the float32 rendering ≤ 3.2e-7 / 1.03e-5
TOL = {"_pe32": (1e-6, 3e-5), "": (1.5e-5, 4e-4), "_f32": (1e-6, 3e-5)}


def _make(cb, df, D, seed):
    from pst_amd._native import Tokenizer
    return Tokenizer(0, cb, df, P.random_blob(D, seed))


@pytest.fixture(scope="module")
def gpu_out():
    return refwide.device_outputs(F, _make)


@pytest.mark.parametrize("var", ["_pe32", "", "_f32"])
@pytest.mark.parametrize("prefix", ["casp_T", "bench256_", "bench512_", "short_"])
def test_gpu_tokens_equal_reference(gpu_out, prefix, var):
    reps = []
    tol_pre, tol_b = TOL[var]
    for c in refwide.cases(F, prefix):
        tok, b, pp = gpu_out[c]
        assert np.abs(b - F[c + "/bounded" + var]).max() < tol_b, c
        if c + "/pre_proj" + var in F.files:
            assert np.abs(pp - F[c + "/pre_proj" + var]).max() < tol_pre, c
        r = refwide.report(F[c + "/bounded" + var], F[c + "/tokens" + var], b, tok)
        assert r["mismatches_explained_by_rounding"], (c, r)
        reps.append(r)
    r = refwide.merge(reps)
    print(prefix, var, {k: r[k] for k in ("tokens", "identical", "min_margin", "max_deviation",
                                          "max_deviation_over_margin")})
    assert r["identical"] == r["tokens"], r


def test_gpu_config4_casp14_k64000():
    """Config 4 on its own: the 31 CASP14 proteins in ONE batch at codebook 64 000, df 1."""
    out = refwide.device_outputs(F, _make, prefix="casp_")
    names = [c for c in refwide.cases(F, "casp_") if "_k64000_" in c]
    assert len(names) == 31
    for c in names:
        assert np.array_equal(out[c][0], F[c + "/tokens"]), c


def _run_bench_sample(S, cb, df):
    """Every protein of a compact bench sample in ONE ragged batch through the C ABI; the report of
    refwide.BenchSample.compare (tokens vs the reference, our deviation on every close token)."""
    from pst_amd import synthetic
    from pst_amd._native import pack_samples
    prots = [int(p) for p in S.proteins]
    samples = [synthetic.synthetic_protein(S.meta["n_res"], S.meta["seed0"] + p) for p in prots]
    pos, flags, off = pack_samples(samples)
    tk = _make(cb, df, S.meta["D"], S.meta["param_seed"])
    tok, nt, nn = tk.tokenize_packed(pos.astype(np.float32), flags, off)
    b = tk.aux(int(off[-1]))["bounded"]
    tk.close()
    assert np.array_equal(nn, S.n_nodes)
    assert all(int(nt[i]) == S.n_tokens(p) for i, p in enumerate(prots))
    sl = [slice(int(off[i]), int(off[i]) + S.n_tokens(p)) for i, p in enumerate(prots)]
    return S.compare(prots, [tok[x] for x in sl], [b[x] for x in sl])


def test_gpu_tokens_equal_reference_bench_sample():
    """The headline workload pinned to the reference: every protein of bench.py's
    synthetic_batch(1024, 256, seed=1000) (forward_ref_bench.npz 'bench256') in ONE ragged batch
    through the C ABI, against the reference's forward (_pe32 rendering). Every token must be
    identical except the listed boundary cases (refwide.KNOWN_BOUNDARY_CASES: the reference's
    float64 latent closer to a rounding boundary than float32 arithmetic resolves, and our
    deviation beyond that margin); an unlisted flip, or a listed case that no longer flips, fails."""
    S = refwide.load_bench_sample("bench256")
    assert [int(p) for p in S.proteins] == list(range(1024))
    r = _run_bench_sample(S, 4096, 1)
    print({k: r[k] for k in ("tokens", "identical", "min_margin", "close_tokens", "max_deviation_close",
                             "max_deviation_over_margin_close", "mismatches")})
    assert r["tokens"] == 256 * len(S)
    assert not r["unexplained"] and not r["unlisted"] and not r["missing_known"], r
    assert r["max_deviation_close"] < TOL["_pe32"][1]
    # every latent of the full-latent subset (32 proteins), not only the close ones
    assert r["full_latent_proteins"] == 32 and r["max_deviation_full"] < TOL["_pe32"][1], r


def test_gpu_tokens_equal_reference_config5_sample():
    """SURVEY config 5 pinned to the reference: every protein of bench.py's 512 x 512-residue
    codebook-64 000 / df-4 workload (forward_ref_bench.npz 'bench512', 512 proteins, 65 536 tokens;
    the df-4 local-window downsampler, model.py:264-318) in one ragged batch through the C ABI,
    against the reference's forward (_pe32 rendering): every token identical except the listed
    boundary cases, and every latent of 32 proteins within the tolerance."""
    S = refwide.load_bench_sample("bench512")
    assert [int(p) for p in S.proteins] == list(range(512))
    r = _run_bench_sample(S, 64000, 4)
    print({k: r[k] for k in ("tokens", "identical", "min_margin", "close_tokens", "max_deviation_close",
                             "max_deviation_full", "mismatches")})
    assert r["tokens"] == 65536
    assert not r["unexplained"] and not r["unlisted"] and not r["missing_known"], r
    assert r["max_deviation_close"] < TOL["_pe32"][1]
    assert r["full_latent_proteins"] == 32 and r["max_deviation_full"] < TOL["_pe32"][1], r


@pytest.mark.parametrize("cb,df", refwide.CASP_DF_CONFIGS)
def test_gpu_tokens_equal_reference_casp_df(cb, df):
    """The 31 CASP14 structures in ONE ragged batch per (codebook, df) at the reference CLI's other
    downsampling settings (df 2 and df 4: the local-window cross-attention downsampler, model.py:
    264-318, modules.py:427-534) through the C ABI, against the reference's forward (_pe32 rendering,
    forward_ref_casp_df.npz): every token identical except the listed boundary cases
    (refwide.KNOWN_CASP_DF_CASES); an unlisted flip or a listed case that no longer flips fails."""
    from pst_amd._native import pack_samples  # noqa: F401  (same binding as the other tests)
    G = refwide.load_casp_df()
    cases = refwide.casp_df_cases(G, cb, df)
    assert len(cases) == 31
    ins = [refwide.casp_inputs(c) for c in cases]
    pos = np.concatenate([p for p, _ in ins]).astype(np.float32)
    fl = np.concatenate([f for _, f in ins])
    off = np.zeros(len(cases) + 1, np.int64)
    off[1:] = np.cumsum([p.shape[0] for p, _ in ins])
    D, seed = (int(v) for v in G[cases[0] + "/meta"][4:6])
    tk = _make(cb, df, D, seed)
    tok, nt, nn = tk.tokenize_packed(pos, fl, off)
    b = tk.aux(int(off[-1]))["bounded"]
    tk.close()
    outs = {}
    for i, c in enumerate(cases):
        n, T = (int(v) for v in G[c + "/meta"][:2])
        assert int(nn[i]) == n and int(nt[i]) == T, c
        a = int(off[i])
        outs[c] = (tok[a:a + T].copy(), b[a:a + T].copy())
    r = refwide.compare_cases(G, outs)
    print({k: r[k] for k in ("cases", "tokens", "identical", "min_margin", "max_deviation", "mismatches")})
    assert not r["unexplained"] and not r["unlisted"] and not r["missing_known"], r
    assert r["max_deviation"] < TOL["_pe32"][1]
