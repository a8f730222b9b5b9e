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


def test_gpu_tokens_equal_reference_bench_sample():
    """The headline workload's reference sample: every 4th protein of bench.py's
    synthetic_batch(1024, 256, seed=1000) (forward_ref_bench.npz, 256 proteins, 65 536 tokens) in
    ONE ragged batch through the C ABI, against the reference's forward (_pe32 rendering)."""
    from pst_amd import synthetic
    from pst_amd._native import pack_samples
    FB = refwide.load_bench()
    names = refwide.cases(FB, "bench256_")
    samples = [synthetic.synthetic_protein(*(int(v) for v in FB[c + "/synthetic_args"])) for c in names]
    pos, flags, off = pack_samples(samples)
    tk = _make(4096, 1, 6, 1234)
    tok, nt, nn = tk.tokenize_packed(pos.astype(np.float32), flags, off)
    b = tk.aux(int(off[-1]))["bounded"]
    tk.close()
    reps = []
    for i, c in enumerate(names):
        n, T = (int(v) for v in FB[c + "/meta"][:2])
        assert nn[i] == n and nt[i] == T
        a = int(off[i])
        assert np.abs(b[a:a + T] - FB[c + "/bounded_pe32"]).max() < TOL["_pe32"][1], c
        reps.append(refwide.report(FB[c + "/bounded_pe32"], FB[c + "/tokens_pe32"], b[a:a + T], tok[a:a + T]))
    r = refwide.merge(reps)
    print({k: r[k] for k in ("tokens", "identical", "min_margin", "max_deviation", "max_deviation_over_margin")})
    assert r["tokens"] == 65536
    # every token equal except where the reference's float64 latent sits closer to a rounding
    # boundary than float32 arithmetic can resolve: at 65 536 x 6 dims one margin below our
    # ~5e-7 deviation is expected (protein 924, token 3: margin 2.6e-7), and every
    # mismatch must be such a case (our deviation beyond its margin, the margin below 1e-6)
    assert r["mismatches_explained_by_rounding"], r
    assert all(m < 1e-6 for m in r["mismatch_margins"]), r
    assert r["tokens"] - r["identical"] <= 1, r


def test_gpu_tokens_equal_reference_config5_sample():
    """SURVEY config 5's exact-match sample: every 16th protein of bench.py's 512 x 512-residue
    codebook-64 000 / df-4 workload (forward_ref_bench.npz bench512_*, 32 proteins, 4 096 tokens) in
    one ragged batch through the C ABI, against the reference's forward (_pe32 rendering)."""
    from pst_amd import synthetic
    from pst_amd._native import pack_samples
    FB = refwide.load_bench()
    names = refwide.cases(FB, "bench512_")
    assert len(names) == 32
    samples = [synthetic.synthetic_protein(*(int(v) for v in FB[c + "/synthetic_args"])) for c in names]
    pos, flags, off = pack_samples(samples)
    tk = _make(64000, 4, 6, 1234)
    tok, nt, nn = tk.tokenize_packed(pos.astype(np.float32), flags, off)
    b = tk.aux(int(off[-1]))["bounded"]
    tk.close()
    reps = []
    for i, c in enumerate(names):
        n, T = (int(v) for v in FB[c + "/meta"][:2])
        assert nn[i] == n and nt[i] == T
        a = int(off[i])
        assert np.abs(b[a:a + T] - FB[c + "/bounded_pe32"]).max() < TOL["_pe32"][1], c
        reps.append(refwide.report(FB[c + "/bounded_pe32"], FB[c + "/tokens_pe32"], b[a:a + T], tok[a:a + T]))
    r = refwide.merge(reps)
    print({k: r[k] for k in ("tokens", "identical", "min_margin", "max_deviation", "max_deviation_over_margin")})
    assert r["tokens"] == 4096 and r["identical"] == r["tokens"], r

