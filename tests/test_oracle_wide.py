"""The CPU oracle against the reference's own forward on the benchmarked configs.

`forward_ref_wide.npz` (`golden/make_forward_wide.py`): the reference `Vq3D.encode_and_quantize`
(model.py:453-479) in float64 under the shim on all 31 CASP14 proteins at codebook 4096 and
64 000 (df 1; BASELINE configs 2 and 4), the first 8 proteins of the bench workload (256
residues, config 3), 2 × 512 residues at 64 000 / df 4 (config 5) and the < 50-residue branch —
13 606 tokens. The oracle executes the canonical float32 sequence the GPU executes bit for bit
(DESIGN.md §4), so this pins the GPU's arithmetic to the reference; the GPU side is
`test_gpu_reference_wide.py`.
"""
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

import refwide
from oracle import oracle as O
from pst_amd import params as P
from pst_amd.config import LEVELS

F = refwide.load()
# Two float64 renderings of the reference (make_forward_wide.py): "pe32" evaluates the sinusoidal
# PE argument in float32 as JAX does with x64 off (the real reference's value), the other in
# float64 — and a third, "_f32", the shim in float32 mode with JAX's float32 PE (make_forward_wide.py
# --f32; mixed precision where NumPy promotes, see there). Measured over all 78 cases (oracle = GPU bits):
#   vs pe32: pre-projection (unit norm, 128-d) ≤ 3.0e-7, bounded latents (|b| < 3.5) ≤ 1.04e-5
#   vs f64:  ≤ 6.1e-6 and ≤ 1.5e-4 — the PE argument's own float32 rounding, not our arithmetic
#   vs f32:  ≤ 3.2e-7 and ≤ 1.03e-5
TOL = {"_pe32": (1e-6, 3e-5), "": (1.5e-5, 4e-4), "_f32": (1e-6, 3e-5)}


def _run(c):
    n, T, cb, df, D, seed = (int(v) for v in F[c + "/meta"])
    out = O.tokenize(P.random_blob(D, seed), LEVELS[cb], df, F[c + "/in_positions"].astype(np.float64),
                     F[c + "/in_flags"])
    return c, out


@pytest.fixture(scope="module")
def oracle_outputs():
    with ThreadPoolExecutor(8) as ex:  # the C oracle releases the GIL
        return dict(ex.map(_run, refwide.cases(F)))


@pytest.mark.parametrize("var", ["_pe32", "", "_f32"])
@pytest.mark.parametrize("prefix", ["casp_", "bench256_", "bench512_", "short_"])
def test_oracle_tokens_equal_reference_wide(oracle_outputs, prefix, var):
    reps = []
    tol_pre, tol_b = TOL[var]
    for c in refwide.cases(F, prefix):
        n, T, cb, df, D, seed = (int(v) for v in F[c + "/meta"])
        out = oracle_outputs[c]
        assert out["graph"]["n"] == n and len(out["tokens"]) == T
        assert np.abs(out["b"] - F[c + "/bounded" + var]).max() < tol_b, c
        if c + "/pre_proj" + var in F.files:
            assert np.abs(out["pre_proj"] - F[c + "/pre_proj" + var]).max() < tol_pre, c
        reps.append(refwide.report(F[c + "/bounded" + var], F[c + "/tokens" + var], out["b"], out["tokens"]))
    r = refwide.merge(reps)
    assert r["mismatches_explained_by_rounding"], r
    assert r["identical"] == r["tokens"], r


def test_fixture_margin_fields():
    for c in refwide.cases(F):
        for var in ("", "_pe32", "_f32"):
            m = refwide.dim_margins(F[c + "/bounded" + var]).min(-1)
            assert np.array_equal(m, F[c + "/margin" + var])
        # the three renderings agree on every token id of the fixture
        assert np.array_equal(F[c + "/tokens"], F[c + "/tokens_pe32"])
        assert np.array_equal(F[c + "/tokens"], F[c + "/tokens_f32"])
        # the float32 rendering's encoder really ran in float32 (its FSQ bound is NumPy-promoted)
        assert list(F[c + "/dtypes_f32"]) == ["float32", "float64"]


def test_deviation_localised_to_encoder_not_fsq_bound(oracle_outputs):
    """Where our bounded-latent deviation comes from (tools/refwide_report.py): our
    float32 FSQ bound (XLA's rational tanh) applied to the reference's OWN z is within 1.3e-6 of
    the reference's bounded latents (the bound term), while our z (encoder + down_proj, float32)
    differs from the reference's by ≤ 4.2e-6, which the bound's slope (up to half_l = 3.5) turns
    into the ≤ 1.04e-5 seen on b. Measured: bound term ≤ 7.6e-7 (pe32) / 1.26e-6 (f32)."""
    import sys
    import os
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    import refwide_report as RR
    for var in ("_pe32", "_f32"):
        loc = RR.localise(refwide.cases(F), oracle_outputs, var)
        assert loc["bound_term_max"] < 2e-6, (var, loc)
        assert loc["max_abs_z_deviation"] < 1e-5, (var, loc)
        assert loc["encoder_term_max"] < 3e-5, (var, loc)


def test_reference_as_computed_torch_matches_fixture():
    """oracle/reference_as_computed.py (the reference's padded, dense computation in plain
    PyTorch-CPU float32 — bench.py's CPU baseline) gives the reference's token ids too."""
    import torch
    from oracle.reference_as_computed import ReferenceAsComputed, padded_graphs
    torch.set_num_threads(8)
    for c in ("short_syn56_missing9_k4096_df2", "casp_T1082_k64000_df1", "bench256_p3_k4096_df1",
              "bench256_p777_k4096_df1", "bench512_p1_k64000_df4", "casp_T1024_k4096_df1"):
        n, T, cb, df, D, seed = (int(v) for v in F[c + "/meta"])
        m = ReferenceAsComputed(P.random_params(D, seed), LEVELS[cb], df)
        o = m.forward(padded_graphs([(F[c + "/in_positions"].astype(np.float64), F[c + "/in_flags"])], df))
        assert np.array_equal(o["tokens"][0, :T], F[c + "/tokens_pe32"]), c
        assert np.array_equal(o["tokens"][0, :T], F[c + "/tokens_f32"]), c
        assert np.abs(o["bounded"][0, :T] - F[c + "/bounded_pe32"]).max() < 1e-4


# ------------------------------------------------------------ the headline workload's sample
# forward_ref_bench.npz (golden/make_forward_bench.py + compact_bench.py): the reference's forward
# (_pe32 rendering) on every protein of bench.py's workload, synthetic_batch(1024, 256, seed=1000)
# at codebook 4096 / df 1 ('bench256'), and every 16th of config 5's ('bench512'). Inputs are not
# stored: they regenerate from the generator (SHA-checked in test_fixture_recipes.py). The C oracle
# runs every 4th headline protein here (65 536 tokens, a few seconds on 8 threads); the GPU test
# runs all of them.


def _oracle_sample(S, prots, levels, df):
    from pst_amd import synthetic

    def run(p):
        s = synthetic.synthetic_protein(S.meta["n_res"], S.meta["seed0"] + p)
        return O.tokenize(P.random_blob(S.meta["D"], S.meta["param_seed"]), levels, df, s.atom37_positions,
                          s.atom_flags())

    with ThreadPoolExecutor(8) as ex:
        outs = list(ex.map(run, prots))
    for p, o in zip(prots, outs):
        assert o["graph"]["n"] == S.n_nodes[S.index[p]] and len(o["tokens"]) == S.n_tokens(p)
    return S.compare(prots, [o["tokens"] for o in outs], [o["b"] for o in outs])


def test_oracle_tokens_equal_reference_bench_sample():
    S = refwide.load_bench_sample("bench256")
    assert S.meta == {"n_res": 256, "seed0": 1000, "codebook": 4096, "df": 1, "D": 6, "param_seed": 1234}
    prots = list(range(0, 1024, 4))
    r = _oracle_sample(S, prots, LEVELS[4096], 1)
    print({k: r[k] for k in ("tokens", "identical", "min_margin", "close_tokens", "max_deviation_close",
                             "max_deviation_over_margin_close", "mismatches")})
    assert r["tokens"] == 65536
    # every token identical except the listed boundary cases (refwide.KNOWN_BOUNDARY_CASES: the
    # reference's float64 latent nearer a rounding boundary than float32 resolves — protein 924,
    # token 3, dim 5: margin 2.6e-7); an unlisted flip or a listed case that no
    # longer flips fails
    assert not r["unexplained"] and not r["unlisted"] and not r["missing_known"], r
    assert r["max_deviation_close"] < TOL["_pe32"][1]
    # the full-latent subset (p % 32 == 0: all 32 are among these 256) bounds the drift of every token
    assert r["full_latent_proteins"] == 32 and r["max_deviation_full"] < TOL["_pe32"][1], r


def test_oracle_tokens_equal_reference_config5_sample():
    """SURVEY config 5 (codebook 64 000, df 4, 512-residue proteins; all 512 proteins of bench.py's
    --codebook 64000 --df 4 --residues 512 --proteins 512 workload are pinned, the GPU test runs them
    all): the C oracle on every 4th protein (128 proteins, 16 384 tokens; the 32 full-latent ones among them)
    against the reference's forward."""
    S = refwide.load_bench_sample("bench512")
    assert S.meta == {"n_res": 512, "seed0": 1000, "codebook": 64000, "df": 4, "D": 6, "param_seed": 1234}
    assert [int(p) for p in S.proteins] == list(range(512))
    r = _oracle_sample(S, list(range(0, 512, 4)), LEVELS[64000], 4)
    print({k: r[k] for k in ("tokens", "identical", "min_margin", "close_tokens", "max_deviation_close",
                             "max_deviation_full", "mismatches")})
    assert r["tokens"] == 16384
    assert not r["unexplained"] and not r["unlisted"] and not r["missing_known"], r
    assert r["full_latent_proteins"] == 32 and r["max_deviation_full"] < TOL["_pe32"][1], r


# ------------------------------------------------------------ CASP14 at df 2 / df 4
# forward_ref_casp_df.npz (golden/make_forward_casp_df.py): the reference's forward (_pe32 rendering)
# on all 31 CASP14 structures at the reference CLI's other downsampling settings — (4096, df 2),
# (4096, df 4), (64000, df 2), (64000, df 4) — which run the local-window cross-attention
# downsampler and its pooling (model.py:264-318, modules.py:427-534) that df 1 does not.
@pytest.mark.parametrize("cb,df", refwide.CASP_DF_CONFIGS)
def test_oracle_tokens_equal_reference_casp_df(cb, df):
    G = refwide.load_casp_df()
    cases = refwide.casp_df_cases(G, cb, df)
    assert len(cases) == 31

    def run(c):
        pos, fl = refwide.casp_inputs(c)
        n, T, mcb, mdf, D, seed = (int(v) for v in G[c + "/meta"])
        assert (mcb, mdf) == (cb, df)
        o = O.tokenize(P.random_blob(D, seed), LEVELS[cb], df, pos.astype(np.float64), fl)
        assert o["graph"]["n"] == n and len(o["tokens"]) == T, c
        return c, (o["tokens"], o["b"])

    with ThreadPoolExecutor(8) as ex:
        outs = dict(ex.map(run, cases))
    r = refwide.compare_cases(G, outs)
    print({k: r[k] for k in ("cases", "tokens", "identical", "min_margin", "max_deviation", "mismatches")})
    assert not r["unexplained"] and not r["unlisted"] and not r["missing_known"], r
    assert r["max_deviation"] < TOL["_pe32"][1]
