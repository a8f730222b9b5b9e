"""The CPU oracle against the reference's own outputs (committed golden fixtures).

graph_golden.npz   — reference `preprocess_sample` (preprocessing.py:42-283) run under the
                     shim: senders/receivers exact, float32 edge features BITWISE equal.
forward_golden_f64.npz — reference `Vq3D.encode_and_quantize` (model.py:453-479) executed in
                     float64 under the shim: the oracle's canonical float32 path must agree to
                     the stated tolerances and give identical token ids.
fsq_golden.npz     — reference `indexes_to_codes` / `codes_to_indexes` (quantize.py:58-79).
"""
import os

import numpy as np
import pytest

from oracle import oracle as O
from pst_amd import params as P
from pst_amd.config import LEVELS

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _cases(npz):
    return sorted({k.split("/")[0] for k in npz.files})


GRAPH = np.load(os.path.join(GOLD, "graph_golden.npz"))
FWD = np.load(os.path.join(GOLD, "forward_golden_f64.npz"))


@pytest.mark.parametrize("case", _cases(GRAPH))
def test_graph_bitwise_vs_reference(case):
    g = O.graph(GRAPH[case + "/in_positions"].astype(np.float64), GRAPH[case + "/in_flags"])
    n = int(GRAPH[case + "/n_node"])
    assert g["n"] == n
    k = 50
    slots = np.arange(n * k)
    r, j = slots // k, slots % k
    valid = j < g["deg"][r]
    assert np.array_equal(g["senders"][valid], GRAPH[case + "/senders"][valid])
    assert np.array_equal(GRAPH[case + "/receivers"][valid], r[valid])
    ours = np.ascontiguousarray(g["feat"][:, :27])
    ref = GRAPH[case + "/edge_features"]
    assert np.array_equal(ours.view(np.uint32), ref.view(np.uint32)), "edge features not bitwise equal"


# Tolerances of the canonical float32 path vs the reference maths in float64.
TOL_PRE_PROJ = 5e-6   # unit-norm 128-d embedding
TOL_BOUNDED = 1e-4    # FSQ-bounded latents (|b| < 4)


@pytest.mark.parametrize("case", _cases(FWD))
def test_forward_vs_reference_f64(case):
    n, T, cb, df, D, seed = (int(v) for v in FWD[case + "/meta"])
    blob = P.random_blob(D, seed)
    out = O.tokenize(blob, LEVELS[cb], df, FWD[case + "/in_positions"].astype(np.float64),
                     FWD[case + "/in_flags"])
    assert out["graph"]["n"] == n and len(out["tokens"]) == T
    assert np.abs(out["pre_proj"] - FWD[case + "/pre_proj"]).max() < TOL_PRE_PROJ
    assert np.abs(out["b"] - FWD[case + "/bounded"]).max() < TOL_BOUNDED
    assert np.array_equal(out["q"], FWD[case + "/quantize"])
    assert np.array_equal(out["tokens"], FWD[case + "/tokens"])


def test_padded_token_id():
    # padded tokens: bounded*mask = 0 -> q = 0 -> sum (L//2)*basis (quantize.py:209)
    F = FWD
    for case in _cases(F):
        cb = int(F[case + "/meta"][2])
        lv = LEVELS[cb]
        basis = np.concatenate(([1], np.cumprod(lv[:-1])))
        pad = int(sum((l // 2) * b for l, b in zip(lv, basis)))
        assert np.all(F[case + "/tokens_padded"] == pad)


def test_fsq_index_map_vs_reference():
    G = np.load(os.path.join(GOLD, "fsq_golden.npz"))
    for tag in _cases(G):
        lv = [int(x) for x in tag.split("x")]
        K = int(np.prod(lv))
        codes = G[tag + "/codes"]  # centred codes in [-1, 1] per reference indexes_to_codes
        basis = np.concatenate(([1], np.cumprod(lv[:-1])))
        half = np.array([l // 2 for l in lv])
        # our token rule: idx = sum (q + L//2) * basis with q = code * (L//2)
        q = np.rint(codes * half).astype(np.int64)
        idx = ((q + half) * basis).sum(-1)
        assert np.array_equal(idx, np.arange(K))
        assert np.array_equal(G[tag + "/roundtrip"], np.arange(K))


def test_fsq_aux_vs_reference():
    """distances / soft_proba / perplexity (quantize.py:211-239) of the oracle's canonical
    formulation vs the reference model's own outputs (f64 run, shim) on the same latents."""
    F = FWD
    c = "syn51_k4096_df1/"
    b = F[c + "bounded"].astype(np.float32)
    a = O.fsq_aux((4,) * 6, b)
    d, p = F[c + "distances"], F[c + "soft_proba"]
    np.testing.assert_allclose(a["distances"], d, rtol=1e-6, atol=1e-5)
    np.testing.assert_allclose(a["soft_proba"], p, rtol=1e-4, atol=1e-6)
    assert np.array_equal(a["argmin"], F[c + "tokens"])
    ppl, _ = O.perplexity(F[c + "tokens"], 4096)
    assert abs(ppl - float(F[c + "perplexity"])) <= 1e-6 * ppl
