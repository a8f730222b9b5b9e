"""Host logic of the reference-format ProteinGraph (pst_amd/graph.py): the padding of
preprocessing.py:191-283 applied to the real graph rows, checked against the reference's own
padded graphs (tests/golden/padded_graph_golden.npz, make_padded_graph_golden.py) — no GPU."""
import os

import numpy as np
import pytest

from pst_amd import graph as Gr
from pst_amd import runner
from pst_amd.sample import ProteinStructureSample

GOLD = os.path.join(os.path.dirname(__file__), "golden")
G = np.load(os.path.join(GOLD, "graph_golden.npz"))
PG = np.load(os.path.join(GOLD, "padded_graph_golden.npz"))
CASES = sorted({k.split("/")[0] for k in PG.files if k.endswith("/n_node")})
FIELDS = ("n_node", "n_edge", "nodes_mask", "nodes_original_coordinates", "node_features",
          "tokens_mask", "senders", "receivers")


def real_rows(c):
    """graph_golden's real part in pst_build_graph's row layout ([n,50] senders, -1 = none)."""
    n = int(G[c + "/n_node"])
    deg = min(n, 50)
    rows = np.full((n, 50), -1, np.int32)
    rows[:, :deg] = G[c + "/senders"].reshape(n, 50)[:, :deg]
    feat = np.zeros((n * 50, 27), np.float32)
    f = G[c + "/edge_features"]
    feat[:len(f)] = f
    return n, rows, feat.reshape(n, 50, 27), G[c + "/node_ca"]


def check_graph(g, c, n_edge_rows=None):
    for f in FIELDS:
        want, got = PG[c + "/" + f], getattr(g, f)
        assert got.shape == want.shape and got.dtype == want.dtype, (c, f, got.shape, want.shape, got.dtype, want.dtype)
        assert np.array_equal(got, want), (c, f)
    assert g.edge_features.shape == tuple(PG[c + "/edge_features_shape"])
    assert str(g.edge_features.dtype) == str(PG[c + "/edge_features_dtype"])
    ne = int(PG[c + "/n_edge"][0])
    ref = G[c + "/edge_features"][:ne]
    assert np.array_equal(g.edge_features[:ne].astype(np.float32).view(np.uint32), ref.view(np.uint32)), c
    assert not np.any(g.edge_features[ne:])


@pytest.mark.parametrize("case", CASES)
def test_padding_matches_reference(case):
    n, rows, feat, ca = real_rows(case)
    check_graph(Gr.pad_protein_graph(n, rows, feat, ca, int(G[case + "/df"])), case)


def test_no_usable_residue_raises_like_reference():
    with pytest.raises(ValueError, match="need at least one array to stack"):
        Gr.pad_protein_graph(0, np.zeros((0, 50)), np.zeros((0, 50, 27)), np.zeros((0, 3)), 1)


def test_batch_collate_unwraps_graph_views():
    c = "syn64_df1"
    pos = G[c + "/in_positions"].astype(np.float64)
    fl = G[c + "/in_flags"]
    n = pos.shape[0]
    s = ProteinStructureSample(None, n, np.zeros((n, 21)), pos, (fl & 1).astype(bool), ((fl >> 1) & 1).astype(bool), 0.0, 1)
    v = Gr.ProteinGraphView(s, 1)
    assert v.nb_residues == n  # structure attributes pass through without a GPU
    b = runner.batch_collate([1, 2], [v, s])
    assert b.samples == (s, s)
    with pytest.raises(TypeError):
        runner.batch_collate([1], [Gr.pad_protein_graph(*real_rows(c), 1)])
