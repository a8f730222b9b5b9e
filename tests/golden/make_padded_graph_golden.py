"""Padded ProteinGraph fixtures: the reference's `preprocess_sample(...).graph` in full
(senders/receivers padded to 512·50 edges, masks, node coordinates padded to 512 rows) for every
`graph_golden.npz` case, run under the import shim.

Run in the build container (needs /root/reference):
    python tests/golden/make_padded_graph_golden.py
Inputs are the atom37 arrays stored in `graph_golden.npz`; the output `padded_graph_golden.npz`
is what `pst_amd.graph.pad_protein_graph` and `build_protein_graphs` are checked against.
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import _refenv  # noqa: E402

K_NEIGHBOR, PAD = 50, 512


def main():
    if not _refenv.available():
        sys.exit("reference not available")
    pss = _refenv.activate(f64=False)
    from structure_tokenizer.data import preprocessing as ref_pp
    from pst_amd.sample import ProteinStructureSample

    G = np.load(os.path.join(HERE, "graph_golden.npz"))
    cases = sorted({k.split("/")[0] for k in G.files if k.endswith("/n_node")})
    out = {}
    for c in cases:
        pos = G[c + "/in_positions"].astype(np.float64)
        fl = G[c + "/in_flags"]
        df = int(G[c + "/df"])
        n = pos.shape[0]
        s = ProteinStructureSample(None, n, np.zeros((n, 21)), pos, (fl & 1).astype(bool),
                                   ((fl >> 1) & 1).astype(bool), 0.0, 1)
        g = ref_pp.preprocess_sample(
            sample=_refenv.to_ref_sample(pss, s), num_neighbor=K_NEIGHBOR, downsampling_ratio=df,
            residue_loc_is_alphac=True, padding_num_residue=PAD, crop_index=PAD,
            noise_level=0.0).graph
        ef = np.asarray(g.edge_features)
        nn = int(g.n_node[0])
        e_real = min(nn, PAD) * K_NEIGHBOR
        assert not np.any(ef[max(int(g.n_edge[0]), e_real):]), "padded edge rows are not zero"
        rec = dict(
            n_node=np.asarray(g.n_node), n_edge=np.asarray(g.n_edge),
            nodes_mask=np.asarray(g.nodes_mask),
            nodes_original_coordinates=np.asarray(g.nodes_original_coordinates),
            node_features=np.asarray(g.node_features),
            edge_features_shape=np.array(ef.shape, np.int64),
            edge_features_dtype=str(ef.dtype),
            tokens_mask=np.asarray(g.tokens_mask),
            senders=np.asarray(g.senders), receivers=np.asarray(g.receivers),
            senders_dtype=str(np.asarray(g.senders).dtype),
        )
        for k, v in rec.items():
            out[f"{c}/{k}"] = v
        print(f"{c}: n_node={nn} n_edge={int(g.n_edge[0])} senders {rec['senders'].shape} "
              f"{rec['senders_dtype']} edge_features {ef.shape} {ef.dtype}")
    np.savez_compressed(os.path.join(HERE, "padded_graph_golden.npz"), **out)


if __name__ == "__main__":
    main()
