"""Autoencoder-pass fixtures from the reference itself (float64 under the NumPy shim).

`InferenceRunner.prepare_ae_fn` (scripts/inference_runner.py:209-222) pmaps `Vq3D.__call__`
(model/model.py:194-259): encode → quantize → decode with the GRAPH's nodes_mask → structure
module with the protein's own features. This runs that unmodified `__call__` on a
`BatchDataVQ3D` whose graph is the reference's `preprocess_sample` graph and whose two features
the structure module reads (`aatype`, `atom37_gt_exists`) are built as
`ProteinStructureSample.make_protein_features` + `preprocess_sample` build them
(protein_structure_sample.py:93-118: gt_exists kept on N, CA, C, O only;
preprocessing.py:285-306: rows of missing-backbone residues dropped, zero-padded to 512). The
rest of `make_protein_features` (atom14 / frames for the training losses) is not read by
`__call__` and needs the AF2 all-atom stack the shim does not carry (_refenv.activate).

Cases are chosen so the node count is NOT a multiple of df (the decode then runs on n_node
residues, not df × tokens) and one residue is UNK (its atoms map to zero, all_atom.py:77-111):

    ae_k64000_df4: 61 residues, 3 without backbone → 58 nodes, 14 tokens (56 ≠ 58)
    ae_k4096_df2:  76 residues, 1 without backbone → 75 nodes, 37 tokens
    ae_k4096_df1:  64 residues, no gaps

Weights: `params.random_full_params(D, seed)`. ~10 minutes per case (the reference pads to 512).

    python tests/golden/make_ae_golden.py [--jobs 3]     # → ae_ref.npz
"""
import argparse
import os
import sys
import time
from multiprocessing import get_context

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "ae_ref.npz")
PAD, K_NEIGHBOR = 512, 50
# (name, codebook, df, n_res, synthetic seed, residues without backbone, UNK residue, param seed)
CASES = [("ae_k64000_df4", 64000, 4, 61, 501, (5, 30, 44), 12, 91),
         ("ae_k4096_df2", 4096, 2, 76, 502, (70,), 3, 92),
         ("ae_k4096_df1", 4096, 1, 64, 503, (), 40, 93)]


def make_inputs(n, seed, gaps, unk):
    """Synthetic backbone; `gaps` lose their O (→ missing backbone, dropped by the graph);
    residue `unk` becomes UNK (restype 20). Returns (positions f32, flags u8, aatype idx)."""
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(HERE)), "protein-structure-tokenizer_amd"))
    from pst_amd import synthetic
    s = synthetic.synthetic_protein(n, seed)
    pos = s.atom37_positions.astype(np.float32)
    fl = s.atom_flags()
    for g in gaps:
        fl[g, 4] = 0  # O (atom37 index 4)
        pos[g, 4] = 0.0
    aa = np.argmax(s.aatype, axis=-1).astype(np.int64)
    aa[unk] = 20
    return pos, fl, aa


def run_case(case):
    os.environ["OMP_NUM_THREADS"] = "2"
    sys.path.insert(0, HERE)
    import _refenv
    pss = _refenv.activate(f64=True)
    import jax
    import haiku as hk
    from structure_tokenizer.data import preprocessing as ref_pp
    from structure_tokenizer.model.model import Vq3D
    from structure_tokenizer.types import BatchDataVQ3D
    from pst_amd import params as P
    from pst_amd.config import LEVELS, load_config, overrides_for
    from pst_amd.sample import sample_from_arrays

    name, cb, df, n, seed, gaps, unk, pseed = case
    t0 = time.time()
    pos32, flags, aa = make_inputs(n, seed, gaps, unk)
    s = sample_from_arrays(pos32.astype(np.float64), flags, aa)
    cfg = load_config("vq3d_inference", overrides=overrides_for(cb, df),
                      config_path=os.path.join(_refenv.REF, "config", "structure_tokenizer"))
    g = ref_pp.preprocess_sample(sample=_refenv.to_ref_sample(pss, s), num_neighbor=K_NEIGHBOR,
                                 downsampling_ratio=df, residue_loc_is_alphac=True,
                                 padding_num_residue=PAD, crop_index=PAD, noise_level=0.0).graph
    gb = jax.tree_util.tree_map(lambda x: np.asarray(x)[None], g)
    gb.edge_features = gb.edge_features.astype(np.float32).astype(np.float64)  # JAX x64-off H2D
    # the two features Vq3D.__call__'s structure module reads (see module docstring)
    gt = np.zeros((n, 37), np.int32)
    for idx in (0, 1, 2, 4):
        gt[:, idx] = s.atom37_gt_exists[:, idx]
    feats = {"aatype": np.asarray(s.aatype, np.float64), "atom37_gt_exists": gt}
    keep = ~s.get_missing_backbone_coords_mask()
    nn = int(keep.sum())
    feats = {k: np.pad(v[keep][:PAD], ((0, PAD - nn),) + ((0, 0),) * (v.ndim - 1)) for k, v in feats.items()}
    feats = {k: v[None] for k, v in feats.items()}
    D = len(LEVELS[cb])
    params = {k: {m: np.asarray(v, np.float64) for m, v in d.items()}
              for k, d in P.params_keys_conversion(P.random_full_params(D, pseed)).items()}

    def fn(batch):
        return Vq3D(config=cfg.model, global_config=cfg.data)(batch, is_training=False, safe_key=None)

    st, q = hk.transform(fn).apply(params, None, BatchDataVQ3D(graph=gb, features=feats))
    n_node = int(g.n_node[0])
    assert n_node == nn
    T = n_node // df
    b = np.asarray(q["continuous_embedding"][0, :T], np.float64)
    out = {"in_positions": pos32, "in_flags": flags, "in_aatype": aa.astype(np.uint8),
           "meta": np.array([n, n_node, T, cb, df, D, pseed], np.int64),
           "tokens": np.asarray(q["tokens"][0, :T]).astype(np.uint32),
           "bounded": b, "margin": np.abs(b - (np.floor(b) + 0.5)).min(axis=-1),
           "quantize_post_proj": np.asarray(q["quantize_post_proj"][0]).astype(np.float32),
           "final_atom_positions": np.asarray(st["final_atom_positions"][0, :n_node]).astype(np.float32),
           "final_atom_mask": np.asarray(st["final_atom_mask"][0]).astype(np.int32)}
    print(name, "done in", round(time.time() - t0), "s", flush=True)
    return name, out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--jobs", type=int, default=3)
    args = ap.parse_args()
    sys.path.insert(0, HERE)
    import _refenv
    if not _refenv.available():
        sys.exit("reference not available")
    res = {}
    with get_context("spawn").Pool(args.jobs) as pool:
        for name, o in pool.imap_unordered(run_case, CASES):
            for k, v in o.items():
                res[f"{name}/{k}"] = v
    np.savez_compressed(OUT, **res)


if __name__ == "__main__":
    main()
