"""Generate golden fixtures by running the REFERENCE's own code under the import shim.

Run in the build container (needs /root/reference):  python tests/golden/make_golden.py
Writes small .npz files next to this script. Inputs are our parsed CASP14 atom37 arrays and
synthetic proteins; expected outputs come from the reference functions named per fixture.
"""
import glob
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import _refenv  # noqa: E402

K_NEIGHBOR, PAD = 50, 512


def graph_case(ref_pp, pss, sample, df):
    g = ref_pp.preprocess_sample(
        sample=_refenv.to_ref_sample(pss, sample), num_neighbor=K_NEIGHBOR,
        downsampling_ratio=df, residue_loc_is_alphac=True, padding_num_residue=PAD,
        crop_index=PAD, noise_level=0.0).graph
    n = int(g.n_node[0])
    rows = min(n, PAD)
    e_real = rows * K_NEIGHBOR
    return dict(
        n_node=np.int32(n), n_edge=np.int32(int(g.n_edge[0])),
        # JAX (x64 off) casts the float64 edge features to float32 on transfer.
        edge_features=np.asarray(g.edge_features[:e_real], dtype=np.float32),
        edge_features_dtype=str(np.asarray(g.edge_features).dtype),
        senders=np.asarray(g.senders[:e_real], dtype=np.int32),
        receivers=np.asarray(g.receivers[:e_real], dtype=np.int32),
        nodes_mask=np.asarray(g.nodes_mask[:, 0]),
        tokens_mask=np.asarray(g.tokens_mask[:, 0]),
        node_ca=np.asarray(g.node_features[:n], dtype=np.float64),
    )


def pack_samples(samples):
    n = [s.nb_residues for s in samples]
    off = np.concatenate([[0], np.cumsum(n)]).astype(np.int64)
    pos = np.concatenate([s.atom37_positions for s in samples]).astype(np.float32)
    flags = np.concatenate([s.atom_flags() for s in samples])
    assert np.array_equal(pos.astype(np.float64), np.concatenate([s.atom37_positions for s in samples]))
    return pos, flags, off


def main():
    if not _refenv.available():
        sys.exit("reference not available")
    pss = _refenv.activate(f64=False)
    from structure_tokenizer.data import preprocessing as ref_pp
    from structure_tokenizer.data import residue_constants as ref_rc
    from pst_amd import residue_constants as rc, synthetic
    from pst_amd.pdb import protein_structure_from_pdb_file

    # --- table parity (restated residue constants vs reference) -------------------------
    assert rc.atom_types == ref_rc.atom_types
    assert rc.restypes == ref_rc.restypes
    assert rc.restype_1to3 == ref_rc.restype_1to3
    assert rc.res_atom37_exist == ref_rc.res_atom37_exist

    # --- CASP14 inputs (parsed by our restated parser) ----------------------------------
    pdbs = sorted(glob.glob(os.path.join(_refenv.REF, "casp14_pdbs", "*.pdb")))
    samples = [protein_structure_from_pdb_file(p) for p in pdbs]
    names = [os.path.basename(p)[:-4] for p in pdbs]
    pos, flags, off = pack_samples(samples)
    np.savez_compressed(os.path.join(HERE, "casp14_atom37.npz"), names=np.array(names),
                        positions=pos, flags=flags, offsets=off,
                        aatype=np.concatenate([s.aatype.argmax(-1) for s in samples]).astype(np.int8))
    print("casp14:", len(samples), "proteins,", off[-1], "residues")

    # --- graph fixtures: reference preprocess_sample ------------------------------------
    cases = {}
    pick = {"T1024": 1, "T1029": 1, "T1041": 4, "T1082": 2}
    for nm, df in pick.items():
        s = samples[names.index(nm)]
        cases[f"casp_{nm}_df{df}"] = (s, df)
    syn = {
        "syn50": synthetic.synthetic_protein(50, 7),
        "syn51": synthetic.synthetic_protein(51, 8),
        "syn64": synthetic.synthetic_protein(64, 9),
        "syn130": synthetic.synthetic_protein(130, 10),
    }
    # ragged/edge cases: missing backbone atoms → fewer than 50 usable residues
    s = synthetic.synthetic_protein(56, 11)
    gt = s.atom37_gt_exists.copy()
    gt[[3, 10, 11, 30, 41, 50, 55], rc.CA_INDEX] = False
    gt[[5, 20], rc.O_INDEX] = False
    pos_ = s.atom37_positions.copy()
    pos_[~gt] = 0.0
    syn["syn56_missing9"] = s._replace(atom37_gt_exists=gt, atom37_positions=pos_)
    # tiny graphs: only the first 5 / 1 residues keep their O atom (n = 5, n = 1)
    for keep in (5, 1):
        s = synthetic.synthetic_protein(60, 12 + keep)
        gt = s.atom37_gt_exists.copy()
        gt[keep:, rc.O_INDEX] = False
        syn[f"syn60_keep{keep}"] = s._replace(atom37_gt_exists=gt)
    for k, v in syn.items():
        cases[k + "_df1"] = (v, 1)
    cases["syn130_df4"] = (syn["syn130"], 4)
    out = {}
    for key, (s, df) in cases.items():
        g = graph_case(ref_pp, pss, s, df)
        for f, v in g.items():
            out[f"{key}/{f}"] = v
        out[f"{key}/in_positions"] = s.atom37_positions.astype(np.float32)
        out[f"{key}/in_flags"] = s.atom_flags()
        out[f"{key}/df"] = np.int32(df)
        print(f"graph {key}: n_node={g['n_node']} edges={len(g['senders'])} dtype={g['edge_features_dtype']}")
    np.savez_compressed(os.path.join(HERE, "graph_golden.npz"), **out)

    # --- FSQ index map: reference codes_to_indexes / indexes_to_codes -------------------
    from structure_tokenizer.model import quantize as ref_q
    fsq = {}
    for levels in ([4] * 6, [8, 8, 8, 5, 5, 5], [4, 4, 3, 3, 3], [4, 4, 4, 3, 3, 3]):
        lv = np.asarray(levels)
        k = int(np.prod(lv))
        basis = np.concatenate(([1], np.cumprod(lv[:-1]))).astype(np.uint32)
        idx = np.arange(k)
        codes = ref_q.indexes_to_codes(lv, idx)  # centred in [-1, 1] (scale_and_shift_inverse)
        back = ref_q.codes_to_indexes(lv, basis, codes)
        tag = "x".join(map(str, levels))
        fsq[f"{tag}/codes"] = np.asarray(codes, dtype=np.float32)
        fsq[f"{tag}/roundtrip"] = np.asarray(back, dtype=np.uint32)
        print("fsq", tag, k, "roundtrip exact:", bool(np.array_equal(back, idx)))
    np.savez_compressed(os.path.join(HERE, "fsq_golden.npz"), **fsq)


FORWARD_CASES = [
    # (name, n_res, seed, codebook, df, keep_aux)
    ("syn51_k4096_df1", 51, 8, 4096, 1, True),
    ("syn64_k4096_df1", 64, 9, 4096, 1, False),
    ("syn96_missing_k4096_df1", 96, 21, 4096, 1, False),
    ("syn130_k64000_df4", 130, 10, 64000, 4, False),
    ("syn90_k4096_df2", 90, 12, 4096, 2, False),
    ("syn60_k432_df1", 60, 13, 432, 1, False),
    ("syn50_k1728_df1", 50, 14, 1728, 1, False),
]
PARAM_SEED = 1234


def forward_main():
    """Reference Vq3D.encode_and_quantize executed under the shim in float64."""
    pss = _refenv.activate(f64=True)
    import jax
    import haiku as hk
    from structure_tokenizer.data import preprocessing as ref_pp
    from structure_tokenizer.model.model import Vq3D
    from pst_amd import synthetic, params as P
    from pst_amd import residue_constants as rc
    from pst_amd.config import load_config, overrides_for, LEVELS

    out = {}
    # the committed inputs are authoritative: `pst_amd.synthetic` was revised after this fixture
    # was made, so re-running regenerates outputs for the stored proteins, never new ones
    path = os.path.join(HERE, "forward_golden_f64.npz")
    stored = np.load(path) if os.path.exists(path) else None
    from pst_amd.sample import sample_from_arrays
    for name, n_res, seed, cb, df, keep_aux in FORWARD_CASES:
        cfg = load_config("vq3d_inference", overrides=overrides_for(cb, df),
                          config_path=os.path.join(_refenv.REF, "config", "structure_tokenizer"))
        if stored is not None and f"{name}/in_positions" in stored.files:
            s = sample_from_arrays(stored[f"{name}/in_positions"].astype(np.float64), stored[f"{name}/in_flags"])
        else:
            s = synthetic.synthetic_protein(n_res, seed)
        if "missing" in name and stored is None:
            gt = s.atom37_gt_exists.copy()
            gt[[2, 17, 40, 41, 77], rc.CA_INDEX] = False
            pos = s.atom37_positions.copy()
            pos[~gt] = 0.0
            s = s._replace(atom37_gt_exists=gt, atom37_positions=pos)
        g = ref_pp.preprocess_sample(sample=_refenv.to_ref_sample(pss, s), num_neighbor=K_NEIGHBOR,
                                     downsampling_ratio=df, residue_loc_is_alphac=True,
                                     padding_num_residue=PAD, crop_index=PAD, noise_level=0.0).graph
        gb = jax.tree_util.tree_map(lambda x: np.asarray(x)[None], g)
        # JAX (x64 disabled) sees float32 edge features; keep those values, in float64
        gb.edge_features = gb.edge_features.astype(np.float32).astype(np.float64)
        D = len(LEVELS[cb])
        params = {m: {k: v.astype(np.float64) for k, v in d.items()}
                  for m, d in P.random_params(D, PARAM_SEED).items()}

        def fn(graph):
            return Vq3D(config=cfg.model, global_config=cfg.data).encode_and_quantize(
                graph, is_training=False, safe_key=None)

        res = hk.transform(fn).apply(params, None, gb)
        n = int(g.n_node[0])
        T = n // df
        pre = f"{name}/"
        out[pre + "in_positions"] = s.atom37_positions.astype(np.float32)
        out[pre + "in_flags"] = s.atom_flags()
        out[pre + "meta"] = np.array([n, T, cb, df, D, PARAM_SEED], np.int64)
        out[pre + "pre_proj"] = np.asarray(res["continuous_embedding_pre_proj"][0, :T])
        out[pre + "bounded"] = np.asarray(res["continuous_embedding"][0, :T])
        out[pre + "quantize"] = np.asarray(res["quantize"][0, :T])
        out[pre + "tokens"] = np.asarray(res["tokens"][0, :T]).astype(np.uint32)
        out[pre + "tokens_padded"] = np.asarray(res["tokens"][0, T:T + 4]).astype(np.uint32)
        if keep_aux:
            out[pre + "distances"] = np.asarray(res["distances"][0, :T], dtype=np.float32)
            out[pre + "soft_proba"] = np.asarray(res["soft_proba"][0, :T], dtype=np.float32)
            out[pre + "perplexity"] = np.asarray(res["perplexity"])
        print(f"forward {name}: n={n} T={T} distinct tokens={len(np.unique(out[pre + 'tokens']))}")
    np.savez_compressed(path, **out)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "forward":
        forward_main()
    elif len(sys.argv) > 1 and sys.argv[1] == "host":
        main()
    else:
        import subprocess
        subprocess.run([sys.executable, __file__, "host"], check=True)
        subprocess.run([sys.executable, __file__, "forward"], check=True)
