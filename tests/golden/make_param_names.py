"""Enumerate every parameter leaf of the reference Vq3D (encoder + decoder + structure module).

Initialises the reference model (imported from /root/reference under the NumPy test shim, see
_refenv.py) with `encode_and_quantize` followed by `decode_and_make_structure` in one
`hk.transform` — the two halves `scripts/inference_runner.py` applies — and writes the
(module, name, shape) list, sorted the way JAX flattens a params dict, to
full_param_names.json. Takes ~10 minutes (the structure module runs in NumPy).

    python tests/golden/make_param_names.py
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, "..", "..", "protein-structure-tokenizer_amd"))


def main():
    import _refenv
    pss = _refenv.activate(f64=False)
    import numpy as np
    import jax
    import haiku as hk
    from structure_tokenizer.data import preprocessing as ref_pp
    from structure_tokenizer.model.model import Vq3D
    from pst_amd import synthetic
    from pst_amd.config import load_config, overrides_for

    cfg = load_config("vq3d_inference", overrides=overrides_for(4096, 1),
                      config_path=os.path.join(_refenv.REF, "config", "structure_tokenizer"))
    s = synthetic.synthetic_protein(60, 3)
    g = ref_pp.preprocess_sample(sample=_refenv.to_ref_sample(pss, s), num_neighbor=50, downsampling_ratio=1,
                                 residue_loc_is_alphac=True, padding_num_residue=512, crop_index=512,
                                 noise_level=0.0).graph
    gb = jax.tree_util.tree_map(lambda x: np.asarray(x)[None], g)

    def fn(graph):
        m = Vq3D(config=cfg.model, global_config=cfg.data)
        q = m.encode_and_quantize(graph, is_training=False, safe_key=None)
        return m.decode_and_make_structure(q["quantize"], graph.nodes_mask, graph.tokens_mask,
                                           is_training=False, safe_key=None)

    params = hk.transform(fn).init(None, gb)
    out = [[k, p, list(params[k][p].shape)] for k in sorted(params) for p in sorted(params[k])]
    with open(os.path.join(HERE, "full_param_names.json"), "w") as f:
        json.dump({"codes_dim": 6, "leaves": out}, f, indent=0)
    print(len(out), "leaves")


if __name__ == "__main__":
    main()
