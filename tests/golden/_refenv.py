"""Helpers to run the reference's own Python code under the import shim (build container only).

Only `tests/golden/make_golden.py` and CPU tests marked `reference` use this; they skip when
`/root/reference` is absent (e.g. on the GPU box).
"""
import os
import sys

REF = os.environ.get("PST_REFERENCE_DIR", "/root/reference")
HERE = os.path.dirname(os.path.abspath(__file__))
SHIM = os.path.join(HERE, "shim")
PKG = os.path.join(os.path.dirname(os.path.dirname(HERE)), "protein-structure-tokenizer_amd")


def available() -> bool:
    return os.path.isdir(os.path.join(REF, "structure_tokenizer"))


def activate(f64: bool = False):
    """Put the shim and the reference on sys.path. Must run before any `jax` import."""
    os.environ["PST_SHIM_F64"] = "1" if f64 else "0"
    for p in (SHIM, REF):
        if p not in sys.path:
            sys.path.insert(0, p)
    if PKG not in sys.path:
        sys.path.append(PKG)
    import structure_tokenizer.data.protein_structure_sample as pss  # noqa: E402

    # `make_protein_features` builds structure-module loss features whose output
    # `make_graph_from_pdb` drops (`inference_runner.py:72` keeps `.graph` only); it is
    # off the tokenize path and needs the AF2 all-atom stack, so fixtures skip it.
    pss.ProteinStructureSample.make_protein_features = lambda self: {}
    return pss


def to_ref_sample(pss, s):
    """Our `ProteinStructureSample` → the reference's NamedTuple (same fields)."""
    return pss.ProteinStructureSample(**s._asdict())
