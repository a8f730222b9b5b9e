"""`dm-tree` subset (test shim)."""
from jax.tree_util import tree_map as _tm


def map_structure(f, *structs):
    return _tm(f, *structs)


def flatten(struct):
    from jax.tree_util import tree_leaves
    return tree_leaves(struct)
