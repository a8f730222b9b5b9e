"""The reference's padded `ProteinGraph` (`structure_tokenizer/types.py:49-75`), built from the
GPU residue graph.

`pst_build_graph` (libpst) runs the graph kernels of the tokenize path and returns, per protein,
the real part of the graph: node count, nearest-first senders, the 27 edge features and the
C-alpha coordinates. `pad_protein_graph` applies the padding of
`preprocessing.py:191-283` (`preprocess_sample`) to it, so `build_protein_graphs` returns what
`preprocess_sample(...).graph` / `make_graph_from_pdb` return in the reference:

  n_node [1], n_edge [1]                  int64
  nodes_mask [512, 1]                     bool
  nodes_original_coordinates = node_features [512, 3]  float64 (C-alpha, zero rows after n)
  edge_features [25600, 27]               float64 holding the float32 values the encoder
                                          consumes (the reference keeps the float64 values on the
                                          host and JAX casts them to float32 on transfer)
  tokens_mask [512 / df, 1]               bool
  senders, receivers [25600]              int64, padded as the reference pads them
"""
from typing import List, NamedTuple, Optional, Sequence

import numpy as np

from .sample import ProteinStructureSample

K_NEIGHBOR = 50
PADDING_NUM_RESIDUE = 512


class ProteinGraph(NamedTuple):
    n_node: np.ndarray
    n_edge: np.ndarray
    nodes_mask: np.ndarray
    nodes_original_coordinates: np.ndarray
    node_features: np.ndarray
    edge_features: np.ndarray
    tokens_mask: np.ndarray
    senders: np.ndarray
    receivers: np.ndarray


def pad_protein_graph(n: int, senders_rows: np.ndarray, features_rows: np.ndarray, ca: np.ndarray,
                      downsampling_ratio: int, num_neighbor: int = K_NEIGHBOR,
                      padding_num_residue: int = PADDING_NUM_RESIDUE) -> ProteinGraph:
    """One protein's graph in the reference layout.

    senders_rows [n, 50] / features_rows [n, 50, 27] / ca [n, 3] are pst_build_graph's rows of
    this protein (for n <= 50 the first n senders of a row are all nodes, self first, and the
    feature rows hold the reference's n x n enumeration row-major).
    """
    if n <= 0:
        # preprocess_sample stacks the per-residue arrays of no residue (np.stack([]))
        raise ValueError("need at least one array to stack")
    k = num_neighbor
    P = padding_num_residue
    deg = min(n, k)  # compute_nearest_neighbors_graph: num_neighbor = n when n <= k
    n_edge = n * deg
    snd_real = np.asarray(senders_rows, np.int64).reshape(n, k)[:, :deg].reshape(-1)
    rcv_real = np.repeat(np.arange(n, dtype=np.int64), deg)
    feat_real = np.asarray(features_rows, np.float32).reshape(n * k, 27)[:n_edge]
    n_pad_edges = k * P

    def pad_edges(x):
        if n < k:  # preprocessing.py:229-260 (pad_directed_edges)
            m = np.pad(x.reshape(n, -1)[:, :k], ((0, 0), (0, k - n)), constant_values=n)
            rows = np.repeat(np.arange(n, P, dtype=np.int64)[:, None], k, axis=-1)
            return np.concatenate([m, rows], axis=0)[:P].reshape(-1)
        return np.concatenate([x, np.repeat(np.arange(n, P, dtype=np.int64), k)])[:n_pad_edges]

    edge_features = np.zeros((n_pad_edges, 27), np.float64)
    edge_features[:min(n_edge, n_pad_edges)] = feat_real[:n_pad_edges]
    nodes_x = np.zeros((P, 3), np.float64)
    nodes_x[:n] = np.asarray(ca, np.float64)[:n]
    nodes_mask = np.zeros((P, 1), bool)
    nodes_mask[:n] = True
    max_tok = P // downsampling_ratio
    tokens_mask = np.zeros((max_tok, 1), bool)
    tokens_mask[:min(n // downsampling_ratio, max_tok)] = True
    return ProteinGraph(
        n_node=np.array([n], np.int64), n_edge=np.array([n_edge], np.int64), nodes_mask=nodes_mask,
        nodes_original_coordinates=nodes_x, node_features=nodes_x, edge_features=edge_features,
        tokens_mask=tokens_mask, senders=pad_edges(snd_real), receivers=pad_edges(rcv_real))


def build_protein_graphs(tokenizer, samples: Sequence[ProteinStructureSample],
                         downsampling_ratio: int) -> List[ProteinGraph]:
    """`preprocess_sample(...).graph` for each sample, graph built on the GPU (pst_build_graph)."""
    from ._native import pack_samples
    pos, flags, off = pack_samples(list(samples))
    snd, feat, ca, nn = tokenizer.build_graph_packed(pos, flags, off)
    out = []
    for b in range(len(samples)):
        a = int(off[b])
        n = int(nn[b])
        out.append(pad_protein_graph(n, snd[a:a + n], feat[a:a + n], ca[a:a + n], downsampling_ratio))
    return out


_GRAPH_CTX = {}
_GRAPH_DEVICE = [None]


def set_graph_device(device: Optional[int]) -> None:
    """The GPU that builds `ProteinGraph`s on demand (`ProteinGraphView.graph`,
    `preprocess_sample`). `InferenceRunner.prepare_tokenize_fn` sets it to the runner's first
    device; None restores the default (LOCAL_RANK modulo the visible devices, else 0)."""
    _GRAPH_DEVICE[0] = device


def graph_device() -> int:
    if _GRAPH_DEVICE[0] is not None:
        return _GRAPH_DEVICE[0]
    import os
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if local == 0:
        return 0
    from . import _native
    return local % max(1, _native.device_count())


def _graph_context(device: Optional[int] = None):
    """A libpst context used only for graph builds (the encoder weights do not enter the graph,
    so they are zeros), on `device` or the caller's graph device (`graph_device()`)."""
    if device is None:
        device = graph_device()
    if device not in _GRAPH_CTX:
        from . import _native, params
        blob = np.zeros(params.param_count(6), np.float32)
        _GRAPH_CTX[device] = _native.Tokenizer(device, 4096, 1, blob)
    return _GRAPH_CTX[device]


class ProteinGraphView:
    """What `runner.make_graph_from_pdb` returns: the parsed structure, which the tokenize path
    hands to the GPU as is, that also reads as the reference's padded `ProteinGraph` — the
    `ProteinGraph` fields are built on first access (pst_build_graph on `graph_device()`, the
    runner's device) and cached.
    Other attributes (`nb_residues`, `atom37_positions`, ...) are the structure's."""

    __slots__ = ("sample", "downsampling_ratio", "_graph")

    def __init__(self, sample: ProteinStructureSample, downsampling_ratio: int):
        self.sample = sample
        self.downsampling_ratio = downsampling_ratio
        self._graph = None

    @property
    def graph(self) -> ProteinGraph:
        if self._graph is None:
            self._graph = build_protein_graphs(_graph_context(), [self.sample], self.downsampling_ratio)[0]
        return self._graph

    def __getattr__(self, name):
        if name in ProteinGraph._fields:
            return getattr(self.graph, name)
        return getattr(self.sample, name)


class BatchDataVQ3D(NamedTuple):
    """`structure_tokenizer/types.py:80-89`; `features` (structure-module loss features,
    `make_protein_features`) are off the tokenize path and left empty."""
    graph: ProteinGraph
    features: dict


def preprocess_sample(sample: ProteinStructureSample, num_neighbor: int, downsampling_ratio: int,
                      residue_loc_is_alphac: bool, padding_num_residue: int, crop_index: int,
                      noise_level: float) -> BatchDataVQ3D:
    """`preprocessing.py:42-283` for the configurations libpst implements (C-alpha locations,
    50 neighbours, 512 residues, no crop beyond 512, no coordinate noise); graph built on the GPU."""
    if not residue_loc_is_alphac:
        raise NotImplementedError("libpst builds the graph on C-alpha locations only")
    if num_neighbor != K_NEIGHBOR or padding_num_residue != PADDING_NUM_RESIDUE or crop_index != PADDING_NUM_RESIDUE:
        raise NotImplementedError("libpst is specialised for num_neighbor=50, padding/crop 512")
    if noise_level != 0.0:
        raise NotImplementedError("coordinate noise (training augmentation) is not implemented")
    return BatchDataVQ3D(build_protein_graphs(_graph_context(), [sample], downsampling_ratio)[0], {})
