"""Host-side mirror of the reference's tokenize runner (`scripts/inference_runner.py`).

Same names, argument meaning and error behaviour as the reference, with the compute moved
into libpst (`include/pst.h`):

  reference (JAX / haiku, pmap over local devices)      here (libpst contexts, one per GPU)
  ----------------------------------------------------  -------------------------------------
  make_graph_from_pdb  (:40-74)  parse + size gates +   parse + the same size gates; returns a
                       preprocess_sample on the host    ProteinGraphView: the graph is built on the
                                                        GPU (k_prep/k_knn) inside pst_tokenize, or
                                                        padded like the reference's ProteinGraph
                                                        on field access (pst_build_graph)
  batch_collate        (:77-83)  stack padded graphs    pack ragged atom37 arrays + offsets
  load_params          (:136-150) npz + pickled treedef npz + leaf order of full_param_spec
  params_keys_conversion (:153-165)                     same (pst_amd.params)
  InferenceRunner.prepare_devices (:169-177)            HIP devices (backend "gpu" only)
  InferenceRunner.prepare_tokenize_fn (:179-191)        TokenizeFn: per-device libpst contexts
  InferenceRunner.prepare_decode_fn / prepare_ae_fn /   DecodeFn / AutoEncodeFn / TokenToCodeFn
    prepare_token_to_code_fn (:193-233)
  InferenceRunner.load_params (:236-248)                ReplicatedParams
  InferenceRunner.tokenize (:250-324)                   same loop, files and layout

There is no CPU fallback: `backend` must be "gpu" (the reference's "cpu"/"tpu" backends are
XLA targets this library does not have) and libpst.so must load.
"""
import concurrent.futures as _cf
import logging
import os
import time
from itertools import cycle, islice
from typing import Any, Callable, Dict, List, NamedTuple, Optional, Sequence, Tuple, Union

import numpy as np

from . import _native
from . import graph as _graph
from . import params as _params
from .config import LEVELS, TokenizerConfig
from .sample import ProteinStructureSample


PARSE_THREADS = int(os.environ.get("PST_PARSE_THREADS", "8"))
WRITE_THREADS = int(os.environ.get("PST_WRITE_THREADS", "1"))  # box: 1 thread 0.34 ms, 4 0.44, 16 0.43 (31 files)


def npy_bytes(a: np.ndarray) -> bytes:
    """The bytes `np.save` writes for a C-contiguous array of a little-endian numeric dtype
    (format 1.0, header padded to a multiple of 64): built directly, without np.save's
    per-call file-object machinery (tests/test_host.py checks byte equality with np.save)."""
    a = np.ascontiguousarray(a)
    shape = "(" + "".join(f"{d}, " for d in a.shape)[:-2] + ("," if a.ndim == 1 else "") + ")"
    d = "{'descr': '%s', 'fortran_order': False, 'shape': %s, }" % (a.dtype.str, shape)
    n = 10 + len(d) + 1
    d = d + " " * ((64 - n % 64) % 64) + "\n"
    return b"\x93NUMPY\x01\x00" + len(d).to_bytes(2, "little") + d.encode("latin1") + a.tobytes()


def save_npy_files(paths: Sequence[str], arrays: Sequence[np.ndarray], threads: int = WRITE_THREADS) -> None:
    """np.save(path, array) for every pair (path gets ".npy" appended as np.save does): the bytes
    built here, the files written by libpst's native host pool (`pst_write_files`; Python threads
    only contend for the GIL on 31 small writes). A path listed twice keeps its last array."""
    last = {p: i for i, p in enumerate(paths)}
    todo = sorted(last.values())
    names = [paths[i] if paths[i].endswith(".npy") else paths[i] + ".npy" for i in todo]
    _native.write_files(names, [npy_bytes(arrays[i]) for i in todo], n_threads=threads)


# ------------------------------------------------------------------------------- graph inputs
def make_graph_from_pdb(pdb_file_path: str, num_neighbor: int, downsampling_ratio: int,
                        residue_loc_is_alphac: bool, padding_num_residue: int,
                        sample: Optional[ProteinStructureSample] = None) -> _graph.ProteinGraphView:
    """Parse one PDB and apply the reference's size gates (`inference_runner.py:40-74`).

    Returns a `ProteinGraphView`: the parsed structure, which `pst_tokenize` turns into the
    residue graph on the GPU inside the tokenize call, and which also reads as the reference's
    padded `ProteinGraph` (fields built by `pst_build_graph` on first access), so callers that
    inspect the graph get the reference's arrays. Parsing uses libpst's native
    parser (`pst_pdb_parse_files`, Biopython semantics as restated in `pst_amd/pdb.py`);
    `sample` skips parsing when the caller parsed a batch already. `residue_loc_is_alphac=False`
    and other `padding_num_residue` / `num_neighbor` values than the shipped 512 / 50 are
    rejected (the device kernels are specialised for them).
    """
    if sample is None:
        if not os.path.exists(pdb_file_path):
            raise FileNotFoundError(pdb_file_path)
        sample = _native.parse_pdb_files([pdb_file_path], n_threads=1).sample(0)
    if sample.nb_residues > 512:
        raise NotImplementedError(
            "We currently don't support protein with more than 512 residues"
            f"given: {sample.nb_residues}")
    if sample.nb_residues < num_neighbor:
        raise NotImplementedError(
            f"We currently don't support protein with less than {num_neighbor} residues"
            f"given: {sample.nb_residues}")
    if bool(np.all(sample.get_missing_backbone_coords_mask())):
        # the reference fails in preprocess_sample (np.stack of no residues) with this message
        raise ValueError("need at least one array to stack")
    if not residue_loc_is_alphac:
        raise NotImplementedError("libpst builds the graph on C-alpha locations only "
                                  "(graph_residue_loc_is_alphac: true in every shipped config)")
    if num_neighbor != 50 or padding_num_residue != 512:
        raise NotImplementedError("libpst is specialised for graph_max_neighbor=50, seq_max_size=512")
    if downsampling_ratio not in (1, 2, 4):
        raise ValueError(f"downsampling_ratio must be 1, 2 or 4, got {downsampling_ratio}")
    return _graph.ProteinGraphView(sample, downsampling_ratio)


class ProteinBatch(NamedTuple):
    """A collated batch: `batch_dims` = [num_device, batch_size_per_device] (or any shape) over
    a flat list of structures, packed per leading index for the device calls."""
    batch_dims: Tuple[int, ...]
    samples: Tuple[ProteinStructureSample, ...]

    def shard(self, i: int) -> List[ProteinStructureSample]:
        per = int(np.prod(self.batch_dims[1:])) if len(self.batch_dims) > 1 else 1
        return list(self.samples[i * per:(i + 1) * per])


def batch_collate(batch_dims: List[int], batch_of_samples: List[ProteinStructureSample]) -> ProteinBatch:
    """Mirror of `inference_runner.py:77-83` (same count check as the reshape there)."""
    if int(np.prod(batch_dims)) != len(batch_of_samples):
        raise ValueError(f"cannot reshape {len(batch_of_samples)} samples into {list(batch_dims)}")
    samples = []
    for s in batch_of_samples:
        if isinstance(s, _graph.ProteinGraphView):
            s = s.sample
        if not isinstance(s, ProteinStructureSample):
            raise TypeError("batch_collate takes the structures make_graph_from_pdb returns "
                            f"(the GPU builds the graph from atom37 arrays), got {type(s).__name__}")
        samples.append(s)
    return ProteinBatch(tuple(int(b) for b in batch_dims), tuple(samples))


# ------------------------------------------------------------------------------------ params
def load_params(filename: str, tree_def: Optional[Sequence[Tuple[str, str]]] = None,
                codes_dim: Optional[int] = None) -> Dict[str, Dict[str, np.ndarray]]:
    """Mirror of `inference_runner.py:136-150`. `tree_def` is the ordered (module, param) leaf
    list; by default the full Vq3D tree (`params.full_param_spec`). Prefix not stripped."""
    return _params.load_params_npz(filename, tree_def, codes_dim=codes_dim, convert=False)


params_keys_conversion = _params.params_keys_conversion


class ReplicatedParams:
    """What `jax.device_put_replicated(params, devices)` returns in the reference: the same
    parameters for every local device. Device copies live in the libpst contexts TokenizeFn
    creates on first use."""

    def __init__(self, params: Dict[str, Dict[str, np.ndarray]], devices: Sequence[int]):
        self.params = params
        self.devices = list(devices)
        self.codes_dim = int(np.asarray(params["vq3_d/down_proj"]["b"]).shape[0])
        self.blob = _params.pack(params, self.codes_dim)


# -------------------------------------------------------------------------------- tokenize fn
def pad_token_value(levels: Sequence[int]) -> int:
    """Token id of a masked (padding) row: bounded = 0 → code 0 → Σ (L//2)·basis
    (`model/quantize.py:183-209`)."""
    basis = np.concatenate(([1], np.cumprod(levels[:-1])))
    return int(sum((l // 2) * b for l, b in zip(levels, basis)))


class TokenizeFn:
    """`jax.pmap(hk.transform(encode_and_quantize).apply)` for libpst.

    `fn(model_params, random_key, batched_graph)` runs shard i of `batched_graph` on
    `devices[i]` (one host thread per device; the C calls release the GIL) and returns a dict
    with "tokens" uint32 [*batch_dims, seq_max_size // df] (padding rows carry the padded-token
    id exactly as the reference's output does) and "n_tokens" int32 [*batch_dims]
    (= tokens_mask.sum(-1) of the reference graph); with `with_n_nodes` (set by AutoEncodeFn, off
    for the reference-shaped `prepare_tokenize_fn` output) also "n_nodes" int32 [*batch_dims] (the
    graph's n_node: residues with N, CA, C and O). `random_key` is accepted and unused, as in
    the reference's inference path (no stochastic op when is_training=False).
    """

    def __init__(self, cfg: TokenizerConfig, devices: Sequence[int], emit_aux: bool = False,
                 with_n_nodes: bool = False):
        self.cfg = cfg
        self.devices = list(devices)
        self.emit_aux = emit_aux
        self.with_n_nodes = with_n_nodes
        self._ctx: Dict[Tuple[int, int], _native.Tokenizer] = {}
        self._pool = _cf.ThreadPoolExecutor(max_workers=max(1, len(self.devices)))

    def _context(self, model_params: ReplicatedParams, dev: int) -> _native.Tokenizer:
        # the entry keeps the params object alive, so its id cannot be reused by other weights
        # while the context built from it is cached
        key = (id(model_params), dev)
        ent = self._ctx.get(key)
        if ent is None or ent[0] is not model_params:
            levels = self.cfg.levels
            if len(levels) != model_params.codes_dim:
                raise ValueError(f"params have codes_dimension {model_params.codes_dim}, config levels {levels}")
            t = _native.Tokenizer(dev, self.cfg.codebook_size, self.cfg.downsampling_ratio,
                                  model_params.blob, levels)
            ent = (model_params, t)
            self._ctx[key] = ent
        return ent[1]

    def tokenize_files(self, model_params: ReplicatedParams, files: Sequence[str], batch_dims: Sequence[int],
                       n_threads: int = 16) -> Dict[str, np.ndarray]:
        """The same outputs as `__call__` on the batch collated from `files` (shard i = files
        i·bs .. i·bs+bs-1 on devices[i]), with the parse on the GPU (pst_tokenize_pdb_files:
        the texts go to HBM, atom37 rows never return to the host). Raises the libpst error of a
        bad file (its message, not necessarily the reference's: InferenceRunner.tokenize then
        re-runs the batch through the reference-shaped path, which raises the reference's)."""
        n_dev, bs = batch_dims[0], int(np.prod(batch_dims[1:]))
        if n_dev > len(self.devices):
            raise ValueError(f"batch has {n_dev} device shards but only {len(self.devices)} devices")
        out_len = self.cfg.seq_max_size // self.cfg.downsampling_ratio
        pad = pad_token_value(self.cfg.levels)

        def run(i):
            t = self._context(model_params, self.devices[i])
            if not hasattr(t, "tokenize_pdb_files"):  # a stand-in context (CPU tests): the collated path
                raise _native.PstError("context without pst_tokenize_pdb_files")
            tok, nt, nn, off = t.tokenize_pdb_files(list(files[i * bs:(i + 1) * bs]), n_threads=n_threads)
            rows = np.full((bs, out_len), pad, np.uint32)
            for b in range(bs):
                rows[b, :nt[b]] = tok[off[b]:off[b] + nt[b]]
            return rows, nt, nn

        res = list(self._pool.map(run, range(n_dev)))
        return {"tokens": np.stack([r[0] for r in res]).reshape(*batch_dims, out_len),
                "n_tokens": np.stack([r[1] for r in res]).reshape(*batch_dims),
                "n_nodes": np.stack([np.asarray(r[2], np.int32) for r in res]).reshape(*batch_dims)}

    def __call__(self, model_params: ReplicatedParams, random_key: Any, batched_graph: ProteinBatch) -> Dict[str, np.ndarray]:
        n_dev = batched_graph.batch_dims[0]
        if n_dev > len(self.devices):
            raise ValueError(f"batch has {n_dev} device shards but only {len(self.devices)} devices")
        out_len = self.cfg.seq_max_size // self.cfg.downsampling_ratio
        pad = pad_token_value(self.cfg.levels)

        def run(i):
            shard = batched_graph.shard(i)
            t = self._context(model_params, self.devices[i])
            pos, flags, off = _native.pack_samples(shard)
            tok, nt, nn = t.tokenize_packed(pos, flags, off)
            rows = np.full((len(shard), out_len), pad, np.uint32)
            for b in range(len(shard)):
                rows[b, :nt[b]] = tok[off[b]:off[b] + nt[b]]
            aux = self._aux(t, shard, off, nt, out_len) if self.emit_aux else None
            return rows, nt, aux, nn

        res = list(self._pool.map(run, range(n_dev)))
        tokens = np.stack([r[0] for r in res]).reshape(*batched_graph.batch_dims, out_len)
        n_tokens = np.stack([r[1] for r in res]).reshape(*batched_graph.batch_dims)
        out = {"tokens": tokens, "n_tokens": n_tokens}
        if self.with_n_nodes:
            out["n_nodes"] = np.stack([np.asarray(r[3], np.int32) for r in res]).reshape(*batched_graph.batch_dims)
        if self.emit_aux:
            for key in res[0][2]:
                if key == "histogram":
                    continue
                out[key] = np.stack([r[2][key] for r in res]).reshape(*batched_graph.batch_dims,
                                                                      *res[0][2][key].shape[1:])
            # perplexity: mean of the per-device normalised histograms (jax.lax.pmean,
            # quantize.py:222-224), replicated per device like the reference's output
            p = np.mean([_normalised(r[2]["histogram"]) for r in res], axis=0)
            ppl = _perplexity(p)
            out["perplexity"] = np.full(n_dev, ppl, np.float32)
            out["straight_through_quantized"] = out["quantize"]
        return out

    def _aux(self, t, shard, off, nt, out_len):
        """Per-shard QuantizerOutput fields, padded to [bpd, out_len, ...] like the reference.
        Padding rows: quantize / continuous_embedding / distances = 0 (masked, quantize.py:184,
        236), soft_proba = softmax of the unmasked distances of a zero latent (:235),
        continuous_embedding_pre_proj = 0 (the reference's value there comes from masked queries
        and is not consumed)."""
        D, K = len(self.cfg.levels), t.codebook_size
        R = int(off[-1])
        a = t.aux(R)
        T = int(nt.sum())
        ca = t.codebook_aux(T)
        bpd = len(shard)
        o = {"quantize": np.zeros((bpd, out_len, D), np.float32),
             "continuous_embedding": np.zeros((bpd, out_len, D), np.float32),
             "continuous_embedding_pre_proj": np.zeros((bpd, out_len, 128), np.float32),
             "distances": np.zeros((bpd, out_len, K), np.float32),
             "soft_proba": np.broadcast_to(_padded_soft_proba(self.cfg.levels), (bpd, out_len, K)).copy()}
        r0 = 0
        for b in range(bpd):
            n = int(nt[b])
            src = slice(int(off[b]), int(off[b]) + n)
            o["quantize"][b, :n] = a["quantize"][src]
            o["continuous_embedding"][b, :n] = a["bounded"][src]
            o["continuous_embedding_pre_proj"][b, :n] = a["pre_proj"][src]
            o["distances"][b, :n] = ca["distances"][r0:r0 + n]
            o["soft_proba"][b, :n] = ca["soft_proba"][r0:r0 + n]
            r0 += n
        o["histogram"] = ca["histogram"].astype(np.float64)
        return o

    def close(self):
        for _, t in self._ctx.values():
            t.close()
        self._ctx.clear()
        self._pool.shutdown(wait=True)


def _padded_soft_proba(levels: Sequence[int]) -> np.ndarray:
    """softmax_k(sum_d c_kd^2): soft_proba of a masked row (its latent is 0)."""
    lv = np.asarray(levels)
    basis = np.concatenate(([1], np.cumprod(lv[:-1])))
    k = np.arange(int(np.prod(lv)))[:, None]
    c = (k // basis) % lv - lv // 2
    d = np.sum(c.astype(np.float32) ** 2, axis=-1)
    e = np.exp(d - d.max())
    return (e / e.sum()).astype(np.float32)


# ------------------------------------------------------------------------------------- runner
def hip_device_count() -> int:
    return _native.device_count()


class InferenceRunner:
    @staticmethod
    def prepare_devices(backend: str = "gpu"):
        """(`inference_runner.py:169-177`) → (local device ordinals, count)."""
        if backend != "gpu":
            raise NotImplementedError(
                f"backend {backend!r}: libpst runs the tokenize path on MI355X GPUs only (backend='gpu')")
        n = hip_device_count()
        if n < 1:
            raise RuntimeError("no HIP device visible")
        rank = int(os.environ.get("RANK", "0"))
        if rank == 0:
            print("---Devices---\n" + f"\tlocal device count: {n}")
        return list(range(n)), n

    @staticmethod
    def prepare_tokenize_fn(cfg: TokenizerConfig, devices: Sequence[int], emit_aux: bool = False) -> Callable:
        """`emit_aux=True` also returns the other QuantizerOutput fields (quantize,
        straight_through_quantized, continuous_embedding, continuous_embedding_pre_proj,
        distances, soft_proba, perplexity) shaped [n_dev, bpd, seq_max/df, ...] as the reference."""
        from .graph import set_graph_device
        set_graph_device(list(devices)[0])  # on-demand ProteinGraph builds run on this runner's GPU
        return TokenizeFn(cfg, devices, emit_aux)

    @staticmethod
    def prepare_decode_fn(cfg: TokenizerConfig, devices: Sequence[int]) -> Callable:
        return DecodeFn(cfg, devices)

    @staticmethod
    def prepare_ae_fn(cfg: TokenizerConfig, devices: Sequence[int]) -> Callable:
        """(`inference_runner.py:209-222`): the whole autoencoder pass, `AutoEncodeFn`."""
        from .graph import set_graph_device
        set_graph_device(list(devices)[0])
        return AutoEncodeFn(cfg, devices)

    @staticmethod
    def prepare_token_to_code_fn(cfg: TokenizerConfig, devices: Sequence[int]) -> Callable:
        return TokenToCodeFn(cfg)

    @staticmethod
    def decode_and_save_pdbs(random_key: Any, decode: Callable, indexes_to_codes_fn: Callable,
                             sequences: List[str], model_params: ReplicatedParams, num_device: int,
                             structure_save_path: str, batch_size_per_device: int, max_seq_len: int,
                             downsampling_ratio: int, pad_token_id: int):
        """(`inference_runner.py:326-437`): token files → `structures/structure_<stem>.pdb`,
        same batching, masks, dummy-ALA residues and PDB format."""
        from .structure_io import atom37_to_pdb
        structure_dir = os.path.join(structure_save_path, "structures")
        os.makedirs(structure_dir, exist_ok=False)
        effective_batch_size = batch_size_per_device * num_device
        num_iteration = len(sequences) // effective_batch_size + int((len(sequences) % effective_batch_size) > 0)
        sequences = list(islice(cycle(sequences), num_iteration * effective_batch_size))
        effective_length = max_seq_len // downsampling_ratio
        for it in range(num_iteration):
            start = it * effective_batch_size
            files = sequences[start:start + effective_batch_size]
            tokens_ids = load_and_build_batch(files, effective_length, pad_token_id)
            tokens_mask = build_tokens_mask_from_sequence(tokens_ids, pad_token_id)
            nodes_mask = build_nodes_mask_from_tokens_mask(tokens_mask, downsampling_ratio)
            number_of_nodes = nodes_mask.sum(axis=-1)
            out = decode(model_params, random_key,
                         tokens_ids.reshape(num_device, batch_size_per_device, effective_length),
                         tokens_mask.reshape(num_device, batch_size_per_device, effective_length))
            pos = out["final_atom_positions"].reshape(effective_batch_size, -1, 37, 3)
            mask = out["final_atom_mask"].reshape(effective_batch_size, -1, 37)
            for k, f in enumerate(files):
                n = int(number_of_nodes[k])
                name = os.path.basename(f).split("_tokens.npy")[0]
                with open(os.path.join(structure_dir, f"structure_{name}.pdb"), "w") as fh:
                    fh.write(atom37_to_pdb(pos[k, :n], mask[k, :n], np.zeros(n, np.int64)))

    @staticmethod
    def load_params(model_dir: str, local_devices: Sequence[int]) -> ReplicatedParams:
        """(`inference_runner.py:236-248`). Reads `model_dir/params.npz` only: the pickled
        treedef in `state_variables.npy` is never unpickled (the leaf order is
        `params.full_param_spec`, the order JAX flattens the Vq3D params dict in)."""
        path = os.path.join(model_dir, "params.npz")
        if not os.path.exists(path):
            raise FileNotFoundError(path)
        p = _params.load_params_npz(path)
        return ReplicatedParams(p, local_devices)

    @staticmethod
    def tokenize(random_key: Any, quantize: Callable, model_params: ReplicatedParams, pdbs: List[str],
                 token_save_path: str, num_device: int, data_config: TokenizerConfig,
                 batch_size_per_device: int = 8, logger: Optional[logging.Logger] = None):
        """(`inference_runner.py:250-324`): same batching (list cycled up to a multiple of
        num_device × batch_size_per_device), same output files: one
        `<pdb stem>_tokens.npy` per PDB, uint32 [1, n_tokens]. PDB parsing of the next batch
        overlaps the GPU work of the current one."""
        if logger is not None:
            logger.info(f"Starting tokenization of {pdbs}")
        os.makedirs(token_save_path, exist_ok=False)
        effective_batch_size = batch_size_per_device * num_device
        num_iteration = len(pdbs) // effective_batch_size + int((len(pdbs) % effective_batch_size) > 0)
        total = num_iteration * effective_batch_size
        pdbs = list(islice(cycle(pdbs), total))

        def load(it):
            files = pdbs[it * effective_batch_size:(it + 1) * effective_batch_size]
            for f in files:
                if not os.path.exists(f):
                    raise FileNotFoundError(f)
            parsed = _native.parse_pdb_files(files, n_threads=PARSE_THREADS)
            graphs = [make_graph_from_pdb(pdb_file_path=f, num_neighbor=data_config.graph_max_neighbor,
                                          downsampling_ratio=data_config.downsampling_ratio,
                                          residue_loc_is_alphac=data_config.residue_loc_is_alphac,
                                          padding_num_residue=data_config.seq_max_size,
                                          sample=parsed.sample(i)) for i, f in enumerate(files)]
            return files, batch_collate([num_device, batch_size_per_device], graphs)

        # libpst's tokenize fn reads, parses and tokenizes each batch with the parse on the GPU
        # (TokenizeFn.tokenize_files); a batch holding a file that fails there (a size gate, a parse
        # error, no residue with a full backbone) is re-run through the reference-shaped path below,
        # which raises the reference's exception for it
        gpu_parse = isinstance(quantize, TokenizeFn) and not quantize.emit_aux

        def gpu_batch(it):
            files = pdbs[it * effective_batch_size:(it + 1) * effective_batch_size]
            for f in files:
                if not os.path.exists(f):
                    raise FileNotFoundError(f)
            try:
                out = quantize.tokenize_files(model_params, files, [num_device, batch_size_per_device],
                                              n_threads=PARSE_THREADS)
            except (ValueError, NotImplementedError, _native.PstError):
                return files, None
            return (files, out) if bool(np.all(out["n_nodes"] > 0)) else (files, None)

        with _cf.ThreadPoolExecutor(max_workers=1) as io:
            nxt = io.submit(load, 0) if num_iteration and not gpu_parse else None
            for it in range(num_iteration):
                start_time = time.perf_counter()
                out = None
                if gpu_parse:
                    files, out = gpu_batch(it)
                if out is None:
                    files, batched = nxt.result() if nxt is not None else load(it)
                    nxt = None
                    if not gpu_parse and it + 1 < num_iteration:
                        nxt = io.submit(load, it + 1)
                    start_time = time.perf_counter()
                    out = quantize(model_params, random_key, batched)
                tokens = out["tokens"].reshape(effective_batch_size, -1)
                n_tok = out["n_tokens"].reshape(effective_batch_size)
                names, arrays = [], []
                for seq_id in range(effective_batch_size):
                    token_array = tokens[seq_id].reshape(1, -1)[:, :n_tok[seq_id]]
                    filename = os.path.basename(files[seq_id]).split(".pdb")[0]
                    names.append(os.path.join(token_save_path, filename + "_tokens"))
                    arrays.append(token_array)
                save_npy_files(names, arrays)  # = np.save per file (inference_runner.py:313-321)
                if logger is not None:
                    logger.info(f"Took {time.perf_counter() - start_time}s to tokenize")


# ------------------------------------------------------------------------------------- decode
def build_tokens_mask_from_sequence(tokens_ids: np.ndarray, pad_token_id: int) -> np.ndarray:
    """`inference_runner.py:86-95`: 1 before the first pad token, 0 from it on."""
    tokens_ids = np.asarray(tokens_ids)
    assert tokens_ids.ndim >= 2
    is_eos = tokens_ids == pad_token_id
    return np.where(np.cumsum(is_eos, axis=-1) == 0, 1, 0)


def build_nodes_mask_from_tokens_mask(tokens_mask: np.ndarray, downsampling_ratio: int) -> np.ndarray:
    """`inference_runner.py:98-111`."""
    batch, seq_len = tokens_mask.shape
    last_true_node = (downsampling_ratio * tokens_mask.sum(axis=-1)).reshape(batch, 1)
    index = np.repeat(np.arange(downsampling_ratio * seq_len)[None], batch, axis=0)
    return np.where(index < last_true_node, 1, 0)


def load_and_build_batch(files_paths: Sequence[str], max_seq_len: int, pad_token_id: int) -> np.ndarray:
    """`inference_runner.py:114-133`: token files → [B, max_seq_len] int32 padded with pad_token_id."""
    def pad(seq, n):
        return np.pad(seq, ((0, 0), (0, n - seq.shape[-1])), mode="constant", constant_values=pad_token_id)
    return np.concatenate([pad(np.load(f, allow_pickle=False).astype(np.int32).reshape(1, -1)[:, :max_seq_len],
                               max_seq_len) for f in files_paths])


class TokenToCodeFn:
    """`prepare_token_to_code_fn` (`inference_runner.py:224-233`): token ids → FSQ codes
    (renorm off: digit − L//2), [..., D] float32. Exact integer arithmetic on the host."""

    def __init__(self, cfg: TokenizerConfig):
        self.levels = np.asarray(cfg.levels)

    def __call__(self, model_params: Any, random_key: Any, tokens: np.ndarray) -> np.ndarray:
        basis = np.concatenate(([1], np.cumprod(self.levels[:-1])))
        t = np.asarray(tokens).astype(np.int64)[..., None]
        return ((t // basis) % self.levels - self.levels // 2).astype(np.float32)


class DecodeFn:
    """`prepare_decode_fn` (`inference_runner.py:193-207`) for libpst: per-device decoder
    contexts; `fn(model_params, random_key, tokens [n_dev, bpd, L], tokens_mask)` →
    {"final_atom_positions" [n_dev, bpd, df·L, 37, 3], "final_atom_mask", "n_nodes"}.
    Token ids (not codes) go to the GPU: indexes_to_codes runs inside the decoder."""

    def __init__(self, cfg: TokenizerConfig, devices: Sequence[int]):
        self.cfg = cfg
        self.devices = list(devices)
        self._ctx: Dict[Tuple[int, int], Any] = {}
        self._pool = _cf.ThreadPoolExecutor(max_workers=max(1, len(self.devices)))

    def _context(self, model_params: ReplicatedParams, dev: int):
        key = (id(model_params), dev)  # strong ref in the entry: see TokenizeFn._context
        ent = self._ctx.get(key)
        if ent is None or ent[0] is not model_params:
            blob = _params.pack_decoder(model_params.params, model_params.codes_dim)
            ent = (model_params, _native.Decoder(dev, self.cfg.codebook_size, self.cfg.downsampling_ratio,
                                                 blob, self.cfg.levels))
            self._ctx[key] = ent
        return ent[1]

    def __call__(self, model_params: ReplicatedParams, random_key: Any, tokens: np.ndarray,
                 tokens_mask: np.ndarray) -> Dict[str, np.ndarray]:
        tokens = np.asarray(tokens)
        n_dev, bpd, L = tokens.shape
        df = self.cfg.downsampling_ratio
        n_tok = np.asarray(tokens_mask).reshape(n_dev, bpd, -1).sum(-1).astype(np.int64)

        def run(i):
            dec = self._context(model_params, self.devices[i])
            return dec.decode([tokens[i, b, :n_tok[i, b]] for b in range(bpd)])

        res = list(self._pool.map(run, range(n_dev)))
        pos = np.zeros((n_dev, bpd, df * L, 37, 3), np.float32)
        mask = np.zeros((n_dev, bpd, df * L, 37), np.float32)
        for i in range(n_dev):
            for b in range(bpd):
                n = res[i][b].shape[0]
                pos[i, b, :n] = res[i][b]
                mask[i, b, :n, [0, 1, 2, 4]] = 1.0  # N, CA, C, O (model.py:547-556)
        return {"final_atom_positions": pos, "final_atom_mask": mask, "n_nodes": df * n_tok}

    def close(self):
        for _, d in self._ctx.values():
            d.close()
        self._ctx.clear()
        self._pool.shutdown(wait=True)


class AutoEncodeFn:
    """`prepare_ae_fn` (`inference_runner.py:209-222`): `Vq3D.__call__` (`model/model.py:194-259`)
    — encode, quantize, decode and structure module in one call — for libpst.

    `fn(model_params, random_key, batched_graph)` → `(decoded_structure, quantized_emb)`:
      * quantized_emb: every `QuantizerOutput` field `prepare_tokenize_fn(emit_aux=True)` returns
        (tokens, quantize, straight_through_quantized, continuous_embedding,
        continuous_embedding_pre_proj, distances, soft_proba, perplexity) plus
        `quantize_post_proj` [n_dev, bpd, seq_max/df, 128] = up_proj(quantize) (model.py:251;
        padding rows, whose quantize is 0, hold the up_proj bias exactly as the reference's);
      * decoded_structure: `final_atom_positions` [n_dev, bpd, seq_max, 37, 3] and
        `final_atom_mask` [n_dev, bpd, seq_max, 37] int32 (folding.py:501-513).
    The tokens are the tokenize path's (libpst encoder, bit-identical to `TokenizeFn`); the
    decoder is libpst's (`pst_decoder_decode_ex`) on the graph's own node count, because
    `__call__` decodes with the graph's `nodes_mask` (n_node residues) rather than df × the token
    count the token-file decode uses. `__call__` passes the protein's real features to the
    structure module, so atom37 positions come from `atom14_to_atom37` with the real `aatype`
    and are masked by its `atom37_gt_exists` (preprocessing.py:285-306,
    protein_structure_sample.py:93-118: the backbone N, CA, C, O of every kept residue): the four
    backbone atoms of standard residues, zero for UNK residues (the UNK row of
    RESTYPE_ATOM37_TO_ATOM14 / RESTYPE_ATOM37_MASK is all zero, all_atom.py:77-111), zero for
    every other atom. The structure module's internal `representations` (unused by the
    reference, folding.py:488-489) are not returned.
    """

    BACKBONE37 = (0, 1, 2, 4)  # N, CA, C, O

    def __init__(self, cfg: TokenizerConfig, devices: Sequence[int]):
        self.cfg = cfg
        self.devices = list(devices)
        self.tokenize = TokenizeFn(cfg, devices, emit_aux=True, with_n_nodes=True)
        self.decode = DecodeFn(cfg, devices)

    def __call__(self, model_params: ReplicatedParams, random_key: Any, batched_graph: ProteinBatch):
        q = self.tokenize(model_params, random_key, batched_graph)
        dims = batched_graph.batch_dims
        n_dev = dims[0]
        flat_tok = q["tokens"].reshape(n_dev, -1, q["tokens"].shape[-1])
        flat_nt = q["n_tokens"].reshape(n_dev, -1)
        flat_nn = q["n_nodes"].reshape(n_dev, -1)
        bpd = flat_tok.shape[1]
        L = self.cfg.seq_max_size
        out_len = flat_tok.shape[-1]

        def run(i):
            dec = self.decode._context(model_params, self.devices[i])
            return dec.decode([flat_tok[i, b, :flat_nt[i, b]] for b in range(bpd)],
                              n_nodes=[int(n) for n in flat_nn[i]], with_up_proj=True)

        res = list(self.decode._pool.map(run, range(n_dev)))
        up_b = np.asarray(model_params.params["vq3_d/up_proj"]["b"], np.float32)
        pos = np.zeros((n_dev, bpd, L, 37, 3), np.float32)
        mask = np.zeros((n_dev, bpd, L, 37), np.int32)
        post = np.broadcast_to(up_b, (n_dev, bpd, out_len, up_b.shape[0])).copy()
        bb = list(self.BACKBONE37)
        for i in range(n_dev):
            atoms, ups = res[i]
            for b in range(bpd):
                s = batched_graph.samples[i * bpd + b]
                kept = ~s.get_missing_backbone_coords_mask()
                aa = np.argmax(np.asarray(s.aatype)[kept], axis=-1)
                n = atoms[b].shape[0]
                std = (aa[:n] < 20).astype(np.float32)  # restype_num: UNK rows map to zero
                pos[i, b, :n, bb] = atoms[b][:, bb].transpose(1, 0, 2) * std[None, :, None]
                mask[i, b, :n, bb] = 1
                post[i, b, :ups[b].shape[0]] = ups[b]
        structure = {"final_atom_positions": pos.reshape(*dims, L, 37, 3),
                     "final_atom_mask": mask.reshape(*dims, L, 37)}
        quantized_emb = {k: v for k, v in q.items() if k not in ("n_nodes",)}
        quantized_emb["quantize_post_proj"] = post.reshape(*dims, out_len, up_b.shape[0])
        return structure, quantized_emb

    def close(self):
        self.tokenize.close()
        self.decode.close()


def _normalised(histogram: np.ndarray) -> np.ndarray:
    h = np.asarray(histogram, np.float64)
    return h / max(h.sum(), 1.0)


def _perplexity(p: np.ndarray) -> float:
    """exp(-Σ p log(p + 1e-10)) of the mean normalised code histogram (quantize.py:222-224)."""
    return float(np.exp(-np.sum(p * np.log(p + 1e-10))))


def global_perplexity(histogram: np.ndarray, group=None) -> float:
    """Codebook perplexity over all ranks of a torchrun job: the reference's pmean of per-device
    normalised histograms (quantize.py:222-224) as ONE all-reduce of K float64 (RCCL over xGMI
    with the nccl backend, gloo on CPU). The only collective of the tokenize path, off the
    token data path. Without an initialised process group it is the local perplexity."""
    p = _normalised(histogram)
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        import torch
        t = torch.from_numpy(p)
        if dist.get_backend(group) == "nccl":
            t = t.cuda()
        dist.all_reduce(t, group=group)
        p = t.cpu().numpy() / dist.get_world_size(group)
    return _perplexity(p)


def lpt_partition(weights: Sequence[float], world_size: int) -> List[List[int]]:
    """Longest-processing-time-first assignment: items by weight, heaviest first
    (ties by index), each to the currently least-loaded rank (ties to the lowest rank). Returns
    per-rank index lists in input order. Deterministic, so every rank computes the same split."""
    if world_size < 1:
        raise ValueError(f"world size {world_size} < 1")
    load = [0.0] * world_size
    parts: List[List[int]] = [[] for _ in range(world_size)]
    for i in sorted(range(len(weights)), key=lambda k: (-float(weights[k]), k)):
        r = min(range(world_size), key=lambda q: (load[q], q))
        parts[r].append(i)
        load[r] += float(weights[i])
    return [sorted(p) for p in parts]


def shard_for_rank(items: Sequence[Any], rank: int, world_size: int,
                   weights: Optional[Sequence[float]] = None) -> List[Any]:
    """Partition of independent proteins across ranks (one process per GPU, no data-path
    collective). With `weights` (residue counts, or PDB file sizes as their proxy) the split is
    LPT-greedy on them (`lpt_partition`), balancing residues per GPU; without, round-robin:
    rank r takes items r, r+W, r+2W, ..."""
    if not 0 <= rank < world_size:
        raise ValueError(f"rank {rank} outside world of {world_size}")
    if weights is None:
        return list(items[rank::world_size])
    if len(weights) != len(items):
        raise ValueError(f"{len(weights)} weights for {len(items)} items")
    return [items[i] for i in lpt_partition(weights, world_size)[rank]]
