"""ctypes binding of libpst.so (the C ABI in include/pst.h).

The library is built in-tree (`protein-structure-tokenizer_amd/pst_amd/_lib/libpst.so`,
`make -C protein-structure-tokenizer_amd/csrc`). There is no CPU fallback: if the library or a
HIP device is missing, loading raises.
"""
import ctypes
import os
import sys
from typing import List, NamedTuple, Optional, Sequence, Tuple

import numpy as np

from . import params as _params
from .config import LEVELS

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("PST_LIB", os.path.join(_HERE, "_lib", "libpst.so"))

PST_OK, PST_E_INVALID, PST_E_TOO_LARGE, PST_E_TOO_SMALL, PST_E_HIP, PST_E_NOMEM = 0, -1, -2, -3, -4, -5
ABI_VERSION = 1


class PstError(RuntimeError):
    pass


class _ModelDesc(ctypes.Structure):
    _fields_ = [("abi_version", ctypes.c_int32), ("codebook_size", ctypes.c_int32),
                ("downsampling_ratio", ctypes.c_int32), ("n_levels", ctypes.c_int32),
                ("levels", ctypes.c_int32 * 8), ("seq_max_size", ctypes.c_int32),
                ("graph_max_neighbor", ctypes.c_int32)]


_lib = None
EXPORTS = ("pst_param_count", "pst_create", "pst_destroy", "pst_last_error", "pst_create_error",
           "pst_tokenize", "pst_tokenize_f32", "pst_tokenize_device", "pst_aux", "pst_codebook_aux", "pst_sync",
           "pst_stream", "pst_debug_fetch", "pst_set_timing", "pst_get_timing", "pst_device_count",
           "pst_codebook_aux_device", "pst_pdb_parse_files", "pst_pdb_parse_strings",
           "pst_pdb_batch_sizes", "pst_pdb_batch_copy", "pst_pdb_batch_error", "pst_pdb_batch_free", "pst_write_files",
           "pst_decoder_param_count", "pst_decoder_create", "pst_decoder_destroy", "pst_decoder_last_error",
           "pst_decoder_create_error", "pst_decoder_decode", "pst_decoder_decode_ex", "pst_decoder_debug",
           "pst_build_graph", "pst_clock_counters", "pst_set_clock_counters", "pst_pdb_batch_copy_f32",
           "pst_decoder_set_timing", "pst_decoder_get_timing", "pst_tokenize_pdb_batch",
           "pst_tokenize_pdb_files", "pst_pdb_files_host_parsed")
STAGES = ("prep", "knn", "mpnn0", "mpnn1", "mpnn2", "down")


def _init_torch_hip_first():
    """PyTorch-ROCm wheels bundle their own HIP/HSA runtime (libamdhip64.so) next to the system
    one libpst links (libamdhip64.so.7). Both can serve one process only if torch's runtime
    opens the GPU first, so when torch is already imported, initialise it before libpst."""
    torch = sys.modules.get("torch")
    if torch is not None:
        try:
            if torch.cuda.is_available():
                torch.cuda.init()
        except Exception:
            pass


def lib():
    """Load libpst.so (raises if it was not built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise PstError(f"libpst.so not found at {LIB_PATH}: build it with "
                           "`make -C protein-structure-tokenizer_amd/csrc` (no CPU fallback exists)")
        _init_torch_hip_first()
        L = ctypes.CDLL(LIB_PATH)
        P = ctypes.c_void_p
        L.pst_param_count.restype = ctypes.c_size_t
        L.pst_param_count.argtypes = [ctypes.c_int32]
        L.pst_create.argtypes = [ctypes.c_int32, ctypes.POINTER(_ModelDesc), P, ctypes.c_size_t, ctypes.POINTER(P)]
        L.pst_destroy.argtypes = [P]
        L.pst_last_error.restype = ctypes.c_char_p
        L.pst_last_error.argtypes = [P]
        L.pst_create_error.restype = ctypes.c_char_p
        L.pst_tokenize.argtypes = [P, P, P, P, ctypes.c_int32, P, P, P]
        L.pst_tokenize_f32.argtypes = [P, P, P, P, ctypes.c_int32, P, P, P]
        L.pst_tokenize_device.argtypes = [P, P, P, P, ctypes.c_int32, P, P, P]
        L.pst_aux.argtypes = [P, P, P, P]
        L.pst_build_graph.argtypes = [P, P, P, P, ctypes.c_int32, P, P, P, P]
        L.pst_codebook_aux.argtypes = [P, P, P, P, P, P, ctypes.c_int64]
        L.pst_codebook_aux_device.argtypes = [P, P, P, P, P, ctypes.c_int64]
        L.pst_sync.argtypes = [P]
        L.pst_stream.restype = P
        L.pst_stream.argtypes = [P]
        L.pst_debug_fetch.argtypes = [P, ctypes.c_int32, P, ctypes.c_size_t]
        L.pst_set_timing.argtypes = [P, ctypes.c_int32]
        L.pst_get_timing.argtypes = [P, P]
        L.pst_device_count.argtypes = [P]
        L.pst_clock_counters.argtypes = [P, P, ctypes.c_int32]
        # entry points added in round 5: absent from older libraries loaded for A/B runs (PST_LIB);
        # tests/test_abi.py requires every EXPORTS symbol of the in-tree build
        for name, at in (("pst_set_clock_counters", [P, ctypes.c_int32]),
                         ("pst_decoder_set_timing", [P, ctypes.c_int32]), ("pst_decoder_get_timing", [P, P]),
                         ("pst_tokenize_pdb_batch", [P, P, P, P, P]),
                         ("pst_tokenize_pdb_files", [P, P, ctypes.c_int32, ctypes.c_int32, P, ctypes.c_int64, P, P, P]),
                         ("pst_pdb_files_host_parsed", [P])):
            if hasattr(L, name):
                getattr(L, name).argtypes = at
        L.pst_pdb_parse_files.argtypes = [P, ctypes.c_int32, ctypes.c_char, ctypes.c_int32, ctypes.POINTER(P)]
        L.pst_pdb_parse_strings.argtypes = [P, P, ctypes.c_int32, ctypes.c_char, ctypes.c_int32, ctypes.POINTER(P)]
        L.pst_pdb_batch_sizes.argtypes = [P, P, P]
        L.pst_pdb_batch_copy.argtypes = [P, P, P, P, P, P]
        L.pst_pdb_batch_copy_f32.argtypes = [P, P, P, P, P, P]
        L.pst_pdb_batch_error.restype = ctypes.c_char_p
        L.pst_pdb_batch_error.argtypes = [P, ctypes.c_int32]
        L.pst_pdb_batch_free.argtypes = [P]
        L.pst_write_files.argtypes = [ctypes.c_int32, P, P, P, ctypes.c_int32]
        L.pst_decoder_param_count.restype = ctypes.c_size_t
        L.pst_decoder_param_count.argtypes = [ctypes.c_int32]
        L.pst_decoder_create.argtypes = [ctypes.c_int32, ctypes.POINTER(_ModelDesc), P, ctypes.c_size_t, ctypes.POINTER(P)]
        L.pst_decoder_destroy.argtypes = [P]
        L.pst_decoder_last_error.restype = ctypes.c_char_p
        L.pst_decoder_last_error.argtypes = [P]
        L.pst_decoder_create_error.restype = ctypes.c_char_p
        L.pst_decoder_decode.argtypes = [P, P, P, ctypes.c_int32, P, P]
        L.pst_decoder_decode_ex.argtypes = [P, P, P, ctypes.c_int32, P, P, P, P]
        L.pst_decoder_debug.argtypes = [P, ctypes.c_int32, P, ctypes.c_size_t]
        _lib = L
    return _lib


def device_count() -> int:
    """Visible HIP devices (pst_device_count)."""
    n = ctypes.c_int32(0)
    lib().pst_device_count(ctypes.byref(n))
    return int(n.value)


def _ptr(a: Optional[np.ndarray]):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def raise_for(code: int, msg: str):
    """Map C ABI codes onto the reference's exception types (inference_runner.py:52-62)."""
    if code == PST_OK:
        return
    if code in (PST_E_TOO_LARGE, PST_E_TOO_SMALL):
        raise NotImplementedError(msg)
    if code == PST_E_INVALID:
        raise ValueError(msg)
    raise PstError(f"libpst error {code}: {msg}")


class PdbBatch(NamedTuple):
    """Packed result of the native parser (pst_pdb_parse_*): ragged atom37 arrays in input order."""
    positions: np.ndarray  # [R,37,3] f64
    flags: np.ndarray      # [R,37] u8
    aatype: np.ndarray     # [R] u8
    offsets: np.ndarray    # [n+1] i64
    status: np.ndarray     # [n] i32 (0 ok)
    errors: List[str]

    def sample(self, i: int):
        """Input i as a ProteinStructureSample (raises ValueError with the parser's message)."""
        from .sample import ProteinStructureSample
        if self.status[i] != PST_OK:
            raise ValueError(self.errors[i])
        a, b = int(self.offsets[i]), int(self.offsets[i + 1])
        n = b - a
        onehot = np.zeros((n, 21))
        onehot[np.arange(n), self.aatype[a:b]] = 1.0
        fl = self.flags[a:b]
        return ProteinStructureSample(None, n, onehot, self.positions[a:b], (fl & 1).astype(bool),
                                      ((fl >> 1) & 1).astype(bool), 0.0, 1)


def _collect_pdb(h, f32: bool = False) -> PdbBatch:
    L = lib()
    try:
        n = ctypes.c_int32()
        r = ctypes.c_int64()
        L.pst_pdb_batch_sizes(h, ctypes.byref(n), ctypes.byref(r))
        n, r = n.value, r.value
        # every element is written by pst_pdb_batch_copy(_f32) (absent atoms as 0.0)
        pos = np.empty((r, 37, 3), np.float32 if f32 else np.float64)
        fl = np.empty((r, 37), np.uint8)
        aa = np.empty(r, np.uint8)
        off = np.zeros(n + 1, np.int64)
        st = np.zeros(n, np.int32)
        copy = L.pst_pdb_batch_copy_f32 if f32 else L.pst_pdb_batch_copy
        copy(h, _ptr(pos), _ptr(fl), _ptr(aa), _ptr(off), _ptr(st))
        errs = [L.pst_pdb_batch_error(h, i).decode() for i in range(n)]
    finally:
        L.pst_pdb_batch_free(h)
    return PdbBatch(pos, fl, aa, off, st, errs)


class PdbHandle:
    """A parsed batch kept inside libpst (pst_pdb_parse_files) for Tokenizer.tokenize_pdb_batch:
    the atom37 arrays go to the GPU without a copy through Python. Free with close()."""

    def __init__(self, h):
        self._h = h
        n = ctypes.c_int32()
        r = ctypes.c_int64()
        lib().pst_pdb_batch_sizes(h, ctypes.byref(n), ctypes.byref(r))
        self.n, self.n_residues = n.value, r.value

    def offsets(self) -> np.ndarray:
        off = np.zeros(self.n + 1, np.int64)
        lib().pst_pdb_batch_copy_f32(self._h, None, None, None, _ptr(off), None)
        return off

    def close(self):
        if self._h:
            lib().pst_pdb_batch_free(self._h)
            self._h = None

    def __del__(self):
        self.close()


def parse_pdb_files_handle(paths: Sequence[str], chain_id: Optional[str] = None, n_threads: int = 8) -> PdbHandle:
    """parse_pdb_files without copying the result out (see PdbHandle)."""
    enc = [os.fsencode(p) for p in paths]
    arr = (ctypes.c_char_p * max(len(enc), 1))(*enc)
    h = ctypes.c_void_p()
    rc = lib().pst_pdb_parse_files(arr, len(enc), (chain_id or "\0").encode()[:1], n_threads, ctypes.byref(h))
    if rc != PST_OK:
        raise PstError(f"pst_pdb_parse_files failed: {rc}")
    return PdbHandle(h)


def parse_pdb_files(paths: Sequence[str], chain_id: Optional[str] = None, n_threads: int = 8,
                    float32: bool = False) -> PdbBatch:
    """Parse PDB files on n_threads host threads with the native parser (pst_pdb_parse_files).
    `float32`: positions as float32 (exact; pst_pdb_batch_copy_f32), the input pst_tokenize_f32 takes."""
    enc = [os.fsencode(p) for p in paths]
    arr = (ctypes.c_char_p * max(len(enc), 1))(*enc)
    h = ctypes.c_void_p()
    rc = lib().pst_pdb_parse_files(arr, len(enc), (chain_id or "\0").encode()[:1], n_threads, ctypes.byref(h))
    if rc != PST_OK:
        raise PstError(f"pst_pdb_parse_files failed: {rc}")
    return _collect_pdb(h, float32)


def parse_pdb_strings(texts: Sequence[str], chain_id: Optional[str] = None, n_threads: int = 8) -> PdbBatch:
    enc = [t.encode() for t in texts]
    arr = (ctypes.c_char_p * max(len(enc), 1))(*enc)
    lens = (ctypes.c_size_t * max(len(enc), 1))(*[len(e) for e in enc])
    h = ctypes.c_void_p()
    rc = lib().pst_pdb_parse_strings(arr, lens, len(enc), (chain_id or "\0").encode()[:1], n_threads, ctypes.byref(h))
    if rc != PST_OK:
        raise PstError(f"pst_pdb_parse_strings failed: {rc}")
    return _collect_pdb(h)


def write_files(paths: Sequence[str], blobs: Sequence[bytes], n_threads: int = 8) -> None:
    """Write whole files from byte strings on libpst's host thread pool (pst_write_files)."""
    n = len(paths)
    if n == 0:
        return
    enc = [os.fsencode(p) for p in paths]
    parr = (ctypes.c_char_p * n)(*enc)
    darr = (ctypes.c_char_p * n)(*blobs)
    larr = (ctypes.c_size_t * n)(*[len(b) for b in blobs])
    rc = lib().pst_write_files(n, parr, darr, larr, n_threads)
    if rc != PST_OK:
        raise OSError(f"pst_write_files failed for one of {n} files (first: {paths[0]})")


def pack_samples(samples) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    """List of ProteinStructureSample → (positions f64 [R,37,3], flags u8 [R,37], offsets i64 [B+1])."""
    n = [s.nb_residues for s in samples]
    off = np.zeros(len(samples) + 1, np.int64)
    off[1:] = np.cumsum(n)
    pos = np.ascontiguousarray(np.concatenate([s.atom37_positions for s in samples]), dtype=np.float64)
    flags = np.ascontiguousarray(np.concatenate([s.atom_flags() for s in samples]), dtype=np.uint8)
    return pos, flags, off


class Tokenizer:
    """One libpst context (one GPU): encoder-half weights resident in HBM."""

    def __init__(self, device: int = 0, codebook_size: int = 4096, downsampling_ratio: int = 1,
                 params_blob: Optional[np.ndarray] = None, levels: Optional[Sequence[int]] = None):
        L = lib()
        self.levels = tuple(levels or LEVELS[codebook_size])
        self.D = len(self.levels)
        self.df = downsampling_ratio
        self.codebook_size = int(np.prod(self.levels))
        if params_blob is None:
            params_blob = _params.random_blob(self.D, 0)
        self.blob = np.ascontiguousarray(params_blob, dtype=np.float32)
        n = L.pst_param_count(self.D)
        if self.blob.size != n:
            raise ValueError(f"parameter blob has {self.blob.size} floats, expected {n}")
        desc = _ModelDesc(ABI_VERSION, self.codebook_size, downsampling_ratio, self.D,
                          (ctypes.c_int32 * 8)(*(list(self.levels) + [0] * (8 - self.D))), 512, 50)
        h = ctypes.c_void_p()
        rc = L.pst_create(device, ctypes.byref(desc), _ptr(self.blob), self.blob.size, ctypes.byref(h))
        if rc != PST_OK:
            raise_for(rc, L.pst_create_error().decode())
        self._h = h
        self.device = device
        self._pdb_tok = np.empty(1 << 16, np.uint32)  # tokenize_pdb_files' token buffer (grown on demand)

    def close(self):
        if getattr(self, "_h", None):
            lib().pst_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc):
        if rc != PST_OK:
            raise_for(rc, lib().pst_last_error(self._h).decode())

    @property
    def stream(self) -> int:
        return lib().pst_stream(self._h)

    def tokenize_packed(self, pos, flags, offsets):
        """Ragged batch → (tokens [R] uint32 in raw-offset layout, n_tokens [B], n_nodes [B]).
        float32 positions go through pst_tokenize_f32 (half the H2D bytes, same results for the
        PDB path's float32 coordinates); anything else is passed as float64 (pst_tokenize)."""
        f32 = isinstance(pos, np.ndarray) and pos.dtype == np.float32
        pos = np.ascontiguousarray(pos, np.float32 if f32 else np.float64)
        flags = np.ascontiguousarray(flags, np.uint8)
        offsets = np.ascontiguousarray(offsets, np.int64)
        B = len(offsets) - 1
        R = int(offsets[-1])
        # every element is written by the call's device-to-host copies (rows past a protein's
        # n_tokens hold unspecified values, as the reference's padded outputs do)
        tok = np.empty(max(R, 1), np.uint32)
        nt = np.empty(B, np.int32)
        nn = np.empty(B, np.int32)
        fn = lib().pst_tokenize_f32 if f32 else lib().pst_tokenize
        self._check(fn(self._h, _ptr(pos), _ptr(flags), _ptr(offsets), B, _ptr(tok), _ptr(nt), _ptr(nn)))
        return tok, nt, nn

    def tokenize_pdb_batch(self, batch: "PdbHandle"):
        """A parsed batch (parse_pdb_files_handle) → (tokens [R] uint32 raw-offset layout,
        n_tokens [n], n_nodes [n]) through pst_tokenize_pdb_batch (page-locked staging inside libpst)."""
        tok = np.empty(max(batch.n_residues, 1), np.uint32)
        nt = np.empty(batch.n, np.int32)
        nn = np.empty(batch.n, np.int32)
        self._check(lib().pst_tokenize_pdb_batch(self._h, batch._h, _ptr(tok), _ptr(nt), _ptr(nn)))
        return tok, nt, nn

    def tokenize_pdb_files(self, paths: Sequence[str], n_threads: int = 16):
        """PDB files → (tokens [R] uint32 raw-offset layout, n_tokens [n], n_nodes [n], offsets
        [n+1]) through pst_tokenize_pdb_files: the texts parsed on the GPU straight into the
        tokenizer's inputs (files outside the GPU fast path through the native host parser)."""
        # the paths as one NUL-separated blob and a pointer array into it (a ctypes c_char_p array
        # costs ~1 us per path); the token buffer is the context's, grown when the call reports a
        # larger R (offsets[n]), so no file is stat'ed here
        n = len(paths)
        enc = [os.fsencode(p) + b"\0" for p in paths]
        blob = np.frombuffer(b"".join(enc), np.uint8)
        starts = np.zeros(max(n, 1), np.uint64)
        if n:
            starts[1:n] = np.cumsum([len(e) for e in enc[:-1]], dtype=np.uint64)
        ptrs = starts + np.uint64(blob.ctypes.data)
        nt = np.empty(n, np.int32)
        nn = np.empty(n, np.int32)
        off = np.zeros(n + 1, np.int64)
        for _ in range(2):
            tok = self._pdb_tok
            rc = lib().pst_tokenize_pdb_files(self._h, _ptr(ptrs), n, n_threads, _ptr(tok), tok.size, _ptr(nt), _ptr(nn),
                                              _ptr(off))
            if rc == PST_E_INVALID and n and int(off[-1]) > tok.size:
                self._pdb_tok = np.empty(int(off[-1]) * 2, np.uint32)
                continue
            self._check(rc)
            break
        return tok[:int(off[-1])].copy(), nt, nn, off

    def pdb_files_host_parsed(self) -> int:
        """Files of the last tokenize_pdb_files call that took the host parser."""
        L = lib()
        L.pst_pdb_files_host_parsed.restype = ctypes.c_int32
        return int(L.pst_pdb_files_host_parsed(self._h))

    def tokenize(self, samples) -> List[np.ndarray]:
        pos, flags, off = pack_samples(samples)
        tok, nt, _ = self.tokenize_packed(pos, flags, off)
        return [tok[off[b]:off[b] + nt[b]].copy() for b in range(len(samples))]

    def tokenize_device(self, d_pos: int, d_flags: int, offsets: np.ndarray, d_tokens: int, d_ntok: int, d_nnodes: int):
        """Device pointers (ints, e.g. torch tensor.data_ptr()); asynchronous on self.stream."""
        offsets = np.ascontiguousarray(offsets, np.int64)
        self._check(lib().pst_tokenize_device(self._h, ctypes.c_void_p(d_pos), ctypes.c_void_p(d_flags), _ptr(offsets),
                                              len(offsets) - 1, ctypes.c_void_p(d_tokens), ctypes.c_void_p(d_ntok),
                                              ctypes.c_void_p(d_nnodes)))

    def set_timing(self, on: bool = True):
        self._check(lib().pst_set_timing(self._h, 1 if on else 0))

    def stage_ms(self):
        """Per-stage device time (ms) of the last call, from HIP events on self.stream."""
        ms = np.zeros(len(STAGES), np.float32)
        self._check(lib().pst_get_timing(self._h, _ptr(ms)))
        return dict(zip(STAGES, ms.tolist()))

    def sync(self):
        self._check(lib().pst_sync(self._h))

    def set_clock_counters(self, on: bool = True):
        """Stamp the fused MPNN launches into the clock counters (off by default: measurement only).
        Libraries from before round 5 (A/B runs) always stamp and lack the switch."""
        if hasattr(lib(), "pst_set_clock_counters"):
            self._check(lib().pst_set_clock_counters(self._h, 1 if on else 0))

    def clock_counters(self, reset: bool = False) -> np.ndarray:
        """Per fused MPNN layer since the last reset, uint64 [3, 8] (pst_clock_counters): shader
        cycles and 100 MHz ticks of the stamping wave (clock = c[l, 0] / c[l, 1] x 0.1 GHz), Σ wave
        lifetimes, earliest start, latest end, waves."""
        out = np.zeros((3, 8), np.uint64)
        self._check(lib().pst_clock_counters(self._h, _ptr(out), 1 if reset else 0))
        return out

    def build_graph_packed(self, pos, flags, offsets):
        """Residue graphs of a packed batch (pst_build_graph): senders [R,50] int32 (node index
        within the protein, -1 = none), edge features [R,50,27] f32, C-alpha [R,3] f64, n_nodes [B]."""
        pos = np.ascontiguousarray(pos, np.float64)
        flags = np.ascontiguousarray(flags, np.uint8)
        offsets = np.ascontiguousarray(offsets, np.int64)
        B = len(offsets) - 1
        R = int(offsets[-1])
        snd = np.zeros((max(R, 1), 50), np.int32)
        feat = np.zeros((max(R, 1), 50, 27), np.float32)
        ca = np.zeros((max(R, 1), 3), np.float64)
        nn = np.zeros(B, np.int32)
        self._check(lib().pst_build_graph(self._h, _ptr(pos), _ptr(flags), _ptr(offsets), B, _ptr(snd), _ptr(feat),
                                          _ptr(ca), _ptr(nn)))
        return snd, feat, ca, nn

    def aux(self, R: int):
        b = np.zeros((R, self.D), np.float32)
        q = np.zeros((R, self.D), np.float32)
        pp = np.zeros((R, 128), np.float32)
        self._check(lib().pst_aux(self._h, _ptr(b), _ptr(q), _ptr(pp)))
        return dict(bounded=b, quantize=q, pre_proj=pp)

    def codebook_aux(self, n_rows: int, distances: bool = True, soft_proba: bool = True):
        """FSQ aux of the last call (pst_codebook_aux): rows compact over real tokens."""
        K = self.codebook_size
        dist = np.zeros((n_rows, K), np.float32) if distances else None
        prob = np.zeros((n_rows, K), np.float32) if soft_proba else None
        arg = np.zeros(n_rows, np.uint32)
        hist = np.zeros(K, np.uint32)
        ppl = np.zeros(1, np.float32)
        self._check(lib().pst_codebook_aux(self._h, _ptr(dist), _ptr(prob), _ptr(arg), _ptr(hist), _ptr(ppl), n_rows))
        return dict(distances=dist, soft_proba=prob, argmin=arg, histogram=hist, perplexity=float(ppl[0]))

    def codebook_aux_device(self, d_dist: int, d_prob: int, d_argmin: int, d_hist: int, row_capacity: int):
        self._check(lib().pst_codebook_aux_device(self._h, ctypes.c_void_p(d_dist or None), ctypes.c_void_p(d_prob or None),
                                                  ctypes.c_void_p(d_argmin or None), ctypes.c_void_p(d_hist or None),
                                                  row_capacity))

    def debug_fetch(self, which: int, R: int):
        if which in (1, 2, 3):
            out = np.zeros((R, 128), np.float32)
        elif which == 10:
            out = np.zeros((R * 50, 32), np.float32)
        elif which == 11:
            out = np.zeros(R * 50, np.int32)
        elif which == 12:
            out = np.zeros(R, np.int32)
        elif which == 13:
            out = np.zeros((R, 37, 3), np.float32)
        elif which == 14:
            out = np.zeros((R, 37), np.uint8)
        else:
            raise ValueError(which)
        self._check(lib().pst_debug_fetch(self._h, which, _ptr(out), out.nbytes))
        return out

    def last_plan(self) -> Tuple[int, int]:
        """(copy ranges of the first chunk — 0 when it was one copy outside the range branch —, pipeline
        chunks) of the last host-buffer tokenize call."""
        p = self.last_plan_detail()
        return p["ranges"], p["chunks"]

    def last_plan_detail(self) -> dict:
        """The last host-buffer tokenize call's plan: copy ranges, chunks, the chunks' protein cuts
        and each chunk's layer schedule ("fused", "fused_half" = two waves per task, "split",
        "fused_queue" = the persistent half-task queue)."""
        out = np.zeros(20, np.int32)
        self._check(lib().pst_debug_fetch(self._h, 20, _ptr(out), out.nbytes))
        C = int(out[1])
        names = {0: "fused", 1: "fused_half", 2: "split", 3: "fused_queue"}
        return {"ranges": int(out[0]), "chunks": C, "cuts": [int(x) for x in out[2:3 + C]],
                "schedules": [names[int(x)] for x in out[11:11 + C]],
                "downsampler": {0: "one_wave", 1: "coop", 2: "pair"}[int(out[19])]}


class Decoder:
    """One libpst decoder context (one GPU): token ids → backbone atom37 coordinates."""

    def __init__(self, device: int = 0, codebook_size: int = 4096, downsampling_ratio: int = 1,
                 params_blob: Optional[np.ndarray] = None, levels: Optional[Sequence[int]] = None):
        L = lib()
        self.levels = tuple(levels or LEVELS[codebook_size])
        self.D = len(self.levels)
        self.df = downsampling_ratio
        self.codebook_size = int(np.prod(self.levels))
        if params_blob is None:
            params_blob = _params.pack_decoder(_params.random_full_params(self.D, 0), self.D)
        self.blob = np.ascontiguousarray(params_blob, dtype=np.float32)
        n = L.pst_decoder_param_count(self.D)
        if self.blob.size != n:
            raise ValueError(f"decoder blob has {self.blob.size} floats, expected {n}")
        desc = _ModelDesc(ABI_VERSION, self.codebook_size, downsampling_ratio, self.D,
                          (ctypes.c_int32 * 8)(*(list(self.levels) + [0] * (8 - self.D))), 512, 50)
        h = ctypes.c_void_p()
        rc = L.pst_decoder_create(device, ctypes.byref(desc), _ptr(self.blob), self.blob.size, ctypes.byref(h))
        if rc != PST_OK:
            raise_for(rc, L.pst_decoder_create_error().decode())
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            lib().pst_decoder_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc):
        if rc != PST_OK:
            raise_for(rc, lib().pst_decoder_last_error(self._h).decode())

    def decode(self, token_lists: Sequence[np.ndarray], n_nodes: Optional[Sequence[int]] = None,
               with_up_proj: bool = False):
        """List of token-id arrays → list of atom37 position arrays [N_b, 37, 3] float32, N_b =
        df·T_b, or `n_nodes[b]` (the graph's node count, df·T_b <= n < df·(T_b+1): the
        autoencoder pass, pst_decoder_decode_ex). With `with_up_proj` also returns the per-protein
        quantize_post_proj rows [T_b, 128]."""
        toks = [np.asarray(t, np.uint32).reshape(-1) for t in token_lists]
        off = np.zeros(len(toks) + 1, np.int64)
        off[1:] = np.cumsum([t.size for t in toks])
        flat = np.ascontiguousarray(np.concatenate(toks) if toks else np.zeros(0, np.uint32), np.uint32)
        nin = None if n_nodes is None else np.ascontiguousarray(n_nodes, np.int32)
        if nin is not None and nin.shape != (len(toks),):
            raise ValueError(f"{nin.shape} node counts for {len(toks)} proteins")
        n_total = int(off[-1]) * self.df if nin is None else int(nin.sum())
        # every row of every protein is written by the call (no zero fill needed); the results are
        # disjoint views of these fresh arrays (no copies)
        out = np.empty((max(n_total, 1), 37, 3), np.float32)
        nn = np.zeros(len(toks), np.int32)
        up = np.empty((max(int(off[-1]), 1), 128), np.float32) if with_up_proj else None
        self._check(lib().pst_decoder_decode_ex(self._h, _ptr(flat if flat.size else np.zeros(1, np.uint32)), _ptr(off),
                                                len(toks), _ptr(nin), _ptr(out), _ptr(nn), _ptr(up)))
        res, o = [], 0
        for n in nn:
            res.append(out[o:o + n])
            o += int(n)
        if not with_up_proj:
            return res
        return res, [up[off[b]:off[b + 1]] for b in range(len(toks))]

    def debug(self, which: int, n_floats: int) -> np.ndarray:
        out = np.zeros(n_floats, np.float32)
        self._check(lib().pst_decoder_debug(self._h, which, _ptr(out), n_floats))
        return out

    def set_timing(self, on: bool = True):
        """Stage timing (pst_decoder_set_timing): direct launches with HIP events while on."""
        self._check(lib().pst_decoder_set_timing(self._h, 1 if on else 0))

    def stage_ms(self) -> dict:
        """ms per stage summed since set_timing(True): upsampler, pair inputs, k_pair_fused, fold."""
        ms = np.zeros(4, np.float32)
        self._check(lib().pst_decoder_get_timing(self._h, _ptr(ms)))
        return dict(zip(("upsampler", "pair_inputs", "k_pair_fused", "fold"), ms.tolist()))
