"""ctypes wrapper of the CPU oracle `oracle/_build/libpst_oracle.so`.

TEST INFRASTRUCTURE: imported only by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, always as the checker / the timed CPU baseline — never by the product.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "_build", "libpst_oracle.so")
_lib = None

K = 50


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            build()
        L = ctypes.CDLL(_SO)
        P = ctypes.c_void_p
        i = ctypes.c_int
        L.pst_oracle_param_count.restype = ctypes.c_size_t
        L.pst_oracle_param_count.argtypes = [i]
        L.pst_oracle_pe_row.argtypes = [i, i, P]
        L.pst_oracle_graph.argtypes = [P, P, i, i, P, P, P, P, P]
        L.pst_oracle_encode.argtypes = [P, i, P, i, i, i, P, P, P, P, P, P, P, P, P]
        L.pst_oracle_tokenize.argtypes = [P, i, P, i, i, P, P, i, P, P, P, P]
        L.pst_oracle_tokenize_batch.argtypes = [P, i, P, i, i, P, P, P, i, P, P, i]
        L.pst_oracle_fsq_aux.argtypes = [P, i, P, ctypes.c_int64, P, P, P]
        for f in ("tanh", "gelu", "exp", "sigmoid"):
            fn = getattr(L, "pst_oracle_" + f)
            fn.restype, fn.argtypes = ctypes.c_float, [ctypes.c_float]
        L.pst_oracle_exp64.restype, L.pst_oracle_exp64.argtypes = ctypes.c_double, [ctypes.c_double]
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def math_fn(name):
    return getattr(lib(), "pst_oracle_" + name)


def pe_row(x, n):
    out = np.zeros(128, np.float32)
    lib().pst_oracle_pe_row(x, n, _p(out))
    return out


def graph(pos, flags, k=K):
    """One protein: raw atom37 (float64 [R,37,3], uint8 flags [R,37]) → dict of graph arrays."""
    pos = np.ascontiguousarray(pos, dtype=np.float64)
    flags = np.ascontiguousarray(flags, dtype=np.uint8)
    R = pos.shape[0]
    n = np.zeros(1, np.int32)
    kept = np.zeros(R, np.int32)
    senders = np.zeros(R * k, np.int32)
    deg = np.zeros(R, np.int32)
    feat = np.zeros((R * k, 32), np.float32)
    rc = lib().pst_oracle_graph(_p(pos), _p(flags), R, k, _p(n), _p(kept), _p(senders), _p(deg), _p(feat))
    if rc != 0:
        raise RuntimeError(f"oracle graph failed: {rc}")
    nn = int(n[0])
    return dict(n=nn, kept=kept[:nn], senders=senders[:nn * k], deg=deg[:nn], feat=feat[:nn * k])


def encode(blob, levels, df, g, k=K, want_layers=False):
    """Graph dict (from `graph`) → dict(tokens, z, b, q, pre_proj[, h_layers])."""
    n = g["n"]
    D = len(levels)
    T = n // df
    lv = np.asarray(levels, np.int32)
    blob = np.ascontiguousarray(blob, np.float32)
    senders = np.ascontiguousarray(g["senders"], np.int32)
    deg = np.ascontiguousarray(g["deg"], np.int32)
    feat = np.ascontiguousarray(g["feat"], np.float32)
    h_layers = np.zeros((4, n, 128), np.float32) if want_layers else None
    pre = np.zeros((T, 128), np.float32)
    z = np.zeros((T, D), np.float32)
    b = np.zeros((T, D), np.float32)
    q = np.zeros((T, D), np.float32)
    tok = np.zeros(T, np.uint32)
    rc = lib().pst_oracle_encode(_p(blob), D, _p(lv), df, n, k, _p(senders), _p(deg), _p(feat),
                                 _p(h_layers) if want_layers else None, _p(pre), _p(z), _p(b), _p(q), _p(tok))
    if rc != T:
        raise RuntimeError(f"oracle encode failed: {rc}")
    out = dict(tokens=tok, z=z, b=b, q=q, pre_proj=pre)
    if want_layers:
        out["h_layers"] = h_layers
    return out


def tokenize(blob, levels, df, pos, flags, k=K, **kw):
    g = graph(pos, flags, k)
    out = encode(blob, levels, df, g, k, **kw)
    out["graph"] = g
    return out


def tokenize_batch(blob, levels, df, pos, flags, offsets, n_threads=1, k=K):
    """Ragged batch (the CPU-baseline entry): tokens laid out like libpst's tokens_out."""
    pos = np.ascontiguousarray(pos, dtype=np.float64)
    flags = np.ascontiguousarray(flags, dtype=np.uint8)
    offsets = np.ascontiguousarray(offsets, dtype=np.int64)
    B = len(offsets) - 1
    tok = np.zeros(int(offsets[-1]), np.uint32)
    nt = np.zeros(B, np.int32)
    lv = np.asarray(levels, np.int32)
    blob = np.ascontiguousarray(blob, np.float32)
    rc = lib().pst_oracle_tokenize_batch(_p(blob), len(levels), _p(lv), df, k, _p(pos), _p(flags),
                                         _p(offsets), B, _p(tok), _p(nt), n_threads)
    if rc != 0:
        raise RuntimeError("oracle batch failed")
    return tok, nt


def fsq_aux(levels, bounded):
    """distances / soft_proba / argmin for rows of continuous embeddings (libpst's canonical
    formulation, see pst_oracle.c)."""
    lv = np.asarray(levels, np.int32)
    b = np.ascontiguousarray(bounded, np.float32).reshape(-1, len(lv))
    T, K = b.shape[0], int(np.prod(lv))
    dist = np.zeros((T, K), np.float32)
    prob = np.zeros((T, K), np.float32)
    arg = np.zeros(T, np.uint32)
    if lib().pst_oracle_fsq_aux(_p(lv), len(lv), _p(b), T, _p(dist), _p(prob), _p(arg)) != 0:
        raise ValueError("fsq_aux needs 4 <= D <= 8")
    return dict(distances=dist, soft_proba=prob, argmin=arg)


def perplexity(tokens, K):
    """quantize.py:211-224 on the real token rows (f64 accumulation)."""
    hist = np.bincount(np.asarray(tokens, np.int64), minlength=K).astype(np.float64)
    p = hist / max(hist.sum(), 1.0)
    return float(np.exp(-np.sum(p * np.log(p + 1e-10)))), hist.astype(np.uint32)
