"""Per-phase wave cycles of the fused k_mpnn layers from a -DPST_STAMP build
(tools/build_variant.sh stamp "-DPST_STAMP"; run with PST_LIB=build/var_stamp/libpst.so).
Phases per 32-edge block: 0 edge update / embedding (to e), 1 message first GEMM(s) (incl. the
e store), 2 message hidden layer, 3 ordered segment sum; 4 = node update per task. Reports mean
cycles per block (phases 0-3) and per task (4) over all waves of the last tokenize call, and the
MFMA floor of each phase (64 cycles per v_mfma_f32_32x32x2_f32 issued by that wave).

    PST_LIB=build/var_stamp/libpst.so python tools/stamp_probe.py --proteins 512
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

os.environ.setdefault("PST_H2D_CHUNKS", "1")  # one chunk: every layer runs the one-wave fused form
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "protein-structure-tokenizer_amd")]
from pst_amd import params as P, synthetic  # noqa: E402
from pst_amd._native import LIB_PATH, Tokenizer, pack_samples  # noqa: E402

# MFMAs per block of each phase (layer 0 / layers 1-2) and per task of the node update
MFMA = {0: [60, 60, 260, 0], 1: [776, 256, 260, 0]}
NODE_MFMA = 256 + 4 * 516 + 4 * 256 + 8


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--proteins", type=int, default=512)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--waves", default="", help="save per-task (start, end, HW_ID|XCC_ID<<32, block) here (.npy)")
    a = ap.parse_args()
    samples = synthetic.synthetic_batch(a.proteins, 256, seed=1000)
    pos, flags, off = pack_samples(samples)
    tk = Tokenizer(0, 4096, 1, P.random_blob(6, 1234))
    lib = ctypes.CDLL(LIB_PATH)
    lib.pst_debug_stamps.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    buf = (ctypes.c_ulonglong * 48)()
    for _ in range(a.reps):
        lib.pst_debug_stamps(buf, 1)
        tk.tokenize_packed(pos.astype(np.float32), flags, off)
        tk.sync()
    lib.pst_debug_stamps(buf, 0)
    st = np.frombuffer(buf, dtype=np.uint64).reshape(3, 16).astype(np.float64)
    out = {"proteins": a.proteins, "lib": LIB_PATH, "layers": {}}
    for L in range(3):
        waves = st[L, 5]
        if waves == 0:
            continue
        blocks = waves * 50
        m = MFMA[0 if L == 0 else 1]
        ph = {f"phase{i}": {"cycles_per_block": round(st[L, i] / blocks), "mfma_floor": 64 * m[i]} for i in range(4)}
        ph["node_update"] = {"cycles_per_task": round(st[L, 4] / waves), "mfma_floor": 64 * NODE_MFMA}
        tot = sum(st[L, :5]) / waves
        ph["total_cycles_per_task"] = round(tot)
        ph["waves"] = int(waves)
        ph["prologue_cycles_per_task"] = round(st[L, 6] / waves)
        span_us = (st[L, 11] - st[L, 10]) / 100.0  # s_memrealtime: 100 MHz
        ph["kernel_span_us"] = round(span_us, 1)
        ph["clock_ghz"] = round(st[L, 9] / st[L, 8] * 0.1, 3)
        # share of the span x 2 048 wave slots (2 per SIMD) that waves occupied
        ph["slot_occupancy"] = round(st[L, 8] / 100.0 / (span_us * 2048), 3)
        ph["stamped_share_of_wave_life"] = round(sum(st[L, :5]) / st[L, 9], 3)
        out["layers"][f"k_mpnn<{L}>"] = ph
    if a.waves:
        lib.pst_debug_waves.argtypes = [ctypes.POINTER(ctypes.c_ulonglong)]
        wb = (ctypes.c_ulonglong * (3 * 16384 * 4))()
        lib.pst_debug_waves(wb)
        np.save(a.waves, np.frombuffer(wb, dtype=np.uint64).reshape(3, 16384, 4))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
