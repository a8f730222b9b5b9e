"""Per-wave timeline of the one-round fused layers (k_mpnn<L, true>) from ab/wstamp/libpst.so
(tools/wave_stamps_build.py): the N = 8 share of the headline (128 x 256 residues) tokenized a few
times, then for each layer the distribution over the 2 048 waves of their start skew, the W1 fill,
the first / steady / last edge block, the wait at the pair barrier, the node update, the end skew.
    PST_LIB=ab/wstamp/libpst.so python tools/wave_stamps_probe.py"""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "protein-structure-tokenizer_amd"))
import torch  # noqa: E402,F401

from pst_amd import params as P, synthetic  # noqa: E402
from pst_amd._native import LIB_PATH, Tokenizer, pack_samples  # noqa: E402

samples = synthetic.synthetic_batch(128, 256, seed=1000)
pos, flags, off = pack_samples(samples)
os.environ["PST_H2D_CHUNKS"] = "1"
tk = Tokenizer(0, 4096, 1, P.random_blob(6, 1234))
for _ in range(4):
    tk.tokenize_packed(pos.astype(np.float32), flags, off)
assert tk.last_plan_detail()["schedules"] == ["fused_half"]
L = ctypes.CDLL(LIB_PATH)
st = np.zeros((3, 2048, 32), np.uint64)
L.pst_x_wave_stamps(st.ctypes.data_as(ctypes.c_void_p))
st = st.astype(np.int64)
nst = np.zeros((3, 2048, 16), np.uint64)
L.pst_x_node_stamps(nst.ctypes.data_as(ctypes.c_void_p))
nst = nst.astype(np.int64)
pct = lambda x: [round(float(v), 1) for v in np.percentile(x, [0, 10, 50, 90, 100])]
for layer in range(3):
    w = st[layer]
    t0 = w[:, 0].min()
    us = lambda a: a / 100.0  # 100 MHz ticks -> us
    blocks = np.diff(w[:, 2:28], axis=1)  # 25 block durations (last one: to the loop end)
    out = {"layer": layer, "span_us": round(us(w[:, 29].max() - t0), 1),
           "start_us_p0_10_50_90_100": pct(us(w[:, 0] - t0)),
           "w1_fill_us": pct(us(w[:, 1] - w[:, 0])),
           "first_block_us": pct(us(blocks[:, 0])),
           "block_2_to_24_us (per block, median over blocks)": pct(us(np.median(blocks[:, 1:-1], axis=1))),
           "last_block_us": pct(us(blocks[:, -1])),
           "edge_phase_end_us": pct(us(w[:, 27] - t0)),
           "barrier_wait_us": pct(us(w[:, 28] - w[:, 27])),
           "node_update_us": pct(us(w[:, 29] - w[:, 28])),
           "end_us": pct(us(w[:, 29] - t0))}
    simd = (w[:, 31] >> 4) & 3
    out["waves_per_simd_slot_check"] = int(len(np.unique(w[:, 31] & 0xffffffff)))
    ns = nst[layer]
    names = ["x_exchange", "ln0", "ffn_chunk0", "ffn_chunk1", "ffn_chunk2", "ffn_chunk3", "residual_exchange",
             "ln1_store", "projections"]
    out["node_phases_us_p10_50_90"] = {nm: [round(float(v), 1) for v in np.percentile(us(ns[:, k + 1] - ns[:, k]), [10, 50, 90])]
                                       for k, nm in enumerate(names) if layer < 2 or nm != "projections"}
    print(json.dumps(out))
tk.close()
