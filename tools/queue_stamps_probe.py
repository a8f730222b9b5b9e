"""Where the persistent queue's waves spend their time (ab/qstamp/libpst.so, tools/queue_stamps_build.py):
the headline batch (1 024 x 256 residues, one chunk) tokenized a few times; per queue layer the
wave-summed edge-phase and node-update times, per unit and per node update, and their share of
the waves' lifetimes.   PST_LIB=ab/qstamp/libpst.so python tools/queue_stamps_probe.py"""
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

pos, flags, off = pack_samples(synthetic.synthetic_batch(1024, 256, seed=1000))
os.environ["PST_H2D_CHUNKS"] = "1"
tk = Tokenizer(0, 4096, 1, P.random_blob(6, 1234))
for _ in range(3):
    tk.tokenize_packed(pos.astype(np.float32), flags, off)
st = np.zeros((3, 4096, 8), np.uint64)
ctypes.CDLL(LIB_PATH).pst_x_queue_stamps(st.ctypes.data_as(ctypes.c_void_p))
st = st.astype(np.int64)
for layer in (1, 2):
    w = st[layer]
    w = w[w[:, 2] > 0]
    life = (w[:, 5] - w[:, 4]).sum()
    out = {"layer": layer, "waves": int(len(w)), "units": int(w[:, 2].sum()), "node_updates": int(w[:, 3].sum()),
           "edge_us_per_unit": round(float(w[:, 0].sum() / w[:, 2].sum() / 100.0), 1),
           "node_us_per_update": round(float(w[:, 1].sum() / max(1, w[:, 3].sum()) / 100.0), 1),
           "edge_share_of_lifetime": round(float(w[:, 0].sum() / life), 4),
           "node_share_of_lifetime": round(float(w[:, 1].sum() / life), 4),
           "span_us": round(float((w[:, 5].max() - w[:, 4].min()) / 100.0), 1)}
    print(json.dumps(out))
tk.close()
