"""Which schedule variant of test_mpnn_queue_identical_at_full_rounds differs from the one-wave
fused form, and from which layer on (diagnostic; PST_LIB selects the library under test)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "protein-structure-tokenizer_amd")]
import torch  # noqa: E402,F401

from pst_amd import params as P, synthetic  # noqa: E402
from pst_amd._native import Tokenizer, pack_samples  # noqa: E402

rng = np.random.default_rng(5)
lens = [int(x) for x in rng.integers(60, 513, 340)]
samples = [synthetic.synthetic_protein(n, 4000 + i) for i, n in enumerate(lens)]
pos, flags, off = pack_samples(samples)
R = int(off[-1])
os.environ["PST_DEBUG"] = "1"
os.environ["PST_H2D_CHUNKS"] = "1"
res = {}
for name, env in (("one_wave", {"PST_MPNN_QUEUE": "0"}), ("queue_all", {"PST_MPNN_QUEUE": "1", "PST_MPNN_QUEUE_LAYERS": "7"}),
                  ("queue_L0", {"PST_MPNN_QUEUE": "1", "PST_MPNN_QUEUE_LAYERS": "1"}),
                  ("queue_L1", {"PST_MPNN_QUEUE": "1", "PST_MPNN_QUEUE_LAYERS": "2"}),
                  ("queue_default", {"PST_MPNN_QUEUE": "1"}),
                  ("queue_4w", {"PST_MPNN_QUEUE": "1", "PST_MPNN_QWAVES": "4"}),
                  ("queue_all_4w", {"PST_MPNN_QUEUE": "1", "PST_MPNN_QUEUE_LAYERS": "7", "PST_MPNN_QWAVES": "4"})):
    for k in ("PST_MPNN_QUEUE", "PST_MPNN_QUEUE_LAYERS", "PST_MPNN_QWAVES"):
        os.environ.pop(k, None)
    os.environ.update(env)
    tk = Tokenizer(0, 4096, 1, P.random_blob(6, 1234))
    tok, nt, nn = tk.tokenize_packed(pos.astype(np.float32), flags, off)
    res[name] = (tok[:R].copy(), [tk.debug_fetch(w, R).copy() for w in (1, 2, 3)])
    tk.close()
base = res["one_wave"]
for name, (tok, hl) in res.items():
    diff = [int(np.sum(h.view(np.uint32) != b.view(np.uint32))) for h, b in zip(hl, base[1])]
    print(name, "tokens differ:", int(np.sum(tok != base[0])), "node-feature words differ per layer:", diff,
          "max |d| L1:", float(np.abs(hl[0] - base[1][0]).max()), flush=True)
