"""Independent proteins on concurrent HIP streams: one batch tokenized by ONE libpst context vs the
same proteins split over K contexts (each with its own stream and workspace) driven from K host
threads at once (ctypes releases the GIL), host buffers in pinned memory as bench.py sends them.
Prints ms per batch (median) for each K and whether the tokens are identical.
    python tools/two_ctx_probe.py [--proteins 128] [--ks 1,2,3,4] [--reps 10]"""
import argparse
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "protein-structure-tokenizer_amd"))
import torch  # noqa: E402

from pst_amd import params as P, synthetic  # noqa: E402
from pst_amd._native import Tokenizer, pack_samples  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--proteins", type=int, default=128)
ap.add_argument("--ks", default="1,2,3,4")
ap.add_argument("--reps", type=int, default=10)
a = ap.parse_args()
samples = synthetic.synthetic_batch(a.proteins, 256, seed=1000)
blob = P.random_blob(6, 1234)


def packed(sub):
    pos, flags, off = pack_samples(sub)
    return (torch.from_numpy(pos.astype(np.float32)).pin_memory().numpy(),
            torch.from_numpy(flags).pin_memory().numpy(), off)


ks = [int(k) for k in a.ks.split(",")]
tks = [Tokenizer(0, 4096, 1, blob) for _ in range(max(ks))]
ref = None
out = {"proteins": a.proteins}
for K in ks:
    parts = [packed(samples[i::K]) for i in range(K)]  # interleaved: equal shares
    res = [None] * K

    def work(i, parts=parts, res=res):
        res[i] = tks[i].tokenize_packed(*parts[i])

    def once(K=K, work=work):
        if K == 1:
            work(0)
            return
        th = [threading.Thread(target=work, args=(i,)) for i in range(K)]
        for t in th:
            t.start()
        for t in th:
            t.join()

    for _ in range(3):
        once()
    ts = []
    for _ in range(a.reps):
        time.sleep(0.005)
        t0 = time.perf_counter()
        once()
        ts.append(time.perf_counter() - t0)
    # tokens back in the original protein order
    toks = [None] * a.proteins
    for i in range(K):
        tok, nt, _ = res[i]
        off = parts[i][2]
        for q, b in enumerate(range(i, a.proteins, K)):
            toks[b] = tok[int(off[q]):int(off[q]) + int(nt[q])].copy()
    if ref is None:
        ref = toks
    same = all(np.array_equal(x, y) for x, y in zip(ref, toks))
    out[f"K{K}"] = {"ms_median": round(float(np.median(ts)) * 1e3, 3), "ms_min": round(min(ts) * 1e3, 3),
                    "tokens_identical_to_K1": same}
    print(json.dumps(out), flush=True)
for t in tks:
    t.close()
