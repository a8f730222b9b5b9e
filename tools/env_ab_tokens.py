"""A/B of a libpst schedule knob read at a context's first call (one context per value):
interleaved rounds of host-to-host timings of pst_tokenize_f32 on synthetic_batch(P, 256), and the
token ids of every value compared with the first value's (must be identical), plus the HIP-event
stage times of each. Prints one JSON line per protein count.

    python tools/env_ab_tokens.py --env PST_HALF_NODE_COOP --values 0 1 [--proteins 128] [--rounds 5]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "protein-structure-tokenizer_amd")]
import torch  # noqa: E402,F401  (pinned buffers)

from pst_amd import params as P, synthetic  # noqa: E402
from pst_amd._native import Tokenizer, pack_samples  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--env", required=True)
    ap.add_argument("--values", nargs="+", required=True)
    ap.add_argument("--proteins", type=int, nargs="+", default=[128])
    ap.add_argument("--residues", type=int, default=256)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    blob = P.random_blob(6, 1234)
    tks = {}
    for v in a.values:
        os.environ[a.env] = v
        tks[v] = Tokenizer(0, 4096, 1, blob)
        tks[v].tokenize_packed(*pack_samples(synthetic.synthetic_batch(8, 256, seed=1)))
    for n in a.proteins:
        samples = synthetic.synthetic_batch(n, a.residues, seed=1000)
        pos, flags, off = pack_samples(samples)
        p32 = torch.from_numpy(pos.astype(np.float32)).pin_memory().numpy()
        fl = torch.from_numpy(flags).pin_memory().numpy()
        ref, same, stages = None, {}, {}
        for v in a.values:
            tok, nt, nn = tks[v].tokenize_packed(p32, fl, off)
            tok = np.concatenate([tok[int(off[i]):int(off[i]) + int(nt[i])] for i in range(n)])
            ref = tok if ref is None else ref
            same[v] = bool(np.array_equal(tok, ref))
        times = {v: [] for v in a.values}
        for _ in range(a.rounds):
            for v in a.values:
                for _ in range(2):
                    tks[v].tokenize_packed(p32, fl, off)
                ts = []
                for _ in range(a.reps):
                    t0 = time.perf_counter()
                    tks[v].tokenize_packed(p32, fl, off)
                    ts.append(time.perf_counter() - t0)
                times[v].append(round(float(np.median(ts)) * 1e3, 3))
        for v in a.values:
            tks[v].set_timing(True)
            acc = None
            for _ in range(5):
                tks[v].tokenize_packed(p32, fl, off)
                st = tks[v].stage_ms()
                acc = st if acc is None else {k: acc[k] + st[k] for k in st}
            tks[v].set_timing(False)
            stages[v] = {k: round(x / 5, 3) for k, x in acc.items()}
        print(json.dumps({"env": a.env, "proteins": n, "residues": int(off[-1]), "tokens_identical_to_first": same,
                          "host_ms_median_per_round": times,
                          "host_ms_median": {v: float(np.median(t)) for v, t in times.items()},
                          "stage_ms": stages}), flush=True)


if __name__ == "__main__":
    main()
