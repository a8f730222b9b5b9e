"""A/B of the one-round two-halves schedule (run(), PST_TWO_HALVES 0 / 1 / 2) at the N = 8 share of
config 3 (128 proteins x 256 residues) and neighbours: one libpst context per mode (the knob is
read at a context's first call), interleaved rounds of host-to-host timings, and the token ids of
every mode compared with mode 0's (must be identical). Prints one JSON line per protein count.

    python tools/two_halves_ab.py [--proteins 128 96 160] [--rounds 5] [--reps 10]
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
    ap.add_argument("--proteins", type=int, nargs="+", default=[128])
    ap.add_argument("--residues", type=int, default=256)
    ap.add_argument("--modes", type=int, nargs="+", default=[0, 1, 2])
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    blob = P.random_blob(6, 1234)
    tks = {}
    for m in a.modes:
        os.environ["PST_TWO_HALVES"] = str(m)
        tks[m] = Tokenizer(0, 4096, 1, blob)
        tks[m].tokenize_packed(*pack_samples(synthetic.synthetic_batch(8, 256, seed=1)))
    for n in a.proteins:
        samples = synthetic.synthetic_batch(n, a.residues, seed=1000)
        pos, flags, off = pack_samples(samples)
        pin = torch.from_numpy(pos.astype(np.float32)).pin_memory()
        pfl = torch.from_numpy(flags).pin_memory()
        p32, fl = pin.numpy(), pfl.numpy()
        ref = None
        same = {}
        for m in a.modes:
            tok, nt, nn = tks[m].tokenize_packed(p32, fl, off)
            tok = np.concatenate([tok[int(off[i]):int(off[i]) + int(nt[i])] for i in range(n)])
            if ref is None:
                ref = tok
            same[m] = bool(np.array_equal(tok, ref))
        times = {m: [] for m in a.modes}
        for _ in range(a.rounds):
            for m in a.modes:
                for _ in range(2):
                    tks[m].tokenize_packed(p32, fl, off)
                ts = []
                for _ in range(a.reps):
                    t0 = time.perf_counter()
                    tks[m].tokenize_packed(p32, fl, off)
                    ts.append(time.perf_counter() - t0)
                times[m].append(round(float(np.median(ts)) * 1e3, 3))
        print(json.dumps({"proteins": n, "residues": int(off[-1]), "tokens_identical_to_mode0": same,
                          "host_ms_median_per_round": times,
                          "host_ms_median": {m: float(np.median(v)) for m, v in times.items()}}), flush=True)


if __name__ == "__main__":
    main()
