"""Host-to-host vs device-resident tokenize on the bench workload (1024 x 256 residues):
where the PCIe-inclusive time goes. Prints one JSON line.

    python tools/pcie_probe.py [--proteins 1024] [--reps 5]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "protein-structure-tokenizer_amd")]
import torch  # noqa: E402

from pst_amd import params as P, synthetic  # noqa: E402
from pst_amd._native import Tokenizer, pack_samples  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--proteins", type=int, default=1024)
    ap.add_argument("--residues", type=int, default=256)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    samples = synthetic.synthetic_batch(a.proteins, a.residues, seed=1000)
    pos, flags, off = pack_samples(samples)
    R = int(off[-1])
    tk = Tokenizer(0, 4096, 1, P.random_blob(6, 1234))
    pin_pos = torch.from_numpy(pos).pin_memory()
    pin_flags = torch.from_numpy(flags).pin_memory()
    ppos, pfl = pin_pos.numpy(), pin_flags.numpy()
    d_pos = torch.from_numpy(pos).cuda()
    d_fl = torch.from_numpy(flags).cuda()
    d_tok = torch.zeros(R, dtype=torch.int32, device="cuda")
    d_nt = torch.zeros(len(samples), dtype=torch.int32, device="cuda")
    d_nn = torch.zeros(len(samples), dtype=torch.int32, device="cuda")
    res = {"residues": R, "h2d_bytes": int(pos.nbytes + flags.nbytes)}

    def timeit(fn):
        fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(a.reps):
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        return round(float(np.median(ts)) * 1e3, 3)

    res["device_ms"] = timeit(lambda: (tk.tokenize_device(d_pos.data_ptr(), d_fl.data_ptr(), off, d_tok.data_ptr(),
                                                          d_nt.data_ptr(), d_nn.data_ptr()), tk.sync()))
    res["host_pageable_ms"] = timeit(lambda: tk.tokenize_packed(pos, flags, off))
    res["host_pinned_ms"] = timeit(lambda: tk.tokenize_packed(ppos, pfl, off))
    dst = torch.empty_like(d_pos)
    res["h2d_pinned_copy_ms"] = timeit(lambda: dst.copy_(pin_pos, non_blocking=True))
    res["h2d_pageable_copy_ms"] = timeit(lambda: dst.copy_(torch.from_numpy(pos)))
    print(json.dumps(res), flush=True)
    tk.close()


if __name__ == "__main__":
    main()
