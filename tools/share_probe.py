"""Host path vs device-resident path on one share of config 3 (default 128 proteins x 256
residues = the N = 8 share): median wall time of each, per-stage HIP-event times of each (the
stage events are recorded on libpst's stream in either path), and the float32 H2D copy alone.
Environment knobs (PST_H2D_*) are read by the context at its first call. Prints one JSON line.

    python tools/share_probe.py [--proteins 128] [--reps 15] [--tag NAME]
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
    ap.add_argument("--proteins", type=int, default=128)
    ap.add_argument("--residues", type=int, default=256)
    ap.add_argument("--reps", type=int, default=15)
    ap.add_argument("--tag", default="")
    a = ap.parse_args()
    samples = synthetic.synthetic_batch(a.proteins, a.residues, seed=1000)
    pos, flags, off = pack_samples(samples)
    R = int(off[-1])
    tk = Tokenizer(0, 4096, 1, P.random_blob(6, 1234))
    pin32 = torch.from_numpy(pos.astype(np.float32)).pin_memory()
    pinf = torch.from_numpy(flags).pin_memory()
    p32, pfl = pin32.numpy(), pinf.numpy()
    d_pos = torch.from_numpy(pos).cuda()
    d_fl = torch.from_numpy(flags).cuda()
    d_tok = torch.zeros(R, dtype=torch.int32, device="cuda")
    d_nt = torch.zeros(len(samples), dtype=torch.int32, device="cuda")
    d_nn = torch.zeros(len(samples), dtype=torch.int32, device="cuda")

    def dev():
        tk.tokenize_device(d_pos.data_ptr(), d_fl.data_ptr(), off, d_tok.data_ptr(), d_nt.data_ptr(), d_nn.data_ptr())
        tk.sync()

    def host():
        tk.tokenize_packed(p32, pfl, off)

    def wall(fn):
        for _ in range(3):
            fn()
        ts = []
        for _ in range(a.reps):
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        return round(float(np.median(ts)) * 1e3, 3)

    def stages(fn):
        tk.set_timing(True)
        acc = None
        for _ in range(5):
            fn()
            st = tk.stage_ms()
            acc = st if acc is None else {k: acc[k] + st[k] for k in st}
        tk.set_timing(False)
        return {k: round(v / 5, 3) for k, v in acc.items()}

    res = {"tag": a.tag, "proteins": a.proteins, "residues": R,
           "env": {k: v for k, v in os.environ.items() if k.startswith("PST_")}}
    res["host_ms"] = wall(host)
    res["device_ms"] = wall(dev)
    res["host_ms_again"] = wall(host)
    res["host_stage_ms"] = stages(host)
    res["device_stage_ms"] = stages(dev)
    res["plan"] = tk.last_plan_detail()
    host()
    res["plan"] = tk.last_plan_detail()
    dst = torch.empty_like(pin32, device="cuda")
    res["h2d_f32_copy_ms"] = wall(lambda: (dst.copy_(pin32, non_blocking=True), torch.cuda.synchronize()))
    print(json.dumps(res), flush=True)
    tk.close()


if __name__ == "__main__":
    main()
