"""Diagnostic: the GPU shader clock while libpst runs the device-resident loop vs the host-buffer
loop (pst_tokenize, H2D inside), sampled by one wave on a side stream (tools/clockprobe). Prints
one JSON line: clock percentiles per mode and a coarse time series (ms, GHz).

    python tools/clock_probe.py [--proteins 256] [--calls 5]
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "protein-structure-tokenizer_amd")]
import torch  # noqa: E402

from pst_amd import params as P, synthetic  # noqa: E402
from pst_amd._native import Tokenizer, pack_samples  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--proteins", type=int, default=256)
    ap.add_argument("--calls", type=int, default=5)
    ap.add_argument("--samples", type=int, default=12000)
    ap.add_argument("--sleep-units", type=int, default=10)
    a = ap.parse_args()
    lib = ctypes.CDLL(os.path.join(ROOT, "tools", "clockprobe", "libclockprobe.so"))
    lib.clock_probe_launch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
    samples = synthetic.synthetic_batch(a.proteins, 256, seed=1000)
    pos, flags, off = pack_samples(samples)
    R = int(off[-1])
    tk = Tokenizer(0, 4096, 1, P.random_blob(6, 1234))
    pin_pos = torch.from_numpy(pos).pin_memory()
    pin_flags = torch.from_numpy(flags).pin_memory()
    ppos, pfl = pin_pos.numpy(), pin_flags.numpy()
    d_pos, d_fl = torch.from_numpy(pos).cuda(), torch.from_numpy(flags).cuda()
    d_tok = torch.zeros(R, dtype=torch.int32, device="cuda")
    d_nt = torch.zeros(len(samples), dtype=torch.int32, device="cuda")
    d_nn = torch.zeros(len(samples), dtype=torch.int32, device="cuda")
    side = torch.cuda.Stream()
    out = {"proteins": a.proteins, "calls": a.calls}

    def device_call():
        tk.tokenize_device(d_pos.data_ptr(), d_fl.data_ptr(), off, d_tok.data_ptr(), d_nt.data_ptr(), d_nn.data_ptr())
        tk.sync()

    def host_call():
        tk.tokenize_packed(ppos, pfl, off)

    for name, fn in (("device", device_call), ("host", host_call), ("device2", device_call)):
        fn()
        torch.cuda.synchronize()
        buf = torch.zeros(2 * a.samples, dtype=torch.int64, device="cuda")
        rc = lib.clock_probe_launch(ctypes.c_void_p(side.cuda_stream), ctypes.c_void_p(buf.data_ptr()), a.samples,
                                    a.sleep_units)
        assert rc == 0, rc
        for _ in range(a.calls):
            fn()
        torch.cuda.synchronize()
        s = buf.cpu().numpy().astype(np.float64).reshape(-1, 2)
        s = s[s[:, 1] > 0]
        dc, dw = np.diff(s[:, 0]), np.diff(s[:, 1])
        ghz = dc / dw * 0.1
        t_ms = (s[1:, 1] - s[0, 1]) / 1e5
        keep = t_ms <= t_ms[-1]
        ghz, t_ms = ghz[keep], t_ms[keep]
        bins = np.arange(0, t_ms[-1] + 5, 5.0)
        idx = np.digitize(t_ms, bins)
        series = [[round(float(bins[i - 1]), 1), round(float(np.median(ghz[idx == i])), 3)] for i in np.unique(idx)]
        out[name] = {"p10": round(float(np.percentile(ghz, 10)), 3), "p50": round(float(np.median(ghz)), 3),
                     "p90": round(float(np.percentile(ghz, 90)), 3), "span_ms": round(float(t_ms[-1]), 1),
                     "series_5ms": series}
    print(json.dumps(out), flush=True)
    tk.close()


if __name__ == "__main__":
    main()
