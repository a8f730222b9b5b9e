"""Wave-slot timeline of the fused k_mpnn layers from tools/stamp_probe.py --waves OUT.npy
(PST_STAMP build): per task the wave's start / end (s_memrealtime, 100 MHz) and the hardware
slot (HW_ID: SIMD, CU, SH, SE; XCC_ID). Prints, per layer: wave duration spread, how the waves
were dealt to SIMDs, and where the span goes (slot occupancy, the ramp and the tail).

    python tools/wave_timeline.py gpurun_out/r03_waves512.npy [n_tasks]
"""
import collections
import json
import sys

import numpy as np


def decode(hw):
    lo = hw & 0xffffffff
    return {"simd": (lo >> 4) & 3, "cu": (lo >> 8) & 15, "sh": (lo >> 12) & 1, "se": (lo >> 13) & 7,
            "xcc": (hw >> 32) & 0xf}


def main():
    W = np.load(sys.argv[1])
    out = {}
    for L in range(3):
        w = W[L]
        n = int(np.count_nonzero(w[:, 1]))
        if n == 0:
            continue
        w = w[:n].astype(np.int64)
        t0 = w[:, 0].min()
        st = (w[:, 0] - t0) / 100.0  # µs
        en = (w[:, 1] - t0) / 100.0
        dur = en - st
        span = en.max()
        simds = collections.defaultdict(list)
        for i in range(n):
            d = decode(int(W[L][i, 2]))
            simds[(d["xcc"], d["se"], d["sh"], d["cu"], d["simd"])].append(i)
        per_simd = np.array([len(v) for v in simds.values()])
        # per SIMD: the time its last wave ended, and its summed wave time / 2 slots
        simd_end = np.array([en[v].max() for v in simds.values()])
        simd_fill = np.array([dur[v].sum() / 2.0 for v in simds.values()])
        # round structure: first waves of each slot vs later ones
        order = np.argsort(st)
        first = order[: min(n, 2 * len(simds))]
        later = order[min(n, 2 * len(simds)):]
        q = lambda x: [round(float(v), 1) for v in np.percentile(x, [0, 10, 50, 90, 100])] if len(x) else None
        out[f"k_mpnn<{L}>"] = {
            "tasks": n, "simds_used": len(simds), "waves_per_simd": q(per_simd),
            "span_us": round(float(span), 1),
            "wave_us_p0_10_50_90_100": q(dur),
            "first_round_start_us": q(st[first]), "first_round_end_us": q(en[first]),
            "later_start_us": q(st[later]) if len(later) else None,
            "later_dur_us": q(dur[later]) if len(later) else None,
            "simd_last_end_us": q(simd_end),
            "simd_busy_us(sum of wave time / 2)": q(simd_fill),
            "occupancy": round(float(dur.sum() / (2 * len(simds) * span)), 3),
        }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
