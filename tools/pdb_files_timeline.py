"""Device timeline of tools/pdb_files_probe.py under rocprofv3 --kernel-trace --memory-copy-trace
(CSV output): calls are split at host gaps > 2 ms; for the median call, every kernel / copy with
its start relative to the call's first device operation and its duration (us), and the idle gaps.

    python tools/pdb_files_timeline.py <rocprof output dir>
"""
import csv
import glob
import sys

import numpy as np

d = sys.argv[1]
ev = []
for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:60]))
for f in glob.glob(f"{d}/**/*memory_copy_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "copy " + r.get("Direction", "")))
ev.sort()
calls, cur = [], [ev[0]]
for e in ev[1:]:
    if e[0] - cur[-1][1] > 2_000_000:
        calls.append(cur)
        cur = [e]
    else:
        cur.append(e)
calls.append(cur)
calls = [c for c in calls if len(c) > 10]
spans = [c[-1][1] - c[0][0] for c in calls]
i = int(np.argsort(spans)[len(spans) // 2])
c = calls[i]
t0 = c[0][0]
print(f"{len(calls)} calls; device span median {np.median(spans) / 1e3:.1f} us")
prev = t0
for s, e, n in c:
    gap = (s - prev) / 1e3
    print(f"{(s - t0) / 1e3:9.1f} +{(e - s) / 1e3:8.1f}  gap {gap:7.1f}  {n}")
    prev = max(prev, e)
