"""Merged kernel + memory-copy timeline of a rocprofv3 --kernel-trace --memory-copy-trace run:
python tools/timeline.py DIR [t_from_ms t_to_ms] — one line per event (start/end ms relative to
the first event, duration, gap since the previous event's end)."""
import csv
import sys

d = sys.argv[1]
ev = []
for r in csv.DictReader(open(d + "/run_kernel_trace.csv")):
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K " + r["Kernel_Name"][:48]))
for r in csv.DictReader(open(d + "/run_memory_copy_trace.csv")):
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "C " + r["Direction"].replace("MEMORY_COPY_", "")))
ev.sort()
t0 = ev[0][0]
lo = float(sys.argv[2]) if len(sys.argv) > 2 else -1
hi = float(sys.argv[3]) if len(sys.argv) > 3 else 1e18
prev_end = t0
for s, e, n in ev:
    a, b = (s - t0) / 1e6, (e - t0) / 1e6
    if lo <= a <= hi:
        print(f"{a:10.3f} {b:10.3f} {(e - s) / 1e6:8.3f} gap {(s - prev_end) / 1e6:8.3f}  {n}")
    prev_end = max(prev_end, e)
