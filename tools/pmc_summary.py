"""Per-dispatch averages of rocprofv3 --pmc CSVs: python tools/pmc_summary.py gpurun_out/<tag>_*"""
import collections
import csv
import glob
import sys

rows = collections.defaultdict(lambda: collections.defaultdict(list))
for d in sys.argv[1:]:
    for f in glob.glob(d + "/run_counter_collection.csv"):
        per = collections.defaultdict(lambda: collections.defaultdict(float))
        with open(f) as fh:
            for r in csv.DictReader(fh):
                per[(r["Kernel_Name"], r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
        for (k, _), cs in per.items():
            for c, v in cs.items():
                rows[k][c].append(v)
for k, cs in rows.items():
    if "pst::" not in k:
        continue
    print(k[:40])
    for c, vs in sorted(cs.items()):
        print(f"    {c:28s} {sum(vs) / len(vs):.4g}")
