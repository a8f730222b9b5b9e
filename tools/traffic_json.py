"""profiles/traffic_k_mpnn1.json (bench.py's roofline `traffic`) from the FETCH_SIZE / WRITE_SIZE passes of
tools/pmc_all.sh (or pmc_traffic.sh): per-dispatch averages of the layer-1 kernel at the full bench size
(PST_H2D_CHUNKS=1, 262 144 residues), FETCH_SIZE x2 (gfx950 wide-read correction, MI355X_MICROARCH.md
HBM section), KB = 1 024 B; MFMA busy from the SQ pass when present.

    python tools/traffic_json.py gpurun_out/TAG SOURCE_NOTE > profiles/traffic_k_mpnn1.json
"""
import collections
import csv
import glob
import json
import sys

tag, note = sys.argv[1], sys.argv[2]
KERNEL = "k_mpnn_q<1, 8>"


def avg(counter):
    vals = collections.defaultdict(float)
    for f in glob.glob(f"{tag}_*/run_counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter and KERNEL in r["Kernel_Name"]:
                vals[r["Dispatch_Id"]] += float(r["Counter_Value"])
    return sum(vals.values()) / len(vals) if vals else None


R = 262144
fetch, write = avg("FETCH_SIZE"), avg("WRITE_SIZE")
busy, gui = avg("SQ_VALU_MFMA_BUSY_CYCLES"), avg("GRBM_GUI_ACTIVE")
out = {"kernel": "k_mpnn_q<1, 8> (layer 1 as the persistent half-task queue)", "residues_per_launch": R,
       "fetch_size_kb_per_launch": fetch, "write_size_kb_per_launch": write,
       "read_bytes_per_residue": round(fetch * 2 * 1024 / R, 1), "write_bytes_per_residue": round(write * 1024 / R, 1),
       "source": note,
       "algorithmic_bytes_per_residue": {"edge_state_read": 25600, "edge_state_write": 25600,
                                         "sender_projection_gathers": 51200, "node_rows": 4608}}
if busy and gui:
    out["mfma_busy_fraction"] = round(busy / (1024 * gui / 8), 4)
print(json.dumps(out, indent=1))
