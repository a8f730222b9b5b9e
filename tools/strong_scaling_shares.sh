# Per-GPU shares of BASELINE config 3's strong scaling (1 024 proteins split over N GPUs), each run
# on one GPU: N = 1, 2, 4, 8 -> 1024, 512, 256, 128 proteins. Since the ranks share nothing on the
# data path, the N-GPU job's step time is the slowest share's (LPT gives equal shares here).
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
for P in 1024 512 256 128; do
  timeout -k 10 300 python -u bench.py --proteins $P --no-cpu-baseline --no-e2e > gpurun_out/shares_$P.json 2>/dev/null
  python - "$P" <<'PY'
import json, sys
P = int(sys.argv[1]); N = 1024 // P
d = json.load(open(f"gpurun_out/shares_{P}.json"))
# `ms_per_step` / `value`: inputs resident in HBM (bench.py's timed region since round 6); before, the
# host-to-host step, now `host_to_host`
h = d.get("host_to_host") or {}
print(json.dumps({"n_gpus_simulated": N, "proteins_per_gpu": P, "ms_per_step": d["ms_per_step"],
                  "per_gpu_residues_per_s": d["value"], "job_residues_per_s_if_N_gpus": round(d["value"] * N, 1),
                  "host_to_host_ms": h.get("ms_per_step"), "stage_ms": d["roofline"]["stage_ms"]}))
PY
done
