# CASP14 device call time vs the split schedule's edge-wave target (PST_EDGE_WAVES).
set -e
mkdir -p gpurun_out
for W in 4096 8192 16384 1000000; do
  PST_EDGE_WAVES=$W timeout -k 10 200 python tools/prof_casp14.py --reps 20 > gpurun_out/ew_tmp.json 2>/dev/null
  python -c "import json; d=json.load(open('gpurun_out/ew_tmp.json')); print($W, d['ms_per_call'], d['stage_ms'])"
done
