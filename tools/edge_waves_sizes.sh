# Split-schedule edge-wave target (PST_EDGE_WAVES) across batch sizes: stage times.
set -e
mkdir -p gpurun_out
for P in 32 64 96; do
  for W in 4096 1000000; do
    PST_EDGE_WAVES=$W timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e --steps 5 --warmup 2 --proteins $P > gpurun_out/ew_tmp.json 2>/dev/null
    python -c "import json; d=json.load(open('gpurun_out/ew_tmp.json')); r=d['roofline']; print($P, $W, d['ms_per_step'], [r['stage_ms'][k] for k in ('mpnn0','mpnn1','mpnn2')])"
  done
done
