# A/B the library variants given as args (paths), 2 rounds each, interleaved
set -e
mkdir -p gpurun_out
for round in 1 2; do
  for lib in "$@"; do
    PST_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --steps 5 --warmup 1 > gpurun_out/ab_tmp.json 2>/dev/null
    python -c "import json,sys; d=json.load(open('gpurun_out/ab_tmp.json')); r=d['roofline']; print('$lib', round(d['value']/1e6,3), 'Mres/s', r['stage_ms'])"
  done
done
