# Throughput and stage times across batch sizes (small CLI-sized batches up to the bench size).
# usage: bash tools/bench_sizes.sh [PST_LIB]
set -e
mkdir -p gpurun_out
[ -n "${1:-}" ] && export PST_LIB=$1
for P in 8 32 128 512 2048; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e --steps 5 --warmup 2 --proteins $P > gpurun_out/sz_tmp.json 2>/dev/null
  python -c "import json; d=json.load(open('gpurun_out/sz_tmp.json')); r=d['roofline']; print($P, 'proteins', round(d['value']/1e6,3), 'Mres/s', d['ms_per_step'], 'ms', r['stage_ms'])"
done
