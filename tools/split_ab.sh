# Fused vs split MPNN schedule across batch sizes (PST_SPLIT_TASKS=0 forces fused, 1e9 forces split).
# usage: bash tools/split_ab.sh
set -e
mkdir -p gpurun_out
for P in ${SIZES:-8 32 64 128 256 512}; do
  for S in 0 1000000000; do
    PST_SPLIT_TASKS=$S timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e --steps 5 --warmup 2 --proteins $P > gpurun_out/ab_tmp.json 2>/dev/null
    python -c "import json; d=json.load(open('gpurun_out/ab_tmp.json')); r=d['roofline']; print($P, 'proteins split' if $S else 'proteins fused', round(d['value']/1e6,3), 'Mres/s', d['ms_per_step'], 'ms', r['stage_ms'])"
  done
done
