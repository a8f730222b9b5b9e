# Default schedule policy (cost model) vs forced fused / split across batch sizes.
# usage: SIZES="128 192 320" bash tools/policy_check.sh
set -e
mkdir -p gpurun_out
for P in ${SIZES:-128 192 256 320 384 512}; do
  for S in auto 0 1000000000; do
    if [ $S = auto ]; then unset PST_SPLIT_TASKS; else export PST_SPLIT_TASKS=$S; fi
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e --steps 5 --warmup 2 --proteins $P > gpurun_out/pc_tmp.json 2>/dev/null
    python -c "import json; d=json.load(open('gpurun_out/pc_tmp.json')); print($P, '$S', round(d['value']/1e6,3), 'Mres/s', d['ms_per_step'], 'ms')"
  done
done
