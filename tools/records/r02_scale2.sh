# Strong-scaling shares with the current policy, then forced two-waves-per-task at larger sizes.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/strong_scaling_shares.sh > gpurun_out/r02_shares2.jsonl
for P in 1024 512 256; do
  for hv in 0 1; do
    PST_HALF_TASKS=$hv timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e --steps 10 --warmup 3 --proteins $P > gpurun_out/ab_tmp.json 2>gpurun_out/ab_err.txt
    python -c "import json; d=json.load(open('gpurun_out/ab_tmp.json')); r=d['roofline']; print('half=$hv', $P, round(d['value']/1e6,4), 'Mres/s dev', d['device_resident']['ms'], r['stage_ms'])" >> gpurun_out/r02_halfforce.txt
  done
done
echo done
