# Split-cost recalibration check: partial-last-round batch sizes, fused vs split.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02pol_pytest.log 2>&1
run() { timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e --steps 10 --warmup 3 --proteins $1 > gpurun_out/ab_tmp.json 2>gpurun_out/ab_err.txt; python -c "import json; d=json.load(open('gpurun_out/ab_tmp.json')); r=d['roofline']; print('$2', $1, d['ms_per_step'], round(d['value']/1e6,4), 'dev', d['device_resident']['ms'], r['stage_ms'])"; }
for P in 960 240 236; do
  unset PST_SPLIT_TASKS
  run $P policy >> gpurun_out/r02_policy2.txt
  PST_SPLIT_TASKS=1000000 run $P split >> gpurun_out/r02_policy2.txt
  PST_SPLIT_TASKS=0 run $P fused >> gpurun_out/r02_policy2.txt
done
echo done
