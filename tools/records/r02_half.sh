# Two-waves-per-task fused layers: GPU tests, then 128 proteins (one round: policy = half tasks)
# vs the previous build (split schedule there), vs this build forced to split, and 1024 proteins.
set -e
TAG=$1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
run() { timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e --steps 10 --warmup 3 --proteins $1 > gpurun_out/ab_tmp.json 2>gpurun_out/ab_err.txt; python -c "import json; d=json.load(open('gpurun_out/ab_tmp.json')); r=d['roofline']; print('$2', $1, round(d['value']/1e6,4), 'Mres/s dev', d['device_resident']['ms'], r['stage_ms'])"; }
for round in 1 2; do
  unset PST_LIB PST_SPLIT_TASKS PST_HALF_TASKS
  run 128 half >> gpurun_out/${TAG}_ab.txt
  PST_LIB=build/var_old/libpst.so run 128 old >> gpurun_out/${TAG}_ab.txt


  run 1024 half_build >> gpurun_out/${TAG}_ab.txt
  PST_LIB=build/var_old/libpst.so run 1024 old >> gpurun_out/${TAG}_ab.txt
done
echo done
