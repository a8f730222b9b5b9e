# 8-wave workgroups with the message MLP's W1 in LDS (build/var_wg8) vs the in-tree build.
set -e
mkdir -p gpurun_out
run() { timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e --steps 10 --warmup 3 --proteins $1 > gpurun_out/ab_tmp.json 2>gpurun_out/ab_err.txt; python -c "import json; d=json.load(open('gpurun_out/ab_tmp.json')); r=d['roofline']; print('$2', $1, round(d['value']/1e6,4), 'dev', d['device_resident']['ms'], r['stage_ms'])"; }
for round in 1 2; do
  unset PST_LIB
  run 1024 base >> gpurun_out/r02_wg8.txt
  PST_LIB=build/var_wg8/libpst.so run 1024 wg8 >> gpurun_out/r02_wg8.txt
  run 128 base >> gpurun_out/r02_wg8.txt
  PST_LIB=build/var_wg8/libpst.so run 128 wg8 >> gpurun_out/r02_wg8.txt
done
echo done
