# Layer 0 as two waves per task at 3 waves/SIMD (build/var_l0h3, PST_HALF_L0=1) vs the default.
set -e
mkdir -p gpurun_out
run() { timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e --steps 10 --warmup 3 --proteins $1 > gpurun_out/ab_tmp.json 2>gpurun_out/ab_err.txt; python -c "import json; d=json.load(open('gpurun_out/ab_tmp.json')); r=d['roofline']; print('$2', $1, round(d['value']/1e6,4), 'dev', d['device_resident']['ms'], r['stage_ms'])"; }
for round in 1 2; do
  unset PST_LIB PST_HALF_L0
  run 1024 base >> gpurun_out/r02_l0h3.txt
  PST_HALF_L0=1 run 1024 half2 >> gpurun_out/r02_l0h3.txt
  PST_LIB=build/var_l0h3/libpst.so PST_HALF_L0=1 run 1024 half3 >> gpurun_out/r02_l0h3.txt
  PST_LIB=build/var_l0h3/libpst.so run 128 half3_128 >> gpurun_out/r02_l0h3.txt
  run 128 base_128 >> gpurun_out/r02_l0h3.txt
done
echo done
