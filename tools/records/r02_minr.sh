# Pipeline threshold (PST_H2D_MIN_ROUNDS) at 2- and 3-round batches.
set -e
mkdir -p gpurun_out
run() { timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e --steps 15 --warmup 3 --proteins $1 > gpurun_out/ab_tmp.json 2>gpurun_out/ab_err.txt; python -c "import json; d=json.load(open('gpurun_out/ab_tmp.json')); print('$2', $1, d['ms_per_step'], round(d['value']/1e6,4), 'dev', d['device_resident']['ms'])"; }
for round in 1 2 3; do
  for P in 256 384; do
    unset PST_H2D_MIN_ROUNDS
    run $P min4 >> gpurun_out/r02_minr.txt
    PST_H2D_MIN_ROUNDS=2 run $P min2 >> gpurun_out/r02_minr.txt
  done
done
echo done
