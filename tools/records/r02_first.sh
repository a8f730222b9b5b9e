# First pipelined chunk size / growth (PST_H2D_FIRST_ROUNDS, PST_H2D_GROWTH) at the bench workload.
set -e
mkdir -p gpurun_out
for round in 1 2 3; do
  for fg in "1 8" "1 3" "1 2" "1 1"; do
    set -- $fg
    PST_H2D_FIRST_ROUNDS=$1 PST_H2D_GROWTH=$2 timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e --steps 15 --warmup 3 > gpurun_out/ab_tmp.json 2>gpurun_out/ab_err.txt
    python -c "import json; d=json.load(open('gpurun_out/ab_tmp.json')); print('first=$1 growth=$2', d['ms_per_step'], round(d['value']/1e6,4), 'dev', d['device_resident']['ms'])" >> gpurun_out/r02_first2.txt
  done
done
echo done
