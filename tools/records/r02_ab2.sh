set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
for round in 1 2; do
  for v in head cur; do
    if [ $v = head ]; then export PST_LIB=build/var_head/libpst.so; else unset PST_LIB; fi
    PST_L0_AGG=0 timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e --steps 5 --warmup 2 > gpurun_out/ab_tmp.json 2>gpurun_out/ab_err.txt
    python -c "import json; d=json.load(open('gpurun_out/ab_tmp.json')); r=d['roofline']; print('$v', round(d['value']/1e6,4), 'Mres/s', r['stage_ms'])"
  done
done
