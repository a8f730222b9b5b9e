# Two-waves-per-task tail launch (PST_HALF_TAIL) A/B, after the GPU suite.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02tail_pytest.log 2>&1
run() { timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e --steps 15 --warmup 3 --proteins $1 > gpurun_out/ab_tmp.json 2>gpurun_out/ab_err.txt; python -c "import json; d=json.load(open('gpurun_out/ab_tmp.json')); r=d['roofline']; print('$2', $1, d['ms_per_step'], round(d['value']/1e6,4), 'dev', d['device_resident']['ms'], r['stage_ms'])"; }
for round in 1 2; do
  for P in 1024 960 384; do
    unset PST_HALF_TAIL
    run $P tail >> gpurun_out/r02_tail.txt
    PST_HALF_TAIL=0 run $P notail >> gpurun_out/r02_tail.txt
  done
done
echo done
