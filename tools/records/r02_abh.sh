# GPU parity tests on the in-tree build, then an A/B against build/var_head (the last commit).
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-abh}
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_reference_wide.py tests/test_gpu_fuzz.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
for round in 1 2; do
  for v in head cur; do
    if [ $v = head ]; then export PST_LIB=build/var_head/libpst.so; else unset PST_LIB; fi
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e --steps 5 --warmup 2 > gpurun_out/ab_tmp.json 2>gpurun_out/ab_err.txt
    python -c "import json; d=json.load(open('gpurun_out/ab_tmp.json')); r=d['roofline']; print('$v', round(d['value']/1e6,4), 'Mres/s', r['stage_ms'])"
  done
done > gpurun_out/${TAG}_ab.txt
echo done
