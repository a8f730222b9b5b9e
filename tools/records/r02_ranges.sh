# Graph per copy range of the first chunk: pipeline + parity tests, then the bench at 1024 / 128 /
# 256 proteins with the default 4 ranges and with one copy (PST_H2D_GRAPH_RANGES=1).
# usage: bash tools/r02_ranges.sh TAG
set -e
TAG=${1:-r02g}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_parity.py tests/test_gpu_fuzz.py -x -v --timeout 200 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
for round in 1 2; do
for P in 1024 128 256; do
  for R in 4 1; do
    PST_H2D_GRAPH_RANGES=$R timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-e2e --proteins $P > gpurun_out/${TAG}_tmp.json 2>> gpurun_out/${TAG}_bench.err
    python -c "import json; d=json.load(open('gpurun_out/${TAG}_tmp.json')); print('round $round proteins $P ranges $R', d['ms_per_step'], 'ms', round(d['value']/1e6,4), 'Mres/s; device-resident', d['device_resident']['ms'], 'ms')" >> gpurun_out/${TAG}_ab.txt
  done
done
done
echo done
