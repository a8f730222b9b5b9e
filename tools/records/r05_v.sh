# Round 5: packed host-buffer inputs (pack_rows): pipeline / parity tests, then bench at 128 and
# 1 024 proteins with PST_H2D_DENSE 1 / 0, alternated
TAG=${1:-r05v}
mkdir -p gpurun_out
export TMPDIR=/tmp
set -e
timeout -k 10 900 python -u -m pytest tests/test_gpu_pipeline.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
echo pytest ok
for i in 1 2; do
  for D in 1 0; do
    PST_H2D_DENSE=$D timeout -k 10 300 python -u bench.py --proteins 128 --no-cpu-baseline --no-e2e > gpurun_out/${TAG}_p128_d${D}_$i.json 2>/dev/null
    PST_H2D_DENSE=$D timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-e2e > gpurun_out/${TAG}_p1024_d${D}_$i.json 2>/dev/null
    echo "dense=$D run $i ok"
  done
done
