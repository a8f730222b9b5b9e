# float32 wire format (pst_tokenize_f32): GPU pipeline tests, then the default bench and the N = 8
# share (128 proteins) with float32 and float64 positions.
# usage: bash tools/r02_f32.sh TAG
set -e
TAG=${1:-r02f}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline.py -x -v --timeout 200 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
for P in 128 256; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-e2e --proteins $P > gpurun_out/${TAG}_p${P}.json 2>> gpurun_out/${TAG}_bench.err
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-e2e --proteins $P --f64-input > gpurun_out/${TAG}_p${P}_f64.json 2>> gpurun_out/${TAG}_bench.err
done
echo done
