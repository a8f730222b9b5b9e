# coexec microbenchmark (VALU density sweep) + the multi-group decode test
set -e
TAG=${1:-r03cx4}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 60 ./tools/micro/coexec > gpurun_out/${TAG}_coexec.txt 2>&1
cat gpurun_out/${TAG}_coexec.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py -x -v --timeout 200 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
tail -3 gpurun_out/${TAG}_pytest.log
