# Final build: pipeline + CLI GPU tests, the per-GPU shares of config 3 (N = 1/2/4/8 on one card),
# and the 2-rank gloo rehearsal of bench.py's spawn path.
set -e
TAG=${1:-r02s}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_cli.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
bash tools/strong_scaling_shares.sh > gpurun_out/${TAG}_shares.jsonl
timeout -k 10 300 python -u bench.py --gpus 2 --dist-backend gloo --no-e2e --steps 10 > gpurun_out/${TAG}_gloo2.json 2> gpurun_out/${TAG}_gloo2.err
echo done
