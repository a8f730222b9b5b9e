set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r03cnt}
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_pipeline.py tests/test_gpu_cli.py tests/test_gpu_parity.py > gpurun_out/${TAG}_pytest.log 2>&1
for i in 1 2; do timeout -k 10 120 python -u tools/share_probe.py --tag counts >> gpurun_out/${TAG}.jsonl; done
timeout -k 10 120 python -u tools/share_probe.py --proteins 1024 --reps 7 --tag counts_1024 >> gpurun_out/${TAG}.jsonl
echo done
