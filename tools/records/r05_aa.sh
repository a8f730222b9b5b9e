# Round 5: decode host side (atom37 host copy on the pool; the binding without zero fills and result
# copies): decode GPU tests, then the decode bench (three shapes)
TAG=${1:-r05aa}
mkdir -p gpurun_out
export TMPDIR=/tmp
set -e
timeout -k 10 600 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_cli.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
echo pytest ok
for s in "--proteins 8 --tokens 256" "--proteins 32 --tokens 128" "--proteins 8 --tokens 512"; do
  timeout -k 10 200 python -u tools/bench_decode.py $s --reps 5 >> gpurun_out/${TAG}_decode.jsonl 2>> gpurun_out/${TAG}_decode.err
done
echo done
