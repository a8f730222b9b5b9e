set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r03dtr}
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_decode.py -k "graph or ipa" > gpurun_out/${TAG}_pytest.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/${TAG}_trace -o run -- python tools/bench_decode.py --proteins 8 --tokens 256 --reps 3 > gpurun_out/${TAG}_trace.log 2>&1
PST_DECODE_NO_GRAPH=1 timeout -k 10 120 python -u tools/bench_decode.py --proteins 8 --tokens 256 --reps 10 > gpurun_out/${TAG}_nograph.json
timeout -k 10 120 python -u tools/bench_decode.py --proteins 8 --tokens 256 --reps 10 > gpurun_out/${TAG}_graph.json
echo done
