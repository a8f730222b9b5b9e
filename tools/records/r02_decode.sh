# Decode: GPU tests, throughput at three shapes (+ the VALU-GEMM fallback), kernel-trace profile.
set -e
TAG=${1:-r02dec}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_decode.py -x -v --timeout 200 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
timeout -k 10 120 python -u tools/bench_decode.py --proteins 8 --tokens 256 > gpurun_out/${TAG}_bench.jsonl
timeout -k 10 120 python -u tools/bench_decode.py --proteins 32 --tokens 128 >> gpurun_out/${TAG}_bench.jsonl
timeout -k 10 120 python -u tools/bench_decode.py --proteins 8 --tokens 512 >> gpurun_out/${TAG}_bench.jsonl
PST_DECODE_NO_MFMA=1 timeout -k 10 120 python -u tools/bench_decode.py --proteins 8 --tokens 256 >> gpurun_out/${TAG}_bench.jsonl
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python tools/bench_decode.py --proteins 8 --tokens 256 > gpurun_out/${TAG}_prof.log 2>&1
echo done
