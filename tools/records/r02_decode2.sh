set -e
TAG=${1:-r02dec5}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_decode.py -x -q -s --timeout 200 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
for s in 8x256 32x128 8x512; do
  P=${s%x*}; T=${s#*x}
  timeout -k 10 120 python -u tools/bench_decode.py --proteins $P --tokens $T >> gpurun_out/${TAG}_bench.jsonl
  PST_DECODE_GEMM_SLICES=1 timeout -k 10 120 python -u tools/bench_decode.py --proteins $P --tokens $T >> gpurun_out/${TAG}_bench.jsonl
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python tools/bench_decode.py --proteins 8 --tokens 256 > gpurun_out/${TAG}_prof.log 2>&1
echo done
