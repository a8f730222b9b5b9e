# Round 4: decode — wide-K GEMM accumulators per wave (PST_DECODE_WIDE_NACC 1/2/4) and the pinned
# atom37 staging; decode tests first.
set -e
TAG=${1:-r04f}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
PST_DECODE_WIDE_NACC=4 timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py -x -q --timeout 200 --timeout-method thread -k "reference or mfma" >> gpurun_out/${TAG}_pytest.log 2>&1
echo pytest ok
for r in 1 2; do
  for n in 1 2 4; do
    for shape in "8 256" "32 128"; do
      set -- $shape
      PST_DECODE_WIDE_NACC=$n timeout -k 10 120 python tools/bench_decode.py --proteins $1 --tokens $2 --reps 5 | sed "s/^/nacc=$n /" >> gpurun_out/${TAG}_decode_ab.txt
    done
  done
done
echo done
