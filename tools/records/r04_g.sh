# Round 4: decode with k_fold_tail on 12 waves: decode tests, A/B vs the separate launches, trace.
set -e
TAG=${1:-r04g}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
echo pytest ok
for r in 1 2; do
  for v in 0 1; do
    for shape in "8 256" "32 128" "8 512"; do
      set -- $shape
      if [ $v = 1 ]; then export PST_DECODE_UNFUSED_TAIL=1; else unset PST_DECODE_UNFUSED_TAIL; fi
      timeout -k 10 120 python tools/bench_decode.py --proteins $1 --tokens $2 --reps 5 | sed "s/^/unfused_tail=$v /" >> gpurun_out/${TAG}_decode_ab.txt
    done
  done
done
unset PST_DECODE_UNFUSED_TAIL
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_decprof -o run -- python tools/bench_decode.py --proteins 8 --tokens 256 --reps 5 > gpurun_out/${TAG}_decprof.log 2>&1
echo done
