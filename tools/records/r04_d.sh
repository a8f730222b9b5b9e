# Round 4 (r04_c.sh without the suite): default bench line, kernel-trace summary of it, and the
# decode A/B of the fused fold tail (k_fold_tail) against the separate launches.
set -e
TAG=${1:-r04c}
mkdir -p gpurun_out
export TMPDIR=/tmp
true

timeout -k 10 400 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
echo bench ok
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
echo decode ok
timeout -k 10 500 bash tools/env_ab.sh 1024 - PST_MPNN_QWAVES=8 - PST_MPNN_QWAVES=8 > gpurun_out/${TAG}_qwaves.txt 2>&1
echo qwaves ok
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-e2e > gpurun_out/${TAG}_prof.log 2>&1
echo done
