# Round 6: split-K k_fold_tail on 16 waves — decode GPU tests, then interleaved A/B of bench_decode against the
# previous build (ab/base = HEAD before the change).
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_decode.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r06k_decode_tests.log 2>&1
for R in 1 2 3; do
  for L in base new; do
    if [ $L = base ]; then export PST_LIB=$PWD/ab/base/libpst.so; else unset PST_LIB; fi
    for S in "8 256" "32 128" "8 512"; do
      set -- $S
      timeout -k 10 120 python tools/bench_decode.py --proteins $1 --tokens $2 --reps 5 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$L', d['proteins'], d['tokens_per_protein'], d['ms_per_batch'], d['stage_ms'])" >> gpurun_out/r06k_decode_ab.txt
    done
  done
done
echo done
