# Round 6: decode on two slots (concurrent groups) — decode GPU tests, then interleaved A/B of bench_decode
# against PST_DECODE_ONE_SLOT=1 (one slot, the round-5 schedule) at the three decode shapes.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_decode.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r06i_decode_tests.log 2>&1
for R in 1 2 3; do
  for L in one two; do
    if [ $L = one ]; then export PST_DECODE_ONE_SLOT=1; else unset PST_DECODE_ONE_SLOT; fi
    for S in "8 256" "32 128" "8 512"; do
      set -- $S
      timeout -k 10 120 python tools/bench_decode.py --proteins $1 --tokens $2 --reps 5 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$L', d['proteins'], d['tokens_per_protein'], d['ms_per_batch'])" >> gpurun_out/r06i_decode_ab.txt
    done
  done
done
echo done
