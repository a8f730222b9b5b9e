# Round 6: k_gemm_tile without split K (S = 1; PST_GEMM_TILE_SMAX): decode GPU tests, bench_decode A/B, 8 x 256 trace.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k decode > gpurun_out/r06x_pytest.txt 2>&1
for R in 1 2; do
  for V in 0 1; do
    export PST_DECODE_GEMM_TILE=$V
    for S in "8 256" "32 128" "8 512"; do
      set -- $S
      timeout -k 10 120 python tools/bench_decode.py --proteins $1 --tokens $2 --reps 5 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('tile=$V', d['proteins'], d['tokens_per_protein'], d['ms_per_batch'], d['stage_ms'])" >> gpurun_out/r06x_ab.txt
    done
  done
done
export PST_DECODE_GEMM_TILE=1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06x_dec -o run -- python tools/bench_decode.py --proteins 8 --tokens 256 --reps 5 > gpurun_out/r06x_dec.log 2>&1
echo done
