# Round 6: per-kernel decode breakdown at 8 x 256 on the current build (rocprofv3 kernel trace).
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06v_dec -o run -- python tools/bench_decode.py --proteins 8 --tokens 256 --reps 5 > gpurun_out/r06v_dec.log 2>&1
echo done
