# Round 6: kernel trace of the two-slot decode (8 x 256) to see how the two streams' kernels overlap.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r06j_trace -o run -- python tools/bench_decode.py --proteins 8 --tokens 256 --reps 3 > gpurun_out/r06j.log 2>&1
echo done
