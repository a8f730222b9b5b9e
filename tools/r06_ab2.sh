# Round 6: kernel + memory-copy timeline of the N = 8 share (128 proteins) host-to-host steps.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/r06ab2_tl -o run -- python bench.py --proteins 128 --steps 6 --warmup 2 --no-cpu-baseline --no-e2e > gpurun_out/r06ab2.log 2>&1
echo done
