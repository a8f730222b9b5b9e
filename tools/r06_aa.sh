# Round 6: kernel + memory-copy timeline of the default bench's host-to-host steps (where the ~1 ms between
# host-to-host and device-resident goes).
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/r06aa_tl -o run -- python bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-e2e > gpurun_out/r06aa.log 2>&1
echo done
