# The N = 8 share of config 3 (128 proteins x 256 residues on one GPU): bench line, then a
# kernel + memory-copy trace of the host-path loop for the timeline (tools/timeline.py).
set -e
TAG=${1:-r03share}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --proteins 128 --no-cpu-baseline --no-e2e > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/${TAG}_trace -o run -- python bench.py --proteins 128 --steps 5 --warmup 2 --no-cpu-baseline --no-e2e > gpurun_out/${TAG}_trace.log 2>&1
echo done
