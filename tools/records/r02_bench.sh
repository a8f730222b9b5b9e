# Default bench (+ stderr progress) and a kernel-trace profile of it.
set -e
TAG=${1:-r02b}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-e2e > gpurun_out/${TAG}_prof.log 2>&1
echo done
