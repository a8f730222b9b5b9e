# GPU check: GPU tests (stop at first failure), default bench (+ stderr progress), kernel-trace profile.
# usage: bash tools/r02_check.sh TAG
set -e
TAG=${1:-r02a}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
timeout -k 10 500 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
# every dispatch at full size (one H2D chunk), so the per-kernel averages are per-launch figures
PST_H2D_CHUNKS=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-e2e > gpurun_out/${TAG}_prof.log 2>&1
echo done
