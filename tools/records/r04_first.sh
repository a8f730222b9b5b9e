# Round 4, first GPU pass: the whole GPU suite, the default bench line (clock, 128-protein
# reference sample, config-2 CPU baseline), and a kernel-trace summary of a short bench run.
set -e
TAG=${1:-r04a}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
echo pytest ok
timeout -k 10 400 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
echo bench ok
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-e2e > gpurun_out/${TAG}_prof.log 2>&1
echo done
