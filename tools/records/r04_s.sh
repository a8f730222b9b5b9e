# Round 4: the reference sample widened to every 4th headline protein (256 proteins): GPU reference
# tests, then the default bench line (exact_match_reference over 265 proteins).
set -e
TAG=${1:-r04s}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_reference_wide.py -x -v -s --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
echo pytest ok
timeout -k 10 400 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
echo done
