# Round 3: the changed GPU tests (drop-in main, ae fn, pipeline plan, decode), then the default bench.
# usage: bash tools/r03_check.sh TAG [pytest selection...]
set -e
TAG=${1:-r03}
shift || true
SEL=${@:-tests/test_gpu_cli.py tests/test_gpu_pipeline.py tests/test_gpu_decode.py}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread $SEL > gpurun_out/${TAG}_pytest.log 2>&1
timeout -k 10 400 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
echo done
