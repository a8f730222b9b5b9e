# Round 5: full GPU suite + smoke on the current tree
TAG=${1:-r05s}
mkdir -p gpurun_out
export TMPDIR=/tmp
set -e
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
echo pytest ok
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
echo done
timeout -k 10 400 python -u bench.py --gpus 2 --dist-backend gloo --no-cpu-baseline --no-e2e --steps 5 > gpurun_out/${TAG}_gloo2.json 2> gpurun_out/${TAG}_gloo2.err
echo gloo ok
