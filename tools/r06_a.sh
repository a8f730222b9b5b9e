# Round 6, first pass: the new no-coordinate PDB tests, the full GPU suite, the default bench line.
# usage: bash tools/r06_a.sh TAG
set -e
TAG=${1:-r06a}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_pdb_parse.py -x -v --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pdb.log 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
timeout -k 10 400 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
echo done
