# Round 5: the PDB-files path's all-host route (PST_PDB_GPU_MAX_FILE) and the GPU parse / CLI tests
TAG=${1:-r05u}
mkdir -p gpurun_out
export TMPDIR=/tmp
set -e
timeout -k 10 600 python -u -m pytest tests/test_gpu_pdb_parse.py tests/test_gpu_cli.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
echo done
