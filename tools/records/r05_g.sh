# Round 5: GPU PDB parse (pst_tokenize_pdb_files): its parity tests, the CLI tests, then the bench
# line (config-2 end-to-end through the GPU parse)
set -e
TAG=${1:-r05g}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
echo pytest ok
timeout -k 10 400 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
echo done
