# Round 5: token ids through a page-locked landing buffer (one sync, host copy on the pool):
# GPU tests of the host-buffer paths, CASP14 pst_tokenize_pdb_files probe, the bench line
set -e
TAG=${1:-r05m}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
echo pytest ok
timeout -k 10 200 python -u tools/pdb_files_probe.py --reps 30 > gpurun_out/${TAG}_probe.json
timeout -k 10 400 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
echo done
