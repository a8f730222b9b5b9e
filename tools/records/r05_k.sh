# Round 5: coalesced GPU PDB scan (16-byte separator words, records staged in LDS, keep flags,
# residue types per run, 8 workgroups per file in k_pdb_write): parity tests, then the CASP14
# pst_tokenize_pdb_files wall time and device timeline
set -e
TAG=${1:-r05k}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_pdb_parse.py tests/test_gpu_cli.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
echo pytest ok
timeout -k 10 200 python -u tools/pdb_files_probe.py --reps 30 > gpurun_out/${TAG}_probe.json
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/${TAG}_tl -o run -- python tools/pdb_files_probe.py --reps 10 > gpurun_out/${TAG}_tl.log 2>&1
python tools/pdb_files_timeline.py gpurun_out/${TAG}_tl > gpurun_out/${TAG}_timeline.txt
echo done
