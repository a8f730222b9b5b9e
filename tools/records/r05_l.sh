# Round 5: GPU PDB scan with the lines / kinds pass fused and prefetched: parity tests, wall time,
# device timeline, per-phase stamps (ab/pdbstamp from tools/pdb_stamps_build.py)
set -e
TAG=${1:-r05l}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_pdb_parse.py tests/test_gpu_cli.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
echo pytest ok
timeout -k 10 200 python -u tools/pdb_files_probe.py --reps 30 > gpurun_out/${TAG}_probe.json
PST_LIB=ab/pdbstamp/libpst.so timeout -k 10 200 python -u tools/pdb_stamp_probe.py > gpurun_out/${TAG}_stamps.txt 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/${TAG}_tl -o run -- python tools/pdb_files_probe.py --reps 10 > gpurun_out/${TAG}_tl.log 2>&1
python tools/pdb_files_timeline.py gpurun_out/${TAG}_tl > gpurun_out/${TAG}_timeline.txt
echo done
