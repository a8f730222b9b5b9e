# Round 5: where pst_tokenize_pdb_files' time goes on CASP14 (config 2): wall per call, then the
# device timeline under rocprofv3 (kernel + memory-copy trace)
set -e
TAG=${1:-r05j}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/pdb_files_probe.py --reps 30 > gpurun_out/${TAG}_probe.json
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/${TAG}_tl -o run -- python tools/pdb_files_probe.py --reps 10 > gpurun_out/${TAG}_tl.log 2>&1
python tools/pdb_files_timeline.py gpurun_out/${TAG}_tl > gpurun_out/${TAG}_timeline.txt
echo done
