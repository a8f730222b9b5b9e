# Round 5: full-size host-path timeline (1 024 proteins, pinned float32 inputs), kernel + memory-copy trace
TAG=${1:-r05ab}
mkdir -p gpurun_out
export TMPDIR=/tmp
set -e
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/${TAG}_tl -o run -- python tools/share_timeline_probe.py --proteins 1024 --reps 6 > gpurun_out/${TAG}_tl.log 2>&1
python tools/pdb_files_timeline.py gpurun_out/${TAG}_tl > gpurun_out/${TAG}_timeline.txt
echo done
