# Round 5: N = 8 share host path, kernel + memory-copy timeline, dense vs packed wire format
TAG=${1:-r05w}
mkdir -p gpurun_out
export TMPDIR=/tmp
set -e
for D in 1 0; do
  PST_H2D_DENSE=$D timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/${TAG}_d$D -o run -- python tools/share_timeline_probe.py > gpurun_out/${TAG}_d$D.log 2>&1
  python tools/pdb_files_timeline.py gpurun_out/${TAG}_d$D > gpurun_out/${TAG}_d${D}_timeline.txt
  echo "dense=$D ok"
done
