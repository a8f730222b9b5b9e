# Round 5: kernel trace of the N = 8 share (128 proteins, host buffers) on the wave-priority build
TAG=${1:-r05ab14}
mkdir -p gpurun_out
export TMPDIR=/tmp
set -e
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_share -o run -- python tools/share_timeline_probe.py --proteins 128 --reps 20 > gpurun_out/${TAG}_share.log 2>&1
echo done
