# rocprof summary of back-to-back device-resident steps at full size (steady state)
set -e
TAG=${1:-r03st}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python tools/steady_prof.py --reps 12 > gpurun_out/${TAG}_prof.log 2>&1
echo done
