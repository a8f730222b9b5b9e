# Round 5 (wave-priority build): layer 0 at full size as the half-task queue (PST_MPNN_QUEUE_LAYERS=7)
# vs k_mpnn<0, false> (default mask 6); bench.py stage times, alternated 3 times
TAG=${1:-r05ab16}
mkdir -p gpurun_out
export TMPDIR=/tmp
set -e
for i in 1 2 3; do
  for V in def q7; do
    unset PST_MPNN_QUEUE_LAYERS
    if [ $V = q7 ]; then export PST_MPNN_QUEUE_LAYERS=7; fi
    timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-e2e > gpurun_out/${TAG}_${V}_$i.json 2> gpurun_out/${TAG}_${V}_$i.err
    echo "$V $i ok"
  done
done
