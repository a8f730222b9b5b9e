# Round 5: layer 0 as the queue when its tasks are not whole rounds (policy, in-tree) vs never (prev);
# bench.py at 1 024 (host path: second chunk 896 proteins = 3.5 rounds; device-resident 4 rounds)
# and host-to-host 512 / 640 / 896 proteins; alternated 3 times, tokens compared
TAG=${1:-r05ab17}
mkdir -p gpurun_out
export TMPDIR=/tmp
set -e
for i in 1 2 3; do
  for V in prev new; do
    if [ $V = new ]; then unset PST_LIB; else export PST_LIB=ab/prev/libpst.so; fi
    timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-e2e > gpurun_out/${TAG}_${V}_bench_$i.json 2> gpurun_out/${TAG}_${V}_bench_$i.err
    for P in 512 640 896; do
      timeout -k 10 120 python -u tools/share_timeline_probe.py --proteins $P --reps 8 --save gpurun_out/${TAG}_${V}_${P}.npy > gpurun_out/${TAG}_${V}_${P}_$i.json 2>&1
    done
    echo "$V $i ok"
  done
done
python - <<PY
import numpy as np
for P in (512, 640, 896):
    print(P, np.array_equal(np.load("gpurun_out/${TAG}_prev_%d.npy" % P), np.load("gpurun_out/${TAG}_new_%d.npy" % P)))
PY
