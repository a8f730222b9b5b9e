# Round 5: wave priority of the node update that follows a task's edge blocks (fused layers and queue
# units): s_setprio 1 (np1) or 3 (np3) vs 0 (in-tree, the last edge block's level); 128 / 256 / 1 024
# proteins, alternated 3 times, tokens compared
TAG=${1:-r05ab11}
mkdir -p gpurun_out
export TMPDIR=/tmp
set -e
VS="base2 np1 np3"
for i in 1 2 3; do
  for V in $VS; do
    export PST_LIB=ab/$V/libpst.so
    for P in 128 256 1024; do
      timeout -k 10 120 python -u tools/share_timeline_probe.py --proteins $P --reps 10 --save gpurun_out/${TAG}_${V}_${P}.npy > gpurun_out/${TAG}_${V}_${P}_$i.json 2>&1
    done
    echo "$V $i ok"
  done
done
python - <<PY
import numpy as np
for P in (128, 256, 1024):
    b = np.load("gpurun_out/${TAG}_base2_%d.npy" % P)
    print(P, {V: bool(np.array_equal(b, np.load("gpurun_out/${TAG}_%s_%d.npy" % (V, P)))) for V in "$VS".split()[1:]})
PY
