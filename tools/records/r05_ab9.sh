# Round 5: graded wave priorities (tail_prio: s_setprio by edge blocks left) in the one-round fused
# layers only (pr_half), plus the multi-round fused layer 0 (pr_full), plus the queue units
# (pr_queue), all three (in-tree) vs none (dec_base); 128 / 256 / 1 024 proteins, alternated 3 times
TAG=${1:-r05ab9}
mkdir -p gpurun_out
export TMPDIR=/tmp
set -e
VS="base pr_half pr_full pr_queue all"
for i in 1 2 3; do
  for V in $VS; do
    if [ $V = all ]; then unset PST_LIB; elif [ $V = base ]; then export PST_LIB=ab/dec_base/libpst.so; else export PST_LIB=ab/$V/libpst.so; fi
    for P in 128 256 1024; do
      timeout -k 10 120 python -u tools/share_timeline_probe.py --proteins $P --reps 10 --save gpurun_out/${TAG}_${V}_${P}.npy > gpurun_out/${TAG}_${V}_${P}_$i.json 2>&1
    done
    echo "$V $i ok"
  done
done
python - <<PY
import numpy as np
for P in (128, 256, 1024):
    b = np.load("gpurun_out/${TAG}_base_%d.npy" % P)
    print(P, {V: bool(np.array_equal(b, np.load("gpurun_out/${TAG}_%s_%d.npy" % (V, P)))) for V in "$VS".split()[1:]})
PY
