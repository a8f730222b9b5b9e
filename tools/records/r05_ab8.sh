# Round 5: graded wave priorities in the one-round fused layers, thresholds (T3, T2, T1): s_setprio 3
# while >= T3 edge blocks remain, 2 while >= T2, 1 while >= T1, else 0; prio8 = (8, 3, 2);
# 128 / 256 proteins, alternated 3 times, tokens compared with the in-tree build
TAG=${1:-r05ab8}
mkdir -p gpurun_out
export TMPDIR=/tmp
set -e
VS="base prio8 p_12_4_2 p_16_8_4 p_6_3_2 p_10_5_2"
for i in 1 2 3; do
  for V in $VS; do
    if [ $V = base ]; then unset PST_LIB; else export PST_LIB=ab/$V/libpst.so; fi
    for P in 128 256; do
      timeout -k 10 120 python -u tools/share_timeline_probe.py --proteins $P --reps 10 --save gpurun_out/${TAG}_${V}_${P}.npy > gpurun_out/${TAG}_${V}_${P}_$i.json 2>&1
    done
    echo "$V $i ok"
  done
done
python - <<PY
import numpy as np
for P in (128, 256):
    b = np.load("gpurun_out/${TAG}_base_%d.npy" % P)
    print(P, {V: bool(np.array_equal(b, np.load("gpurun_out/${TAG}_%s_%d.npy" % (V, P)))) for V in "$VS".split()[1:]})
PY
