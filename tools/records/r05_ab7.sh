# Round 5: one-round fused layers (k_mpnn<L, true>) with wave priorities that favour the wave with
# more edge blocks left (s_setprio 3 while >= PRIO_TAIL blocks remain, then 2 / 1 / 0), so the two
# waves sharing a SIMD end together; N = 8 share (128) and 256 / 1 024 proteins, alternated 3 times
TAG=${1:-r05ab7}
mkdir -p gpurun_out
export TMPDIR=/tmp
set -e
for i in 1 2 3; do
  for V in base prio4 prio8; do
    if [ $V = base ]; then unset PST_LIB; else export PST_LIB=ab/$V/libpst.so; fi
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
    print(P, {V: bool(np.array_equal(b, np.load("gpurun_out/${TAG}_%s_%d.npy" % (V, P)))) for V in ("prio4", "prio8")})
PY
