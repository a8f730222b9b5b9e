# Round 5: the N = 8 share's one-round layers as the persistent half-task queue (all three layers,
# 8-wave or 4-wave workgroups) vs the one-round fused form (default), with the wave priorities in
# both; 128 / 256 proteins host to host, alternated 3 times, tokens compared
TAG=${1:-r05ab15}
mkdir -p gpurun_out
export TMPDIR=/tmp
set -e
for i in 1 2 3; do
  for V in def q8 q4; do
    unset PST_HALF_TASKS PST_MPNN_QUEUE PST_MPNN_QUEUE_LAYERS PST_MPNN_QWAVES
    if [ $V != def ]; then export PST_HALF_TASKS=0 PST_MPNN_QUEUE=1 PST_MPNN_QUEUE_LAYERS=7; fi
    if [ $V = q4 ]; then export PST_MPNN_QWAVES=4; fi
    for P in 128 256; do
      timeout -k 10 120 python -u tools/share_timeline_probe.py --proteins $P --reps 10 --save gpurun_out/${TAG}_${V}_${P}.npy > gpurun_out/${TAG}_${V}_${P}_$i.json 2>&1
    done
    echo "$V $i ok"
  done
done
python - <<PY
import numpy as np
for P in (128, 256):
    b = np.load("gpurun_out/${TAG}_def_%d.npy" % P)
    print(P, {V: bool(np.array_equal(b, np.load("gpurun_out/${TAG}_%s_%d.npy" % (V, P)))) for V in ("q8", "q4")})
PY
