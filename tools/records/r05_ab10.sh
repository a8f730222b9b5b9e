# Round 5: tail_prio in the split schedule's edge kernel (k_mpnn_edge, blocks_per_wave blocks per
# wave) vs the in-tree build: CASP14 resident (prof_casp14), CASP14 files end to end
# (pdb_files_probe), 16 / 64 proteins host to host; alternated 3 times, tokens compared
TAG=${1:-r05ab10}
mkdir -p gpurun_out
export TMPDIR=/tmp
set -e
for i in 1 2 3; do
  for V in base2 edgeprio; do
    export PST_LIB=ab/$V/libpst.so
    timeout -k 10 120 python -u tools/prof_casp14.py --reps 30 > gpurun_out/${TAG}_${V}_casp_$i.json 2>&1
    timeout -k 10 120 python -u tools/pdb_files_probe.py > gpurun_out/${TAG}_${V}_files_$i.json 2>&1
    for P in 16 64; do
      timeout -k 10 120 python -u tools/share_timeline_probe.py --proteins $P --reps 20 --save gpurun_out/${TAG}_${V}_${P}.npy > gpurun_out/${TAG}_${V}_${P}_$i.json 2>&1
    done
    echo "$V $i ok"
  done
done
python - <<PY
import numpy as np
for P in (16, 64):
    print(P, np.array_equal(np.load("gpurun_out/${TAG}_base2_%d.npy" % P), np.load("gpurun_out/${TAG}_edgeprio_%d.npy" % P)))
PY
