# Round 5: N = 8 share (128 proteins) — in-tree k_mpnn<L, true> vs k_mpnn_pair with stealing off
# (fixed halves in 8-wave workgroups, all of W1 in LDS: ab/pair_fix) and on (ab/pair_steal)
TAG=${1:-r05p}
mkdir -p gpurun_out
export TMPDIR=/tmp
set -e
for i in 1 2; do
  for V in base pair_fix pair_steal; do
    if [ $V = base ]; then unset PST_LIB; else export PST_LIB=ab/$V/libpst.so; fi
    timeout -k 10 300 python -u bench.py --proteins 128 --no-cpu-baseline --no-e2e > gpurun_out/${TAG}_${V}_$i.json 2>/dev/null
    echo "$V run $i ok"
  done
done
