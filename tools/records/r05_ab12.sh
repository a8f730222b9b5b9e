# Round 5: layer 0 at full size (k_mpnn<0, false>, 50-block tasks, 4 rounds of waves): wave priorities
# off (l0off) / thresholds x1 (l0s1) / x2 (in-tree, cur); bench stage times, alternated 3 times
TAG=${1:-r05ab12}
mkdir -p gpurun_out
export TMPDIR=/tmp
set -e
for i in 1 2 3; do
  for V in cur l0off l0s1; do
    export PST_LIB=ab/$V/libpst.so
    timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-e2e > gpurun_out/${TAG}_${V}_$i.json 2> gpurun_out/${TAG}_${V}_$i.err
    echo "$V $i ok"
  done
done
