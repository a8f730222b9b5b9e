# Round 5: one-round MPNN layers (N = 8 share, 128 proteins) with the second wave slot of each SIMD
# started late (tools/variants/desync.patch, DESYNC_SLEEPS x s_sleep(127)), alternated twice
TAG=${1:-r05o}
mkdir -p gpurun_out
export TMPDIR=/tmp
set -e
for i in 1 2; do
  for D in 0 7 14; do
    PST_LIB=ab/desync$D/libpst.so timeout -k 10 300 python -u bench.py --proteins 128 --no-cpu-baseline --no-e2e > gpurun_out/${TAG}_d${D}_$i.json 2>/dev/null
    echo "d=$D run $i ok"
  done
done
