# HBM traffic of k_mpnn<1> at the full bench size: one rocprofv3 --pmc pass per counter
# (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950), kernel-trace only.
# usage: bash tools/pmc_traffic.sh TAG   → gpurun_out/TAG_{FETCH_SIZE,WRITE_SIZE}/
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-traffic}
export PST_H2D_CHUNKS=1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 400 rocprofv3 --pmc $c --output-format csv -d gpurun_out/${TAG}_$c -o run -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_$c.log 2>&1
done
echo done
