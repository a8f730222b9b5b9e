# k_fsq_aux (config 4 aux: CASP14, K = 64 000): in-tree vs the rows written one tensor at a time
# (build/var_auxsplit), interleaved, plus a kernel-trace profile of the in-tree build.
set -e
TAG=${1:-r03aux}
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2; do
  timeout -k 10 120 python -u tools/bench_aux.py --codebook 64000 --reps 20 | sed 's/^/base /' >> gpurun_out/${TAG}_ab.txt
  PST_LIB=build/var_auxsplit/libpst.so timeout -k 10 120 python -u tools/bench_aux.py --codebook 64000 --reps 20 | sed 's/^/split /' >> gpurun_out/${TAG}_ab.txt
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python tools/bench_aux.py --codebook 64000 --reps 20 > gpurun_out/${TAG}_prof.log 2>&1
echo done
