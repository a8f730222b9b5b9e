# Decode launch trims (k_affine_update folded into k_sc_geom, no k_zero, query scale in the GEMM
# epilogue, one packed index upload per group) vs the previous build (build/var_head): decode GPU
# tests, then 8 x 256 decode throughput interleaved, three rounds.
set -e
TAG=${1:-r03dec2}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_decode.py -x -v --timeout 200 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
for r in 1 2 3; do
  PST_LIB=build/var_head/libpst.so timeout -k 10 120 python -u tools/bench_decode.py --proteins 8 --tokens 256 --reps 10 | sed 's/^/head /' >> gpurun_out/${TAG}_ab.txt
  timeout -k 10 120 python -u tools/bench_decode.py --proteins 8 --tokens 256 --reps 10 | sed 's/^/new /' >> gpurun_out/${TAG}_ab.txt
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python tools/bench_decode.py --proteins 8 --tokens 256 --reps 5 > gpurun_out/${TAG}_prof.log 2>&1
echo done
