# Round 4: IPA projections on transposed weights (k_gemm_mfma_t): decode GPU tests, then interleaved
# A/B against the row-major k_gemm_mfma (PST_DECODE_GEMM_T=0) and the 8-k trip build, and a trace.
set -e
TAG=${1:-r04l}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_decode.py -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
echo pytest ok
for r in 1 2; do
  for v in - PST_DECODE_GEMM_T=0 PST_LIB=ab/libpst_gt8.so; do
    for shape in "8 256" "32 128"; do
      set -- $shape
      if [ "$v" = "-" ]; then envs=""; else envs="$v"; fi
      env $envs timeout -k 10 120 python tools/bench_decode.py --proteins $1 --tokens $2 --reps 5 | sed "s|^|$v |" >> gpurun_out/${TAG}_ab.txt
    done
  done
done
echo ab ok
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_decprof -o run -- python tools/bench_decode.py --proteins 8 --tokens 256 --reps 5 > gpurun_out/${TAG}_decprof.log 2>&1
echo done
