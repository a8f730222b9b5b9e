# Round 4: IPA projections on the LDS-staged GEMM (k_gemm_lds): decode GPU tests, interleaved A/B
# against k_gemm_mfma (PST_DECODE_GEMM_LDS=0) at 8 x 256, 32 x 128, 8 x 512, and a kernel trace.
set -e
TAG=${1:-r04m}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_decode.py -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
echo pytest ok
for r in 1 2; do
  for v in - PST_DECODE_GEMM_LDS=0 PST_LIB=ab/libpst_d2.so; do
    for shape in "8 256" "32 128" "8 512"; do
      set -- $shape
      if [ "$v" = "-" ]; then envs=""; else envs="$v"; fi
      env $envs timeout -k 10 120 python tools/bench_decode.py --proteins $1 --tokens $2 --reps 5 | sed "s|^|$v |" >> gpurun_out/${TAG}_ab.txt
    done
  done
done
echo ab ok
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_decprof -o run -- python tools/bench_decode.py --proteins 8 --tokens 256 --reps 5 > gpurun_out/${TAG}_decprof.log 2>&1
echo done
