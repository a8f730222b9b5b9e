# Round 6: CASP14 df 2 / df 4 reference tests on the GPU (new fixture) + the reference-wide suite.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_reference_wide.py -v -s --timeout 300 --timeout-method thread -k "casp_df or bench_sample or config4 or tokens_equal_reference" > gpurun_out/r06g_refwide.log 2>&1 || true
echo done
