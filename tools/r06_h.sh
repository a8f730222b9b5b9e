# Round 6: the randomised GPU parity sweep widened to 256 seeds (tests/test_gpu_fuzz.py, PST_FUZZ_SEEDS).
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
PST_FUZZ_SEEDS=256 timeout -k 10 1100 python -u -m pytest tests/test_gpu_fuzz.py -v --timeout 120 --timeout-method thread > gpurun_out/r06h_fuzz.log 2>&1
echo done
