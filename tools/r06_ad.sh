# Round 6: the GPU fuzz sweep (random ragged batches, gaps, short proteins, both wire formats; tokens,
# graph and layer outputs bitwise vs the oracle) over 256 seeds on the final build.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
PST_FUZZ_SEEDS=256 timeout -k 10 900 python -u -m pytest tests/test_gpu_fuzz.py -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r06ad_fuzz.txt 2>&1
echo done
