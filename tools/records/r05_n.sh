# Round 5: the headline workload pinned on all 1 024 proteins: the reference-wide GPU tests (every
# mismatch printed), then the bench line (exact_match_reference over 262 144 tokens)
TAG=${1:-r05n}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_reference_wide.py -m gpu -v -s --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
echo "pytest rc $?"
timeout -k 10 400 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
echo "bench rc $?"
