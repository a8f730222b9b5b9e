# Round 5: k_mpnn_pair (stealing pairs for one-round batches): parity vs the fixed halves, then
# the N = 8 share of config 3 (128 proteins) with PST_MPNN_PAIR 0 / 1, alternated
set -e
TAG=${1:-r05h}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "pair or fused_and_split" > gpurun_out/${TAG}_pytest.log 2>&1
echo pytest ok
for i in 1 2; do
  for PR in 0 1; do
    PST_MPNN_PAIR=$PR timeout -k 10 300 python -u bench.py --proteins 128 --no-cpu-baseline --no-e2e > gpurun_out/${TAG}_p128_pair${PR}_$i.json 2>/dev/null
    echo "pair=$PR run $i ok"
  done
done
