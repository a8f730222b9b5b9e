# Round 5: one-round layers (k_mpnn<L, true>) with the node update on the second finisher alone
# (in-workgroup hand-off) vs the pair node update (ab/half_pair = previous build): parity tests,
# then the N = 8 share, alternated
TAG=${1:-r05y}
mkdir -p gpurun_out
export TMPDIR=/tmp
set -e
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pipeline.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
echo pytest ok
for i in 1 2 3; do
  for V in new old; do
    if [ $V = new ]; then unset PST_LIB; else export PST_LIB=ab/half_pair/libpst.so; fi
    timeout -k 10 300 python -u bench.py --proteins 128 --no-cpu-baseline --no-e2e > gpurun_out/${TAG}_${V}_$i.json 2>/dev/null
    echo "$V run $i ok"
  done
done
