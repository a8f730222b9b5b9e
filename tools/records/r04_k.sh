# Round 4: layers 1-2 as one persistent queue (k_mpnn_x, PST_MPNN_XLAYER=1): the queue parity test
# (includes the joint launch, 4- and 8-wave), then A/B at 1024 / 512 / 256 / 128 proteins.
set -e
TAG=${1:-r04k}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread -k "queue" > gpurun_out/${TAG}_pytest.log 2>&1
echo pytest ok
for P in 1024 512 256; do
  echo "== $P" >> gpurun_out/${TAG}_ab.txt
  timeout -k 10 900 bash tools/env_ab.sh $P - PST_MPNN_XLAYER=1 "PST_MPNN_XLAYER=1 PST_MPNN_QWAVES=4" >> gpurun_out/${TAG}_ab.txt 2>&1
  echo "$P ok"
done
echo "== 128" >> gpurun_out/${TAG}_ab.txt
timeout -k 10 900 bash tools/env_ab.sh 128 - "PST_HALF_TASKS=0 PST_MPNN_XLAYER=1" "PST_HALF_TASKS=0 PST_MPNN_XLAYER=1 PST_MPNN_QWAVES=4" "PST_HALF_TASKS=0" >> gpurun_out/${TAG}_ab.txt 2>&1
echo done
