# Round 4: queue on layers 1-2 only (layer 0 as k_mpnn<0, false>): queue parity tests, then A/B at
# 1024 / 512 / 256 proteins: default, queue on all layers, group sizes 128 / 512, the committed build.
set -e
TAG=${1:-r04i}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_reference_wide.py -x -q --timeout 200 --timeout-method thread -k "queue or fused or reference" > gpurun_out/${TAG}_pytest.log 2>&1
echo pytest ok
for P in 1024 512 256; do
  echo "== $P" >> gpurun_out/${TAG}_ab.txt
  timeout -k 10 900 bash tools/env_ab.sh $P - PST_MPNN_QUEUE_LAYERS=7 PST_MPNN_QGROUP=128 PST_MPNN_QGROUP=512 PST_LIB=ab/libpst_head.so >> gpurun_out/${TAG}_ab.txt 2>&1
  echo "$P ok"
done
echo done
