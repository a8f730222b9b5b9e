# Round 4: queue unit order (groups of one XCD's wave slots, first halves before second halves) and
# the opaque lane index: queue parity tests, then stage-time A/B at 1024 / 512 / 256 proteins against
# the committed build (ab/libpst_head.so), adjacent halves (PST_MPNN_QGROUP=0), the fused form
# without the queue, and the build with every lane index opaque (ab/libpst_olane.so).
set -e
TAG=${1:-r04h}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_reference_wide.py -x -q --timeout 200 --timeout-method thread -k "queue or fused or reference" > gpurun_out/${TAG}_pytest.log 2>&1
echo pytest ok
for P in 256 512 1024; do
  echo "== $P" >> gpurun_out/${TAG}_ab.txt
  timeout -k 10 900 bash tools/env_ab.sh $P PST_LIB=ab/libpst_head.so - PST_MPNN_QGROUP=0 PST_MPNN_QUEUE=0 PST_LIB=ab/libpst_olane.so >> gpurun_out/${TAG}_ab.txt 2>&1
  echo "$P ok"
done
echo done
