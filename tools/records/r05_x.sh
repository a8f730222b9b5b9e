# Round 5: per-wave edge / node time sums of the persistent queue layers at full size
TAG=${1:-r05x}
mkdir -p gpurun_out
export TMPDIR=/tmp
set -e
PST_LIB=ab/qstamp/libpst.so timeout -k 10 300 python -u tools/queue_stamps_probe.py > gpurun_out/${TAG}_qstamps.jsonl 2> gpurun_out/${TAG}_qstamps.err
echo done
