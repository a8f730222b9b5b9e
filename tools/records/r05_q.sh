# Round 5: per-wave, per-block stamps of the one-round fused layers at the N = 8 share
TAG=${1:-r05q}
mkdir -p gpurun_out
export TMPDIR=/tmp
set -e
PST_LIB=ab/wstamp/libpst.so timeout -k 10 300 python -u tools/wave_stamps_probe.py > gpurun_out/${TAG}_wstamps.jsonl 2> gpurun_out/${TAG}_wstamps.err
echo done
