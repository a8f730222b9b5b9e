# k_down_coop (four waves per 32-token tile) vs k_down<1> (one wave per tile) at the N = 8 / 4
# shares: PST_DOWN_COOP threshold default (0.375 x SIMDs = 384 tiles) vs 1024 / 2048 tiles.
set -e
TAG=${1:-r02d}
mkdir -p gpurun_out
export TMPDIR=/tmp
for round in 1 2; do
for P in 128 256; do
  for T in -1 1024 2048; do
    if [ $T = -1 ]; then unset PST_DOWN_COOP; else export PST_DOWN_COOP=$T; fi
    timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-e2e --proteins $P --steps 15 > gpurun_out/${TAG}_tmp.json 2>> gpurun_out/${TAG}_bench.err
    python -c "import json; d=json.load(open('gpurun_out/${TAG}_tmp.json')); print('round $round proteins $P down_coop $T', d['ms_per_step'], 'ms; device-resident', d['device_resident']['ms'], 'ms; down', d['roofline']['stage_ms']['down'], 'ms')" >> gpurun_out/${TAG}_ab.txt
  done
done
done
unset PST_DOWN_COOP
echo done
