# H2D policy with the float32 wire format and graph ranges: host-to-host ms at 256 / 512 / 1024
# proteins with the default pipeline (chunks from 2 rounds) vs no chunking (PST_H2D_MIN_ROUNDS=64),
# at 4 and 8 graph ranges; two interleaved rounds.
# usage: bash tools/r02_h2d_policy.sh TAG
set -e
TAG=${1:-r02h}
mkdir -p gpurun_out
export TMPDIR=/tmp
for round in 1 2; do
for P in 256 512 1024; do
  for MR in 2 64; do
    for GR in 4 8; do
      PST_H2D_MIN_ROUNDS=$MR PST_H2D_GRAPH_RANGES=$GR timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-e2e --proteins $P --steps 15 > gpurun_out/${TAG}_tmp.json 2>> gpurun_out/${TAG}_bench.err
      python -c "import json; d=json.load(open('gpurun_out/${TAG}_tmp.json')); print('round $round proteins $P min_rounds $MR ranges $GR', d['ms_per_step'], 'ms', round(d['value']/1e6,4), 'Mres/s; device-resident', d['device_resident']['ms'], 'ms')" >> gpurun_out/${TAG}_ab.txt
    done
  done
done
done
echo done
timeout -k 10 200 python -u tools/casp14_e2e.py > gpurun_out/${TAG}_casp14.txt 2>&1 || true
