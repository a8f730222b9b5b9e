# Round 4: wave-slot occupancy of the MPNN launches (bench roofline.wave_slot_occupancy) at 1024 /
# 256 / 128 proteins on the current build.
set -e
TAG=${1:-r04j}
mkdir -p gpurun_out
export TMPDIR=/tmp
for P in 1024 256 128; do
  timeout -k 10 300 python -u bench.py --proteins $P --no-cpu-baseline --no-e2e > gpurun_out/${TAG}_$P.json 2> gpurun_out/${TAG}_$P.err
  python -c "import json; d=json.load(open('gpurun_out/${TAG}_$P.json')); r=d['roofline']; print($P, d['value'], d['ms_per_step'], r['stage_ms'], r['wave_slot_occupancy'], d['pipeline_plan']['schedules'])"
done
