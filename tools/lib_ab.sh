# Stage times of several libpst builds across batch sizes.
# usage: bash tools/lib_ab.sh "P1 P2 ..." LIB1 LIB2 ...   ("default" = the in-tree build)
set -e
mkdir -p gpurun_out
SIZES=$1; shift
for P in $SIZES; do
  for L in "$@"; do
    if [ "$L" = default ]; then unset PST_LIB; else export PST_LIB=$L; fi
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e --steps 5 --warmup 2 --proteins $P > gpurun_out/ab_tmp.json 2>/dev/null
    python -c "import json; d=json.load(open('gpurun_out/ab_tmp.json')); r=d['roofline']; print($P, '$L'.split('/')[-2] if '/' in '$L' else '$L', d['ms_per_step'], r['stage_ms'])"
  done
done
