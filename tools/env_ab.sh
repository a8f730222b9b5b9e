# A/B of environment settings on the bench (stage times), two interleaved rounds.
# usage: bash tools/env_ab.sh PROTEINS "NAME=VAL ..." "NAME=VAL ..." ...   ("-" = no extra setting)
set -e
mkdir -p gpurun_out
P=$1; shift
for round in 1 2; do
  for setting in "$@"; do
    if [ "$setting" = "-" ]; then envs=""; else envs="$setting"; fi
    env $envs timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e --steps 5 --warmup 2 --proteins $P > gpurun_out/envab_tmp.json 2>gpurun_out/envab_err.txt
    python -c "import json; d=json.load(open('gpurun_out/envab_tmp.json')); r=d['roofline']; print('$setting', round(d['value']/1e6,4), 'Mres/s', r['stage_ms'])"
  done
done
