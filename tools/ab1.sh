# one round over the library variants given as args
set -e
mkdir -p gpurun_out
for lib in "$@"; do
  PST_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --steps 5 --warmup 1 > gpurun_out/ab_tmp.json 2>/dev/null
  python -c "import json,sys; d=json.load(open('gpurun_out/ab_tmp.json')); r=d['roofline']; print('$lib'.split('/')[-1], round(d['value']/1e6,3), 'Mres/s', r['stage_ms'])"
done
