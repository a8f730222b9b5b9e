# A/B libpst variants (build/var_<name>/libpst.so from tools/build_variant.sh) against the
# in-tree build on a reduced bench; two interleaved rounds.
# usage: bash tools/ab_variants.sh PROTEINS name1 name2 ...
set -e
mkdir -p gpurun_out
P=$1; shift
for round in 1 2; do
  for v in base "$@"; do
    if [ $v = base ]; then unset PST_LIB; else export PST_LIB=build/var_$v/libpst.so; fi
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e --steps 5 --warmup 2 --proteins $P > gpurun_out/ab_tmp.json 2>gpurun_out/ab_err.txt
    python -c "import json; d=json.load(open('gpurun_out/ab_tmp.json')); r=d['roofline']; print('$v', round(d['value']/1e6,4), 'Mres/s', r['stage_ms'])"
  done
done
