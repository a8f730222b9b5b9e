# Round 6: ablation — every k_fold_tail / k_transition128 / k_ln_proj2 weight load from the first 16 rows
# (L1-hot; results differ) vs the product, to bound what the decode's per-tile weight stream costs.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
for R in 1 2 3; do
  for L in prod hot; do
    if [ $L = hot ]; then export PST_LIB=$PWD/ab/fthot/libpst.so; else unset PST_LIB; fi
    timeout -k 10 120 python tools/bench_decode.py --proteins 8 --tokens 256 --reps 5 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$L', d['proteins'], d['tokens_per_protein'], d['ms_per_batch'], d['stage_ms'])" >> gpurun_out/r06m_ft_hot.txt
  done
done
echo done
