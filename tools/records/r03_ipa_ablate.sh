# k_ipa_attn phase ablations (timing only): decode 8 x 256 with the in-tree build and with the
# value sums / logits / pair sums removed (build/var_*: tools/build_variant.sh).
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out/${1:-r03ipa}.txt
for round in 1 2; do
  for v in base novals nolog nopair; do
    if [ $v = base ]; then unset PST_LIB; else export PST_LIB=build/var_$v/libpst.so; fi
    echo "$v $(timeout -k 10 120 python tools/bench_decode.py --proteins 8 --tokens 256 --reps 10)" >> $O
  done
done
echo done
