# Round 5: k_ipa_attn phase ablations (timing only, results differ): no z pass / no logits, kernel trace, 8 x 256 decode
TAG=${1:-r05ab2}
mkdir -p gpurun_out
export TMPDIR=/tmp
set -e
for V in base ipa_noz ipa_nologit; do
  if [ $V = base ]; then unset PST_LIB; else export PST_LIB=ab/$V/libpst.so; fi
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_$V -o run -- python -u tools/bench_decode.py --proteins 8 --tokens 256 --reps 5 > gpurun_out/${TAG}_$V.json 2>/dev/null
  echo "$V ok"
done
