# Round 5: CASP14 device-resident vs the split schedule's edge-wave target (PST_EDGE_WAVES: about one
# round of multi-block waves instead of ~4.3 rounds of one-block waves), alternated twice
TAG=${1:-r05t}
mkdir -p gpurun_out
export TMPDIR=/tmp
set -e
for i in 1 2; do
  for W in 0 2048 1536 1024; do
    if [ $W = 0 ]; then unset PST_EDGE_WAVES; else export PST_EDGE_WAVES=$W; fi
    timeout -k 10 200 python -u tools/prof_casp14.py --reps 30 > gpurun_out/${TAG}_w${W}_$i.json 2>/dev/null
    echo "w=$W run $i ok"
  done
done
