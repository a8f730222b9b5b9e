# Round 5: deeper weight-load ring in the cooperative block GEMMs (PST_COOP_DEPTH 16 -> 32 / 48: the
# one-round pair node update, k_mpnn_node_coop, k_down_coop / k_down_pair), N = 8 share + CASP14 device
TAG=${1:-r05r}
mkdir -p gpurun_out
export TMPDIR=/tmp
set -e
for i in 1 2; do
  for V in base coop32 coop48; do
    if [ $V = base ]; then unset PST_LIB; else export PST_LIB=ab/$V/libpst.so; fi
    timeout -k 10 300 python -u bench.py --proteins 128 --no-cpu-baseline --no-e2e > gpurun_out/${TAG}_${V}_$i.json 2>/dev/null
    timeout -k 10 200 python -u tools/prof_casp14.py --reps 30 > gpurun_out/${TAG}_${V}_casp_$i.json 2>/dev/null
    echo "$V run $i ok"
  done
done
