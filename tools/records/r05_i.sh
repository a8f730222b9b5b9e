# Round 5: k_mpnn_range (split-regime batches as receiver ranges per wave): schedule parity, then
# CASP14 device-resident (tools/prof_casp14.py) and small bench sizes, range vs edge/seg_sum, alternated
set -e
TAG=${1:-r05i}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pdb_parse.py -m gpu -x -v --timeout 300 --timeout-method thread -k "fused_and_split or node_coop or casp14 or fast_path" > gpurun_out/${TAG}_pytest.log 2>&1
echo pytest ok
for i in 1 2; do
  for R in 0 auto; do
    if [ $R = auto ]; then unset PST_MPNN_RANGE; else export PST_MPNN_RANGE=$R; fi
    timeout -k 10 200 python -u tools/prof_casp14.py --reps 30 > gpurun_out/${TAG}_casp_r${R}_$i.json 2>/dev/null
    for P in 16 64; do
      timeout -k 10 200 python -u bench.py --proteins $P --steps 10 --warmup 3 --no-cpu-baseline --no-e2e > gpurun_out/${TAG}_p${P}_r${R}_$i.json 2>/dev/null
    done
    echo "range=$R run $i ok"
  done
done
unset PST_MPNN_RANGE
for W in 6 8 16; do
  PST_MPNN_RANGE=$W timeout -k 10 200 python -u tools/prof_casp14.py --reps 30 > gpurun_out/${TAG}_casp_w$W.json 2>/dev/null
done
echo done
