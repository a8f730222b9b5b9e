# Round 5: decode — k_fold_tail / k_transition128 / k_ln_proj2 weight prefetch depth (FT_PF groups of
# 16 k ahead: 4 = in-tree, 8, 12), 8 x 256 decode, alternated twice
TAG=${1:-r05z}
mkdir -p gpurun_out
export TMPDIR=/tmp
set -e
for i in 1 2; do
  for V in base ftpf8 ftpf12; do
    if [ $V = base ]; then unset PST_LIB; else export PST_LIB=ab/$V/libpst.so; fi
    timeout -k 10 200 python -u tools/bench_decode.py --proteins 8 --tokens 256 --reps 5 > gpurun_out/${TAG}_${V}_$i.json 2>/dev/null
    echo "$V run $i ok"
  done
done
