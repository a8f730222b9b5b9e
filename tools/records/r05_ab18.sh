# Round 5: the fold iterations' sidechain half (k_fold_side + the angle normalisation) on a side
# stream beside the next iteration (k_fold_tail keeps the transition, LN and affine update; the
# frame update is its own small kernel): GPU decode tests, then decode A/B vs the previous build
# (prev), alternated twice, and a kernel trace of the new build
TAG=${1:-r05ab18}
mkdir -p gpurun_out
export TMPDIR=/tmp
set -e
timeout -k 10 600 python -u -m pytest tests/test_gpu_decode.py -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
echo tests ok
for i in 1 2; do
  for V in prev new; do
    if [ $V = new ]; then unset PST_LIB; else export PST_LIB=ab/prev/libpst.so; fi
    for S in "8 256" "32 128" "8 512"; do
      set -- $S
      timeout -k 10 200 python -u tools/bench_decode.py --proteins $1 --tokens $2 --reps 5 > gpurun_out/${TAG}_${V}_${1}x${2}_$i.json 2>/dev/null
    done
    echo "$V run $i ok"
  done
done
unset PST_LIB
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_tr -o run -- python -u tools/bench_decode.py --proteins 8 --tokens 256 --reps 3 > /dev/null 2>&1
echo done
