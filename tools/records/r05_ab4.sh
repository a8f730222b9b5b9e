# Round 5: k_ipa_attn with IPA_QB queries per workgroup (one read of each key's rows for all of
# them): the GPU decode tests on the in-tree build (QB 4), then decode A/B vs the round's previous
# build (one query per workgroup) and QB 2 / 8, alternated twice, then kernel traces
TAG=${1:-r05ab4}
mkdir -p gpurun_out
export TMPDIR=/tmp
set -e
timeout -k 10 600 python -u -m pytest tests/test_gpu_decode.py -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
echo tests ok
for i in 1 2; do
  for V in dec_base qb4 ipa_q2 ipa_q8; do
    if [ $V = qb4 ]; then unset PST_LIB; else export PST_LIB=ab/$V/libpst.so; fi
    for S in "8 256" "32 128"; do
      set -- $S
      timeout -k 10 200 python -u tools/bench_decode.py --proteins $1 --tokens $2 --reps 5 > gpurun_out/${TAG}_${V}_${1}x${2}_$i.json 2>/dev/null
    done
    if [ $V != ipa_q8 ]; then
      timeout -k 10 200 python -u tools/bench_decode.py --proteins 8 --tokens 512 --reps 3 > gpurun_out/${TAG}_${V}_8x512_$i.json 2>/dev/null
    fi
    echo "$V run $i ok"
  done
done
for V in dec_base qb4 ipa_q2; do
  if [ $V = qb4 ]; then unset PST_LIB; else export PST_LIB=ab/$V/libpst.so; fi
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_tr_$V -o run -- python -u tools/bench_decode.py --proteins 8 --tokens 256 --reps 3 > /dev/null 2>&1
  echo "$V trace ok"
done
