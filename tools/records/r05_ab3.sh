# Round 5: decode A/B, 8 x 256: IPA output projection K slices (16 in-tree, 10, 8) and k_ipa_attn's
# attention rows in dynamic LDS sized to the group's longest protein (dynatt; dynatt8u1 also caps it
# at 64 VGPRs for 8 waves/SIMD); alternated twice, then one kernel trace per variant
TAG=${1:-r05ab3}
mkdir -p gpurun_out
export TMPDIR=/tmp
set -e
for i in 1 2; do
  for V in base dec_s10 dec_s8 dec_dynatt dec_dynatt8u1; do
    if [ $V = base ]; then unset PST_LIB; else export PST_LIB=ab/$V/libpst.so; fi
    timeout -k 10 200 python -u tools/bench_decode.py --proteins 8 --tokens 256 --reps 5 > gpurun_out/${TAG}_${V}_$i.json 2>/dev/null
    echo "$V run $i ok"
  done
done
for V in base dec_s10 dec_s8 dec_dynatt dec_dynatt8u1; do
  if [ $V = base ]; then unset PST_LIB; else export PST_LIB=ab/$V/libpst.so; fi
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_tr_$V -o run -- python -u tools/bench_decode.py --proteins 8 --tokens 256 --reps 3 > /dev/null 2>&1
  echo "$V trace ok"
done
