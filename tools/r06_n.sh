# Round 6: the two-slot decode variant with direct launches (PST_DECODE_NO_GRAPH=1): does hipGraphLaunch
# serialise the two slots? one slot / two slots x graph / direct, bench_decode 8 x 256 and 32 x 128.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
export PST_LIB=$PWD/ab/twoslot/libpst.so
for R in 1 2; do
  for G in graph direct; do
    if [ $G = direct ]; then export PST_DECODE_NO_GRAPH=1; else unset PST_DECODE_NO_GRAPH; fi
    for L in one two; do
      if [ $L = one ]; then export PST_DECODE_ONE_SLOT=1; else unset PST_DECODE_ONE_SLOT; fi
      for S in "8 256" "32 128"; do
        set -- $S
        timeout -k 10 120 python tools/bench_decode.py --proteins $1 --tokens $2 --reps 5 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$G', '$L', d['proteins'], d['tokens_per_protein'], d['ms_per_batch'])" >> gpurun_out/r06n.txt
      done
    done
  done
done
echo done
