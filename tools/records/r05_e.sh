# Round 5: GELU tail A/B at 1024 x 256 (interleaved, two rounds): the product (asm final fma +
# s_nop 1), the C-level final fma (ab/v3_cfinal), the pre-doubled-GELU build (ab/44af52d)
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2; do
  timeout -k 10 900 bash tools/lib_ab.sh "1024" default $PWD/ab/v3_cfinal/libpst.so $PWD/ab/44af52d/libpst.so >> gpurun_out/r05e_ab.txt 2>&1
done
echo done
