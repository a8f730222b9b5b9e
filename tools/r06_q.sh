# Round 6: layer-0 gather ablations on the pair-table build (timing only, wrong bits): the per-edge
# V row (1), T row (2), feature row (4) or all three (7) read from one hot row.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
for R in 1 2; do
  timeout -k 10 900 bash tools/lib_ab.sh "1024" default $PWD/ab/l0hot1/libpst.so $PWD/ab/l0hot2/libpst.so $PWD/ab/l0hot4/libpst.so $PWD/ab/l0hot7/libpst.so >> gpurun_out/r06q_ab.txt
done
echo done
