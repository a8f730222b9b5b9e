# Round 6: the segment sums' two chains as one packed FMA per edge (SEG_PACKED): GPU suite on the new
# build, then interleaved stage times against the previous build (ab/blk).
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06t_pytest.txt 2>&1
for R in 1 2 3; do
  timeout -k 10 900 bash tools/lib_ab.sh "1024 128" $PWD/ab/blk/libpst.so default >> gpurun_out/r06t_ab.txt
done
echo done
