# Round 6: layer 0's edge features in a 32-edge blocked layout (feat_f4: one lane-linear 1 KB load per
# k-step quad instead of 128-byte-strided rows): GPU suite on the new build (blocked + one-block-ahead
# prefetch), then interleaved stage times: ab/l0pf0 (row layout, no prefetch), ab/blkpf0 (blocked, no
# prefetch), default (blocked + prefetch).
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06s_pytest.txt 2>&1
for R in 1 2 3; do
  timeout -k 10 900 bash tools/lib_ab.sh "1024 128" $PWD/ab/l0pf0/libpst.so $PWD/ab/blkpf0/libpst.so default >> gpurun_out/r06s_ab.txt
done
echo done
