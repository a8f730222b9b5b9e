# Round 6: layer 0 features loaded one block ahead (L0_FEAT_PREFETCH): GPU suite on the new build,
# then interleaved stage times against the pair-table build without it (ab/l0pf0).
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06r_pytest.txt 2>&1
for R in 1 2 3; do
  timeout -k 10 900 bash tools/lib_ab.sh "1024 128" $PWD/ab/l0pf0/libpst.so default >> gpurun_out/r06r_ab.txt
done
echo done
