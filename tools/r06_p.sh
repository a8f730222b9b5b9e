# Round 6: layer 0's message chain start from the per-(receiver, sender) pair table (L0_PAIR_TABLE,
# one gathered row per edge instead of three tables and two adds): GPU suite on the new build, then
# interleaved stage times against the previous build (ab/l0base).
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06p_pytest.txt 2>&1
for R in 1 2 3; do
  timeout -k 10 900 bash tools/lib_ab.sh "1024 128" $PWD/ab/l0base/libpst.so default >> gpurun_out/r06p_ab.txt
done
echo done
