# ACT_GROUP=8 (four activation chains per 8-k-step group) vs the default 4: parity on the variant
# library, then interleaved bench stage times at 1024 proteins (default pipeline).
set -e
TAG=${1:-r04g}
mkdir -p gpurun_out
export TMPDIR=/tmp
PST_LIB=$PWD/ab/libpst_g8.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
echo pytest ok
timeout -k 10 700 bash tools/lib_ab.sh "1024" default $PWD/ab/libpst_g8.so default $PWD/ab/libpst_g8.so > gpurun_out/${TAG}_ab.txt 2>&1
echo done
