# GPU tests, then A/B of the in-tree build vs build/var_old at 1024 and 128 proteins, and a
# CASP14 device-resident probe of both.
set -e
TAG=$1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
timeout -k 10 600 bash tools/ab_variants.sh 1024 old > gpurun_out/${TAG}_ab1024.txt 2>&1
timeout -k 10 600 bash tools/ab_variants.sh 128 old > gpurun_out/${TAG}_ab128.txt 2>&1
echo done
