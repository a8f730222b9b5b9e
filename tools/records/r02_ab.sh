# GPU tests, then an A/B of the in-tree build against build/var_<name> variants at P proteins.
# usage: bash tools/r02_ab.sh TAG P name1 name2 ...
set -e
TAG=$1; P=$2; shift 2
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
timeout -k 10 600 bash tools/ab_variants.sh $P "$@" > gpurun_out/${TAG}_ab.txt 2>&1
echo done
