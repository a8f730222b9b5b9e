# GELU as pinned scalar f32 (c_gelu2_sasm, build/var_sasm) vs pinned packed (in-tree): parity tests
# on the variant, then the bench A/B at 1 024 proteins (two interleaved rounds).
set -e
TAG=${1:-r03sasm}
mkdir -p gpurun_out
export TMPDIR=/tmp
PST_LIB=build/var_sasm/libpst.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
bash tools/ab_variants.sh 1024 sasm > gpurun_out/${TAG}_ab.txt 2>&1
echo done
