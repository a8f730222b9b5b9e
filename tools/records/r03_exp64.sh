# f64 exp Horner with SGPR coefficients in k_knn's edge features (-DPST_EXP64_SCONST, build/var_exp64)
# vs in-tree: graph/parity tests on the variant, then the bench A/B at 1 024 proteins.
set -e
TAG=${1:-r03exp}
mkdir -p gpurun_out
export TMPDIR=/tmp
PST_LIB=build/var_exp64/libpst.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_cli.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
bash tools/ab_variants.sh 1024 exp64 > gpurun_out/${TAG}_ab.txt 2>&1
echo done
