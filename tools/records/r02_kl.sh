# Message-MLP W1 fragments partly in LDS (W1_LDS_KSTEPS: in-tree 32, variants 0 / 16 / 40), after the GPU suite.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02kl_pytest.log 2>&1
timeout -k 10 700 bash tools/ab_variants.sh 1024 kl0 > gpurun_out/r02_kl.txt 2>&1
echo done
