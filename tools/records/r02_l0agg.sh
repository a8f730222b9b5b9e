set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py -k wide -q -s --timeout 200 --timeout-method thread > gpurun_out/r02g_decwide.log 2>&1 || true
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --deselect tests/test_gpu_decode.py::test_decode_matches_reference_wide > gpurun_out/r02g_pytest.log 2>&1
timeout -k 10 600 bash tools/env_ab.sh 1024 - PST_L0_AGG=0 > gpurun_out/r02g_ab.txt 2>&1
echo done
