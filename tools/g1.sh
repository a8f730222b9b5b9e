set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_reference_wide.py tests/test_gpu_decode.py "tests/test_gpu_cli.py::test_cli_casp14" > gpurun_out/g1_pytest.log 2>&1
timeout -k 10 300 python -u tools/pcie_probe.py > gpurun_out/g1_probe.json 2> gpurun_out/g1_probe.err
echo done
