# k_seg_sum (the split schedule's message gather/scatter, SURVEY north-star "HBM GB/s on the
# scatter") re-measured on the current build: the split-schedule GPU tests, the CASP14 device path
# under --kernel-trace --stats, then PMC passes (FETCH_SIZE; WRITE_SIZE) for the HBM traffic.
set -e
TAG=${1:-r03seg}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_fuzz.py > gpurun_out/${TAG}_pytest.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python tools/prof_casp14.py --reps 20 > gpurun_out/${TAG}_prof.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${TAG}_pmcF -o run -- python tools/prof_casp14.py --reps 5 > gpurun_out/${TAG}_pmcF.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${TAG}_pmcW -o run -- python tools/prof_casp14.py --reps 5 > gpurun_out/${TAG}_pmcW.log 2>&1
python tools/pmc_summary.py gpurun_out/${TAG}_pmcF > gpurun_out/${TAG}_pmcF_summary.txt
python tools/pmc_summary.py gpurun_out/${TAG}_pmcW > gpurun_out/${TAG}_pmcW_summary.txt
echo done
