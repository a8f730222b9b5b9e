set -e
TAG=${1:-aux}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/${TAG}_pytest.log 2>&1
timeout -k 10 300 python tools/bench_aux.py > gpurun_out/${TAG}_bench_aux.json 2>gpurun_out/${TAG}_bench_aux.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_auxprof -o run -- python tools/bench_aux.py --reps 5 > gpurun_out/${TAG}_auxprof.log 2>&1
bash tools/pmc_traffic.sh ${TAG}_traffic
echo done
