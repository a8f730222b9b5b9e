# k_mpnn one-wave workgroups (PST_MPNN_SOLO bit mask, default 7) vs four-wave workgroups, plus the
# decode after the k_sc_geom / k_zero fusions: parity tests, bench A/B at 1 024 proteins, decode
# throughput.
set -e
TAG=${1:-r03solo}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_decode.py -x -v --timeout 200 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
bash tools/env_ab.sh 1024 "PST_MPNN_SOLO=0" "-" "PST_MPNN_SOLO=6" > gpurun_out/${TAG}_ab.txt 2>&1
for i in 1 2; do timeout -k 10 120 python -u tools/bench_decode.py --proteins 8 --tokens 256 --reps 5 >> gpurun_out/${TAG}_decode.jsonl; done
echo done
