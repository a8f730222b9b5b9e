# k_mpnn_q (persistent half-task queue) vs k_mpnn<L,false>: bitwise tests, then bench A/B
# (interleaved, two rounds) at 1024 and 512 proteins, default pipeline and one chunk.
set -e
TAG=${1:-r04q}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pipeline.py -x -v --timeout 200 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
echo pytest ok
timeout -k 10 600 bash tools/env_ab.sh 1024 - PST_MPNN_QUEUE=1 "PST_H2D_CHUNKS=1" "PST_H2D_CHUNKS=1 PST_MPNN_QUEUE=1" > gpurun_out/${TAG}_ab1024.txt 2>&1
echo ab1024 ok
timeout -k 10 300 bash tools/env_ab.sh 512 - PST_MPNN_QUEUE=1 > gpurun_out/${TAG}_ab512.txt 2>&1
echo done
