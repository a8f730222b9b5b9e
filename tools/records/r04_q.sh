# Round 4: libpst-pinned inputs (pst_host_alloc) and the zero-copy first chunk: pipeline GPU tests,
# then A/B at 1 024 and 128 proteins: default (libpst-pinned, zero-copy), copy path on libpst-pinned
# buffers (PST_H2D_ZERO_COPY=0), torch-pinned buffers as in round 3 (PST_BENCH_TORCH_PIN=1).
set -e
TAG=${1:-r04q}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_pipeline.py -x -v --timeout 200 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
echo pytest ok
for P in 1024 128; do
  echo "== $P" >> gpurun_out/${TAG}_ab.txt
  timeout -k 10 700 bash tools/env_ab.sh $P - PST_H2D_ZERO_COPY=0 PST_BENCH_TORCH_PIN=1 >> gpurun_out/${TAG}_ab.txt 2>&1
done
echo done
