# Round 5: GPU suite on the final GELU / feature-slot / parser build, bench line, CASP14 probe,
# queue-variant diagnostic, and an interleaved A/B against the start-of-round build (ab/44af52d)
set -e
TAG=${1:-r05f}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
echo pytest ok
timeout -k 10 400 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
echo bench ok
timeout -k 10 300 python -u tools/casp14_e2e.py > gpurun_out/${TAG}_casp.json 2> gpurun_out/${TAG}_casp.err
timeout -k 10 300 python -u tools/queue_diag.py > gpurun_out/${TAG}_diag.txt 2>&1
for r in 1 2; do
  timeout -k 10 900 bash tools/lib_ab.sh "1024" default $PWD/ab/44af52d/libpst.so >> gpurun_out/${TAG}_ab.txt 2>&1
done
echo done
