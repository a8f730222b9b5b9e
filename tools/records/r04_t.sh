# Round 4: the 2-rank bench spawn path rehearsed on one card (gloo for the timing reductions), and
# the config-4 aux line (CASP14, codebook 64 000) on the final build.
set -e
TAG=${1:-r04t}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --gpus 2 --dist-backend gloo --no-cpu-baseline --no-e2e --steps 5 > gpurun_out/${TAG}_gloo2.json 2> gpurun_out/${TAG}_gloo2.err
echo gloo ok
timeout -k 10 300 python -u tools/bench_aux.py > gpurun_out/${TAG}_aux.json 2> gpurun_out/${TAG}_aux.err
echo done
