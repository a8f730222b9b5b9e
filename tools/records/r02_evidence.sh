# Round-2 evidence: PMC passes on the full bench, the per-GPU share of an 8-GPU strong-scaling run
# (128 proteins), and a 2-rank (gloo, one GPU shared) rehearsal of the multi-rank bench.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/pmc_all.sh r02pmc
python tools/pmc_summary.py gpurun_out/r02pmc_* > gpurun_out/r02_pmc_summary.txt
timeout -k 10 200 python -u bench.py --proteins 128 --no-cpu-baseline --no-e2e > gpurun_out/r02_bench_p128.json 2> gpurun_out/r02_bench_p128.err
timeout -k 10 300 python -u bench.py --gpus 2 --dist-backend gloo --no-cpu-baseline --no-e2e > gpurun_out/r02_bench_gloo2.json 2> gpurun_out/r02_bench_gloo2.err
echo done
