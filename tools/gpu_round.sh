# Round-end evidence in one GPU call: full GPU tests, default bench (+ JSON), kernel-trace profile of
# the bench, SURVEY config 5 bench (df 4, codebook 64000, 512-residue proteins).
# usage: bash tools/gpu_round.sh TAG
set -e
TAG=${1:-round}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -q > gpurun_out/${TAG}_pytest.log 2>&1
timeout -k 10 400 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-e2e > gpurun_out/${TAG}_prof.log 2>&1
timeout -k 10 400 python bench.py --codebook 64000 --df 4 --residues 512 --proteins 512 --no-e2e --cpu-sample 64 > gpurun_out/${TAG}_bench_cfg5.json 2> gpurun_out/${TAG}_bench_cfg5.err
echo done
