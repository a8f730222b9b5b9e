# Round 4: host-path timeline of the bench (kernel + memory-copy trace) and an A/B of the first
# pipeline chunk's size (1 round = 128 proteins, default; 2 rounds = 256) at 1 024 proteins.
set -e
TAG=${1:-r04n}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 bash tools/env_ab.sh 1024 - PST_H2D_FIRST_ROUNDS=2 "PST_H2D_FIRST_ROUNDS=2 PST_H2D_GRAPH_RANGES=8" > gpurun_out/${TAG}_ab.txt 2>&1
echo ab ok
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/${TAG}_tl -o run -- python bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-e2e > gpurun_out/${TAG}_tl.log 2>&1
echo done
