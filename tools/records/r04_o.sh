# Round 4: the first chunk's exposed copy (~0.9 ms of the host-path step, tools/r04_n.sh timeline):
# A/B of two copy streams and of 2 / 8 graph ranges at 1 024 proteins.
set -e
TAG=${1:-r04o}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 800 bash tools/env_ab.sh 1024 - PST_H2D_COPY_STREAMS=2 PST_H2D_GRAPH_RANGES=2 PST_H2D_GRAPH_RANGES=8 "PST_H2D_COPY_STREAMS=2 PST_H2D_GRAPH_RANGES=8" > gpurun_out/${TAG}_ab.txt 2>&1
echo done
