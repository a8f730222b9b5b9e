# Round 4: layer 0 as the queue in 4-wave workgroups (W1 k-steps 0-39 in LDS, as k_mpnn<0, false>)
# with the grouped unit order, against the default (layer 0 one wave per task) at 1 024 / 512 proteins.
set -e
TAG=${1:-r04u}
mkdir -p gpurun_out
export TMPDIR=/tmp
for P in 1024 512; do
  echo "== $P" >> gpurun_out/${TAG}_ab.txt
  timeout -k 10 600 bash tools/env_ab.sh $P - "PST_MPNN_QUEUE_LAYERS=7 PST_MPNN_QWAVES_L0=4" PST_MPNN_QUEUE_LAYERS=7 >> gpurun_out/${TAG}_ab.txt 2>&1
done
echo done
