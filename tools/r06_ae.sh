# Round 6: the multi-rank bench path with the device-resident timed loop, rehearsed as 2 ranks sharing
# the one GPU over gloo (the driver's 8-GPU run uses RCCL, one GPU per rank).
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py --gpus 2 --dist-backend gloo --no-e2e --cpu-sample 16 > gpurun_out/r06ae_gloo2.json 2> gpurun_out/r06ae_gloo2.err
echo done
