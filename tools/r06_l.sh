# Round 6: the N = 2 launch / rendezvous / sharding path on one card (2 ranks sharing the GPU, gloo for the
# barrier and reductions), as bench.py --gpus 2 spawns it.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py --gpus 2 --dist-backend gloo --no-e2e --cpu-sample 16 > gpurun_out/r06l_gloo2.json 2> gpurun_out/r06l_gloo2.err
echo done
