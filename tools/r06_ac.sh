# Round 6: bench.py with the device-resident timed region (value) and the host-to-host step beside it:
# full size and the N = 8 share.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-e2e > gpurun_out/r06ac_full.json 2> gpurun_out/r06ac_full.err
timeout -k 10 300 python -u bench.py --proteins 128 --steps 10 --warmup 3 --no-cpu-baseline --no-e2e > gpurun_out/r06ac_share.json 2> gpurun_out/r06ac_share.err
echo done
