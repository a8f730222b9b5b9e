# Round 5 evidence on the final build (wave priorities by edge blocks left; decode host-side trims):
# GPU suite + smoke, the default bench line, full-size kernel trace (one chunk), CASP14 kernel trace,
# the decode bench (three shapes, with its k_pair_fused roofline), the strong-scaling shares
set -e
TAG=${1:-r05ev3}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
echo pytest ok
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
echo smoke ok
timeout -k 10 400 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
echo bench ok
PST_H2D_CHUNKS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof1 -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-e2e > gpurun_out/${TAG}_prof1.log 2>&1
echo prof ok
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_casp -o run -- python tools/prof_casp14.py --reps 20 > gpurun_out/${TAG}_casp.log 2>&1
echo casp ok
for s in "--proteins 8 --tokens 256" "--proteins 32 --tokens 128" "--proteins 8 --tokens 512"; do
  timeout -k 10 200 python -u tools/bench_decode.py $s --reps 5 >> gpurun_out/${TAG}_decode.jsonl 2>> gpurun_out/${TAG}_decode.err
done
echo decode ok
timeout -k 10 900 bash tools/strong_scaling_shares.sh > gpurun_out/${TAG}_shares.jsonl 2>&1
echo done
