# Round 6 evidence on the final build: GPU suite + smoke, the default bench line, full-size kernel trace (one
# chunk) and the default bench's kernel trace, PMC passes (traffic + issue counters), config-4 aux, decode bench
# (three shapes), strong-scaling shares, CASP14 kernel trace, the config-5 bench line. PST_HEAD (the commit) comes from the command line.
# usage: PST_HEAD=<commit> bash tools/r06_ev.sh TAG [PYTEST_K]
set -e
TAG=${1:-r06ev}
K=${2:-}
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "$K" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "$K" > gpurun_out/${TAG}_pytest.log 2>&1
else
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
fi
echo pytest ok
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
echo smoke ok
timeout -k 10 400 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
echo bench ok
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-e2e > gpurun_out/${TAG}_prof.log 2>&1
PST_H2D_CHUNKS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof1 -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-e2e > gpurun_out/${TAG}_prof1.log 2>&1
echo prof ok
bash tools/pmc_all.sh ${TAG}_pmc
echo pmc ok
timeout -k 10 300 python tools/bench_aux.py > gpurun_out/${TAG}_bench_aux.json 2> gpurun_out/${TAG}_bench_aux.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_auxprof -o run -- python tools/bench_aux.py --reps 5 > gpurun_out/${TAG}_auxprof.log 2>&1
echo aux ok
for s in "--proteins 8 --tokens 256" "--proteins 32 --tokens 128" "--proteins 8 --tokens 512"; do
  timeout -k 10 200 python -u tools/bench_decode.py $s --reps 5 >> gpurun_out/${TAG}_decode.jsonl 2>> gpurun_out/${TAG}_decode.err
done
echo decode ok
timeout -k 10 900 bash tools/strong_scaling_shares.sh > gpurun_out/${TAG}_shares.jsonl 2>&1
echo shares ok
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_casp -o run -- python tools/prof_casp14.py --reps 20 > gpurun_out/${TAG}_casp.log 2>&1
echo casp ok
timeout -k 10 400 python -u bench.py --codebook 64000 --df 4 --residues 512 --proteins 512 --no-e2e --cpu-sample 32 > gpurun_out/${TAG}_bench_cfg5.json 2> gpurun_out/${TAG}_bench_cfg5.err
echo done
