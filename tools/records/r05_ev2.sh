# Round 5 evidence on the final MPNN build (one-round node update hand-off): GPU suite + smoke, the
# default bench line, full-size kernel trace, strong-scaling shares
set -e
TAG=${1:-r05ev2}
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
timeout -k 10 900 bash tools/strong_scaling_shares.sh > gpurun_out/${TAG}_shares.jsonl 2>&1
echo done
