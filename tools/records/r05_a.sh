# Round 5, first GPU pass after the product-tree cleanup (k_mpnn_x and the decode A/B switches
# moved to tools/variants/, clock stamps off unless enabled): GPU suite + smoke, bench line,
# decode bench.
set -e
TAG=${1:-r05a}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
echo pytest ok
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
echo smoke ok
timeout -k 10 400 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
echo bench ok
timeout -k 10 300 python -u tools/bench_decode.py > gpurun_out/${TAG}_decode.jsonl 2> gpurun_out/${TAG}_decode.err
echo done
