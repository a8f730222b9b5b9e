# Round 6: later pipeline chunks' graphs on a side stream (PST_GRAPH_STREAM=1): the GPU suite and the
# bench's exact-match check with it on, then an interleaved host-to-host A/B against it off.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
export PST_GRAPH_STREAM=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06o_pytest.txt 2>&1
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/r06o_bench_on.json
unset PST_GRAPH_STREAM
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/r06o_bench_off.json
timeout -k 10 600 python tools/env_ab_tokens.py --env PST_GRAPH_STREAM --values 0 1 --proteins 1024 512 --rounds 7 > gpurun_out/r06o_ab.txt
echo done
