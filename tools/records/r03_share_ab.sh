# N = 8 share probes: host vs device path, stage times in both, copy-stream / range variants.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out/${1:-r03shab}.jsonl
timeout -k 10 120 python -u tools/share_probe.py --tag default >> $O
PST_H2D_COPY_STREAMS=2 timeout -k 10 120 python -u tools/share_probe.py --tag copy2 >> $O
PST_H2D_GRAPH_RANGES=1 timeout -k 10 120 python -u tools/share_probe.py --tag ranges1 >> $O
PST_H2D_GRAPH_RANGES=8 PST_H2D_COPY_STREAMS=2 timeout -k 10 120 python -u tools/share_probe.py --tag ranges8_copy2 >> $O
timeout -k 10 120 python -u tools/share_probe.py --tag default_again >> $O
echo done
