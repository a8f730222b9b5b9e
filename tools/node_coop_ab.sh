# MPNN stage times (split schedule), k_mpnn_node (PST_NODE_COOP=0) vs k_mpnn_node_coop (PST_NODE_COOP=1000000),
# across batch sizes (256-residue proteins, 8 tasks each).
set -e
mkdir -p gpurun_out
for P in 8 32 64 128; do
  for C in 0 1000000; do
    PST_NODE_COOP=$C timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e --steps 5 --warmup 2 --proteins $P > gpurun_out/nc_tmp.json 2>/dev/null
    python -c "import json; d=json.load(open('gpurun_out/nc_tmp.json')); r=d['roofline']; print($P, 'proteins coop<=', $C, 'mpnn', [r['stage_ms'][k] for k in ('mpnn0','mpnn1','mpnn2')], 'ms total', d['ms_per_step'])"
  done
done
