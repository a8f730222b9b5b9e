# Round 6: one-round layers ending at the edge halves + k_mpnn_node_coop (PST_HALF_NODE_COOP) A/B.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/env_ab_tokens.py --env PST_HALF_NODE_COOP --values 0 1 --proteins 128 > gpurun_out/r06e_half_node_coop.jsonl 2> gpurun_out/r06e.err
echo done
