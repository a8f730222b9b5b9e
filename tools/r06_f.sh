# Round 6: layer 0 as the persistent queue (PST_MPNN_QUEUE_LAYERS=7) vs the one-wave form (6, default), with the
# wave priorities in both (round 5 added them after the round-4 A/B), at 1 024 and 512 proteins.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u tools/env_ab_tokens.py --env PST_MPNN_QUEUE_LAYERS --values 6 7 --proteins 1024 512 256 --rounds 8 --reps 5 > gpurun_out/r06f_l0_queue2.jsonl 2> gpurun_out/r06f.err
echo done
