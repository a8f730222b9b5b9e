# Round 6: two-halves schedule A/B at the N = 8 share (+ parity of the halves vs one stream).
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/two_halves_ab.py --proteins 128 96 160 64 > gpurun_out/r06b_two_halves.jsonl 2> gpurun_out/r06b_two_halves.err
echo done
