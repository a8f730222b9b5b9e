# Round 5: independent proteins on concurrent contexts / streams (tools/two_ctx_probe.py): the N = 8
# share (128 proteins) and 256 / 1 024 proteins, one context vs K contexts from K host threads
TAG=${1:-r05ab6}
mkdir -p gpurun_out
export TMPDIR=/tmp
set -e
for P in 128 256; do
  timeout -k 10 200 python -u tools/two_ctx_probe.py --proteins $P --ks 1,2,3,4 --reps 10 > gpurun_out/${TAG}_$P.jsonl 2>&1
  echo "$P ok"
done
timeout -k 10 200 python -u tools/two_ctx_probe.py --proteins 1024 --ks 1,2 --reps 6 > gpurun_out/${TAG}_1024.jsonl 2>&1
echo done
