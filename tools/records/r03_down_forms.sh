# Downsampler forms vs tile count (df 1): one wave per tile, coop (4 waves/tile), pair (2 waves/tile).
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out/${1:-r03df}.jsonl
for P in 16 48 64 96 128 256; do
  PST_DOWN_COOP=0 PST_DOWN_PAIR=0 timeout -k 10 120 python -u tools/share_probe.py --proteins $P --reps 9 --tag "one_wave_$P" >> $O
  PST_DOWN_COOP=1000000 timeout -k 10 120 python -u tools/share_probe.py --proteins $P --reps 9 --tag "coop_$P" >> $O
  PST_DOWN_COOP=0 PST_DOWN_PAIR=1 timeout -k 10 120 python -u tools/share_probe.py --proteins $P --reps 9 --tag "pair_$P" >> $O
done
echo done
