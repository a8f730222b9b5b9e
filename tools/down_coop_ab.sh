# Downsampler stage time, k_down<1> (PST_DOWN_COOP=0) vs k_down_coop (PST_DOWN_COOP=1000000),
# across batch sizes (256-residue proteins, 8 tiles each).
set -e
mkdir -p gpurun_out
for P in 8 32 64 128 256 512; do
  for C in 0 1000000; do
    PST_DOWN_COOP=$C timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e --steps 5 --warmup 2 --proteins $P > gpurun_out/dc_tmp.json 2>/dev/null
    python -c "import json; d=json.load(open('gpurun_out/dc_tmp.json')); r=d['roofline']; print($P, 'proteins coop<=', $C, 'down', r['stage_ms']['down'], 'ms total', d['ms_per_step'])"
  done
done
