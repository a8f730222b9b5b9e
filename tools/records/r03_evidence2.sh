# Round-3 evidence, part 2: PMC passes over the bench at full size (one counter group per pass; the
# first with the kernel trace, for per-dispatch cycles vs duration), decode throughput at three
# shapes, and the per-GPU shares of config 3 at N = 2 / 4 / 8.
set -e
TAG=${1:-r03f}
mkdir -p gpurun_out
export TMPDIR=/tmp
export PST_H2D_CHUNKS=1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/${TAG}pmc_SQ_WAVES -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/${TAG}pmc_a.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d gpurun_out/${TAG}pmc_SQ_BUSY_CYCLES -o run -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/${TAG}pmc_b.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${TAG}pmc_FETCH_SIZE -o run -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/${TAG}pmc_c.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${TAG}pmc_WRITE_SIZE -o run -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/${TAG}pmc_d.log 2>&1
unset PST_H2D_CHUNKS
python tools/pmc_summary.py gpurun_out/${TAG}pmc_* > gpurun_out/${TAG}_pmc_summary.txt
for shape in "8 256" "32 128" "8 512"; do
  set -- $shape
  timeout -k 10 120 python -u tools/bench_decode.py --proteins $1 --tokens $2 --reps 10 >> gpurun_out/${TAG}_decode.jsonl
done
for P in 512 256 128; do
  timeout -k 10 300 python -u bench.py --proteins $P --no-cpu-baseline --no-e2e > gpurun_out/${TAG}_share_$P.json 2>/dev/null
done
echo done
