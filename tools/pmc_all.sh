# PMC passes (one counter group per pass, kernel-trace only) over the default bench at full size.
# usage: bash tools/pmc_all.sh TAG  → gpurun_out/TAG_<first counter>/
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-pmc}
# one chunk per host call: every k_mpnn dispatch then has the full 8 192 tasks (per-dispatch averages)
export PST_H2D_CHUNKS=1
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE" "SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES" "FETCH_SIZE" "WRITE_SIZE"; do
  t=$(echo $set | cut -d' ' -f1)
  timeout -k 10 400 rocprofv3 --pmc $set --output-format csv -d gpurun_out/${TAG}_$t -o run -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/${TAG}_$t.log 2>&1
done
echo done
