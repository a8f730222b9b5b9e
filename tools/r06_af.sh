# Round 6: PMC passes over the 8 x 256 decode (k_pair_fused, the fold's kernels): issue mix, MFMA busy,
# wait cycles, LDS and cache counters; one counter group per pass.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE" "SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD" "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum" "FETCH_SIZE" "WRITE_SIZE"; do
  t=$(echo $set | cut -d' ' -f1)
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d gpurun_out/r06af_$t -o run -- python tools/bench_decode.py --proteins 8 --tokens 256 --reps 1 > gpurun_out/r06af_$t.log 2>&1
done
echo done
