set -e
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || true
grep -oE "^[[:space:]]*(SQ_[A-Z0-9_]+|TCC_[A-Z0-9_]+|TA_[A-Z0-9_]+|GRBM_[A-Z0-9_]+|TCP_[A-Z0-9_]+|FETCH_SIZE|WRITE_SIZE)" gpurun_out/counters_list.txt | sort -u > gpurun_out/counter_names.txt || true
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE" "SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_VALU_MFMA_BUSY_CYCLES" "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum" "FETCH_SIZE" "WRITE_SIZE"; do
  tag=$(echo $set | cut -d' ' -f1)
  timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d gpurun_out/pmc_$tag -o run -- python bench.py --steps 1 --warmup 0 --proteins 256 --no-cpu-baseline > gpurun_out/pmc_$tag.log 2>&1 || echo "pmc set $tag failed"
done
