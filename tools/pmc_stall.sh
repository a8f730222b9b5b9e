# Issue/stall PMC passes over a reduced bench (256 proteins): where do k_mpnn's non-MFMA cycles go?
# usage: bash tools/pmc_stall.sh TAG [PST_LIB]
set -e
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
TAG=${1:-st}
[ -n "${2:-}" ] && export PST_LIB=$2
i=0
for set in "SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT" \
           "SQ_INST_LEVEL_VMEM SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU2 SQ_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d gpurun_out/${TAG}_p$i -o run -- python bench.py --steps 1 --warmup 0 --proteins 256 --no-cpu-baseline --no-e2e > gpurun_out/${TAG}_p$i.log 2>&1
done
python tools/pmc_summary.py gpurun_out/${TAG}_p*
