# Instruction-cache PMC pass over a reduced bench (256 proteins): is the k_mpnn loop body fetch-bound?
set -e
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
TAG=${1:-ic}
[ -n "${2:-}" ] && export PST_LIB=$2
timeout -s KILL 120 rocprofv3 --list-avail > gpurun_out/${TAG}_avail.txt 2>&1 || true
for set in "SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE" "SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU"; do
  t=$(echo $set | cut -d' ' -f1)
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d gpurun_out/${TAG}_$t -o run -- python bench.py --steps 1 --warmup 0 --proteins ${PROTEINS:-256} --no-cpu-baseline --no-e2e > gpurun_out/${TAG}_$t.log 2>&1 || echo "pmc set $t failed"
done
python tools/pmc_summary.py gpurun_out/${TAG}_*
