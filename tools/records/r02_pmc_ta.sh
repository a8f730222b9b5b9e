# Texture-address / L1 (TA, TD, TCP) PMC passes over the default bench at full size: is the
# per-lane row gather of k_mpnn<0> bound by the L1 address path? One counter group per pass.
# usage: bash tools/r02_pmc_ta.sh TAG  → gpurun_out/TAG_<first counter>/
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-pmcta}
export PST_H2D_CHUNKS=1
for set in "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE" \
           "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum" \
           "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_LFIFO_STALL_CYCLES_sum"; do
  t=$(echo $set | cut -d' ' -f1)
  timeout -s KILL 300 rocprofv3 --pmc $set --output-format csv -d gpurun_out/${TAG}_$t -o run -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/${TAG}_$t.log 2>&1
done
python tools/pmc_summary.py gpurun_out/${TAG}_* > gpurun_out/${TAG}_summary.txt
echo done
