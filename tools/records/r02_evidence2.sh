# Final evidence of the round: GPU suite, default bench line, per-launch rocprof summary (one
# H2D chunk), PMC summary and the HBM-traffic passes of k_mpnn<1>.
set -e
TAG=${1:-r02z}
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/r02_check.sh $TAG
bash tools/pmc_all.sh ${TAG}pmc
python tools/pmc_summary.py gpurun_out/${TAG}pmc_* > gpurun_out/${TAG}_pmc_summary.txt
echo done
