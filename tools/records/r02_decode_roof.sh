# Decode roofline evidence (8 x 256 tokens): kernel-trace stats and one PMC pass (MFMA count,
# MFMA busy, clock) over tools/bench_decode.py.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/dec_prof -o run -- python tools/bench_decode.py --reps 5 > gpurun_out/dec_prof.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/dec_pmc -o run -- python tools/bench_decode.py --reps 2 > gpurun_out/dec_pmc.log 2>&1
python tools/pmc_summary.py gpurun_out/dec_pmc > gpurun_out/dec_pmc_summary.txt
echo done
