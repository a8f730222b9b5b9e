# Decode (round 3): GPU tests, throughput with the MFMA pair sum vs the VALU form at three shapes,
# kernel-trace profile and one PMC pass (MFMA instructions per kernel) of 8 x 256.
set -e
TAG=${1:-r03dec}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_decode.py -x -v --timeout 200 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
for shape in "8 256" "32 128" "8 512"; do
  set -- $shape
  timeout -k 10 120 python -u tools/bench_decode.py --proteins $1 --tokens $2 --reps 5 >> gpurun_out/${TAG}_bench.jsonl
  PST_DECODE_IPA_VALU=1 timeout -k 10 120 python -u tools/bench_decode.py --proteins $1 --tokens $2 --reps 5 >> gpurun_out/${TAG}_bench_valu.jsonl
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python tools/bench_decode.py --proteins 8 --tokens 256 --reps 5 > gpurun_out/${TAG}_prof.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/${TAG}_pmc -o run -- python tools/bench_decode.py --reps 2 > gpurun_out/${TAG}_pmc.log 2>&1
python tools/pmc_summary.py gpurun_out/${TAG}_pmc > gpurun_out/${TAG}_pmc_summary.txt
echo done
