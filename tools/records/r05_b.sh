# Round 5: the doubled-GELU + 14-k-step features + GELU asm hazard guard build (same bits): GPU
# suite (bitwise vs the oracle), bench line, decode bench with its roofline, CASP14 host probe,
# PMC instruction counts per launch for profiles/r05_pmc_summary.txt.
set -e
TAG=${1:-r05b}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
echo pytest ok
timeout -k 10 400 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
echo bench ok
for s in "8 256" "32 128" "8 512"; do
  set -- $s
  timeout -k 10 200 python -u tools/bench_decode.py --proteins $1 --tokens $2 >> gpurun_out/${TAG}_decode.jsonl 2>> gpurun_out/${TAG}_decode.err
done
echo decode ok
timeout -k 10 300 python -u tools/casp14_e2e.py > gpurun_out/${TAG}_casp.json 2> gpurun_out/${TAG}_casp.err
export PST_H2D_CHUNKS=1
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE" "SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES"; do
  t=$(echo $set | cut -d' ' -f1)
  timeout -k 10 400 rocprofv3 --pmc $set --output-format csv -d gpurun_out/${TAG}_pmc_$t -o run -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/${TAG}_pmc_$t.log 2>&1
done
echo done
