# Decode A/B: bitwise test of the MFMA pair sum, then 8x256 / 32x128 / 8x512 MFMA vs VALU form.
set -e
TAG=${1:-r03deca}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py -x -v --timeout 200 --timeout-method thread -k "ipa or wide" > gpurun_out/${TAG}_pytest.log 2>&1
for shape in "8 256" "32 128" "8 512"; do
  set -- $shape
  timeout -k 10 120 python -u tools/bench_decode.py --proteins $1 --tokens $2 --reps 5 >> gpurun_out/${TAG}_bench.jsonl
  PST_DECODE_IPA_VALU=1 timeout -k 10 120 python -u tools/bench_decode.py --proteins $1 --tokens $2 --reps 5 >> gpurun_out/${TAG}_bench_valu.jsonl
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python tools/bench_decode.py --proteins 8 --tokens 256 --reps 5 > gpurun_out/${TAG}_prof.log 2>&1
echo done
