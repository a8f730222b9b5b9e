# Multi-query IPA attention: bitwise A/B of the decode outputs vs the previous build
# (build/var_decold), the decode GPU tests, and decode throughput of both builds.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python tools/decode_ab_check.py new > gpurun_out/ipa_ab.log 2>&1
PST_LIB=build/var_decold/libpst.so timeout -k 10 200 python tools/decode_ab_check.py old >> gpurun_out/ipa_ab.log 2>&1
python tools/decode_ab_check.py --compare new old >> gpurun_out/ipa_ab.log 2>&1
timeout -k 10 500 python -u -m pytest tests/test_gpu_decode.py -x -q --timeout 300 --timeout-method thread > gpurun_out/ipa_pytest.log 2>&1
for t in 256 512; do
  timeout -k 10 200 python tools/bench_decode.py --tokens $t --reps 5 >> gpurun_out/ipa_bench.txt 2>/dev/null
  PST_LIB=build/var_decold/libpst.so timeout -k 10 200 python tools/bench_decode.py --tokens $t --reps 5 >> gpurun_out/ipa_bench_old.txt 2>/dev/null
done
echo done
