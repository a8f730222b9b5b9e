# k_down_coop with the original track in LDS (two waves per SIMD) vs the previous build
# (build/var_oldcoop): parity tests, then the down stage at 32 / 128 proteins (256 / 1 024 tiles)
# under the default policy and with coop forced up to 1 024 tiles.
set -e
TAG=${1:-r02o}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_cli.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
for round in 1 2; do
for P in 32 128; do
  for v in base oldcoop; do
    for T in -1 1024; do
      if [ $v = base ]; then unset PST_LIB; else export PST_LIB=build/var_$v/libpst.so; fi
      if [ $T = -1 ]; then unset PST_DOWN_COOP; else export PST_DOWN_COOP=$T; fi
      timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-e2e --proteins $P --steps 15 > gpurun_out/${TAG}_tmp.json 2>> gpurun_out/${TAG}_bench.err
      python -c "import json; d=json.load(open('gpurun_out/${TAG}_tmp.json')); print('round $round proteins $P $v down_coop $T', d['ms_per_step'], 'ms; device-resident', d['device_resident']['ms'], 'ms; down', d['roofline']['stage_ms']['down'], 'ms')" >> gpurun_out/${TAG}_ab.txt
    done
  done
done
done
unset PST_LIB PST_DOWN_COOP
echo done
