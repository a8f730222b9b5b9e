# f32 MFMA vs scalar / packed f32 VALU on the two waves of a SIMD (tools/micro/coexec.hip), then
# optionally the round check (tools/r03_check.sh TAG tests/).
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 60 ./tools/micro/coexec > gpurun_out/${1:-r03cx}_coexec.txt 2>&1
cat gpurun_out/${1:-r03cx}_coexec.txt
if [ -n "$2" ]; then bash tools/r03_check.sh ${1:-r03cx} $2; fi
