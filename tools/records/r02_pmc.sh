set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/pmc_all.sh r02pmc1
python tools/pmc_summary.py gpurun_out/r02pmc1_* > gpurun_out/r02_pmc_summary.txt
echo done
