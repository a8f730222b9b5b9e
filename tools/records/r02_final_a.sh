# GPU suite, then the strong-scaling shares with the current pipeline policy.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02fa_pytest.log 2>&1
bash tools/strong_scaling_shares.sh > gpurun_out/r02_shares3.jsonl
echo done
