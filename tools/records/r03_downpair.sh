# k_down_pair: identity test, then the N = 8 share with the pair form (default at one round of
# tiles) vs k_down<1> (PST_DOWN_PAIR=0).
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r03dp}
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "down_coop or fused_and_split" > gpurun_out/${TAG}_pytest.log 2>&1
O=gpurun_out/${TAG}.jsonl
for i in 1 2; do
  timeout -k 10 120 python -u tools/share_probe.py --tag pair >> $O
  PST_DOWN_PAIR=0 timeout -k 10 120 python -u tools/share_probe.py --tag one_wave >> $O
done
echo done
