# Round 6: layer 0's queue tasks strided over the XCDs (PST_L0_XCD_STRIDE=1: XCD q takes tasks q, q+8, ...,
# so concurrent tasks of one XCD share receiver positions and their pair-table rows): GPU suite with it on
# (the default), then an interleaved host-to-host A/B with stage times.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06u_pytest.txt 2>&1
timeout -k 10 600 python tools/env_ab_tokens.py --env PST_L0_XCD_STRIDE --values 0 1 --proteins 1024 512 --rounds 7 > gpurun_out/r06u_ab.txt
echo done
