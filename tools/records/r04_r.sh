# Round 4: SURVEY config 5's exact-match sample (forward_ref_bench.npz bench512_*): the GPU reference
# tests, then the config-5 bench line (512 x 512 residues, codebook 64 000, df 4).
set -e
TAG=${1:-r04r}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_reference_wide.py -x -v -s --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
echo pytest ok
timeout -k 10 400 python -u bench.py --codebook 64000 --df 4 --residues 512 --proteins 512 --no-e2e > gpurun_out/${TAG}_bench_config5.json 2> gpurun_out/${TAG}_bench_config5.err
echo done
