# Secondary configs on the final build: config 5 (512 x 512 residues, codebook 64 000, df 4) and
# config 4's aux (CASP14, 64 000); the gloo rehearsal of the 2-rank bench spawn path on one card.
set -e
TAG=${1:-r03cfg}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --proteins 512 --residues 512 --codebook 64000 --df 4 --no-cpu-baseline --no-e2e > gpurun_out/${TAG}_config5.json 2> gpurun_out/${TAG}_config5.err
timeout -k 10 120 python -u tools/bench_aux.py --codebook 64000 --reps 20 > gpurun_out/${TAG}_aux_config4.json
timeout -k 10 400 python -u bench.py --gpus 2 --dist-backend gloo --no-cpu-baseline --no-e2e --steps 5 > gpurun_out/${TAG}_gloo2.json 2> gpurun_out/${TAG}_gloo2.err
echo done
