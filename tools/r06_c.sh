# Round 6: kernel traces of the two-halves schedule (modes 0, 2) at 128 proteins.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
for M in 0 2; do
  timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/r06c_m$M -o run -- python -u tools/two_halves_ab.py --proteins 128 --modes $M --rounds 1 --reps 3 > gpurun_out/r06c_m$M.log 2>&1
done
echo done
