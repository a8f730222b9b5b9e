# Round 4, after k_mpnn_q: schedule policy A/Bs around the new queue form, ACT_GROUP=8 A/B, and
# the default bench line.
set -e
TAG=${1:-r04b}
mkdir -p gpurun_out
export TMPDIR=/tmp
# one round (the N = 8 share): two waves per task (default) vs the queue
timeout -k 10 200 bash tools/env_ab.sh 128 - "PST_HALF_TASKS=0" > gpurun_out/${TAG}_ab128.txt 2>&1
# half a round to two rounds: split (the policy's pick below one round) vs the queue
for P in 192 256 320 384; do
  timeout -k 10 200 bash tools/env_ab.sh $P - "PST_SPLIT_TASKS=0" "PST_SPLIT_TASKS=0 PST_HALF_TASKS=0" >> gpurun_out/${TAG}_absplit.txt 2>&1
done
echo policy ok
timeout -k 10 400 bash tools/lib_ab.sh "1024" default $PWD/ab/libpst_g8.so default $PWD/ab/libpst_g8.so > gpurun_out/${TAG}_g8.txt 2>&1
echo g8 ok
timeout -k 10 400 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
echo done
