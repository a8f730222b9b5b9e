# Round 5: which queue variant differs after the doubled-GELU / feature-slot changes (queue_diag.py
# on the pre-GELU build, the GELU commit's build and the working tree's build)
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
for lib in ab/44af52d/libpst.so ab/402d1a8/libpst.so protein-structure-tokenizer_amd/pst_amd/_lib/libpst.so; do
  echo "== $lib" >> gpurun_out/r05c_diag.txt
  PST_LIB=$PWD/$lib timeout -k 10 300 python -u tools/queue_diag.py >> gpurun_out/r05c_diag.txt 2>&1
done
echo done
