# Round 5: queue diagnostic on the C-GELU variant; CASP14 host-path probe of the working tree
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "== ab/v1_cgelu" > gpurun_out/r05d_diag.txt
PST_LIB=$PWD/ab/v1_cgelu/libpst.so timeout -k 10 300 python -u tools/queue_diag.py >> gpurun_out/r05d_diag.txt 2>&1
timeout -k 10 300 python -u tools/casp14_e2e.py > gpurun_out/r05d_casp.json 2> gpurun_out/r05d_casp.err
timeout -k 10 300 python -u tools/parse_probe.py > gpurun_out/r05d_parse.json 2> gpurun_out/r05d_parse.err
echo done
