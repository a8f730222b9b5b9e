# Sanitizer builds + runs of the host code and the oracle (CPU). Log: profiles/r03_sanitize.log
set -e
cd "$(dirname "$0")/.."
make -s -C protein-structure-tokenizer_amd/csrc asan tsan
make -s -C oracle asan
D=$(mktemp -d)
tar -xzf tests/golden/casp14_pdbs.tar.gz -C "$D"
{
  echo "== $(date -u +%FT%TZ) $(g++ --version | head -1)"
  echo "== ASan+UBSan: parser / host pool / writer, 31 CASP14 files + malformed variants"
  protein-structure-tokenizer_amd/pst_amd/_lib/san/pdb_harness_asan "$D" "$D"/casp14_pdbs/*.pdb 2>&1
  echo "rc=$?"
  echo "== TSan: parser / host pool / writer, 31 CASP14 files + malformed variants, 2 host threads"
  protein-structure-tokenizer_amd/pst_amd/_lib/san/pdb_harness_tsan "$D" "$D"/casp14_pdbs/*.pdb 2>&1
  echo "rc=$?"
  echo "== ASan+UBSan: C oracle (tests/test_sanitize.py::test_oracle_under_asan_ubsan)"
  python -m pytest -q -p no:cacheprovider tests/test_sanitize.py 2>&1 | tail -3
} | tee profiles/r03_sanitize.log
rm -rf "$D"
