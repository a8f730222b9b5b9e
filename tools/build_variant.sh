# Build a libpst variant with extra compiler flags into build/var_<name>/libpst.so (for A/B runs via PST_LIB).
# usage: bash tools/build_variant.sh NAME "-DFOO -fno-slp-vectorize"
set -e
NAME=$1; EXTRA=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/build/var_$NAME
mkdir -p $OUT
make -s -C $ROOT/protein-structure-tokenizer_amd/csrc OUT=$OUT FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -Wall -Wno-unused-result $EXTRA" -j8 $OUT/libpst.so
echo $OUT/libpst.so
