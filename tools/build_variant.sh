# Build a libpst variant into build/var_<name>/libpst.so (for A/B runs via PST_LIB).
#   bash tools/build_variant.sh NAME "EXTRA_FLAGS" [PATCH ...]
# EXTRA_FLAGS go to hipcc (tunables such as -DW1_LDS_KSTEPS_L0=32 that keep the product's bits);
# each PATCH names tools/variants/PATCH.patch (timing-only ablations and diagnostic builds, kept
# out of the product sources), applied to a copy of the tree under build/var_<name>/tree.
set -e
NAME=$1; EXTRA=$2; shift 2 || shift $#
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/build/var_$NAME
mkdir -p $OUT
SRC=$ROOT
if [ $# -gt 0 ]; then
  SRC=$OUT/tree
  rm -rf $SRC
  mkdir -p $SRC/protein-structure-tokenizer_amd
  cp -r $ROOT/include $SRC/
  cp -r $ROOT/protein-structure-tokenizer_amd/csrc $SRC/protein-structure-tokenizer_amd/
  for p in "$@"; do
    patch -s -p1 -d $SRC < $ROOT/tools/variants/$p.patch
  done
fi
make -s -C $SRC/protein-structure-tokenizer_amd/csrc OUT=$OUT FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -Wall -Wno-unused-result $EXTRA" -j8 $OUT/libpst.so
echo $OUT/libpst.so
