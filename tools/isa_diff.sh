# Disassemble the gfx950 code object of two hipcc objects (or .so) and diff them per kernel.
#   bash tools/isa_diff.sh OLD.o NEW.o     -> "identical ISA" or the kernels whose code differs
# Used to show that a source cleanup changes no instruction, and to identify what a build variant changed.
set -e
B=/opt/rocm/lib/llvm/bin
T=$(mktemp -d)
for i in 1 2; do
  src=$1; [ $i = 2 ] && src=$2
  $B/llvm-objcopy --dump-section .hip_fatbin=$T/$i.fb "$src"
  $B/clang-offload-bundler --unbundle --type=o --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --input=$T/$i.fb --output=$T/$i.co
  $B/llvm-objdump -d --no-show-raw-insn $T/$i.co | grep -v 'file format' > $T/$i.s
done
if cmp -s $T/1.s $T/2.s; then
  echo "identical ISA ($(wc -l < $T/1.s) lines)"
else
  python3 - "$T/1.s" "$T/2.s" <<'EOF'
import re, sys
def funcs(p):
    out, cur = {}, None
    for ln in open(p):
        m = re.match(r"^[0-9a-f]+ <(.+)>:", ln)
        if m:
            cur = m.group(1); out[cur] = []
        elif cur and ln.strip():
            out[cur].append(re.sub(r"//.*", "", ln).strip())
    return out
a, b = funcs(sys.argv[1]), funcs(sys.argv[2])
for k in sorted(set(a) | set(b)):
    if a.get(k) != b.get(k):
        print(f"differs: {k}  ({len(a.get(k, []))} -> {len(b.get(k, []))} instructions)")
EOF
fi
rm -rf $T
