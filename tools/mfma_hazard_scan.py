"""Scan a built code object for a VALU write followed by an MFMA reading that VGPR as its A or B
operand with fewer than 2 wait states in between (s_nop N counts N+1, any other instruction 1).
hipcc pads this hazard for its own code but not after inline asm, so a hit means an asm block's
output reaches an MFMA too early (the MFMA reads the stale register).

    python tools/mfma_hazard_scan.py protein-structure-tokenizer_amd/pst_amd/_lib/pst_kernels.o [...]
exit 1 if any kernel has a hit."""
import os
import re
import subprocess
import sys
import tempfile

B = "/opt/rocm/lib/llvm/bin"


def disasm(obj):
    with tempfile.TemporaryDirectory() as d:
        fb, co = os.path.join(d, "fb"), os.path.join(d, "co")
        subprocess.run([f"{B}/llvm-objcopy", "--dump-section", f".hip_fatbin={fb}", obj], check=True)
        subprocess.run([f"{B}/clang-offload-bundler", "--unbundle", "--type=o",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--input={fb}", f"--output={co}"], check=True)
        return subprocess.run([f"{B}/llvm-objdump", "-d", "--no-show-raw-insn", co], check=True,
                              capture_output=True, text=True).stdout


def funcs(text):
    out, cur = {}, None
    for ln in text.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.+)>:", ln)
        if m:
            cur = m.group(1)
            out[cur] = []
        elif cur and ln.strip():
            out[cur].append(re.sub(r"//.*", "", ln).strip())
    return out


def regs(op):
    s = set()
    for a, b in re.findall(r"v\[(\d+):(\d+)\]", op):
        s |= set(range(int(a), int(b) + 1))
    for a in re.findall(r"(?<![\w\[])v(\d+)", op):
        s.add(int(a))
    return s


def hits(ins, need=2):
    res = []
    for i, l in enumerate(ins):
        if not l.startswith("v_") or l.startswith("v_mfma") or l.startswith(("v_readlane", "v_readfirstlane")):
            continue
        parts = l.split(None, 1)
        if len(parts) < 2:
            continue
        dst = regs(parts[1].split(",")[0])
        ws = 0
        for j in range(i + 1, min(len(ins), i + 6)):
            n = ins[j]
            if n.startswith("s_nop"):
                ws += int(n.split()[1]) + 1
            elif n.startswith("v_mfma"):
                ops = n.split(None, 1)[1].split(",")
                if dst & (regs(ops[1]) | regs(ops[2])) and ws < need:
                    res.append((l, n, ws))
                ws += 1
            else:
                ws += 1
            if ws >= need:
                break
    return res


bad = 0
for obj in sys.argv[1:]:
    for k, ins in funcs(disasm(obj)).items():
        h = hits(ins)
        if h:
            bad += len(h)
            print(f"{os.path.basename(obj)} {k}: {len(h)} VALU->MFMA operand reads with < 2 wait states, e.g. {h[0]}")
print("hazard hits:", bad)
sys.exit(1 if bad else 0)
