"""Build ab/pdbstamp/libpst.so: the current sources with per-phase s_memrealtime stamps in
k_pdb_scan (pst_x_pdb_stamps; read by tools/pdb_stamp_probe.py). Diagnostic only: the stamped
source is written to a scratch tree, never to csrc/."""
import os
import shutil
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tree = os.path.join(ROOT, "build", "pdbstamp_tree")
shutil.rmtree(tree, ignore_errors=True)
os.makedirs(os.path.join(tree, "protein-structure-tokenizer_amd"))
shutil.copytree(os.path.join(ROOT, "include"), os.path.join(tree, "include"))
shutil.copytree(os.path.join(ROOT, "protein-structure-tokenizer_amd", "csrc"),
                os.path.join(tree, "protein-structure-tokenizer_amd", "csrc"))
p = os.path.join(tree, "protein-structure-tokenizer_amd", "csrc", "pst_pdb_gpu.hip")
s = open(p).read()
s = s.replace("namespace pst {\n\nnamespace {", "namespace pst {\n__device__ unsigned long long g_stamp[64 * 16];\n"
              "#define STAMP(k) if (threadIdx.x == 0 && blockIdx.x < 64) g_stamp[blockIdx.x * 16 + (k)] = "
              "__builtin_amdgcn_s_memrealtime();\nnamespace {", 1)
marks = [("  for (int c = tid; c < 256; c += PDB_THREADS) s_chain_seg[c] = 0;\n  __syncthreads();\n", 0),
         ("  const int n_lines = at;  // separators + 1 (the last line may be empty)\n  __syncthreads();\n", 1),
         ("  const int stop = min(s_stop, n_lines);\n", 3),
         ("  __syncthreads();\n  n_rec = min(n_rec, rec_cap);\n", 4),
         ("    n_run += tile;\n  }\n  __syncthreads();\n", 5),
         ("  for (int r = tid; r < n_run * 37; r += PDB_THREADS) a.slot[37 * rb + r] = PDB_INT_MAX;\n  __syncthreads();\n", 6)]
for m, k in marks:
    assert m in s, k
    s = s.replace(m, m + f"  STAMP({k});\n", 1)
s = s.replace("  const int start = s_start;", "  STAMP(2);\n  const int start = s_start;", 1)
s = s.replace("  __syncthreads();\n  // ---- kept residues", "  __syncthreads();\n  STAMP(7);\n  // ---- kept residues", 1)
s = s.replace("  if (tid == 0) {\n    a.n_res[f] = n_keep;", "  STAMP(8);\n  if (tid == 0) {\n    a.n_res[f] = n_keep;", 1)
s = s.replace("void launch_pdb_scan(", 'extern "C" int pst_x_pdb_stamps(unsigned long long* out) {\n'
              "  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stamp), sizeof(g_stamp)) == hipSuccess ? 0 : -1;\n}\n"
              "void launch_pdb_scan(", 1)
assert s.count("STAMP(") == 10, s.count("STAMP(")
open(p, "w").write(s)
out = os.path.join(ROOT, "ab", "pdbstamp")
os.makedirs(out, exist_ok=True)
subprocess.run(["make", "-s", "-C", os.path.dirname(p), f"OUT={out}", "-j8", f"{out}/libpst.so"], check=True)
for f in os.listdir(out):
    if f.endswith(".o"):
        os.remove(os.path.join(out, f))
print(f"{out}/libpst.so")
