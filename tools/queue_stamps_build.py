"""Build ab/qstamp/libpst.so: the current sources with per-wave time sums in the persistent queue
kernel k_mpnn_q<L, NW> (pst_x_queue_stamps; read by tools/queue_stamps_probe.py). Per wave (u64,
100 MHz ticks): [0] Σ edge phases (the units' 25 blocks), [1] Σ node updates, [2] units, [3] node
updates, [4] first start, [5] last end. Diagnostic only: scratch-tree build, never csrc/."""
import os
import shutil
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tree = os.path.join(ROOT, "build", "qstamp_tree")
shutil.rmtree(tree, ignore_errors=True)
os.makedirs(os.path.join(tree, "protein-structure-tokenizer_amd"))
shutil.copytree(os.path.join(ROOT, "include"), os.path.join(tree, "include"))
shutil.copytree(os.path.join(ROOT, "protein-structure-tokenizer_amd", "csrc"),
                os.path.join(tree, "protein-structure-tokenizer_amd", "csrc"))
p = os.path.join(tree, "protein-structure-tokenizer_amd", "csrc", "pst_kernels.hip")
s = open(p).read()


def rep(a, b):
    global s
    assert s.count(a) == 1, (s.count(a), a[:60])
    s = s.replace(a, b, 1)


rep("namespace pst {\n", "namespace pst {\n__device__ unsigned long long g_qst[3][4096][8];\n")
rep("""  int q = __builtin_amdgcn_readfirstlane((int)(__builtin_amdgcn_s_getreg(0xf814) & 7));
  int empty = 0;""", """  int q = __builtin_amdgcn_readfirstlane((int)(__builtin_amdgcn_s_getreg(0xf814) & 7));
  int empty = 0;
  const int64_t qw = (int64_t)blockIdx.x * NW + w;
  unsigned long long qe = 0, qn = 0, qu = 0, qnu = 0, qt0 = __builtin_amdgcn_s_memrealtime();""")
rep("""    mpnn_edge_blocks<LAYER, KL, NW>(a, task, ln, 25 * hh, 25 * hh + 25, w1_lds, lds_scratch, w);""",
    """    const unsigned long long te0 = __builtin_amdgcn_s_memrealtime();
    mpnn_edge_blocks<LAYER, KL, NW>(a, task, ln, 25 * hh, 25 * hh + 25, w1_lds, lds_scratch, w);
    qe += __builtin_amdgcn_s_memrealtime() - te0;
    ++qu;""")
rep("""      mpnn_node_tile<LAYER>(a, task * 32, ln, a.agg + task * 32 * 128);
    }
  }""", """      const unsigned long long tn0 = __builtin_amdgcn_s_memrealtime();
      mpnn_node_tile<LAYER>(a, task * 32, ln, a.agg + task * 32 * 128);
      qn += __builtin_amdgcn_s_memrealtime() - tn0;
      ++qnu;
    }
  }
  if (lane == 0 && qw < 4096) {
    g_qst[LAYER][qw][0] = qe;
    g_qst[LAYER][qw][1] = qn;
    g_qst[LAYER][qw][2] = qu;
    g_qst[LAYER][qw][3] = qnu;
    g_qst[LAYER][qw][4] = qt0;
    g_qst[LAYER][qw][5] = __builtin_amdgcn_s_memrealtime();
  }""")
s = s.replace("void launch_mpnn(", 'extern "C" int pst_x_queue_stamps(unsigned long long* out) {\n'
              "  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_qst), sizeof(g_qst)) == hipSuccess ? 0 : -1;\n}\n"
              "void launch_mpnn(", 1)
open(p, "w").write(s)
out = os.path.join(ROOT, "ab", "qstamp")
os.makedirs(out, exist_ok=True)
subprocess.run(["make", "-s", "-C", os.path.dirname(p), f"OUT={out}", "-j8", f"{out}/libpst.so"], check=True)
for f in os.listdir(out):
    if f.endswith(".o"):
        os.remove(os.path.join(out, f))
print(f"{out}/libpst.so")
