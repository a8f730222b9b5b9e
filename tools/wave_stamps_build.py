"""Build ab/wstamp/libpst.so: the current sources with per-wave, per-edge-block s_memrealtime stamps
in the one-round fused kernel k_mpnn<L, true> (pst_x_wave_stamps; read by tools/wave_stamps_probe.py).
Diagnostic only: the stamped source goes to a scratch tree, never to csrc/.
Stamps per wave (u64, 100 MHz): [0] start, [1] after the W1 LDS fill, [2 + b] start of its b-th edge
block (b < 25), [27] edge loop done, [28] past the pair barrier, [29] end; [31] HW_ID | XCC_ID << 32."""
import os
import shutil
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tree = os.path.join(ROOT, "build", "wstamp_tree")
shutil.rmtree(tree, ignore_errors=True)
os.makedirs(os.path.join(tree, "protein-structure-tokenizer_amd"))
shutil.copytree(os.path.join(ROOT, "include"), os.path.join(tree, "include"))
shutil.copytree(os.path.join(ROOT, "protein-structure-tokenizer_amd", "csrc"),
                os.path.join(tree, "protein-structure-tokenizer_amd", "csrc"))
p = os.path.join(tree, "protein-structure-tokenizer_amd", "csrc", "pst_kernels.hip")
s = open(p).read()


def rep(a, b):
    global s
    assert s.count(a) >= 1, a[:60]
    s = s.replace(a, b, 1)


rep("namespace pst {\n", "namespace pst {\n__device__ unsigned long long g_wst[3][2048][32];\n"
    "#define WST(k) if (HALF && lane == 0 && wid < 2048) g_wst[LAYER][wid][k] = __builtin_amdgcn_s_memrealtime();\n")
head = """  const int hh = w & 1;  // HALF: which half of the task's edge blocks
  // the first KL k-steps of the message MLP's W1 fragments (msg_hidden), read by every block of
  // the workgroup's four waves from LDS instead of L2; filled before any wave may leave
  constexpr int KL = w1_lds_ksteps<LAYER>();
  __shared__ float4 w1_lds_buf[(KL > 0 ? KL : 1) * 64];
  const float4* w1_lds = KL > 0 ? w1_lds_buf : nullptr;
  if (KL > 0) {
    for (int i = threadIdx.x; i < KL * 64; i += 256) w1_lds_buf[i] = a.msg.w1[i];
    __syncthreads();
  }
"""
rep(head, head.replace("  const int hh = w & 1;", "  const int64_t wid = (int64_t)blockIdx.x * 4 + w;\n  WST(0);\n  const int hh = w & 1;")
    + "  WST(1);\n  if (HALF && lane == 0 && wid < 2048) g_wst[LAYER][wid][31] = (unsigned long long)__builtin_amdgcn_s_getreg(0xf804) | ((unsigned long long)__builtin_amdgcn_s_getreg(0xf814) << 32);\n")
i = s.index("template <int LAYER, bool HALF>\n__global__ __launch_bounds__(256, MPNN_MIN_BLOCKS) void k_mpnn(MpnnArgs a)")
j = s.index("// Fused layer as a persistent work queue")
body = s[i:j]
body = body.replace("    const int32_t s_cur = s_next;\n", "    WST(2 + blk - blk_lo);\n    const int32_t s_cur = s_next;\n", 1)
body = body.replace("  if (HALF) {\n    __builtin_amdgcn_fence(__ATOMIC_RELEASE, \"workgroup\");",
                    "  WST(27);\n  if (HALF) {\n    __builtin_amdgcn_fence(__ATOMIC_RELEASE, \"workgroup\");", 1)
body = body.replace("    node_update_pair<LAYER>(a, g0, hh, lds_scratch[w & 2]);\n    cs.stop(a.clk);",
                    "    WST(28);\n    node_update_pair<LAYER>(a, g0, hh, lds_scratch[w & 2]);\n    WST(29);\n    cs.stop(a.clk);", 1)
assert body.count("WST(") == 6, body.count("WST(")
s = s[:i] + body + s[j:]
# node_update_pair phases: stamps 8 + k of a per-wave side array g_nst (after the x exchange, LN0,
# each FFN chunk, the residual exchange, LN1 + h store, the projections)
rep("__device__ unsigned long long g_wst[3][2048][32];\n",
    "__device__ unsigned long long g_wst[3][2048][32];\n__device__ unsigned long long g_nst[3][2048][16];\n")
i = s.index("template <int LAYER>\n__device__ __forceinline__ void node_update_pair(const MpnnArgs& a, int64_t g0, int h, float* xs) {")
j = s.index("template <int LAYER>\n__global__ __launch_bounds__(256, 1) void k_mpnn_node_coop")
nb = s[i:j]
nb = nb.replace("  const int lane = lane_id();\n", "  const int lane = lane_id();\n  const int64_t nw = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);\n"
                "#define NST(k) if (lane == 0 && nw < 2048) g_nst[LAYER][nw][k] = __builtin_amdgcn_s_memrealtime();\n  NST(0);\n", 1)
nb = nb.replace("    pair_exchange(x, xp0, xp1, xs, h);\n  }\n  tile_layer_norm(x, a.ln0_s, a.ln0_o);  // V_i_0\n",
                "    pair_exchange(x, xp0, xp1, xs, h);\n  }\n  NST(1);\n  tile_layer_norm(x, a.ln0_s, a.ln0_o);  // V_i_0\n  NST(2);\n", 1)
nb = nb.replace("      blk_gemm(out1, hid, a.ff_w2 + ck * 64 * 64, b1);\n    }\n  }\n",
                "      blk_gemm(out1, hid, a.ff_w2 + ck * 64 * 64, b1);\n    }\n    NST(3 + ck);\n  }\n", 1)
nb = nb.replace("  tile_layer_norm(x, a.ln1_s, a.ln1_o);  // V_i_1\n", "  NST(7);\n  tile_layer_norm(x, a.ln1_s, a.ln1_o);  // V_i_1\n", 1)
nb = nb.replace("  if (a.P_out) {\n#pragma unroll 1\n    for (int p = 0; p < 4; ++p) {\n      f32x16 pr0, pr1;",
                "  NST(8);\n  if (a.P_out) {\n#pragma unroll 1\n    for (int p = 0; p < 4; ++p) {\n      f32x16 pr0, pr1;", 1)
nb = nb.rstrip()
assert nb.endswith("}"), nb[-40:]
nb = nb[:-1] + "  NST(9);\n#undef NST\n}\n\n"
assert nb.count("NST(") == 8, nb.count("NST(")
s = s[:i] + nb + s[j:]
s = s.replace("void launch_mpnn(", 'extern "C" int pst_x_wave_stamps(unsigned long long* out) {\n'
              "  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_wst), sizeof(g_wst)) == hipSuccess ? 0 : -1;\n}\n"
              'extern "C" int pst_x_node_stamps(unsigned long long* out) {\n'
              "  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_nst), sizeof(g_nst)) == hipSuccess ? 0 : -1;\n}\n"
              "void launch_mpnn(", 1)
open(p, "w").write(s)
out = os.path.join(ROOT, "ab", "wstamp")
os.makedirs(out, exist_ok=True)
subprocess.run(["make", "-s", "-C", os.path.dirname(p), f"OUT={out}", "-j8", f"{out}/libpst.so"], check=True)
for f in os.listdir(out):
    if f.endswith(".o"):
        os.remove(os.path.join(out, f))
print(f"{out}/libpst.so")
