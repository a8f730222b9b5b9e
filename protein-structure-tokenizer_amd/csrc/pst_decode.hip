// pst_decode.hip — token ids → backbone atom37 coordinates on the GPU (the reference's decode path:
// Vq3D.indexes_to_codes → decode → structure_module, model/model.py:481-569 + folding.py), C ABI in
// include/pst.h (pst_decoder_*).
//
// Per protein (T tokens, N = df·T nodes; only real rows are computed — every masked row/key of the
// reference contributes exact zeros to them):
//   codes → up_proj → "original" = Linear([PE(t; 512/df) | up])               modules.py:453-480
//   3 cross-attention blocks: nodes (PE(i; 512) queries) attend over tokens, gated; transitions
//                                                                              modules.py:537-636
//   spherical norm → s; pair: LN → left/right (256) → P = left[i]⊙right[j] → LN(MLP(P) + Lin(P))
//   → [PE(j−i) | pair] → Linear → Transition = z                    sequence_decoder.py, modules.py:639-740
//   structure module: 8 fold iterations (IPA with pair bias and point attention, transitions,
//   quaternion backbone update, backbone torsions → frames → atom14 → atom37)        folding.py
// Kernels are plain fp32 (no bitwise claim): the pair chain as one fused f32-MFMA kernel
// (k_pair_fused), per-node GEMMs on the in-tree f32-MFMA k_gemm_mfma (no library GEMM), the rest
// hand-written (LayerNorm, gated cross-attention, IPA, frame geometry).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include <array>
#include <map>

#include "../../include/pst.h"
#include "pst_backbone_tables.h"
#include "pst_pool.h"
#include "pst_device.h"
#include "pst_frag.h"
#include "pst_pe.h"

namespace pst {
namespace dec {

// F_QSCALE: output × key_dim^-0.5 (the upsampler's query scaling, modules.py:346) in the epilogue,
// the same multiply the separate k_scale pass did
enum { F_RELU_OUT = 1, F_RELU_IN = 2, F_ACCUM = 4, F_SIGMOID_OUT = 8, F_QSCALE = 16 };
#define Q_SCALE 0.176776695296637f

__global__ void k_zero(float* x, int64_t n) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) x[i] = 0.0f;
}

// Y[M,N] (op)= act(act_in(X[M,K]) · W[K,N] + b): fp32 fma chain over k ascending, 64×64 tile per
// workgroup, 4×4 outputs per thread, K staged through LDS 16 at a time.
__global__ __launch_bounds__(256) void k_gemm(const float* __restrict__ X, int ldx, const float* __restrict__ W,
                                              int ldw, const float* __restrict__ b, float* __restrict__ Y, int ldy,
                                              int M, int N, int K, int flags) {
  __shared__ float Xs[16][64 + 1];
  __shared__ float Ws[16][64];
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  const int row0 = blockIdx.y * 64, col0 = blockIdx.x * 64;
  float acc[4][4] = {};
  for (int k0 = 0; k0 < K; k0 += 16) {
    for (int e = threadIdx.x; e < 64 * 16; e += 256) {
      int r = e >> 4, kk = e & 15;
      int gr = row0 + r, gk = k0 + kk;
      float v = (gr < M && gk < K) ? X[(int64_t)gr * ldx + gk] : 0.0f;
      if (flags & F_RELU_IN) v = v > 0.0f ? v : 0.0f;
      Xs[kk][r] = v;
      int wk = e >> 6, wc = e & 63;
      int gwk = k0 + wk, gwc = col0 + wc;
      Ws[wk][wc] = (gwk < K && gwc < N) ? W[(int64_t)gwk * ldw + gwc] : 0.0f;
    }
    __syncthreads();
    const int kmax = min(16, K - k0);
    for (int kk = 0; kk < kmax; ++kk) {
      float xv[4], wv[4];
#pragma unroll
      for (int a = 0; a < 4; ++a) xv[a] = Xs[kk][ty * 4 + a];
#pragma unroll
      for (int c = 0; c < 4; ++c) wv[c] = Ws[kk][tx * 4 + c];
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int c = 0; c < 4; ++c) acc[a][c] = __builtin_fmaf(xv[a], wv[c], acc[a][c]);
    }
    __syncthreads();
  }
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    const int r = row0 + ty * 4 + a;
    if (r >= M) continue;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int col = col0 + tx * 4 + c;
      if (col >= N) continue;
      float v = acc[a][c];
      if (b) v = v + b[col];
      if (flags & F_RELU_OUT) v = v > 0.0f ? v : 0.0f;
      if (flags & F_SIGMOID_OUT) v = 1.0f / (1.0f + expf(-v));
      if (flags & F_QSCALE) v = v * Q_SCALE;
      float* y = Y + (int64_t)r * ldy + col;
      *y = (flags & F_ACCUM) ? *y + v : v;
    }
  }
}

// The same GEMM on f32 MFMA (v_mfma_f32_32x32x2_f32), split over K: a block owns one
// 32 × (32·NACC) output tile and its SLICES waves take consecutive K ranges of `kslice` (a
// multiple of 4), so a wave's dependent MFMA chain is K / SLICES / 2 long instead of K / 2 — these
// GEMMs have a few thousand rows at most, and their time is that chain and the re-reads of X (one
// per column tile: NACC accumulators per wave cut them), not MFMA throughput. A fragments come
// straight from X rows (one float4 = two k-steps of a lane: k = 4s + h and 4s + 2 + h for lane
// half h), B fragments from W columns (coalesced 128-byte rows); act_in is applied on load. The
// slices' partial tiles are summed in slice order through LDS, then bias / activation /
// accumulation. Needs K % 4 == 0, ldx % 4 == 0 and a 16-byte aligned X (gemm_any checks; k_gemm
// otherwise).
template <int SLICES, int NACC>
__global__ __launch_bounds__(64 * SLICES) void k_gemm_mfma(const float* __restrict__ X, int ldx,
                                                           const float* __restrict__ W, int ldw,
                                                           const float* __restrict__ b, float* __restrict__ Y,
                                                           int ldy, int M, int N, int K, int flags, int kslice) {
  __shared__ float part[SLICES][16][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  // 1-D grid of ncol x nrow tiles. Workgroups are dispatched round-robin over the 8 XCDs (bid % 8),
  // each with its own L2: when nrow % 8 == 0, XCD x takes row tiles x, x + 8, ... with all their
  // column tiles, so each 32-row slab of X is fetched into one L2 instead of all eight (the
  // out_proj GEMM's X is 17 MB at 8 x 256 residues).
  const int ncol = (N + 32 * NACC - 1) / (32 * NACC), nrow = (M + 31) / 32;
  int tr, tc;
  if ((nrow & 7) == 0) {
    const int x = blockIdx.x & 7, idx = blockIdx.x >> 3;
    tr = x + 8 * (idx / ncol);
    tc = idx % ncol;
  } else {
    tr = blockIdx.x / ncol;
    tc = blockIdx.x % ncol;
  }
  const int row0 = tr * 32, col0 = tc * 32 * NACC;
  const int i = lane & 31, h = lane >> 5;
  const float* xr = X + (int64_t)min(row0 + i, M - 1) * ldx;  // rows past M: clamped, not stored
  bool cv[NACC];
  const float* wc[NACC];
#pragma unroll
  for (int t = 0; t < NACC; ++t) {
    const int c = col0 + 32 * t + i;
    cv[t] = c < N;
    wc[t] = W + (cv[t] ? c : 0) + (int64_t)h * ldw;
  }
  const bool relu_in = flags & F_RELU_IN;
  const int k0 = w * kslice, k1 = min(K, k0 + kslice);
  f32x16 acc[NACC];
#pragma unroll
  for (int t = 0; t < NACC; ++t) acc[t] = f32x16{};
  int k = k0;
  for (; k + 8 <= k1; k += 8) {  // 2 fragment groups per trip, loads ahead of their MFMAs
    float4 xa[2];
    float bw[2][NACC][2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      xa[u] = *reinterpret_cast<const float4*>(xr + k + 4 * u);
#pragma unroll
      for (int t = 0; t < NACC; ++t) {
        bw[u][t][0] = cv[t] ? wc[t][(int64_t)(k + 4 * u) * ldw] : 0.0f;
        bw[u][t][1] = cv[t] ? wc[t][(int64_t)(k + 4 * u + 2) * ldw] : 0.0f;
      }
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      float4 x = xa[u];
      if (relu_in) {
        x.x = x.x > 0.0f ? x.x : 0.0f;
        x.y = x.y > 0.0f ? x.y : 0.0f;
        x.z = x.z > 0.0f ? x.z : 0.0f;
        x.w = x.w > 0.0f ? x.w : 0.0f;
      }
#pragma unroll
      for (int t = 0; t < NACC; ++t) acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(h ? x.y : x.x, bw[u][t][0], acc[t], 0, 0, 0);
#pragma unroll
      for (int t = 0; t < NACC; ++t) acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(h ? x.w : x.z, bw[u][t][1], acc[t], 0, 0, 0);
    }
  }
  for (; k < k1; k += 4) {
    float4 x = *reinterpret_cast<const float4*>(xr + k);
    if (relu_in) {
      x.x = x.x > 0.0f ? x.x : 0.0f;
      x.y = x.y > 0.0f ? x.y : 0.0f;
      x.z = x.z > 0.0f ? x.z : 0.0f;
      x.w = x.w > 0.0f ? x.w : 0.0f;
    }
#pragma unroll
    for (int t = 0; t < NACC; ++t) {
      const float b0 = cv[t] ? wc[t][(int64_t)k * ldw] : 0.0f, b1 = cv[t] ? wc[t][(int64_t)(k + 2) * ldw] : 0.0f;
      acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(h ? x.y : x.x, b0, acc[t], 0, 0, 0);
      acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(h ? x.w : x.z, b1, acc[t], 0, 0, 0);
    }
  }
  // one accumulator at a time through LDS; wave w finishes registers r = w, w + SLICES, ... of it
  // (slice sums in slice order)
#pragma unroll
  for (int t = 0; t < NACC; ++t) {
    if (t) __syncthreads();
#pragma unroll
    for (int r = 0; r < 16; ++r) part[w][r][lane] = acc[t][r];
    __syncthreads();
    const int c = col0 + 32 * t + i;
    for (int r = w; r < 16; r += SLICES) {
      float v = part[0][r][lane];
      for (int q = 1; q < SLICES; ++q) v = v + part[q][r][lane];
      const int row = row0 + (r & 3) + 8 * (r >> 2) + 4 * h;
      if (row >= M || c >= N) continue;
      if (b) v = v + b[c];
      if (flags & F_RELU_OUT) v = v > 0.0f ? v : 0.0f;
      if (flags & F_SIGMOID_OUT) v = 1.0f / (1.0f + expf(-v));
      if (flags & F_QSCALE) v = v * Q_SCALE;
      float* y = Y + (int64_t)row * ldy + c;
      *y = (flags & F_ACCUM) ? *y + v : v;
    }
  }
}

// hk.LayerNorm over the last axis (C ≤ 512): mean, centred variance, eps 1e-5; one wave per row
__global__ __launch_bounds__(256) void k_layernorm(const float* __restrict__ X, int ldx, float* __restrict__ Y,
                                                   int ldy, int M, int C, const float* __restrict__ s,
                                                   const float* __restrict__ o) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const float* x = X + row * ldx;
  float v[8];
  const int per = (C + 63) / 64;
  float sum = 0.0f;
  for (int i = 0; i < per; ++i) {
    int c = lane + 64 * i;
    v[i] = c < C ? x[c] : 0.0f;
    sum += v[i];
  }
  for (int m = 32; m >= 1; m >>= 1) sum += __shfl_xor(sum, m);
  const float mean = sum / (float)C;
  float sq = 0.0f;
  for (int i = 0; i < per; ++i) {
    int c = lane + 64 * i;
    if (c < C) {
      float d = v[i] - mean;
      sq += d * d;
    }
  }
  for (int m = 32; m >= 1; m >>= 1) sq += __shfl_xor(sq, m);
  const float rs = 1.0f / sqrtf(sq / (float)C + 1e-5f);
  float* y = Y + row * ldy;
  for (int i = 0; i < per; ++i) {
    int c = lane + 64 * i;
    if (c < C) y[c] = (s[c] * rs) * (v[i] - mean) + o[c];
  }
}

// y = x / (|x|_2 + 1e-6) (model.py:148-162, "spherical"), 128 channels, one wave per row
__global__ void k_spherical(float* __restrict__ X, int M) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  float* x = X + row * 128;
  float a = x[lane], b = x[lane + 64];
  float s = a * a + b * b;
  for (int m = 32; m >= 1; m >>= 1) s += __shfl_xor(s, m);
  const float d = sqrtf(s) + 1e-6f;
  x[lane] = a / d;
  x[lane + 64] = b / d;
}

// A group of proteins decoded together: rows of every per-token / per-node / per-pair tensor are
// the proteins' rows concatenated; per-protein kernels find their protein through these maps.
struct DecBatch {
  int32_t B;
  const int64_t* tok_off;   // [B+1]
  const int64_t* node_off;  // [B+1]
  const int64_t* pair_off;  // [B+1] (N_b² rows per protein)
  const int32_t* tok_prot;  // [T_total]
  const int32_t* node_prot; // [N_total]
};

__device__ __forceinline__ int pair_protein(const DecBatch& bt, int64_t p) {
  int lo = 0, hi = bt.B - 1;
  while (lo < hi) {  // last b with pair_off[b] <= p
    const int mid = (lo + hi + 1) >> 1;
    if (bt.pair_off[mid] <= p) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

// codes (FSQ grid, renorm off: digit - L/2) → up_proj → [PE(t; T_pad) | up] rows of `orig_in`
__global__ void k_up_init(const uint32_t* __restrict__ tokens, DecBatch bt, int64_t T_total,
                          const int* __restrict__ levels, int D, const float* __restrict__ w_up,
                          const float* __restrict__ b_up, const float* __restrict__ pe_tok, float* __restrict__ orig_in) {
  const int64_t t = blockIdx.x;
  const int c = threadIdx.x;  // 128 threads
  if (t >= T_total) return;
  const int64_t tl = t - bt.tok_off[bt.tok_prot[t]];
  uint32_t tok = tokens[t];
  float code[8];
  uint32_t basis = 1;
  for (int d = 0; d < D; ++d) {
    const uint32_t L = (uint32_t)levels[d];
    const int digit = (int)((tok / basis) % L);
    code[d] = (float)(digit - (int)(L / 2));
    basis *= L;
  }
  float acc = 0.0f;
  for (int d = 0; d < D; ++d) acc = __builtin_fmaf(code[d], w_up[d * 128 + c], acc);
  orig_in[t * 256 + c] = pe_tok[tl * 128 + c];
  orig_in[t * 256 + 128 + c] = acc + b_up[c];
}

// resampled track init: node i of its protein gets PE(i_local; 512)
__global__ void k_node_pe(const float* __restrict__ pe_node, DecBatch bt, int64_t N_total, float* __restrict__ res) {
  const int64_t i = blockIdx.x;
  if (i >= N_total) return;
  const int64_t il = i - bt.node_off[bt.node_prot[i]];
  res[i * 128 + threadIdx.x] = pe_node[il * 128 + threadIdx.x];
}

// Upsampler attention, gated (modules.py:271-382): one wave per (node i, head h) over the T
// tokens of i's protein (the only unmasked keys)
__global__ __launch_bounds__(256) void k_up_attn(const float* __restrict__ q, const float* __restrict__ k,
                                                 const float* __restrict__ v, const float* __restrict__ gate,
                                                 float* __restrict__ out, DecBatch bt, int64_t N_total) {
  __shared__ float wsh[4][512];
  const int lane = threadIdx.x & 63, h = threadIdx.x >> 6;
  const int64_t i = blockIdx.x;
  if (i >= N_total) return;
  const int b = bt.node_prot[i];
  const int64_t t0 = bt.tok_off[b];
  const int T = (int)(bt.tok_off[b + 1] - t0);
  const float* qi = q + i * 128 + h * 32;
  float l[8];
  float mx = -INFINITY;
  for (int s = 0; s < 8; ++s) {
    int j = lane + 64 * s;
    float acc = 0.0f;
    if (j < T) {
      const float* kj = k + (t0 + j) * 128 + h * 32;
      for (int c = 0; c < 32; ++c) acc = __builtin_fmaf(qi[c], kj[c], acc);
    }
    l[s] = j < T ? acc : -INFINITY;
    mx = fmaxf(mx, l[s]);
  }
  for (int m = 32; m >= 1; m >>= 1) mx = fmaxf(mx, __shfl_xor(mx, m));
  float sum = 0.0f;
  for (int s = 0; s < 8; ++s) {
    int j = lane + 64 * s;
    float e = j < T ? expf(l[s] - mx) : 0.0f;
    l[s] = e;
    sum += e;
  }
  for (int m = 32; m >= 1; m >>= 1) sum += __shfl_xor(sum, m);
  for (int s = 0; s < 8; ++s) {
    int j = lane + 64 * s;
    if (j < T) wsh[h][j] = l[s] / sum;
  }
  __syncthreads();
  if (lane < 32) {
    float acc = 0.0f;
    for (int j = 0; j < T; ++j) acc = __builtin_fmaf(wsh[h][j], v[(t0 + j) * 128 + h * 32 + lane], acc);
    out[i * 128 + h * 32 + lane] = acc * gate[i * 128 + h * 32 + lane];
  }
}

// ---------------------------------------------------------------- fused pair representation
// The whole per-pair chain of the sequence decoder and the structure module's pair inputs in one
// pass over 32-pair wave tiles (pst_device.h layout, f32 MFMA), instead of ~12 library GEMMs and
// elementwise passes over N² × 256 tensors in HBM (sequence_decoder.py:69-99, folding.py:260-275):
//   P      = left[i] ⊙ right[j]                                  (256)
//   pair0  = LN_out( out2(relu(out1(P))) + right1(P) )           (128)
//   lin    = seq_linear([PE(j − i) | pair0]) = U[j − i] + pair0 · W_seq[128:256]
//            (U = PE · W_seq[0:128] + b, a 1 023-row table built at pst_decoder_create)
//   z      = pt2(relu(pt1(LN_pt(lin))))                          (Transition output, 128)
//   zln    = LN_pair(z);  b2d = (zln · W_att2d + b) / sqrt(3)     (12 heads)
// Only zln and b2d go to HBM (z too when the decoder keeps debug intermediates).
struct PairArgs {
  const float* left;   // [N][256] natural
  const float* right;  // [N][256]
  const float4* f_out1[2][2];  // [k chunk][out chunk]
  const float* pb_out1[2];     // perm bias chunks (applied with the ReLU, just in time)
  const float4* f_out2[2];
  const float4* bf_out2;
  const float4* f_r1[2];
  const float* pb_r1;
  const float *ln1_s, *ln1_o;  // pair representation out LN (perm)
  const float* U;              // [1023][128] perm
  const float4* f_seqb;
  const float *ln2_s, *ln2_o;  // transition input LN
  const float4* f_pt1[2];
  const float* pb_pt1[2];
  const float4* f_pt2[2];
  const float4* bf_pt2;
  const float *ln3_s, *ln3_o;  // structure-module pair LN
  const float* f_att2d;        // narrow fragments [64][64]
  const float* b_att2d;        // [12]
  float* z;                    // [NP][128] natural, or null
  float* zln;                  // [NP][128] natural
  float* b2d;                  // [NP][12]
  int64_t NP;
  DecBatch bt;
};

// natural-order 128-channel rows <-> the wave tile (lane half h holds channels 32M + 8q + 4h + i)
__device__ __forceinline__ void tile_load_nat(Tile& t, const float* __restrict__ row) {
  const int h = lane_id() >> 5;
#pragma unroll
  for (int M = 0; M < 4; ++M)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float4 v = *reinterpret_cast<const float4*>(row + 32 * M + 8 * q + 4 * h);
      t.m[M][4 * q + 0] = v.x;
      t.m[M][4 * q + 1] = v.y;
      t.m[M][4 * q + 2] = v.z;
      t.m[M][4 * q + 3] = v.w;
    }
}
__device__ __forceinline__ void tile_store_nat(const Tile& t, float* __restrict__ row) {
  const int h = lane_id() >> 5;
#pragma unroll
  for (int M = 0; M < 4; ++M)
#pragma unroll
    for (int q = 0; q < 4; ++q)
      *reinterpret_cast<float4*>(row + 32 * M + 8 * q + 4 * h) =
          make_float4(t.m[M][4 * q], t.m[M][4 * q + 1], t.m[M][4 * q + 2], t.m[M][4 * q + 3]);
}
__device__ __forceinline__ void tile_mul_nat(Tile& t, const float* __restrict__ row) {
  const int h = lane_id() >> 5;
#pragma unroll
  for (int M = 0; M < 4; ++M)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float4 v = *reinterpret_cast<const float4*>(row + 32 * M + 8 * q + 4 * h);
      t.m[M][4 * q + 0] *= v.x;
      t.m[M][4 * q + 1] *= v.y;
      t.m[M][4 * q + 2] *= v.z;
      t.m[M][4 * q + 3] *= v.w;
    }
}

__global__ __launch_bounds__(256) void k_pair_fused(PairArgs a) {
  const int lane = threadIdx.x & 63;
  const int64_t p = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 32 + (lane & 31);
  if (((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 32 >= a.NP) return;  // wave-uniform
  const bool valid = p < a.NP;
  const int64_t pc = valid ? p : a.NP - 1;
  const int b = pair_protein(a.bt, pc);
  const int64_t n0 = a.bt.node_off[b];
  const int64_t Nb = a.bt.node_off[b + 1] - n0, loc = pc - a.bt.pair_off[b];
  const int64_t il = loc / Nb, jl = loc - il * Nb;
  const float* lrow = a.left + (n0 + il) * 256;
  const float* rrow = a.right + (n0 + jl) * 256;
  Tile A0, A1, H, Q;
  tile_load_nat(A0, lrow);
  tile_mul_nat(A0, rrow);
  tile_load_nat(A1, lrow + 128);
  tile_mul_nat(A1, rrow + 128);
  // pair0 = out2(relu(out1(P) + b1)) + b2 + right1(P) + b_r1, then LN
  tile_zero(H);
  tile_gemm(H, A0, a.f_out1[0][0]);
  tile_gemm(H, A1, a.f_out1[1][0]);
  tile_gemm_bf(Q, H, a.f_out2[0], a.bf_out2, ActBiasRelu{a.pb_out1[0]});
  tile_zero(H);
  tile_gemm(H, A0, a.f_out1[0][1]);
  tile_gemm(H, A1, a.f_out1[1][1]);
  tile_gemm_f(Q, H, a.f_out2[1], ActBiasRelu{a.pb_out1[1]});
  tile_gemm(Q, A0, a.f_r1[0]);
  tile_gemm(Q, A1, a.f_r1[1]);
  tile_add_vec(Q, a.pb_r1);
  tile_layer_norm(Q, a.ln1_s, a.ln1_o);
  // seq_linear over [PE(j - i) | pair0]
  tile_load_perm(A0, a.U + (jl - il + 511) * 128);
  tile_gemm(A0, Q, a.f_seqb);
  tile_layer_norm(A0, a.ln2_s, a.ln2_o);
  // transition (no residual): z = pt2(relu(pt1(x) + b1)) + b2
  tile_zero(H);
  tile_gemm(H, A0, a.f_pt1[0]);
  tile_gemm_bf(Q, H, a.f_pt2[0], a.bf_pt2, ActBiasRelu{a.pb_pt1[0]});
  tile_zero(H);
  tile_gemm(H, A0, a.f_pt1[1]);
  tile_gemm_f(Q, H, a.f_pt2[1], ActBiasRelu{a.pb_pt1[1]});
  if (a.z && valid) tile_store_nat(Q, a.z + p * 128);
  tile_layer_norm(Q, a.ln3_s, a.ln3_o);
  if (valid) tile_store_nat(Q, a.zln + p * 128);
  // attention 2-D bias: 12 outputs of one narrow accumulator (rows = output channels)
  f32x16 acc = {};
  tile_gemm_narrow(acc, Q, a.f_att2d);
  if (valid) {
    const int h = lane >> 5;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int o = (r & 3) + 8 * (r >> 2) + 4 * h;
      if (o < 12) a.b2d[p * 12 + o] = (acc[r] + a.b_att2d[o]) * 0.577350269189626f;
    }
  }
}

// ---------------------------------------------------------------- structure module helpers
__device__ __forceinline__ void quat_to_rot(const float* q, float* r) {
  // QUAT_TO_ROT contraction (quat_affine.py:43-56, 143-157)
  const float w = q[0], x = q[1], y = q[2], z = q[3];
  r[0] = w * w + x * x - y * y - z * z;
  r[1] = 2.0f * (x * y) - 2.0f * (w * z);
  r[2] = 2.0f * (x * z) + 2.0f * (w * y);
  r[3] = 2.0f * (x * y) + 2.0f * (w * z);
  r[4] = w * w - x * x + y * y - z * z;
  r[5] = 2.0f * (y * z) - 2.0f * (w * x);
  r[6] = 2.0f * (x * z) - 2.0f * (w * y);
  r[7] = 2.0f * (y * z) + 2.0f * (w * x);
  r[8] = w * w - x * x - y * y + z * z;
}

// affine tensor [N][7] (unit quaternion, translation) → rotation [N][9]; identity init
__global__ void k_affine_init(float* __restrict__ aff, float* __restrict__ rot, int N) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  const float a[7] = {1.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int c = 0; c < 7; ++c) aff[i * 7 + c] = a[c];
  quat_to_rot(a, rot + i * 9);
}

// QuatAffine.pre_compose (quat_affine.py:288-317): q += q ⊗ (0, v); t += R·dt; renormalise
__device__ __forceinline__ void affine_update(float* __restrict__ aff, float* __restrict__ rot, const float* u, int i) {
  float* a = aff + i * 7;
  float* R = rot + i * 9;
  const float q0 = a[0], q1 = a[1], q2 = a[2], q3 = a[3];
  const float v1 = u[0], v2 = u[1], v3 = u[2];
  float nq[4];
  nq[0] = q0 + (-(q1 * v1) - q2 * v2 - q3 * v3);
  nq[1] = q1 + (q0 * v1 + q2 * v3 - q3 * v2);
  nq[2] = q2 + (q0 * v2 - q1 * v3 + q3 * v1);
  nq[3] = q3 + (q0 * v3 + q1 * v2 - q2 * v1);
  float dt[3];
  for (int r = 0; r < 3; ++r) dt[r] = R[3 * r] * u[3] + R[3 * r + 1] * u[4] + R[3 * r + 2] * u[5];
  const float nrm = sqrtf(nq[0] * nq[0] + nq[1] * nq[1] + nq[2] * nq[2] + nq[3] * nq[3]);
  for (int c = 0; c < 4; ++c) a[c] = nq[c] / nrm;
  for (int c = 0; c < 3; ++c) a[4 + c] = a[4 + c] + dt[c];
  quat_to_rot(a, R);
}

// IPA points to the global frame (apply_to_point, quat_affine.py): q [N][12][4][3], kv [N][12][12][3].
// Also writes the keys k_ipa_attn's logits read, transposed to [feature][N] so its
// thread-per-key loads coalesce: kT [192][N] (scalar keys, head-major) and kpT [144][N] (the
// 4 key points of each head, xyz).
__global__ void k_ipa_points(const float* __restrict__ qpl /*[N][144]*/, const float* __restrict__ kvpl /*[N][432]*/,
                             const float* __restrict__ aff, const float* __restrict__ rot, float* __restrict__ qpg,
                             float* __restrict__ kvpg, const float* __restrict__ kvs /*[N][384]*/,
                             float* __restrict__ kT, float* __restrict__ kpT, int N, int ld) {
  const int i = blockIdx.x, t = threadIdx.x;  // 192 threads: 48 q points + 144 kv points
  if (i >= N) return;
  kT[(int64_t)t * N + i] = kvs[(int64_t)i * ld + (t / 16) * 32 + t % 16];
  const float* R = rot + i * 9;
  const float* tr = aff + i * 7 + 4;
  float x, y, z;
  float* dst;
  int kp = -1;  // row of kpT for key points
  if (t < 48) {
    x = qpl[(int64_t)i * ld + t];
    y = qpl[(int64_t)i * ld + 48 + t];
    z = qpl[(int64_t)i * ld + 96 + t];
    dst = qpg + ((int64_t)i * 48 + t) * 3;
  } else {
    const int p = t - 48;
    x = kvpl[(int64_t)i * ld + p];
    y = kvpl[(int64_t)i * ld + 144 + p];
    z = kvpl[(int64_t)i * ld + 288 + p];
    dst = kvpg + ((int64_t)i * 144 + p) * 3;
    if (p % 12 < 4) kp = ((p / 12) * 4 + p % 12) * 3;
  }
  for (int r = 0; r < 3; ++r) {
    const float v = R[3 * r] * x + R[3 * r + 1] * y + R[3 * r + 2] * z + tr[r];
    dst[r] = v;
    if (kp >= 0) kpT[(int64_t)(kp + r) * N + i] = v;
  }
}

// Invariant point attention for query residue i (folding.py:69-289): logits over all N residues,
// softmax, then the 2112 output features [scalar 192 | local points x,y,z 3×96 | norms 96 |
// pair 1536]. One workgroup per i.
// The attention weights live in LDS transposed, attT[j][ATT_LD] (heads 0..11 of key j, row
// stride 13 words: odd, so a wave's 64 consecutive keys of one head hit 32 distinct banks in the
// softmax, and the MFMA operand reads below conflict at most 2-way).
// The pair attention Σ_j att[h][j]·z_ij[c] (12 heads × 128 channels, the largest of the weighted
// sums) runs on v_mfma_f32_16x16x4_f32 — D[c][h] = Σ_j z[j][c]·att[h][j], wave w owning channels
// 32w..32w+31 as two 16-row blocks, the 12 heads in columns 0..11 of the 16. That instruction is
// a k-ascending fmaf chain (tools/probe/mfma_probe.hip: 256/256 bitwise), so every sum is the
// in-order chain over j from 0 (round 3 measured it bitwise equal to per-query VALU fmaf chains;
// that form is tools/variants/decode_ab.patch). The attention weights go to att_out for the
// value sums and the local frames (k_ipa_values).
constexpr int ATT_LD = 13;
typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_ipa_attn(const float* __restrict__ qs /*[N][192]*/,
                                                  const float* __restrict__ qpg,
                                                  const float* __restrict__ b2d_all /*[pairs][12], × sqrt(1/3)*/,
                                                  const float* __restrict__ zln_all /*[pairs][128]*/,
                                                  const float* __restrict__ pw /*[12]*/,
                                                  const float* __restrict__ aff, const float* __restrict__ rot,
                                                  float* __restrict__ feat /*[N][2112]*/, DecBatch bt,
                                                  const float* __restrict__ kT_all /*[192][Ntot]*/,
                                                  const float* __restrict__ kpT_all /*[144][Ntot]*/, int Ntot,
                                                  int ld /*row stride of qs*/,
                                                  float* __restrict__ att_out /*[pairs][12]*/) {
  __shared__ float attT[512 * ATT_LD];
  const int64_t ig = blockIdx.x;
  const int tid = threadIdx.x;
  const int bprot = bt.node_prot[ig];
  const int64_t n0 = bt.node_off[bprot];
  const int N = (int)(bt.node_off[bprot + 1] - n0);
  const int il = (int)(ig - n0);
  // protein-local views: pair rows (il, j) of b2d/zln
  const float* b2d = b2d_all + (bt.pair_off[bprot] + (int64_t)il * N) * 12;
  const float* zln = zln_all + (bt.pair_off[bprot] + (int64_t)il * N) * 128;
  const float sw = 0.144337567297406f;  // sqrt(1 / (3 * 16))
  // logits: one key per thread, all 12 heads, from 16-byte loads of the key's rows; the query
  // (scaled scalar part and global points) is shared through LDS
  __shared__ float qsh[192 + 144];
  for (int e = tid; e < 192; e += 256) qsh[e] = sw * qs[ig * ld + e];
  for (int e = tid; e < 144; e += 256) qsh[192 + e] = qpg[ig * 144 + e];
  __syncthreads();
  const float* kT = kT_all + n0;  // column j = key j of this protein
  const float* kpT = kpT_all + n0;
  for (int j = tid; j < N; j += 256) {
    const float4* brow = reinterpret_cast<const float4*>(b2d + (int64_t)j * 12);
    float bb[12];
#pragma unroll
    for (int u = 0; u < 3; ++u) {
      const float4 v = brow[u];
      bb[4 * u] = v.x; bb[4 * u + 1] = v.y; bb[4 * u + 2] = v.z; bb[4 * u + 3] = v.w;
    }
#pragma unroll 2
    for (int h = 0; h < 12; ++h) {
      // transposed key rows: lanes read consecutive keys (coalesced)
      float k[16], kp[12];
#pragma unroll
      for (int c = 0; c < 16; ++c) k[c] = kT[(int64_t)(h * 16 + c) * Ntot + j];
#pragma unroll
      for (int c = 0; c < 12; ++c) kp[c] = kpT[(int64_t)(h * 12 + c) * Ntot + j];
      float sc = 0.0f;
#pragma unroll
      for (int c = 0; c < 16; ++c) sc = __builtin_fmaf(qsh[h * 16 + c], k[c], sc);
      float pt = 0.0f;
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        const float* qp = qsh + 192 + (h * 4 + p) * 3;
        const float dx = qp[0] - kp[3 * p], dy = qp[1] - kp[3 * p + 1], dz = qp[2] - kp[3 * p + 2];
        const float d2 = (dx * dx + dy * dy) + dz * dz;
        pt += pw[h] * d2;
      }
      attT[j * ATT_LD + h] = (sc + (-0.5f * pt)) + bb[h];
    }
  }
  __syncthreads();
  // softmax per head (waves 0..3 take heads h, h+4, h+8)
  {
    const int lane = tid & 63, w = tid >> 6;
    for (int h = w; h < 12; h += 4) {
      float mx = -INFINITY;
      for (int j = lane; j < N; j += 64) mx = fmaxf(mx, attT[j * ATT_LD + h]);
      for (int m = 32; m >= 1; m >>= 1) mx = fmaxf(mx, __shfl_xor(mx, m));
      float s = 0.0f;
      for (int j = lane; j < N; j += 64) {
        float e = expf(attT[j * ATT_LD + h] - mx);
        attT[j * ATT_LD + h] = e;
        s += e;
      }
      for (int m = 32; m >= 1; m >>= 1) s += __shfl_xor(s, m);
      for (int j = lane; j < N; j += 64) attT[j * ATT_LD + h] = attT[j * ATT_LD + h] / s;
    }
  }
  __syncthreads();
  float* f = feat + ig * 2112;
  {
    // the attention weights of query i for k_ipa_values: att_out[(pair row (i, j)) * 12 + h]
    float* ao = att_out + (bt.pair_off[bprot] + (int64_t)il * N) * 12;
    for (int e = tid; e < N * 12; e += 256) ao[e] = attT[(e / 12) * ATT_LD + e % 12];
  }
  {
    // pair attention on the matrix cores: lane (i = lane & 15, g = lane >> 4) feeds A = z[4s+g][c0+i]
    // and B = att[head i][4s+g] (0 for the 4 padding heads); after the chain it holds
    // D[c0 + 4g + r][head i], r = 0..3
    const int lane = tid & 63, w = tid >> 6;
    const int i = lane & 15, g = lane >> 4;
    const int cA = 32 * w + i, cB = cA + 16;
    const bool hv = i < 12;
    f32x4 accA = {0.f, 0.f, 0.f, 0.f}, accB = {0.f, 0.f, 0.f, 0.f};
    const float* zrow = zln + (int64_t)g * 128;
    int s = 0;
    const int S = N / 4;  // whole k-steps; a tail of N % 4 keys runs as one zero-padded step
    for (; s + 8 <= S; s += 8) {  // 8 k-steps of z loads in flight per trip
      float za[8], zb[8], bt4[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const float* zr = zrow + (int64_t)(4 * (s + u)) * 128;
        za[u] = zr[cA];
        zb[u] = zr[cB];
        bt4[u] = hv ? attT[(4 * (s + u) + g) * ATT_LD + i] : 0.0f;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        accA = __builtin_amdgcn_mfma_f32_16x16x4f32(za[u], bt4[u], accA, 0, 0, 0);
        accB = __builtin_amdgcn_mfma_f32_16x16x4f32(zb[u], bt4[u], accB, 0, 0, 0);
      }
    }
    for (; 4 * s < N; ++s) {
      // last steps (and a partial one): keys j >= N enter as 0·0 products, which leave the chain unchanged
      const int j = 4 * s + g;
      const bool jv = j < N;
      const float* zr = zrow + (int64_t)(4 * s) * 128;
      const float za = jv ? zr[cA] : 0.0f, zb = jv ? zr[cB] : 0.0f;
      const float bv = hv && jv ? attT[j * ATT_LD + i] : 0.0f;
      accA = __builtin_amdgcn_mfma_f32_16x16x4f32(za, bv, accA, 0, 0, 0);
      accB = __builtin_amdgcn_mfma_f32_16x16x4f32(zb, bv, accB, 0, 0, 0);
    }
    if (hv) {
      float* o = f + 576 + i * 128 + 32 * w + 4 * g;
      *reinterpret_cast<float4*>(o) = make_float4(accA[0], accA[1], accA[2], accA[3]);
      *reinterpret_cast<float4*>(o + 16) = make_float4(accB[0], accB[1], accB[2], accB[3]);
    }
  }
}

// IPA value sums, batched over queries (the per-query form re-read every key's values from L2:
// 1 GB per fold iteration at 8 x 256 residues). One wave per (16 queries of one protein, head h):
// D[q][o] = Σ_j att[q][h][j] · V_h[j][o] on v_mfma_f32_16x16x4_f32 for the 16 scalar values and
// the 8 value points × xyz (24) of head h — three 16-wide output blocks (8 columns unused). The
// instruction is a k-ascending fmaf chain, so each sum is the in-order chain over j from 0 that
// a per-query VALU loop would run: identical bits. Scalar outputs go to feat[q][16h + o]. The
// global-frame value points then go to each query's local frame (invert_point) with their norms
// (folding.py:256-275) in this launch (round 6; they were the separate k_ipa_local launch, through
// a [N][288] buffer): the 16 x 24 point coordinates through LDS, two (query, point) pairs per lane,
// the same operations in the same order as before.
__global__ __launch_bounds__(64) void k_ipa_values(const float* __restrict__ att_all, const float* __restrict__ kvs_all,
                                                   const float* __restrict__ kvpg_all, float* __restrict__ feat,
                                                   const float* __restrict__ aff, const float* __restrict__ rot,
                                                   DecBatch bt, const int32_t* __restrict__ vt_prot,
                                                   const int32_t* __restrict__ vt_q0, int ld) {
  __shared__ float sp[16][25];  // [query][point coordinate o = 3p + xyz] (+1 pad)
  const int tile = blockIdx.x, h = blockIdx.y;
  const int lane = threadIdx.x, i = lane & 15, g = lane >> 4;
  const int b = vt_prot[tile], q0 = vt_q0[tile];
  const int64_t n0 = bt.node_off[b];
  const int N = (int)(bt.node_off[b + 1] - n0);
  const int qa = q0 + i;  // A-operand row (query) of this lane
  const int qc = qa < N ? qa : N - 1;
  const float* arow = att_all + (bt.pair_off[b] + (int64_t)qc * N) * 12 + h;
  const float* vs = kvs_all + n0 * ld + h * 32 + 16 + i;
  const float* vp = kvpg_all + n0 * 432 + (h * 12 + 4) * 3 + i;
  f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = acc0, acc2 = acc0;
  // 8 k-steps of operands loaded per trip, then their 24 MFMAs (one memory round trip per 32 keys;
  // 16 per trip measured slower: 183 -> 202 us per 8 x 256 decode)
  const int S = (N + 3) / 4;
  for (int s0 = 0; s0 < S; s0 += 8) {
    float a[8], b0[8], b1[8], b2[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int j = 4 * (s0 + u) + g;
      const bool jv = j < N;
      a[u] = jv ? arow[(int64_t)j * 12] : 0.0f;
      b0[u] = jv ? vs[(int64_t)j * ld] : 0.0f;
      b1[u] = jv ? vp[(int64_t)j * 432] : 0.0f;
      b2[u] = jv && i < 8 ? vp[(int64_t)j * 432 + 16] : 0.0f;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u], b0[u], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u], b1[u], acc1, 0, 0, 0);
      acc2 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u], b2[u], acc2, 0, 0, 0);
    }
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int q = 4 * g + r;
    sp[q][i] = acc1[r];
    if (i < 8) sp[q][16 + i] = acc2[r];
    if (q0 + q >= N) continue;
    feat[(n0 + q0 + q) * 2112 + h * 16 + i] = acc0[r];
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int e = lane + 64 * k, q = e >> 3, p = e & 7;
    if (q0 + q >= N) continue;
    const int64_t ig = n0 + q0 + q;
    const float* R = rot + ig * 9;
    const float* tr = aff + ig * 7 + 4;
    const float gx = sp[q][3 * p + 0] - tr[0];
    const float gy = sp[q][3 * p + 1] - tr[1];
    const float gz = sp[q][3 * p + 2] - tr[2];
    const float lx = R[0] * gx + R[3] * gy + R[6] * gz;
    const float ly = R[1] * gx + R[4] * gy + R[7] * gz;
    const float lz = R[2] * gx + R[5] * gy + R[8] * gz;
    float* f = feat + ig * 2112;
    const int c = h * 8 + p;
    f[192 + c] = lx;
    f[288 + c] = ly;
    f[384 + c] = lz;
    f[480 + c] = sqrtf(((1e-8f + lx * lx) + ly * ly) + lz * lz);
  }
}

// Backbone torsions → frames → atom14 → atom37 (folding.py:674-746, all_atom.py:473-595, :122-135)
// plus the trajectory row (affine × [1,1,1,1,10,10,10]).
// One node i: this iteration's backbone update (affine_update, from the 6 update values `u6`), then
// the torsions (the 6 unnormalised sin / cos values `un6`), trajectory row and, on the last
// iteration, the atoms. Runs at the end of k_fold_tail (round 6; it was the k_sc_geom launch).
__device__ void sc_geom_node(float* __restrict__ aff, float* __restrict__ rot, const float* u6, const float* un6,
                             float* __restrict__ angles /*[N][3][2]*/, float* __restrict__ traj /*[N][7]*/,
                             float* __restrict__ atom37 /*[N][37][3] or null*/,
                             float* __restrict__ atom14 /*[N][14][3] or null*/, int i) {
  affine_update(aff, rot, u6, i);
  const float* a = aff + i * 7;
  const float* R = rot + i * 9;
  float sn[4] = {0.f, 0.f, 0.f, 0.f}, cs[4] = {1.f, 1.f, 1.f, 1.f};
  for (int t = 0; t < 3; ++t) {
    const float s = un6[2 * t], c = un6[2 * t + 1];
    const float d = sqrtf(fmaxf(s * s + c * c, 1e-12f));
    sn[t + 1] = s / d;
    cs[t + 1] = c / d;
    angles[(i * 3 + t) * 2 + 0] = sn[t + 1];
    angles[(i * 3 + t) * 2 + 1] = cs[t + 1];
  }
  for (int c = 0; c < 4; ++c) traj[i * 7 + c] = a[c];
  for (int c = 0; c < 3; ++c) traj[i * 7 + 4 + c] = a[4 + c] * 10.0f;
  if (!atom37 && !atom14) return;
  const float T0[3] = {a[4] * 10.0f, a[5] * 10.0f, a[6] * 10.0f};  // scale_translation(position_scale)
  float fr[4][12];  // per group: rot (9, row-major) + trans (3), to global
  for (int g = 0; g < 4; ++g) {
    // default frame ∘ rotation about x by torsion g (group 0: identity rotation)
    float m[9], mt[3];
    for (int r = 0; r < 3; ++r) {
      for (int c = 0; c < 3; ++c) m[3 * r + c] = kDefaultFrame[g][r][c];
      mt[r] = kDefaultFrame[g][r][3];
    }
    const float rx[9] = {1.f, 0.f, 0.f, 0.f, cs[g], -sn[g], 0.f, sn[g], cs[g]};
    float mb[9];
    for (int r = 0; r < 3; ++r)
      for (int c = 0; c < 3; ++c) mb[3 * r + c] = m[3 * r] * rx[c] + m[3 * r + 1] * rx[3 + c] + m[3 * r + 2] * rx[6 + c];
    // backbone-to-global ∘ frame-to-backbone
    for (int r = 0; r < 3; ++r) {
      for (int c = 0; c < 3; ++c)
        fr[g][3 * r + c] = R[3 * r] * mb[c] + R[3 * r + 1] * mb[3 + c] + R[3 * r + 2] * mb[6 + c];
      fr[g][9 + r] = (R[3 * r] * mt[0] + R[3 * r + 1] * mt[1] + R[3 * r + 2] * mt[2]) + T0[r];
    }
  }
  float p14[14][3];
  for (int at = 0; at < 14; ++at) {
    const float* F = fr[kAtom14Group[at]];
    for (int r = 0; r < 3; ++r) {
      const float v = F[3 * r] * kAtom14Pos[at][0] + F[3 * r + 1] * kAtom14Pos[at][1] + F[3 * r + 2] * kAtom14Pos[at][2] +
                      F[9 + r];
      p14[at][r] = v * kAtom14Mask[at];
    }
  }
  if (atom14)
    for (int at = 0; at < 14; ++at)
      for (int r = 0; r < 3; ++r) atom14[(i * 14 + at) * 3 + r] = p14[at][r];
  if (atom37) {
    // atom14_to_atom37 for the dummy ALA aatype, then × atom37_gt_exists (N, CA, C, O)
    for (int at = 0; at < 37; ++at) {
      const float gt = (at == 0 || at == 1 || at == 2 || at == 4) ? 1.0f : 0.0f;
      for (int r = 0; r < 3; ++r) atom37[(i * 37 + at) * 3 + r] = (p14[kAla37To14[at]][r] * kAla37Mask[at]) * gt;
    }
  }
}

}  // namespace dec
}  // namespace pst

// ======================================================================== host side / C ABI
using namespace pst::dec;

namespace {

struct Lin {
  const float* w = nullptr;
  const float* b = nullptr;
  int in = 0, out = 0;
};
struct LnP {
  const float* s = nullptr;
  const float* o = nullptr;
};

struct DecWeights {
  Lin up_proj;
  // upsampler block b: norms and attention weights are [3][...] stacked
  LnP qn[3], dn[3];
  const float *wq[3], *wk[3], *wv[3], *wg[3], *gb[3], *wo[3], *ob[3];
  LnP rt_ln[3], ot_ln[3];
  Lin rt1[3], rt2[3], ot1[3], ot2[3];
  Lin proj_original;
  Lin seq_linear;
  LnP pt_ln;
  Lin pt1, pt2;
  LnP pr_ln_in, pr_ln_out;
  Lin left, right, right1, out1, out2;
  Lin affine_update;
  LnP att_ln;
  const float* tpw;
  Lin att2d, kv_point, kv_scalar, out_proj, q_point, q_scalar;
  Lin sc_in, sc_in1, rb1, rb1_1, rb2, rb2_1, angles;
  Lin tr[3];
  LnP tr_ln;
  Lin init_proj;
  LnP pair_ln, single_ln;
};

}  // namespace

struct pst_decoder {
  int device = 0;
  pst_model_desc desc{};
  int D = 6, df = 1;
  hipStream_t stream = nullptr;
  std::string err;
  float* d_blob = nullptr;
  int* d_levels = nullptr;
  float* d_pe_node = nullptr;  // PE(i; 512) [512][128]
  float* d_pe_tok = nullptr;   // PE(t; 512/df) [512/df][128]
  float* d_pe_rel = nullptr;   // PE(d; 512), d = -511..511 [1023][128]
  float* d_pw = nullptr;       // IPA point weights [12]
  float* d_ipa_w = nullptr;  // [384][1152]: q_scalar | kv_scalar | q_point | kv_point weights
  float* d_ipa_b = nullptr;  // [1152] their biases
  DecWeights W{};
  float* d_pair = nullptr;  // fused pair kernel: fragments, perm vectors, U table (k_pair_fused)
  PairArgs pair{};          // pointers into d_pair (per-call fields filled by decode_group)
  // scratch (grow-only, sized for N = 512)
  void* ws = nullptr;
  size_t ws_bytes = 0;
  // last call's intermediates (per protein offsets) for pst_decoder_debug
  std::vector<float> last_single, last_pair, last_traj, last_angles, last_atom14;
  // pinned staging of a group's index arrays (one H2D copy per group) and the event of its copy
  char* h_up = nullptr;
  size_t h_up_bytes = 0;
  float* h_atoms = nullptr;  // pinned staging of a group's atom37 output (D2H at full rate)
  size_t h_atoms_floats = 0;
  hipEvent_t up_ev = nullptr;
  // decode_group's kernel sequence as HIP graphs, keyed by the group's shape (decode_group)
  std::map<std::vector<int64_t>, hipGraphExec_t> graphs;
  // stage timing (pst_decoder_set_timing; measurement): HIP events around the upsampler, the pair
  // chain's inputs, k_pair_fused and the 8 fold iterations, launched directly (no graph replay)
  // while enabled; ms summed over the groups of the calls since enabling
  bool timing = false;
  hipEvent_t tev[PST_DECODER_N_STAGES + 1] = {};
  float tms[PST_DECODER_N_STAGES] = {};
};

namespace {

std::string g_dec_create_error;

#define DCHK(x)                                                               \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      dec->err = std::string(#x) + ": " + hipGetErrorString(e_);              \
      return PST_E_HIP;                                                       \
    }                                                                         \
  } while (0)

int dfail(pst_decoder* dec, int code, const std::string& m) {
  dec->err = m;
  return code;
}

// walk the decoder-half blob in pst_amd.params.decoder_param_spec order
size_t walk_decoder(const float* base, int D, DecWeights* W) {
  size_t o = 0;
  auto take = [&](size_t n) {
    const float* p = base ? base + o : nullptr;
    o += n;
    return p;
  };
  auto lin = [&](Lin& l, int in, int out) {
    l.in = in;
    l.out = out;
    l.w = take((size_t)in * out);
    l.b = take(out);
  };
  const int H = 128;
  lin(W->up_proj, D, H);
  // _scaler_spec(US/cross_attn_scaler_iteration, 3)
  const float *qs = take(3 * H), *qo = take(3 * H), *ds = take(3 * H), *dso = take(3 * H);
  const float *wq = take(3 * H * H), *wk = take(3 * H * H), *wv = take(3 * H * H), *wg = take(3 * H * H);
  const float *gb = take(3 * H), *wo = take(3 * H * H), *ob = take(3 * H);
  const float *rls = take(3 * H), *rlo = take(3 * H), *r1w = take(3 * H * 2 * H), *r1b = take(3 * 2 * H);
  const float *r2w = take(3 * 2 * H * H), *r2b = take(3 * H);
  const float *ols = take(3 * H), *olo = take(3 * H), *o1w = take(3 * H * 2 * H), *o1b = take(3 * 2 * H);
  const float *o2w = take(3 * 2 * H * H), *o2b = take(3 * H);
  if (base)
    for (int b = 0; b < 3; ++b) {
      W->qn[b] = {qs + b * H, qo + b * H};
      W->dn[b] = {ds + b * H, dso + b * H};
      W->wq[b] = wq + (size_t)b * H * H;
      W->wk[b] = wk + (size_t)b * H * H;
      W->wv[b] = wv + (size_t)b * H * H;
      W->wg[b] = wg + (size_t)b * H * H;
      W->gb[b] = gb + b * H;
      W->wo[b] = wo + (size_t)b * H * H;
      W->ob[b] = ob + b * H;
      W->rt_ln[b] = {rls + b * H, rlo + b * H};
      W->rt1[b] = {r1w + (size_t)b * H * 2 * H, r1b + b * 2 * H, H, 2 * H};
      W->rt2[b] = {r2w + (size_t)b * 2 * H * H, r2b + b * H, 2 * H, H};
      W->ot_ln[b] = {ols + b * H, olo + b * H};
      W->ot1[b] = {o1w + (size_t)b * H * 2 * H, o1b + b * 2 * H, H, 2 * H};
      W->ot2[b] = {o2w + (size_t)b * 2 * H * H, o2b + b * H, 2 * H, H};
    }
  lin(W->proj_original, 2 * H, H);
  lin(W->seq_linear, 2 * H, H);
  W->pt_ln = {take(H), take(H)};
  lin(W->pt1, H, 2 * H);
  lin(W->pt2, 2 * H, H);
  W->pr_ln_in = {take(H), take(H)};
  W->pr_ln_out = {take(H), take(H)};
  lin(W->left, H, 2 * H);
  lin(W->right, H, 2 * H);
  lin(W->right1, 2 * H, H);
  lin(W->out1, 2 * H, 2 * H);
  lin(W->out2, 2 * H, H);
  const int S = 384;
  lin(W->affine_update, S, 6);
  W->att_ln = {take(S), take(S)};
  W->tpw = take(12);
  lin(W->att2d, H, 12);
  lin(W->kv_point, S, 432);
  lin(W->kv_scalar, S, S);
  lin(W->out_proj, 2112, S);
  lin(W->q_point, S, 144);
  lin(W->q_scalar, S, 192);
  lin(W->sc_in, S, H);
  lin(W->sc_in1, H, H);
  lin(W->rb1, H, H);
  lin(W->rb1_1, H, H);
  lin(W->rb2, H, H);
  lin(W->rb2_1, H, H);
  lin(W->angles, H, 6);
  for (int t = 0; t < 3; ++t) lin(W->tr[t], S, S);
  W->tr_ln = {take(S), take(S)};
  lin(W->init_proj, H, S);
  W->pair_ln = {take(H), take(H)};
  W->single_ln = {take(H), take(H)};
  return o;
}

// Every decode GEMM is in-tree: k_gemm_mfma (f32 MFMA), or the LDS-tiled VALU k_gemm when the
// operands do not meet its alignment (or PST_DECODE_NO_MFMA=1, for the A/B test). Both compute
// the same fma chains.
thread_local bool t_mfma = true;  // set by decode_group for the current call

// ---- fused fold-iteration tail (k_fold_tail): everything between the IPA output projection and
// the frame update of one structure-module iteration (folding.py:291-455), per 16-node tile, with
// the activations held in LDS across the chained linears:
//   act = LN_att(act);  act += tr2(relu(tr1(relu(tr0(act)))));  act = LN_tr(act)   (Transition)
//   upd = affine_update(act)                                                        (6)
//   sc  = sc_in(relu(act)) + sc_in1(relu(init_act)); sc += rb2(relu(rb1(relu(sc)))) twice
//   unnorm = angles(relu(sc))                                                       (6)
// 11 linears and 2 LayerNorms that ran as 13 launches. The GEMMs run on v_mfma_f32_16x16x4_f32 with
// D[out channel][node]: A = weight rows W[k][n] (the [in][out] layout every decode Lin has), B =
// activations from LDS, one fma chain over k ascending per output (plain fp32, no bitwise claim:
// the decode's tolerance tests hold it to the reference). 8 waves share each GEMM's 16-wide output
// blocks. LDS activations are stored [node][k & 3][k >> 2] (+4 pad) so a lane reads 4 k-steps of
// its B operand with one ds_read_b128.
constexpr int FT_NODES = 16;
typedef float f32x4t __attribute__((ext_vector_type(4)));

struct FoldTailArgs {
  float* act;              // [N][384]: in, act after the IPA output projection; out, after LN_tr
  const float* init_relu;  // [N][128]: relu(initial act)
  float* upd;              // [N][6]
  float* unnorm;           // [N][6]
  int N;
  const float *att_ln_s, *att_ln_o, *tr_ln_s, *tr_ln_o;
  const float *w_tr[3], *b_tr[3];
  const float *w_aff, *b_aff;
  const float *w_sc, *b_sc, *w_sc1, *b_sc1;
  const float *w_rb[4], *b_rb[4];  // rb1, rb2, rb1_1, rb2_1
  const float *w_ang, *b_ang;
  // the iteration's geometry (sc_geom_node) for the tile's nodes after the angles
  float *aff, *rot, *angles, *traj, *atom37, *atom14;
};

// strides of a [16 nodes][C] LDS activation (C = 384 or 128): plane j = k & 3 of node n starts at
// n * ft_sn(C) + j * ft_sj(C)
__host__ __device__ constexpr int ft_sj(int C) { return C / 4 + 4; }
__host__ __device__ constexpr int ft_sn(int C) { return 4 * ft_sj(C); }
__device__ __forceinline__ int ft_at(int C, int node, int c) { return node * ft_sn(C) + (c & 3) * ft_sj(C) + (c >> 2); }

// acc[b] = X (16 nodes x K, LDS, optional ReLU on load) · W[:, 16·blk_b .. +15], blk_b = b0 + b·bstep.
// Fully unrolled over K; the weight operands run PF groups of 4 k-steps (16 k) ahead in a register
// ring (the weights are L2-resident: a fetch is ~1 us, ~4 groups of this wave's MFMAs).
// prefetch depth in groups of 16 k (a build tunable: 8 and 12 measured no faster, fold stage 2.60 ms
// either way; profiles/r05_ab_decode_ft_prefetch.txt)
#ifndef FT_PF
#define FT_PF 4
#endif
template <int NB, bool RELU_IN, int K>
__device__ __forceinline__ void ft_gemm(f32x4t (&acc)[NB], const float* X, const float* __restrict__ W, int N,
                                        int b0, int bstep, int lane) {
  constexpr int G = K / 16, PF = G < FT_PF ? G : FT_PF;
  const int node = lane & 15, j = lane >> 4;
  const float* xb = X + node * ft_sn(K) + j * ft_sj(K);
  int col[NB];
  bool cv[NB];
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    col[b] = 16 * (b0 + b * bstep) + (lane & 15);
    cv[b] = col[b] < N;
    acc[b] = f32x4t{0.f, 0.f, 0.f, 0.f};
  }
  float ring[PF][4][NB];
  auto load = [&](float (&a)[4][NB], int g) {
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int b = 0; b < NB; ++b) a[u][b] = cv[b] ? W[(int64_t)(4 * (4 * g + u) + j) * N + col[b]] : 0.0f;
  };
#pragma unroll
  for (int p = 0; p < PF; ++p) load(ring[p], p);
#pragma unroll
  for (int g = 0; g < G; ++g) {
    f32x4t xv = *reinterpret_cast<const f32x4t*>(xb + 4 * g);
    if (RELU_IN) {
#pragma unroll
      for (int u = 0; u < 4; ++u) xv[u] = xv[u] > 0.0f ? xv[u] : 0.0f;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int b = 0; b < NB; ++b) acc[b] = __builtin_amdgcn_mfma_f32_16x16x4f32(ring[g % PF][u][b], xv[u], acc[b], 0, 0, 0);
    if (g + PF < G) load(ring[g % PF], g + PF);
  }
}

// epilogue into an LDS activation: y = acc + bias (ReLU if RELU_OUT); Y = y, or Y += y (RESID)
template <int NB, bool RELU_OUT, bool RESID>
__device__ __forceinline__ void ft_store(const f32x4t (&acc)[NB], float* Y, int C, const float* __restrict__ bias,
                                         int b0, int bstep, int lane) {
  const int node = lane & 15;
#pragma unroll
  for (int b = 0; b < NB; ++b)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int n = 16 * (b0 + b * bstep) + 4 * (lane >> 4) + r;
      float v = acc[b][r] + bias[n];
      if (RELU_OUT) v = v > 0.0f ? v : 0.0f;
      float* y = Y + ft_at(C, node, n);
      *y = RESID ? *y + v : v;
    }
}

// the same epilogue for a 6-wide output (one block, wave 0) to global rows [N][6] and the tile's
// LDS copy [16][6]
__device__ __forceinline__ void ft_store6(const f32x4t& acc, float* __restrict__ out, float* lds,
                                          const float* __restrict__ bias, int64_t node0, int N, int lane) {
  const int64_t node = node0 + (lane & 15);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int n = 4 * (lane >> 4) + r;
    if (n < 6) {
      const float v = acc[r] + bias[n];
      lds[(lane & 15) * 6 + n] = v;
      if (node < N) out[node * 6 + n] = v;
    }
  }
}

// hk.LayerNorm over the 384 channels of each node, in place in LDS; the operation order of
// k_layernorm (per-lane sums over c = lane + 64 i in i order, then the xor-shuffle reduction)
__device__ __forceinline__ void ft_layernorm384(float* X, int node, const float* __restrict__ s,
                                                const float* __restrict__ o, int lane) {
  float v[6];
  float sum = 0.0f;
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    v[i] = X[ft_at(384, node, lane + 64 * i)];
    sum += v[i];
  }
  for (int m = 32; m >= 1; m >>= 1) sum += __shfl_xor(sum, m);
  const float mean = sum / 384.0f;
  float sq = 0.0f;
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    const float d = v[i] - mean;
    sq += d * d;
  }
  for (int m = 32; m >= 1; m >>= 1) sq += __shfl_xor(sq, m);
  const float rs = 1.0f / sqrtf(sq / 384.0f + 1e-5f);
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    const int c = lane + 64 * i;
    X[ft_at(384, node, c)] = (s[c] * rs) * (v[i] - mean) + o[c];
  }
}

// hk.LayerNorm over 128 channels of one node held in LDS ([node][k & 3][k >> 2] layout), written
// to Y (may be X); k_layernorm's operation order (lane sums c = lane, lane + 64, xor reduction)
__device__ __forceinline__ void ft_layernorm128(const float* X, float* Y, int node, const float* __restrict__ s,
                                                const float* __restrict__ o, int lane) {
  const float v0 = X[ft_at(128, node, lane)], v1 = X[ft_at(128, node, lane + 64)];
  float sum = 0.0f;
  sum += v0;
  sum += v1;
  for (int m = 32; m >= 1; m >>= 1) sum += __shfl_xor(sum, m);
  const float mean = sum / 128.0f;
  float sq = 0.0f;
  const float d0 = v0 - mean, d1 = v1 - mean;
  sq += d0 * d0;
  sq += d1 * d1;
  for (int m = 32; m >= 1; m >>= 1) sq += __shfl_xor(sq, m);
  const float rs = 1.0f / sqrtf(sq / 128.0f + 1e-5f);
  Y[ft_at(128, node, lane)] = (s[lane] * rs) * d0 + o[lane];
  Y[ft_at(128, node, lane + 64)] = (s[lane + 64] * rs) * d1 + o[lane + 64];
}

// The upsampler's Transition on 128-channel rows, fused (modules.py:599-636): x += W2(relu(W1(LN(x))
// + b1)) + b2, hidden 256, per 16-row tile in LDS (the k_fold_tail machinery); one launch instead
// of LayerNorm + two GEMMs.
struct Trans128Args {
  float* x;  // [M][128], updated in place
  int M;
  const float *ln_s, *ln_o, *w1, *b1, *w2, *b2;  // w1 [128][256], w2 [256][128]
};

__global__ __launch_bounds__(512) void k_transition128(Trans128Args a) {
  __shared__ __attribute__((aligned(16))) float X[FT_NODES * ft_sn(128)];
  __shared__ __attribute__((aligned(16))) float Xn[FT_NODES * ft_sn(128)];
  __shared__ __attribute__((aligned(16))) float Hs[FT_NODES * ft_sn(256)];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t row0 = (int64_t)blockIdx.x * FT_NODES;
  for (int e = threadIdx.x; e < FT_NODES * 128; e += 512) {
    const int n = e >> 7, c = e & 127;
    X[ft_at(128, n, c)] = row0 + n < a.M ? a.x[(row0 + n) * 128 + c] : 0.0f;
  }
  __syncthreads();
  ft_layernorm128(X, Xn, 2 * w, a.ln_s, a.ln_o, lane);
  ft_layernorm128(X, Xn, 2 * w + 1, a.ln_s, a.ln_o, lane);
  __syncthreads();
  {
    f32x4t acc[2];
    ft_gemm<2, false, 128>(acc, Xn, a.w1, 256, w, 8, lane);
    ft_store<2, true, false>(acc, Hs, 256, a.b1, w, 8, lane);
  }
  __syncthreads();
  {
    f32x4t acc[1];
    ft_gemm<1, false, 256>(acc, Hs, a.w2, 128, w, 1, lane);
    ft_store<1, false, true>(acc, X, 128, a.b2, w, 1, lane);
  }
  __syncthreads();
  for (int e = threadIdx.x; e < FT_NODES * 128; e += 512) {
    const int n = e >> 7, c = e & 127;
    if (row0 + n < a.M) a.x[(row0 + n) * 128 + c] = X[ft_at(128, n, c)];
  }
}

// LayerNorm of 128-channel rows and two 128 -> 128 projections of the normalised rows, fused (the
// upsampler's query / gate and key / value inputs, modules.py:537-598): y_i = f_i(LN(x)·W_i + b_i)
// with f = identity, × key_dim^-0.5 (F_QSCALE) or sigmoid (F_SIGMOID_OUT); b_i may be null. One
// launch instead of a LayerNorm and two GEMMs.
struct LnProj2Args {
  const float* x;  // [M][128]
  int M;
  const float *ln_s, *ln_o;
  const float *w[2], *b[2];
  int flags[2];
  float* y[2];  // [M][128] each
};

__global__ __launch_bounds__(512) void k_ln_proj2(LnProj2Args a) {
  __shared__ __attribute__((aligned(16))) float X[FT_NODES * ft_sn(128)];
  __shared__ __attribute__((aligned(16))) float Y[2][FT_NODES * ft_sn(128)];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t row0 = (int64_t)blockIdx.x * FT_NODES;
  for (int e = threadIdx.x; e < FT_NODES * 128; e += 512) {
    const int n = e >> 7, c = e & 127;
    X[ft_at(128, n, c)] = row0 + n < a.M ? a.x[(row0 + n) * 128 + c] : 0.0f;
  }
  __syncthreads();
  ft_layernorm128(X, X, 2 * w, a.ln_s, a.ln_o, lane);
  ft_layernorm128(X, X, 2 * w + 1, a.ln_s, a.ln_o, lane);
  __syncthreads();
  for (int p = 0; p < 2; ++p) {  // wave w: output block w of both projections
    f32x4t acc[1];
    ft_gemm<1, false, 128>(acc, X, a.w[p], 128, w, 1, lane);
    const int node = lane & 15;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int n = 16 * w + 4 * (lane >> 4) + r;
      float v = acc[0][r];
      if (a.b[p]) v = v + a.b[p][n];
      if (a.flags[p] & F_SIGMOID_OUT) v = 1.0f / (1.0f + expf(-v));
      if (a.flags[p] & F_QSCALE) v = v * Q_SCALE;
      Y[p][ft_at(128, node, n)] = v;
    }
  }
  __syncthreads();
  for (int p = 0; p < 2; ++p)
    for (int e = threadIdx.x; e < FT_NODES * 128; e += 512) {
      const int n = e >> 7, c = e & 127;
      if (row0 + n < a.M) a.y[p][(row0 + n) * 128 + c] = Y[p][ft_at(128, n, c)];
    }
}

// 12 waves: the 384-wide linears' 24 output blocks two per wave; the 128-wide ones on waves 0-7
constexpr int FT_WAVES = 12;
__global__ __launch_bounds__(64 * FT_WAVES) void k_fold_tail(FoldTailArgs a) {
  __shared__ __attribute__((aligned(16))) float A0[FT_NODES * ft_sn(384)];
  __shared__ __attribute__((aligned(16))) float T1[FT_NODES * ft_sn(384)];
  __shared__ __attribute__((aligned(16))) float T2[FT_NODES * ft_sn(384)];
  __shared__ __attribute__((aligned(16))) float S0[FT_NODES * ft_sn(128)];
  __shared__ __attribute__((aligned(16))) float S1[FT_NODES * ft_sn(128)];
  __shared__ __attribute__((aligned(16))) float IR[FT_NODES * ft_sn(128)];
  __shared__ float UPD[FT_NODES * 6], UN[FT_NODES * 6];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // FT_WAVES waves
  const int64_t node0 = (int64_t)blockIdx.x * FT_NODES;
  // rows in (nodes past N: zeros, never stored)
  for (int e = threadIdx.x; e < FT_NODES * 384; e += 64 * FT_WAVES) {
    const int n = e / 384, c = e - 384 * (e / 384);
    A0[ft_at(384, n, c)] = node0 + n < a.N ? a.act[(node0 + n) * 384 + c] : 0.0f;
  }
  for (int e = threadIdx.x; e < FT_NODES * 128; e += 64 * FT_WAVES) {
    const int n = e >> 7, c = e & 127;
    IR[ft_at(128, n, c)] = node0 + n < a.N ? a.init_relu[(node0 + n) * 128 + c] : 0.0f;
  }
  __syncthreads();
  for (int nd = w; nd < FT_NODES; nd += FT_WAVES) ft_layernorm384(A0, nd, a.att_ln_s, a.att_ln_o, lane);
  __syncthreads();
  {  // Transition: three 384 x 384 linears, wave w owns output blocks w, w + 12
    f32x4t acc[2];
    ft_gemm<2, false, 384>(acc, A0, a.w_tr[0], 384, w, FT_WAVES, lane);
    ft_store<2, true, false>(acc, T1, 384, a.b_tr[0], w, FT_WAVES, lane);
    __syncthreads();
    ft_gemm<2, false, 384>(acc, T1, a.w_tr[1], 384, w, FT_WAVES, lane);
    ft_store<2, true, false>(acc, T2, 384, a.b_tr[1], w, FT_WAVES, lane);
    __syncthreads();
    ft_gemm<2, false, 384>(acc, T2, a.w_tr[2], 384, w, FT_WAVES, lane);
    ft_store<2, false, true>(acc, A0, 384, a.b_tr[2], w, FT_WAVES, lane);  // act += ...
    __syncthreads();
  }
  for (int nd = w; nd < FT_NODES; nd += FT_WAVES) ft_layernorm384(A0, nd, a.tr_ln_s, a.tr_ln_o, lane);
  __syncthreads();
  for (int e = threadIdx.x; e < FT_NODES * 384; e += 64 * FT_WAVES) {  // act out (the next iteration's input)
    const int n = e / 384, c = e - 384 * (e / 384);
    if (node0 + n < a.N) a.act[(node0 + n) * 384 + c] = A0[ft_at(384, n, c)];
  }
  {
    f32x4t acc[1], acc2[1];
    if (w == 8) {  // backbone affine update (6 outputs)
      ft_gemm<1, false, 384>(acc, A0, a.w_aff, 6, 0, 1, lane);
      ft_store6(acc[0], a.upd, UPD, a.b_aff, node0, a.N, lane);
    }
    // sidechain input: sc_in(relu(act)) + sc_in1(relu(init_act)), wave w owns block w of 8
    if (w < 8) {
    ft_gemm<1, true, 384>(acc, A0, a.w_sc, 128, w, 1, lane);
    ft_gemm<1, false, 128>(acc2, IR, a.w_sc1, 128, w, 1, lane);
      const int node = lane & 15;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = 16 * w + 4 * (lane >> 4) + r;
        S0[ft_at(128, node, n)] = (acc[0][r] + a.b_sc[n]) + (acc2[0][r] + a.b_sc1[n]);
      }
    }
    __syncthreads();
    // two residual blocks: sc += rb2(relu(rb1(relu(sc)))), waves 0-7 one block each
    for (int rb = 0; rb < 2; ++rb) {
      if (w < 8) {
        ft_gemm<1, true, 128>(acc, S0, a.w_rb[2 * rb], 128, w, 1, lane);
        ft_store<1, true, false>(acc, S1, 128, a.b_rb[2 * rb], w, 1, lane);
      }
      __syncthreads();
      if (w < 8) {
        ft_gemm<1, false, 128>(acc, S1, a.w_rb[2 * rb + 1], 128, w, 1, lane);
        ft_store<1, false, true>(acc, S0, 128, a.b_rb[2 * rb + 1], w, 1, lane);
      }
      __syncthreads();
    }
    if (w == 0) {  // torsion angles (unnormalised, 6 outputs)
      ft_gemm<1, true, 128>(acc, S0, a.w_ang, 6, 0, 1, lane);
      ft_store6(acc[0], a.unnorm, UN, a.b_ang, node0, a.N, lane);
    }
  }
  __syncthreads();
  if (threadIdx.x < FT_NODES && node0 + threadIdx.x < a.N)
    sc_geom_node(a.aff, a.rot, UPD + threadIdx.x * 6, UN + threadIdx.x * 6, a.angles, a.traj, a.atom37, a.atom14,
                 (int)(node0 + threadIdx.x));
}

__global__ __launch_bounds__(256) void k_relu_copy(const float* __restrict__ X, int ldx, float* __restrict__ Y,
                                                   int64_t M, int K) {
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= M) return;
  for (int c = threadIdx.x & 63; c < K; c += 64) {
    const float v = X[r * ldx + c];
    Y[r * K + c] = v > 0.0f ? v : 0.0f;
  }
}

inline void gemm_any(hipStream_t st, const float* X, int ldx, const float* Wt, int K, int N, const float* b, float* Y,
                     int ldy, int M, int flags) {
  if (M <= 0) return;
  if (t_mfma && K % 4 == 0 && ldx % 4 == 0 && ((uintptr_t)X & 15) == 0) {
    // one 32-column accumulator per wave and K split into slices of <= ~130: the operand loads
    // per MFMA are the same for any split, while more slices mean more waves in flight and
    // shorter dependent chains (measured on 8 x 256 decodes: four accumulators per wave with 4/16
    // slices 7.05 ms, one with 4/8 slices 6.08 ms)
    auto go = [&](auto kern, int slices, int nacc = 1) {
      // slice width rounded UP (to whole 4-k fragment groups): ks · slices >= K, so no tail of K is
      // dropped; the last slices may be short or empty (k1 = min(K, k0 + ks) in the kernel)
      const int ks = ((K + slices - 1) / slices + 3) / 4 * 4;
      const dim3 grid((unsigned)(((N + 32 * nacc - 1) / (32 * nacc)) * ((M + 31) / 32)));  // 1-D, XCD-aware in the kernel
      hipLaunchKernelGGL(kern, grid, dim3(64 * slices), 0, st, X, ldx, Wt, N, b, Y, ldy, M, N, K, flags, ks);
    };
    if (K >= 1024)  // the IPA output projection (K = 2112); 2 or 4 column tiles per wave: no gain (round 4)
      go(k_gemm_mfma<16, 1>, 16);
    else if (K >= 256)
      go(k_gemm_mfma<8, 1>, 8);
    else
      go(k_gemm_mfma<4, 1>, 4);
    return;
  }
  dim3 grid((N + 63) / 64, (M + 63) / 64);
  hipLaunchKernelGGL(k_gemm, grid, dim3(256), 0, st, X, ldx, Wt, N, b, Y, ldy, M, N, K, flags);
}

inline void gemm(hipStream_t st, const float* X, int ldx, const Lin& L, float* Y, int ldy, int M, int flags,
                 const float* b_override = nullptr, bool use_bias = true) {
  gemm_any(st, X, ldx, L.w, L.in, L.out, use_bias ? (b_override ? b_override : L.b) : nullptr, Y, ldy, M, flags);
}

inline void gemm_raw(hipStream_t st, const float* X, int ldx, const float* Wt, int K, int N, const float* b, float* Y,
                     int ldy, int M, int flags) {
  gemm_any(st, X, ldx, Wt, K, N, b, Y, ldy, M, flags);
}
inline void layernorm(hipStream_t st, const float* X, int ldx, float* Y, int ldy, int M, int C, const LnP& p) {
  hipLaunchKernelGGL(k_layernorm, dim3((M + 3) / 4), dim3(256), 0, st, X, ldx, Y, ldy, M, C, p.s, p.o);
}

// group capacities: a group holds proteins while Σ N_b ≤ kNodeCap and Σ N_b² ≤ kPairCap
// (one 512-residue protein is 2^18 pairs; the pair buffers are ≈ 5.7 KB per pair)
constexpr int64_t kNodeCap = 8192;
constexpr int64_t kPairCap = int64_t(1) << 20;

struct Scratch {
  float *orig_in, *orig, *res, *ln_a, *q, *k, *v, *gate, *wavg;
  float *left, *right, *z, *zln, *b2d;
  float *act, *init_act, *qs, *kvs, *qpl, *kvpl, *qpg, *kvpg, *feat, *upd;
  float *aff, *rot, *unnorm, *angles, *traj, *atom37, *atom14, *kT, *kpT, *init_relu, *ipa_in;
  int64_t *tok_off, *node_off, *pair_off;
  int32_t *tok_prot, *node_prot, *vt_prot, *vt_q0;
  float *att;
  uint32_t* tokens;
};

int ensure_ws(pst_decoder* dec, Scratch* S) {
  const size_t NN = kNodeCap, NP = kPairCap;
  struct It {
    void** p;
    size_t bytes;
  };
  const size_t F = sizeof(float);
  It items[] = {{(void**)&S->orig_in, NN * 256 * F}, {(void**)&S->orig, NN * 128 * F}, {(void**)&S->res, NN * 128 * F},
                {(void**)&S->ln_a, NN * 128 * F},    {(void**)&S->q, NN * 128 * F},
                {(void**)&S->k, NN * 128 * F},       {(void**)&S->v, NN * 128 * F},    {(void**)&S->gate, NN * 128 * F},
                {(void**)&S->wavg, NN * 128 * F},    {(void**)&S->left, NN * 256 * F},
                {(void**)&S->right, NN * 256 * F},   {(void**)&S->z, NP * 128 * F},    {(void**)&S->zln, NP * 128 * F},
                {(void**)&S->b2d, NP * 12 * F},      {(void**)&S->act, NN * 384 * F},     {(void**)&S->init_act, NN * 128 * F},
                {(void**)&S->ipa_in, NN * 1152 * F},
                {(void**)&S->qpg, NN * 144 * F},
                {(void**)&S->kvpg, NN * 432 * F},    {(void**)&S->feat, NN * 2112 * F}, {(void**)&S->upd, NN * 6 * F},
                {(void**)&S->aff, NN * 7 * F},       {(void**)&S->rot, NN * 9 * F},    {(void**)&S->unnorm, NN * 6 * F},
                {(void**)&S->angles, 8 * NN * 6 * F}, {(void**)&S->traj, 8 * NN * 7 * F},
                {(void**)&S->atom37, NN * 111 * F},  {(void**)&S->atom14, NN * 42 * F},
                {(void**)&S->kT, NN * 192 * F}, {(void**)&S->kpT, NN * 144 * F},
                {(void**)&S->init_relu, NN * 128 * F},
                {(void**)&S->tok_off, (NN + 1) * sizeof(int64_t)}, {(void**)&S->node_off, (NN + 1) * sizeof(int64_t)},
                {(void**)&S->pair_off, (NN + 1) * sizeof(int64_t)}, {(void**)&S->tok_prot, NN * sizeof(int32_t)},
                {(void**)&S->node_prot, NN * sizeof(int32_t)}, {(void**)&S->tokens, NN * sizeof(uint32_t)},
                {(void**)&S->vt_prot, 2 * NN * sizeof(int32_t)}, {(void**)&S->vt_q0, 2 * NN * sizeof(int32_t)},
                {(void**)&S->att, NP * 12 * F}};
  size_t total = 0;
  for (auto& it : items) total += (it.bytes + 255) / 256 * 256;
  if (!dec->ws) {
    hipError_t e = hipMalloc(&dec->ws, total);
    if (e != hipSuccess) return dfail(dec, PST_E_NOMEM, std::string("decoder workspace: ") + hipGetErrorString(e));
    dec->ws_bytes = total;
  }
  char* p = (char*)dec->ws;
  for (auto& it : items) {
    *it.p = p;
    p += (it.bytes + 255) / 256 * 256;
  }
  S->qs = S->ipa_in;  // column blocks of the fused projection output
  S->kvs = S->ipa_in + 192;
  S->qpl = S->ipa_in + 576;
  S->kvpl = S->ipa_in + 720;
  return PST_OK;
}

// Host view of one group: proteins [b0, b1) of the call.
struct Group {
  std::vector<int64_t> tok_off, node_off, pair_off;
  std::vector<int32_t> tok_prot, node_prot, vt_prot, vt_q0;  // k_ipa_values tiles: 16 queries of one protein
  std::vector<uint32_t> tokens;
  int64_t T = 0, N = 0, NP = 0;
  int B = 0;
};

// decode a group; atom37 of its nodes are left in S.atom37 (group order)
int decode_group(pst_decoder* dec, Scratch& S, const Group& G, bool keep_debug) {
  const DecWeights& W = dec->W;
  hipStream_t st = dec->stream;
  const int64_t T = G.T, N = G.N, NP = G.NP;
  t_mfma = !getenv("PST_DECODE_NO_MFMA");
  std::vector<int32_t> vt_prot, vt_q0;
  for (int b = 0; b < G.B; ++b)
    for (int64_t q0 = 0; q0 < G.node_off[b + 1] - G.node_off[b]; q0 += 16) {
      vt_prot.push_back(b);
      vt_q0.push_back((int32_t)q0);
    }
  const int n_vt = (int)vt_prot.size();
  {
    // The group's index arrays travel as ONE copy from a pinned staging buffer: they are laid out
    // back to back from the start of the workspace's index region (tok_off ... vt_q0, allocated
    // consecutively with room for kNodeCap entries each, so the packed form always fits), and the
    // S pointers are set to that layout (a function of the group's shape, so the graph cache key
    // still covers every kernel argument). Eight pageable copies cost ~10 us each before.
    char* const d0 = reinterpret_cast<char*>(S.tok_off);
    const struct {
      void** dst;
      const void* src;
      size_t bytes;
    } parts[] = {{(void**)&S.tok_off, G.tok_off.data(), sizeof(int64_t) * (G.B + 1)},
                 {(void**)&S.node_off, G.node_off.data(), sizeof(int64_t) * (G.B + 1)},
                 {(void**)&S.pair_off, G.pair_off.data(), sizeof(int64_t) * (G.B + 1)},
                 {(void**)&S.tok_prot, G.tok_prot.data(), sizeof(int32_t) * T},
                 {(void**)&S.node_prot, G.node_prot.data(), sizeof(int32_t) * N},
                 {(void**)&S.tokens, G.tokens.data(), sizeof(uint32_t) * T},
                 {(void**)&S.vt_prot, vt_prot.data(), sizeof(int32_t) * n_vt},
                 {(void**)&S.vt_q0, vt_q0.data(), sizeof(int32_t) * n_vt}};
    size_t total = 0;
    for (const auto& q : parts) total += (q.bytes + 255) / 256 * 256;
    if (dec->up_ev) DCHK(hipEventSynchronize(dec->up_ev));  // the previous group's copy has left the buffer
    if (total > dec->h_up_bytes) {
      if (dec->h_up) DCHK(hipHostFree(dec->h_up));
      dec->h_up = nullptr;
      dec->h_up_bytes = 0;
      DCHK(hipHostMalloc((void**)&dec->h_up, total));
      dec->h_up_bytes = total;
    }
    size_t off = 0;
    for (const auto& q : parts) {
      *q.dst = d0 + off;
      if (q.bytes) std::memcpy(dec->h_up + off, q.src, q.bytes);
      off += (q.bytes + 255) / 256 * 256;
    }
    DCHK(hipMemcpyAsync(d0, dec->h_up, total, hipMemcpyHostToDevice, st));
    if (!dec->up_ev) DCHK(hipEventCreateWithFlags(&dec->up_ev, hipEventDisableTiming));
    DCHK(hipEventRecord(dec->up_ev, st));
  }
  DecBatch bt{G.B, S.tok_off, S.node_off, S.pair_off, S.tok_prot, S.node_prot};
  const int Ni = (int)N;
  auto mark = [&](int i) {
    if (dec->timing) (void)hipEventRecord(dec->tev[i], st);
  };
  auto launch = [&]() -> int {
    mark(0);
    // ---- upsampler (CrossAttentionScaler, use_original_posenc)
    hipLaunchKernelGGL(k_up_init, dim3((unsigned)T), dim3(128), 0, st, S.tokens, bt, T, dec->d_levels, dec->D,
                       W.up_proj.w, W.up_proj.b, dec->d_pe_tok, S.orig_in);
    gemm(st, S.orig_in, 256, W.proj_original, S.orig, 128, (int)T, 0);
    hipLaunchKernelGGL(k_node_pe, dim3((unsigned)N), dim3(128), 0, st, dec->d_pe_node, bt, N, S.res);
    for (int b = 0; b < 3; ++b) {
      // LayerNorm + both projections per operand in one launch (k_ln_proj2; q · key_dim^-0.5)
      LnProj2Args qa{S.res, Ni, W.qn[b].s, W.qn[b].o, {W.wq[b], W.wg[b]}, {nullptr, W.gb[b]},
                     {F_QSCALE, F_SIGMOID_OUT}, {S.q, S.gate}};
      hipLaunchKernelGGL(k_ln_proj2, dim3((unsigned)((N + FT_NODES - 1) / FT_NODES)), dim3(512), 0, st, qa);
      LnProj2Args ka{S.orig, (int)T, W.dn[b].s, W.dn[b].o, {W.wk[b], W.wv[b]}, {nullptr, nullptr}, {0, 0},
                     {S.k, S.v}};
      hipLaunchKernelGGL(k_ln_proj2, dim3((unsigned)((T + FT_NODES - 1) / FT_NODES)), dim3(512), 0, st, ka);
      hipLaunchKernelGGL(k_up_attn, dim3((unsigned)N), dim3(256), 0, st, S.q, S.k, S.v, S.gate, S.wavg, bt, N);
      gemm_raw(st, S.wavg, 128, W.wo[b], 128, 128, W.ob[b], S.res, 128, Ni, F_ACCUM);
      // the two Transitions fused (k_transition128)
      Trans128Args ta{S.res, Ni, W.rt_ln[b].s, W.rt_ln[b].o, W.rt1[b].w, W.rt1[b].b, W.rt2[b].w, W.rt2[b].b};
      hipLaunchKernelGGL(k_transition128, dim3((unsigned)((N + FT_NODES - 1) / FT_NODES)), dim3(512), 0, st, ta);
      Trans128Args tb{S.orig, (int)T, W.ot_ln[b].s, W.ot_ln[b].o, W.ot1[b].w, W.ot1[b].b, W.ot2[b].w, W.ot2[b].b};
      hipLaunchKernelGGL(k_transition128, dim3((unsigned)((T + FT_NODES - 1) / FT_NODES)), dim3(512), 0, st, tb);
    }
    hipLaunchKernelGGL(k_spherical, dim3((unsigned)((N + 3) / 4)), dim3(256), 0, st, S.res, Ni);  // s_i
    mark(1);
    // ---- sequence decoder: pair representation over each protein's N_b² pairs
    layernorm(st, S.res, 128, S.ln_a, 128, Ni, 128, W.pr_ln_in);
    gemm(st, S.ln_a, 128, W.left, S.left, 256, Ni, 0);
    gemm(st, S.ln_a, 128, W.right, S.right, 256, Ni, 0);
    layernorm(st, S.res, 128, S.init_act, 128, Ni, 128, W.single_ln);
    gemm(st, S.init_act, 128, W.init_proj, S.act, 384, Ni, 0);
    PairArgs pa = dec->pair;
    pa.left = S.left;
    pa.right = S.right;
    pa.z = keep_debug ? S.z : nullptr;
    pa.zln = S.zln;
    pa.b2d = S.b2d;
    pa.NP = NP;
    pa.bt = bt;
    const int64_t tiles = (NP + 31) / 32;
    mark(2);
    hipLaunchKernelGGL(k_pair_fused, dim3((unsigned)((tiles + 3) / 4)), dim3(256), 0, st, pa);
    mark(3);
    hipLaunchKernelGGL(k_affine_init, dim3((unsigned)((N + 63) / 64)), dim3(64), 0, st, S.aff, S.rot, Ni);
    // relu(init_act) feeds the angle resnet of every iteration: once, not 8 copies
    hipLaunchKernelGGL(k_relu_copy, dim3((unsigned)((N + 3) / 4)), dim3(256), 0, st, S.init_act, 128, S.init_relu,
                       (int64_t)Ni, 128);
    for (int it = 0; it < 8; ++it) {
      // the four IPA input projections as one 384 -> 1152 GEMM: [q_scalar | kv_scalar | q_point |
      // kv_point] columns of ipa_in (row stride 1152)
      gemm_raw(st, S.act, 384, dec->d_ipa_w, 384, 1152, dec->d_ipa_b, S.ipa_in, 1152, Ni, 0);
      hipLaunchKernelGGL(k_ipa_points, dim3((unsigned)N), dim3(192), 0, st, S.qpl, S.kvpl, S.aff, S.rot, S.qpg, S.kvpg,
                         S.kvs, S.kT, S.kpT, Ni, 1152);
      hipLaunchKernelGGL(k_ipa_attn, dim3((unsigned)N), dim3(256), 0, st, S.qs, S.qpg, S.b2d, S.zln,
                         dec->d_pw, S.aff, S.rot, S.feat, bt, S.kT, S.kpT, Ni, 1152, S.att);
      hipLaunchKernelGGL(k_ipa_values, dim3((unsigned)n_vt, 12), dim3(64), 0, st, S.att, S.kvs, S.kvpg, S.feat, S.aff,
                         S.rot, bt, S.vt_prot, S.vt_q0, 1152);
      gemm(st, S.feat, 2112, W.out_proj, S.act, 384, Ni, F_ACCUM);  // act += IPA
      // the rest of the iteration's linears and norms in one launch (k_fold_tail)
      const bool last = it == 7;
      FoldTailArgs ft{S.act, S.init_relu, S.upd, S.unnorm, Ni, W.att_ln.s, W.att_ln.o, W.tr_ln.s, W.tr_ln.o,
                      {W.tr[0].w, W.tr[1].w, W.tr[2].w}, {W.tr[0].b, W.tr[1].b, W.tr[2].b},
                      W.affine_update.w, W.affine_update.b, W.sc_in.w, W.sc_in.b, W.sc_in1.w, W.sc_in1.b,
                      {W.rb1.w, W.rb2.w, W.rb1_1.w, W.rb2_1.w}, {W.rb1.b, W.rb2.b, W.rb1_1.b, W.rb2_1.b},
                      W.angles.w, W.angles.b, S.aff, S.rot, S.angles + it * kNodeCap * 6, S.traj + it * kNodeCap * 7,
                      last ? S.atom37 : nullptr, last ? S.atom14 : nullptr};
      hipLaunchKernelGGL(k_fold_tail, dim3((unsigned)((N + FT_NODES - 1) / FT_NODES)), dim3(64 * FT_WAVES), 0, st, ft);
    }
    mark(4);
    DCHK(hipGetLastError());
    return PST_OK;
  };
  // The ~200 launches of one group are captured once per group shape into a HIP graph and
  // replayed (the decode was partly launch-bound: kernel time 5.0 ms of ~5.7 ms per 8 x 256
  // decode). Inputs are uploaded above, outside the graph; every kernel argument is a function of
  // the shape (per-protein token / node counts) and the decoder's fixed buffers.
  const bool use_graph = !keep_debug && !dec->timing && !getenv("PST_DECODE_NO_GRAPH");
  if (!use_graph) {
    int rc = launch();
    if (rc) return rc;
    if (dec->timing) {
      DCHK(hipEventSynchronize(dec->tev[PST_DECODER_N_STAGES]));
      for (int i = 0; i < PST_DECODER_N_STAGES; ++i) {
        float ms = 0.0f;
        DCHK(hipEventElapsedTime(&ms, dec->tev[i], dec->tev[i + 1]));
        dec->tms[i] += ms;
      }
    }
  } else {
    std::vector<int64_t> key{(int64_t)t_mfma, G.B};
    key.insert(key.end(), G.node_off.begin(), G.node_off.end());
    key.insert(key.end(), G.tok_off.begin(), G.tok_off.end());
    auto it = dec->graphs.find(key);
    if (it == dec->graphs.end()) {
      if (dec->graphs.size() >= 16) {  // bounded cache: start over
        for (auto& kv : dec->graphs) (void)hipGraphExecDestroy(kv.second);
        dec->graphs.clear();
      }
      DCHK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
      const int rc = launch();
      hipGraph_t graph = nullptr;
      const hipError_t ec = hipStreamEndCapture(st, &graph);
      if (rc) {
        if (graph) (void)hipGraphDestroy(graph);
        return rc;
      }
      DCHK(ec);
      hipGraphExec_t exec = nullptr;
      const hipError_t ei = hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0);
      (void)hipGraphDestroy(graph);
      DCHK(ei);
      it = dec->graphs.emplace(key, exec).first;
    }
    DCHK(hipGraphLaunch(it->second, st));
  }
  if (keep_debug) {
    std::vector<float> h((size_t)NP * 128 > (size_t)8 * N * 7 ? (size_t)NP * 128 : (size_t)8 * N * 7);
    auto grab = [&](const float* src, size_t n) -> int {
      DCHK(hipMemcpyAsync(h.data(), src, n * sizeof(float), hipMemcpyDeviceToHost, st));
      DCHK(hipStreamSynchronize(st));
      return PST_OK;
    };
    if (grab(S.res, (size_t)N * 128)) return PST_E_HIP;
    dec->last_single.insert(dec->last_single.end(), h.begin(), h.begin() + N * 128);
    if (grab(S.z, (size_t)NP * 128)) return PST_E_HIP;
    dec->last_pair.insert(dec->last_pair.end(), h.begin(), h.begin() + NP * 128);
    if (grab(S.atom14, (size_t)N * 42)) return PST_E_HIP;
    dec->last_atom14.insert(dec->last_atom14.end(), h.begin(), h.begin() + N * 42);
    // per-protein [8][N_b][...] blocks from the [8][kNodeCap][...] device layout
    std::vector<float> tr((size_t)8 * kNodeCap * 7), an((size_t)8 * kNodeCap * 6);
    DCHK(hipMemcpyAsync(tr.data(), S.traj, tr.size() * sizeof(float), hipMemcpyDeviceToHost, st));
    DCHK(hipMemcpyAsync(an.data(), S.angles, an.size() * sizeof(float), hipMemcpyDeviceToHost, st));
    DCHK(hipStreamSynchronize(st));
    for (int b = 0; b < G.B; ++b) {
      const int64_t n0 = G.node_off[b], nb = G.node_off[b + 1] - n0;
      for (int it = 0; it < 8; ++it) {
        const float* t7 = tr.data() + ((size_t)it * kNodeCap + n0) * 7;
        dec->last_traj.insert(dec->last_traj.end(), t7, t7 + nb * 7);
        const float* a6 = an.data() + ((size_t)it * kNodeCap + n0) * 6;
        dec->last_angles.insert(dec->last_angles.end(), a6, a6 + nb * 6);
      }
    }
  }
  return PST_OK;
}

}  // namespace

extern "C" {

int pst_decoder_set_timing(pst_decoder* dec, int32_t enable) {
  if (!dec) return PST_E_INVALID;
  DCHK(hipSetDevice(dec->device));
  if (enable && !dec->tev[0])
    for (int i = 0; i <= PST_DECODER_N_STAGES; ++i) DCHK(hipEventCreate(&dec->tev[i]));
  dec->timing = enable != 0;
  for (float& v : dec->tms) v = 0.0f;
  return PST_OK;
}

int pst_decoder_get_timing(pst_decoder* dec, float* ms) {
  if (!dec || !ms) return PST_E_INVALID;
  for (int i = 0; i < PST_DECODER_N_STAGES; ++i) ms[i] = dec->tms[i];
  return PST_OK;
}

size_t pst_decoder_param_count(int32_t n_levels) {
  DecWeights W;
  return walk_decoder(nullptr, n_levels, &W);
}

const char* pst_decoder_create_error(void) { return g_dec_create_error.c_str(); }

namespace {
// Pack the pair-chain weights for k_pair_fused (host weights Wh from walk_decoder on the blob).
int build_pair_arena(pst_decoder* dec, const DecWeights& Wh) {
  using namespace pst_host;
  const int H = 128;
  std::vector<float> A;
  auto add = [&](const std::vector<float>& v) {
    const size_t o = A.size();
    A.insert(A.end(), v.begin(), v.end());
    A.resize((A.size() + 63) / 64 * 64, 0.0f);
    return o;
  };
  size_t f_out1[2][2], f_out2[2], f_r1[2], f_pt1[2], f_pt2[2], pb_out1[2], pb_pt1[2];
  for (int kc = 0; kc < 2; ++kc)
    for (int oc = 0; oc < 2; ++oc) f_out1[kc][oc] = add(frag(Wh.out1.w, 2 * H, H * kc, H, H, H * oc, H));
  for (int kc = 0; kc < 2; ++kc) {
    f_out2[kc] = add(frag(Wh.out2.w, H, H * kc, H, H, 0, H));
    f_r1[kc] = add(frag(Wh.right1.w, H, H * kc, H, H, 0, H));
    f_pt2[kc] = add(frag(Wh.pt2.w, H, H * kc, H, H, 0, H));
    f_pt1[kc] = add(frag(Wh.pt1.w, 2 * H, 0, H, H, H * kc, H));
    pb_out1[kc] = add(perm(Wh.out1.b + H * kc));
    pb_pt1[kc] = add(perm(Wh.pt1.b + H * kc));
  }
  const size_t bf_out2 = add(bfrag(Wh.out2.b)), bf_pt2 = add(bfrag(Wh.pt2.b)), pb_r1 = add(perm(Wh.right1.b));
  const size_t f_seqb = add(frag(Wh.seq_linear.w, H, H, H, H, 0, H));
  const size_t ln1s = add(perm(Wh.pr_ln_out.s)), ln1o = add(perm(Wh.pr_ln_out.o));
  const size_t ln2s = add(perm(Wh.pt_ln.s)), ln2o = add(perm(Wh.pt_ln.o));
  const size_t ln3s = add(perm(Wh.pair_ln.s)), ln3o = add(perm(Wh.pair_ln.o));
  const size_t f_att = add(frag_narrow(Wh.att2d.w, 12, 12));
  const size_t b_att = add(std::vector<float>(Wh.att2d.b, Wh.att2d.b + 12));
  // U[d] = PE(d - 511; 512) · W_seq[0:128] + b_seq (float64 accumulation, rounded once)
  std::vector<float> pe = pst::pe_rows(-511, 1023, 512), U((size_t)1023 * H);
  for (int d = 0; d < 1023; ++d)
    for (int o = 0; o < H; ++o) {
      double acc = Wh.seq_linear.b[o];
      for (int c = 0; c < H; ++c) acc += (double)pe[(size_t)d * H + c] * (double)Wh.seq_linear.w[(size_t)c * H + o];
      U[(size_t)d * H + o] = (float)acc;
    }
  const size_t u_tab = add(perm_rows(U, 1023));
  if (hipMalloc(&dec->d_pair, A.size() * sizeof(float)) != hipSuccess ||
      hipMemcpy(dec->d_pair, A.data(), A.size() * sizeof(float), hipMemcpyHostToDevice) != hipSuccess)
    return 1;
  const float* D = dec->d_pair;
  auto F4 = [&](size_t o) { return reinterpret_cast<const float4*>(D + o); };
  PairArgs& P = dec->pair;
  for (int kc = 0; kc < 2; ++kc) {
    for (int oc = 0; oc < 2; ++oc) P.f_out1[kc][oc] = F4(f_out1[kc][oc]);
    P.f_out2[kc] = F4(f_out2[kc]);
    P.f_r1[kc] = F4(f_r1[kc]);
    P.f_pt1[kc] = F4(f_pt1[kc]);
    P.f_pt2[kc] = F4(f_pt2[kc]);
    P.pb_out1[kc] = D + pb_out1[kc];
    P.pb_pt1[kc] = D + pb_pt1[kc];
  }
  P.bf_out2 = F4(bf_out2);
  P.bf_pt2 = F4(bf_pt2);
  P.pb_r1 = D + pb_r1;
  P.f_seqb = F4(f_seqb);
  P.ln1_s = D + ln1s;
  P.ln1_o = D + ln1o;
  P.ln2_s = D + ln2s;
  P.ln2_o = D + ln2o;
  P.ln3_s = D + ln3s;
  P.ln3_o = D + ln3o;
  P.f_att2d = D + f_att;
  P.b_att2d = D + b_att;
  P.U = D + u_tab;
  return 0;
}
}  // namespace

int pst_decoder_create(int32_t device, const pst_model_desc* desc, const float* params, size_t n_params,
                       pst_decoder** out) {
  g_dec_create_error.clear();
  if (!desc || !params || !out) {
    g_dec_create_error = "null argument";
    return PST_E_INVALID;
  }
  const int D = desc->n_levels, df = desc->downsampling_ratio;
  if (desc->abi_version != PST_ABI_VERSION || D < 1 || D > 8 || (df != 1 && df != 2 && df != 4) ||
      desc->seq_max_size != 512) {
    g_dec_create_error = "unsupported model description";
    return PST_E_INVALID;
  }
  if (n_params != pst_decoder_param_count(D)) {
    g_dec_create_error = "decoder blob has " + std::to_string(n_params) + " floats, expected " +
                         std::to_string(pst_decoder_param_count(D));
    return PST_E_INVALID;
  }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) {
    g_dec_create_error = "no such HIP device: " + std::to_string(device);
    return PST_E_HIP;
  }
  pst_decoder* dec = new pst_decoder();
  dec->device = device;
  dec->desc = *desc;
  dec->D = D;
  dec->df = df;
  auto bad = [&](const char* what, int code = PST_E_HIP) {
    g_dec_create_error = what;
    pst_decoder_destroy(dec);
    return code;
  };
  if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&dec->stream, hipStreamNonBlocking) != hipSuccess)
    return bad("hip stream creation failed");
  if (hipMalloc(&dec->d_blob, n_params * sizeof(float)) != hipSuccess ||
      hipMemcpy(dec->d_blob, params, n_params * sizeof(float), hipMemcpyHostToDevice) != hipSuccess)
    return bad("decoder weight upload failed");
  walk_decoder(dec->d_blob, D, &dec->W);
  {
    if (hipMalloc(&dec->d_ipa_w, 384 * 1152 * sizeof(float)) != hipSuccess ||
        hipMalloc(&dec->d_ipa_b, 1152 * sizeof(float)) != hipSuccess)
      return bad("IPA projection buffer allocation failed");
    int col = 0;
    for (const Lin* L : {&dec->W.q_scalar, &dec->W.kv_scalar, &dec->W.q_point, &dec->W.kv_point}) {
      if (L->in != 384) return bad("IPA projection input width is not 384", PST_E_INVALID);
      if (hipMemcpy2D(dec->d_ipa_w + col, 1152 * sizeof(float), L->w, L->out * sizeof(float), L->out * sizeof(float),
                      384, hipMemcpyDeviceToDevice) != hipSuccess ||
          (L->b ? hipMemcpy(dec->d_ipa_b + col, L->b, L->out * sizeof(float), hipMemcpyDeviceToDevice)
                : hipMemset(dec->d_ipa_b + col, 0, L->out * sizeof(float))) != hipSuccess)
        return bad("IPA projection weight packing failed");
      col += L->out;
    }
    if (col != 1152) return bad("IPA projection widths do not add up to 1152", PST_E_INVALID);
  }
  // host-side constants: PE tables, levels, IPA point weights
  auto up = [&](float** d, const std::vector<float>& h) {
    return hipMalloc(d, h.size() * sizeof(float)) == hipSuccess &&
           hipMemcpy(*d, h.data(), h.size() * sizeof(float), hipMemcpyHostToDevice) == hipSuccess;
  };
  if (!up(&dec->d_pe_node, pst::pe_rows(0, 512, 512)) || !up(&dec->d_pe_tok, pst::pe_rows(0, 512 / df, 512 / df)) ||
      !up(&dec->d_pe_rel, pst::pe_rows(-511, 1023, 512)))
    return bad("PE table upload failed");
  if (hipMalloc(&dec->d_levels, 8 * sizeof(int)) != hipSuccess ||
      hipMemcpy(dec->d_levels, desc->levels, 8 * sizeof(int), hipMemcpyHostToDevice) != hipSuccess)
    return bad("levels upload failed");
  {
    // point_weights = sqrt(1 / (3 · 4 · 9/2)) · softplus(trainable_point_weights)   (folding.py:178-197)
    DecWeights Wh;
    walk_decoder(params, D, &Wh);
    std::vector<float> pw(12);
    const float base = (float)std::sqrt(1.0 / (3.0 * 4.0 * 9.0 / 2.0));
    for (int h = 0; h < 12; ++h) {
      const double x = Wh.tpw[h];
      const float sp = (float)(x > 20.0 ? x : std::log1p(std::exp(x)));
      pw[h] = base * sp;
    }
    if (!up(&dec->d_pw, pw)) return bad("point weight upload failed");
    if (build_pair_arena(dec, Wh)) return bad("pair fragment upload failed");
  }
  *out = dec;
  return PST_OK;
}

int pst_decoder_destroy(pst_decoder* dec) {
  if (!dec) return PST_OK;
  (void)hipSetDevice(dec->device);
  if (dec->stream) (void)hipStreamSynchronize(dec->stream);
  for (void* p : {(void*)dec->d_blob, (void*)dec->d_levels, (void*)dec->d_pe_node, (void*)dec->d_pe_tok,
                  (void*)dec->d_pe_rel, (void*)dec->d_pw, (void*)dec->d_pair, dec->ws, (void*)dec->d_ipa_w,
                  (void*)dec->d_ipa_b})
    if (p) (void)hipFree(p);
  for (auto& kv : dec->graphs) (void)hipGraphExecDestroy(kv.second);
  dec->graphs.clear();
  if (dec->h_up) (void)hipHostFree(dec->h_up);
  if (dec->h_atoms) (void)hipHostFree(dec->h_atoms);
  if (dec->up_ev) (void)hipEventDestroy(dec->up_ev);
  for (auto& e : dec->tev)
    if (e) (void)hipEventDestroy(e);
  if (dec->stream) (void)hipStreamDestroy(dec->stream);
  delete dec;
  return PST_OK;
}

const char* pst_decoder_last_error(const pst_decoder* dec) { return dec ? dec->err.c_str() : "null decoder"; }

int pst_decoder_decode(pst_decoder* dec, const uint32_t* tokens, const int64_t* token_offsets, int32_t n_prot,
                       float* atom37_out, int32_t* n_nodes_out) {
  return pst_decoder_decode_ex(dec, tokens, token_offsets, n_prot, nullptr, atom37_out, n_nodes_out, nullptr);
}

int pst_decoder_decode_ex(pst_decoder* dec, const uint32_t* tokens, const int64_t* token_offsets, int32_t n_prot,
                          const int32_t* n_nodes_in, float* atom37_out, int32_t* n_nodes_out, float* up_proj_out) {
  if (!dec) return PST_E_INVALID;
  dec->err.clear();
  if (!tokens || !token_offsets || n_prot < 1 || !atom37_out) return dfail(dec, PST_E_INVALID, "null argument");
  const int64_t max_tok = 512 / dec->df;
  int64_t K = 1;
  for (int d = 0; d < dec->D; ++d) K *= dec->desc.levels[d];
  if (token_offsets[0] != 0) return dfail(dec, PST_E_INVALID, "token_offsets[0] must be 0");
  for (int b = 0; b < n_prot; ++b) {
    const int64_t T = token_offsets[b + 1] - token_offsets[b];
    if (T < 0 || T > max_tok)
      return dfail(dec, PST_E_INVALID, "protein " + std::to_string(b) + ": token count outside [0, " +
                                           std::to_string(max_tok) + "]");
    if (n_nodes_in) {
      // the graph's node count n gives T = floor(n / df) tokens (preprocessing.py:212-216)
      const int64_t n = n_nodes_in[b];
      if (n < T * dec->df || n >= (T + 1) * dec->df || n > 512 || (T == 0 && n != 0))
        return dfail(dec, PST_E_INVALID, "protein " + std::to_string(b) + ": " + std::to_string(n) +
                                             " nodes do not give " + std::to_string(T) + " tokens at df " +
                                             std::to_string(dec->df));
    }
  }
  DCHK(hipSetDevice(dec->device));
  Scratch S;
  int rc = ensure_ws(dec, &S);
  if (rc) return rc;
  const bool keep = getenv("PST_DEBUG") && getenv("PST_DEBUG")[0] == '1';
  dec->last_single.clear();
  dec->last_pair.clear();
  dec->last_traj.clear();
  dec->last_angles.clear();
  dec->last_atom14.clear();
  int64_t out_node = 0;
  int b = 0;
  while (b < n_prot) {
    Group G;
    G.tok_off.push_back(0);
    G.node_off.push_back(0);
    G.pair_off.push_back(0);
    const int64_t out0 = out_node;
    const int b0 = b;
    while (b < n_prot) {
      const int64_t T = token_offsets[b + 1] - token_offsets[b], N = n_nodes_in ? n_nodes_in[b] : T * dec->df;
      if (G.B > 0 && (G.N + N > kNodeCap || G.NP + N * N > kPairCap)) break;
      if (n_nodes_out) n_nodes_out[b] = (int32_t)N;
      if (T > 0) {  // empty proteins take no rows
        // indexes_to_codes extracts digits as (id // basis_d) mod L_d (quantize.py:70-79), which
        // decodes any uint32 id as id mod K: ids >= K are accepted, not rejected
        for (int64_t t = token_offsets[b]; t < token_offsets[b + 1]; ++t)
          G.tokens.push_back((uint32_t)((uint64_t)tokens[t] % (uint64_t)K));
        G.tok_prot.insert(G.tok_prot.end(), (size_t)T, G.B);
        G.node_prot.insert(G.node_prot.end(), (size_t)N, G.B);
        G.T += T;
        G.N += N;
        G.NP += N * N;
        G.tok_off.push_back(G.T);
        G.node_off.push_back(G.N);
        G.pair_off.push_back(G.NP);
        ++G.B;
      }
      out_node += N;
      ++b;
    }
    if (G.B == 0) continue;
    rc = decode_group(dec, S, G, keep);
    if (rc) return rc;
    // atom37 D2H into a pinned staging buffer, then one host copy (a pageable-destination D2H is
    // staged by the runtime in small pieces)
    const size_t na = (size_t)G.N * 111;
    if (na > dec->h_atoms_floats) {
      if (dec->h_atoms) DCHK(hipHostFree(dec->h_atoms));
      dec->h_atoms = nullptr;
      dec->h_atoms_floats = 0;
      DCHK(hipHostMalloc((void**)&dec->h_atoms, sizeof(float) * na));
      dec->h_atoms_floats = na;
    }
    DCHK(hipMemcpyAsync(dec->h_atoms, S.atom37, sizeof(float) * na, hipMemcpyDeviceToHost, dec->stream));
    if (up_proj_out)  // quantize_post_proj: the up_proj half of each token's [PE | up_proj] row
      DCHK(hipMemcpy2DAsync(up_proj_out + token_offsets[b0] * 128, 128 * sizeof(float), S.orig_in + 128,
                            256 * sizeof(float), 128 * sizeof(float), (size_t)G.T, hipMemcpyDeviceToHost,
                            dec->stream));
    DCHK(hipStreamSynchronize(dec->stream));
    // the host copy on libpst's host pool in 64 K-float parts (one thread copies ~6 GB/s; a 8 x 512
    // decode returns 1.8 MB)
    constexpr size_t PART = size_t(1) << 16;
    const int parts = (int)((na + PART - 1) / PART);
    float* dst = atom37_out + out0 * 111;
    const float* src = dec->h_atoms;
    pst::HostPool::get().run(parts, std::min(parts, 8), [&](int i) {
      const size_t a = (size_t)i * PART, e = std::min(na, a + PART);
      std::memcpy(dst + a, src + a, sizeof(float) * (e - a));
    });
  }
  return PST_OK;
}

int pst_decoder_debug(pst_decoder* dec, int32_t which, float* out, size_t n_floats) {
  if (!dec || !out) return PST_E_INVALID;
  const std::vector<float>* v = which == 0 ? &dec->last_single
                                : which == 1 ? &dec->last_pair
                                : which == 2 ? &dec->last_traj
                                : which == 3 ? &dec->last_angles
                                : which == 4 ? &dec->last_atom14
                                             : nullptr;
  if (!v) return dfail(dec, PST_E_INVALID, "unknown debug id");
  if (v->empty()) return dfail(dec, PST_E_INVALID, "no intermediates kept (set PST_DEBUG=1)");
  if (n_floats < v->size()) return dfail(dec, PST_E_INVALID, "debug buffer too small");
  std::copy(v->begin(), v->end(), out);
  return PST_OK;
}

}  // extern "C"
