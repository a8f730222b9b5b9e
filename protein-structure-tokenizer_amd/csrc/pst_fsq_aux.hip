// pst_fsq_aux.hip — FSQ auxiliary outputs over the implicit codebook (model/quantize.py:205-239):
//   distances[row, k]  = sum_d (b_d - c_kd)^2          (quantize.py:226-231, 236)
//   soft_proba[row, k] = softmax_k(distances[row, :])   (quantize.py:235, sign as in the reference)
//   argmin[row]        = nearest code, histogram[k] += 1 per real token (perplexity, :211-224)
//
// The codebook is the grid c_kd = digit_d(k) - L_d/2 (renorm: false in every shipped config), so
// a row is separable over dimensions. Split the dimensions into a low group (0..2, K_lo codes)
// and a high group (3..D-1, K_hi codes), k = k_lo + K_lo * k_hi:
//   distance(k) = A[k_lo] + B[k_hi]          A, B = sequential sums of (b_d - c)^2 over the group
//   soft_proba  = EA[k_lo] * EB[k_hi] * (1 / (S_A * S_B)),  EA = exp(A - max A), S_A = sum EA
// (exp(A + B - max) factorises; max A + max B is the row maximum by monotone rounding). Each
// row therefore needs K_lo + K_hi exponentials, not K, and no reduction over K: the kernel is a
// pure streaming write of 2 x 4K bytes per token row (HBM-write roofline). A GEMM formulation
// (|b|^2 - 2 b.c + |c|^2 on MFMA) would add cancellation error and cannot beat the write bound.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pst_device.h"
#include "pst_kernels.h"

namespace pst {

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v = fmaxf(v, __shfl_xor(v, m));
  return v;
}

// canonical row sum: per lane sequential over i = lane, lane+64, ... from +0, then a xor
// butterfly 32, 16, 8, 4, 2, 1 (every lane ends with the same value)
__device__ __forceinline__ float wave_sum_butterfly(float v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v = v + __shfl_xor(v, m);
  return v;
}

__global__ __launch_bounds__(256) void k_fsq_aux(FsqAuxArgs a) {
  __shared__ float sA[FSQ_AUX_MAX_LO], sEA[FSQ_AUX_MAX_LO], sB[FSQ_AUX_MAX_HI], sEB[FSQ_AUX_MAX_HI];
  __shared__ float sSum[2];
  const int tile = blockIdx.x >> 5;
  const int b = a.tile_prot[tile];
  const int t = a.tile_t0[tile] + (int)(blockIdx.x & 31);
  const int T = a.n_nodes[b] / a.df;
  if (t >= T) return;  // uniform over the block
  const int64_t src = a.offsets[b] + t;
  const int64_t row = a.row_start[b] + t;
  float bv[8];
#pragma unroll
  for (int d = 0; d < 8; ++d) bv[d] = d < a.D ? a.bounded[src * 8 + d] : 0.0f;

  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (w < 2) {  // wave 0: low group table, wave 1: high group table
    const int d0 = w == 0 ? 0 : 3, d1 = w == 0 ? 3 : a.D;
    const int n = w == 0 ? a.K_lo : a.K_hi;
    float* S = w == 0 ? sA : sB;
    float* E = w == 0 ? sEA : sEB;
    float mx = -__builtin_inff();
    for (int i = lane; i < n; i += 64) {
      int rem = i;
      float s = 0.0f;
      for (int d = d0; d < d1; ++d) {
        const int L = a.L[d];
        const int digit = rem % L;
        rem /= L;
        const float diff = bv[d] - (float)(digit - L / 2);
        const float sq = diff * diff;
        s = d == d0 ? sq : s + sq;
      }
      S[i] = s;
      mx = fmaxf(mx, s);
    }
    mx = wave_max(mx);
    float part = 0.0f;
    for (int i = lane; i < n; i += 64) {
      const float e = c_exp(S[i] - mx);
      E[i] = e;
      part = part + e;
    }
    part = wave_sum_butterfly(part);
    if (lane == 0) sSum[w] = part;
  }
  __syncthreads();
  const float inv_s = 1.0f / (sSum[0] * sSum[1]);
  if (threadIdx.x == 0) {
    if (a.argmin) {  // per-dimension nearest level, lowest digit on ties
      uint32_t k = 0;
      for (int d = 0; d < a.D; ++d) {
        const int L = a.L[d];
        int best = 0;
        float bd = __builtin_inff();
        for (int g = 0; g < L; ++g) {
          const float diff = bv[d] - (float)(g - L / 2);
          const float sq = diff * diff;
          if (sq < bd) {
            bd = sq;
            best = g;
          }
        }
        k += (uint32_t)best * (uint32_t)a.basis[d];
      }
      a.argmin[row] = k;
    }
    if (a.hist) atomicAdd(&a.hist[a.tokens[src]], 1u);
  }
  const int nq = a.K >> 2;
  f32x4* dist = a.dist ? reinterpret_cast<f32x4*>(a.dist + row * (int64_t)a.K) : nullptr;
  f32x4* prob = a.prob ? reinterpret_cast<f32x4*>(a.prob + row * (int64_t)a.K) : nullptr;
  const f32x4* A4 = reinterpret_cast<const f32x4*>(sA);
  const f32x4* E4 = reinterpret_cast<const f32x4*>(sEA);
  const int qlo = a.K_lo >> 2;
  for (int q = threadIdx.x; q < nq; q += 256) {
    const int khi = q / qlo;
    const int ql = q - khi * qlo;
    if (dist) {
      const float bb = sB[khi];
      f32x4 v = A4[ql];
      v.x = v.x + bb;
      v.y = v.y + bb;
      v.z = v.z + bb;
      v.w = v.w + bb;
      __builtin_nontemporal_store(v, dist + q);
    }
    if (prob) {
      const float eb = sEB[khi];
      f32x4 v = E4[ql];
      v.x = (v.x * eb) * inv_s;
      v.y = (v.y * eb) * inv_s;
      v.z = (v.z * eb) * inv_s;
      v.w = (v.w * eb) * inv_s;
      __builtin_nontemporal_store(v, prob + q);
    }
  }
}

// compact output row of each protein's first token: exclusive scan of n_nodes / df
__global__ void k_row_start(const int32_t* n_nodes, int64_t* row_start, int B, int df) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    int64_t acc = 0;
    for (int b = 0; b < B; ++b) {
      row_start[b] = acc;
      acc += n_nodes[b] / df;
    }
    row_start[B] = acc;
  }
}

void launch_fsq_aux(const FsqAuxArgs& a, int n_prot, hipStream_t st) {
  hipLaunchKernelGGL(k_row_start, dim3(1), dim3(64), 0, st, a.n_nodes, const_cast<int64_t*>(a.row_start), n_prot,
                     a.df);
  if (a.n_rows_grid > 0) hipLaunchKernelGGL(k_fsq_aux, dim3((unsigned)a.n_rows_grid), dim3(256), 0, st, a);
}

}  // namespace pst
