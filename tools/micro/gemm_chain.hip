// Microbenchmark: MFMA utilisation of the wave-tile GEMM chain used by k_mpnn.
// 8192 waves x 50 blocks x 6 GEMMs (128x128 on a 32-column tile), 2 waves/SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include "../../protein-structure-tokenizer_amd/csrc/pst_device.h"
using namespace pst;

template <int MODE>  // 0: plain chain, 1: JIT bias+gelu, 2: plain, weights from LDS, 3: gelu+LDS
__global__ __launch_bounds__(256, 2) void k_chain(const float4* W, const float* b, float* out, int nblk) {
  __shared__ float4 wl[64 * 64];
  Tile x, acc;
  tile_zero(x);
  for (int M = 0; M < 4; ++M) for (int r = 0; r < 16; ++r) x.m[M][r] = 0.001f * (threadIdx.x + r);
  const float4* src = W;
  if (MODE >= 2) {
    for (int i = threadIdx.x; i < 64 * 64; i += 256) wl[i] = W[i];
    __syncthreads();
  }
  for (int blk = 0; blk < nblk; ++blk) {
#pragma unroll 1
    for (int g = 0; g < 6; ++g) {
      tile_zero(acc);
      if (MODE == 0) tile_gemm(acc, x, src + (g % 3) * 4096);
      if (MODE == 1) tile_gemm_f(acc, x, src + (g % 3) * 4096, ActBiasGelu{b});
      if (MODE == 2) {
        const float4* w = wl + lane_id();
#pragma unroll
        for (int t = 0; t < 64; ++t) {
          float4 a = w[t * 64];
          float bb = x.m[t / 16][t % 16];
          acc.m[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, bb, acc.m[0], 0, 0, 0);
          acc.m[1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, bb, acc.m[1], 0, 0, 0);
          acc.m[2] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.z, bb, acc.m[2], 0, 0, 0);
          acc.m[3] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.w, bb, acc.m[3], 0, 0, 0);
        }
      }
      x = acc;
    }
  }
  tile_store_blk(x, out + (size_t)(blockIdx.x * 4 + (threadIdx.x >> 6)) * 4096);
}

int main() {
  const int waves = 8192, nblk = 50;
  float4* W; float* b; float* out;
  hipMalloc(&W, 3 * 4096 * 16); hipMalloc(&b, 512); hipMalloc(&out, (size_t)waves * 4096 * 4);
  std::vector<float> h(3 * 4096 * 4);
  for (size_t i = 0; i < h.size(); ++i) h[i] = 0.01f * ((i * 7919) % 101 - 50) / 50.0f;
  hipMemcpy(W, h.data(), h.size() * 4, hipMemcpyHostToDevice);
  hipMemset(b, 0, 512);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  for (int mode = 0; mode < 3; ++mode) {
    for (int rep = 0; rep < 3; ++rep) {
      hipEventRecord(e0);
      if (mode == 0) k_chain<0><<<waves / 4, 256>>>(W, b, out, nblk);
      if (mode == 1) k_chain<1><<<waves / 4, 256>>>(W, b, out, nblk);
      if (mode == 2) k_chain<2><<<waves / 4, 256>>>(W, b, out, nblk);
      hipEventRecord(e1); hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1);
      double flops = (double)waves * nblk * 6 * 2.0 * 128 * 128 * 32;
      if (rep == 2) printf("mode %d: %.3f ms  %.1f TFLOP/s (%.1f%% of 157.3)\n", mode, ms, flops / ms / 1e9, flops / ms / 1e9 / 157.3 * 100);
    }
  }
  return 0;
}
