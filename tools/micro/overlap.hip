// Do fp32 MFMA and fp32 VALU from DIFFERENT waves on one SIMD overlap on gfx950?
// Workgroup of 8 waves (2 per SIMD). Role per wave: 'M' = MFMA chain only, 'V' = VALU GELU only.
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../../protein-structure-tokenizer_amd/csrc/pst_device.h"
using namespace pst;

__device__ void do_mfma(const float4* W, float* out, int iters) {
  Tile x, acc;
  for (int M = 0; M < 4; ++M) for (int r = 0; r < 16; ++r) x.m[M][r] = 0.001f * (threadIdx.x + r);
  for (int it = 0; it < iters; ++it) {
    tile_zero(acc);
    tile_gemm(acc, x, W);
    x = acc;
  }
  tile_store_blk(x, out);
}
__device__ void do_valu(float* out, int iters) {
  f32x2 v = {0.001f * threadIdx.x, 0.002f * threadIdx.x};
  f32x2 s = {0.f, 0.f};
  for (int it = 0; it < iters; ++it) {
#pragma unroll 8
    for (int k = 0; k < 64; ++k) {  // 64 gelus per 'iteration' ~ one GEMM's worth of JIT activations
      v = c_gelu2(v + (f32x2){1e-3f, -1e-3f});
      s = s + v;
    }
  }
  out[threadIdx.x] = s.x + s.y;
}
template <int ROLE>  // 0: all M, 1: all V, 2: waves 0-3 M + 4-7 V (each SIMD gets one of each)
__global__ __launch_bounds__(512, 1) void k(const float4* W, float* out, int iters) {
  int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  float* o = out + (size_t)(blockIdx.x * 8 + w) * 4096;
  bool m = ROLE == 0 || (ROLE == 2 && w < 4);
  if (m) do_mfma(W, o, iters); else do_valu(o, iters);
}
int main() {
  float4* W; float* out;
  hipMalloc(&W, 4096 * 16); hipMalloc(&out, (size_t)256 * 8 * 4096 * 4);
  hipMemset(W, 0, 4096 * 16);
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  const int iters = 400;
  for (int role = 0; role < 3; ++role) {
    for (int rep = 0; rep < 3; ++rep) {
      hipEventRecord(a);
      if (role == 0) k<0><<<256, 512>>>(W, out, iters);
      if (role == 1) k<1><<<256, 512>>>(W, out, iters);
      if (role == 2) k<2><<<256, 512>>>(W, out, iters);
      hipEventRecord(b); hipEventSynchronize(b);
      float ms; hipEventElapsedTime(&ms, a, b);
      if (rep == 2) printf("role %s: %.3f ms\n", role == 0 ? "all-MFMA" : role == 1 ? "all-VALU" : "half/half", ms);
    }
  }
}
