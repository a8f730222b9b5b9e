// Does an f32 MFMA stream on one wave of a SIMD leave issue room for f32 VALU from the other
// wave of the same SIMD, and does it matter whether that VALU is packed (v_pk_fma_f32) or scalar
// (v_fma_f32)? 8 waves per workgroup (2 per SIMD), one workgroup per CU. Wave roles per SIMD pair:
//   M = v_mfma_f32_32x32x2_f32 on 4 independent accumulators (throughput-bound)
//   S = v_fma_f32 on 16 independent registers, P = v_pk_fma_f32 on 8 independent pairs
//       (the same FLOPs per iteration: 16 scalar FMAs = 8 packed)
// Pairs: MM, SS, PP, M+S, M+P, and each role alone with the partner slot idle (M_, S_, P_).
// Build: hipcc -O3 --offload-arch=gfx950 tools/micro/coexec.hip -o tools/micro/coexec
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

__device__ float run_m(int iters) {
  f32x16 a0 = {}, a1 = {}, a2 = {}, a3 = {};
  float x = 1e-3f * (threadIdx.x & 63), y = 1.0001f;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      a0 = __builtin_amdgcn_mfma_f32_32x32x2f32(x, y, a0, 0, 0, 0);
      a1 = __builtin_amdgcn_mfma_f32_32x32x2f32(y, x, a1, 0, 0, 0);
      a2 = __builtin_amdgcn_mfma_f32_32x32x2f32(x, x, a2, 0, 0, 0);
      a3 = __builtin_amdgcn_mfma_f32_32x32x2f32(y, y, a3, 0, 0, 0);
    }
  }
  float s = 0.f;
  for (int r = 0; r < 16; ++r) s += a0[r] + a1[r] + a2[r] + a3[r];
  return s;
}

// 64 scalar FMAs per iteration (16 chains x 4) = 4 MFMA-iteration's... calibrated by timing alone
__device__ float run_s(int iters) {
  float v[16];
  for (int i = 0; i < 16; ++i) v[i] = 1e-3f * (threadIdx.x + i);
  const float m = 0.9999f, c = 1e-4f;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int i = 0; i < 16; ++i) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(v[i]) : "v"(m), "v"(c));
  }
  float s = 0.f;
  for (int i = 0; i < 16; ++i) s += v[i];
  return s;
}

__device__ float run_p(int iters) {
  f32x2 v[8];
  for (int i = 0; i < 8; ++i) v[i] = (f32x2){1e-3f * (threadIdx.x + i), 2e-3f * i};
  const f32x2 m = {0.9999f, 0.9998f}, c = {1e-4f, 2e-4f};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int i = 0; i < 8; ++i) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(v[i]) : "v"(m), "v"(c));
  }
  float s = 0.f;
  for (int i = 0; i < 8; ++i) s += v[i].x + v[i].y;
  return s;
}

// role codes: 0 idle, 1 M, 2 S, 3 P; waves 0-3 take role A, waves 4-7 role B (wave w and w+4
// land on the same SIMD: waves are assigned round-robin over the 4 SIMDs)
__global__ __launch_bounds__(512, 1) void k(float* out, int ra, int rb, int im, int is, int ip) {
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int role = w < 4 ? ra : rb;
  float s = 0.f;
  if (role == 1) s = run_m(im);
  else if (role == 2) s = run_s(is);
  else if (role == 3) s = run_p(ip);
  out[blockIdx.x * 512 + threadIdx.x] = s;
}

int main() {
  float* out;
  hipMalloc(&out, 256 * 512 * 4);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const int im = 2000, is = 8000, ip = 8000;
  const char* nm = "_MSP";
  const int pairs[][2] = {{1, 0}, {2, 0}, {3, 0}, {1, 1}, {2, 2}, {3, 3}, {1, 2}, {1, 3}, {2, 3}};
  for (auto& p : pairs) {
    float best = 1e9f;
    for (int rep = 0; rep < 4; ++rep) {
      hipEventRecord(a);
      k<<<256, 512>>>(out, p[0], p[1], im, is, ip);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      if (rep > 0 && ms < best) best = ms;
    }
    printf("%c+%c: %.3f ms\n", nm[p[0]], nm[p[1]], best);
  }
  printf("per iteration: M = 16 MFMA 32x32x2 f32 (1024 cyc at 64/MFMA), S = 64 v_fma_f32, P = 32 v_pk_fma_f32\n");
  return 0;
}
