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

// P with an s_nop 0 after every packed FMA (the compiler puts one after each inline-asm block)
__device__ float run_pn(int iters) {
  f32x2 v[8];
  for (int i = 0; i < 8; ++i) v[i] = (f32x2){1e-3f * (threadIdx.x + i), 2e-3f * i};
  const f32x2 m = {0.9999f, 0.9998f}, c = {1e-4f, 2e-4f};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int i = 0; i < 8; ++i) asm volatile("v_pk_fma_f32 %0, %0, %1, %2\n\ts_nop 0" : "+v"(v[i]) : "v"(m), "v"(c));
  }
  float s = 0.f;
  for (int i = 0; i < 8; ++i) s += v[i].x + v[i].y;
  return s;
}

// transcendental: v_rcp_f32 on 16 independent registers (64 per iteration, as S)
__device__ float run_t(int iters) {
  float v[16];
  for (int i = 0; i < 16; ++i) v[i] = 1.0f + 1e-3f * (threadIdx.x + i);
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int i = 0; i < 16; ++i) asm volatile("v_rcp_f32 %0, %0" : "+v"(v[i]));
  }
  float s = 0.f;
  for (int i = 0; i < 16; ++i) s += v[i];
  return s;
}

// the same wave interleaving its MFMAs with independent VALU work: KIND 0 = 2 v_pk_fma_f32 per
// MFMA, 1 = 4 v_fma_f32 per MFMA, 2 = one s_nop 0 per MFMA, 3 = one v_rcp_f32 per MFMA
template <int KIND, int NP = 2, int NS = 4>
__device__ float run_mix(int iters) {
  f32x16 a0 = {}, a1 = {}, a2 = {}, a3 = {};
  float x = 1e-3f * (threadIdx.x & 63), y = 1.0001f;
  f32x2 v0 = {x, y}, v1 = {y, x}, v2 = {x, x}, v3 = {y, y};
  float s0 = x, s1 = y, s2 = x + y, s3 = x * y, s4 = x - y, s5 = 2 * x, s6 = 2 * y, s7 = x + 1;
  const f32x2 m = {0.9999f, 0.9998f}, c = {1e-4f, 2e-4f};
  const float ms = 0.9999f, cs = 1e-4f;
#define MIX_STEP(acc, A, B, SR)                                                                   \
  acc = __builtin_amdgcn_mfma_f32_32x32x2f32(A, B, acc, 0, 0, 0);                              \
  if (KIND == 0) {                                                                              \
    if (NP > 0) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(v0) : "v"(m), "v"(c));       \
    if (NP > 1) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(v1) : "v"(m), "v"(c));       \
    if (NP > 2) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(v2) : "v"(m), "v"(c));       \
    if (NP > 3) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(v3) : "v"(m), "v"(c));       \
  } else if (KIND == 1) {                                                                       \
    if (NS > 0) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(s0) : "v"(ms), "v"(cs));         \
    if (NS > 1) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(s1) : "v"(ms), "v"(cs));         \
    if (NS > 2) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(s2) : "v"(ms), "v"(cs));         \
    if (NS > 3) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(s3) : "v"(ms), "v"(cs));         \
    if (NS > 4) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(s4) : "v"(ms), "v"(cs));         \
    if (NS > 5) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(s5) : "v"(ms), "v"(cs));         \
    if (NS > 6) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(s6) : "v"(ms), "v"(cs));         \
    if (NS > 7) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(s7) : "v"(ms), "v"(cs));         \
  } else if (KIND == 2) {                                                                       \
    asm volatile("s_nop 0");                                                                    \
  } else {                                                                                      \
    asm volatile("v_rcp_f32 %0, %0" : "+v"(SR));                                                \
  }                                                                                             \
  __builtin_amdgcn_sched_barrier(0);
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      MIX_STEP(a0, x, y, s0)
      MIX_STEP(a1, y, x, s1)
      MIX_STEP(a2, x, x, s2)
      MIX_STEP(a3, y, y, s3)
    }
  }
  float s = v0.x + v0.y + v1.x + v1.y + v2.x + v2.y + v3.x + v3.y + s0 + s1 + s2 + s3 + s4 + s5 + s6 + s7;
  for (int r = 0; r < 16; ++r) s += a0[r] + a1[r] + a2[r] + a3[r];
  return s;
}

// role codes: 0 idle, 1 M, 2 S, 3 P, 4 P+nop, 5 T (v_rcp_f32), 6-9 run_mix<0..3>; waves 0-3 take role A, waves 4-7 role B (wave w and w+4
// land on the same SIMD: waves are assigned round-robin over the 4 SIMDs)
__global__ __launch_bounds__(512, 1) void k(float* out, int ra, int rb, int im, int is, int ip) {
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int role = w < 4 ? ra : rb;
  float s = 0.f;
  if (role == 1) s = run_m(im);
  else if (role == 2) s = run_s(is);
  else if (role == 3) s = run_p(ip);
  else if (role == 4) s = run_pn(ip);
  else if (role == 5) s = run_t(is);
  else if (role == 6) s = run_mix<0>(im);
  else if (role == 7) s = run_mix<1>(im);
  else if (role == 8) s = run_mix<2>(im);
  else if (role == 9) s = run_mix<3>(im);
  else if (role == 10) s = run_mix<0, 1>(im);
  else if (role == 11) s = run_mix<0, 4>(im);
  else if (role == 12) s = run_mix<1, 2, 1>(im);
  else if (role == 13) s = run_mix<1, 2, 2>(im);
  else if (role == 14) s = run_mix<1, 2, 8>(im);
  out[blockIdx.x * 512 + threadIdx.x] = s;
}

int main() {
  float* out;
  hipMalloc(&out, 256 * 512 * 4);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const int im = 2000, is = 8000, ip = 8000;
  const char* nm = "_MSPNTabcdefghi";
  const int pairs[][2] = {{1, 0}, {2, 0}, {3, 0}, {4, 0}, {5, 0}, {1, 1}, {2, 2}, {3, 3}, {4, 4}, {5, 5}, {1, 2}, {1, 3}, {1, 4}, {1, 5}, {2, 3}, {6, 0}, {7, 0}, {8, 0}, {9, 0}, {6, 6}, {7, 7}, {8, 8}, {9, 9}, {10, 10}, {11, 11}, {12, 12}, {13, 13}, {14, 14}};
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
  printf("per iteration: M = 16 MFMA 32x32x2 f32 (1024 cyc at 64/MFMA), S = 64 v_fma_f32, P = 32 v_pk_fma_f32, N = P + s_nop 0 after each, T = 64 v_rcp_f32; a/b/c/d = M with 2 v_pk_fma / 4 v_fma / 1 s_nop / 1 v_rcp after each MFMA in the same wave; e/f = 1 / 4 v_pk_fma, g/h/i = 1 / 2 / 8 v_fma_f32 after each MFMA\n");
  return 0;
}
