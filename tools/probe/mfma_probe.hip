// Probe: is v_mfma_f32_32x32x2_f32 bit-identical to a k-ordered fmaf chain, and which
// lane half supplies the first k? Also checks f32 div/sqrt are correctly rounded.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <random>
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// A: [32][K] row-major, B: [K][32], C init [32][32]; D out [32][32]. K even.
__global__ void k32(const float* A, const float* B, const float* C, float* D, int K) {
  int l = threadIdx.x; int i = l & 31, h = l >> 5;
  f32x16 acc;
  for (int r = 0; r < 16; ++r) { int row = (r & 3) + 8 * (r >> 2) + 4 * h; acc[r] = C[row * 32 + i]; }
  for (int s = 0; s < K / 2; ++s) {
    float a = A[i * K + 2 * s + h];
    float b = B[(2 * s + h) * 32 + i];
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
  }
  for (int r = 0; r < 16; ++r) { int row = (r & 3) + 8 * (r >> 2) + 4 * h; D[row * 32 + i] = acc[r]; }
}
// 16x16x4: A [16][K], B [K][16]
__global__ void k16(const float* A, const float* B, const float* C, float* D, int K) {
  int l = threadIdx.x; int i = l & 15, q = l >> 4;
  f32x4 acc;
  for (int r = 0; r < 4; ++r) acc[r] = C[(4 * q + r) * 16 + i];
  for (int s = 0; s < K / 4; ++s) {
    float a = A[i * K + 4 * s + q];
    float b = B[(4 * s + q) * 16 + i];
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc, 0, 0, 0);
  }
  for (int r = 0; r < 4; ++r) D[(4 * q + r) * 16 + i] = acc[r];
}
__global__ void kdiv(const float* x, const float* y, float* q, float* s, int n) {
  int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t < n) { q[t] = x[t] / y[t]; s[t] = sqrtf(fabsf(x[t])); }
}
static float chain(const float* a, const float* b, float c, const int* order, int K) {
  for (int t = 0; t < K; ++t) c = fmaf(a[order[t]], b[order[t]], c);
  return c;
}
int main() {
  std::mt19937 g(123); std::uniform_real_distribution<float> U(-1.f, 1.f);
  const int K = 64;
  for (int shape = 0; shape < 2; ++shape) {
    int M = shape == 0 ? 32 : 16, KS = shape == 0 ? 2 : 4;
    std::vector<float> A(M * K), B(K * M), C(M * M), D(M * M);
    for (auto& v : A) v = U(g) * (1 << (g() % 20)); for (auto& v : B) v = U(g) * (1 << (g() % 20));
    for (auto& v : C) v = U(g);
    float *dA, *dB, *dC, *dD;
    hipMalloc(&dA, A.size() * 4); hipMalloc(&dB, B.size() * 4); hipMalloc(&dC, C.size() * 4); hipMalloc(&dD, D.size() * 4);
    hipMemcpy(dA, A.data(), A.size() * 4, hipMemcpyHostToDevice); hipMemcpy(dB, B.data(), B.size() * 4, hipMemcpyHostToDevice);
    hipMemcpy(dC, C.data(), C.size() * 4, hipMemcpyHostToDevice);
    if (shape == 0) k32<<<1, 64>>>(dA, dB, dC, dD, K); else k16<<<1, 64>>>(dA, dB, dC, dD, K);
    hipMemcpy(D.data(), dD, D.size() * 4, hipMemcpyDeviceToHost);
    // candidate orders within a k-step: ascending lane group, descending
    int asc[64], desc[64];
    for (int s = 0; s < K / KS; ++s) for (int j = 0; j < KS; ++j) { asc[s * KS + j] = s * KS + j; desc[s * KS + j] = s * KS + (KS - 1 - j); }
    long ok_asc = 0, ok_desc = 0, tot = 0;
    for (int i = 0; i < M; ++i) for (int j = 0; j < M; ++j) {
      float a[64], b[64]; for (int k = 0; k < K; ++k) { a[k] = A[i * K + k]; b[k] = B[k * M + j]; }
      float ra = chain(a, b, C[i * M + j], asc, K), rd = chain(a, b, C[i * M + j], desc, K);
      float d = D[i * M + j];
      ok_asc += !memcmp(&ra, &d, 4); ok_desc += !memcmp(&rd, &d, 4); ++tot;
    }
    printf("mfma %dx%dx%d: match asc-lane-group chain %ld/%ld, desc %ld/%ld\n", M, M, KS, ok_asc, tot, ok_desc, tot);
  }
  const int n = 1 << 22;
  std::vector<float> x(n), y(n), q(n), s(n);
  for (int i = 0; i < n; ++i) { x[i] = U(g) * powf(2.f, (int)(g() % 60) - 30); y[i] = U(g) * powf(2.f, (int)(g() % 60) - 30); }
  float *dx, *dy, *dq, *ds; hipMalloc(&dx, n * 4); hipMalloc(&dy, n * 4); hipMalloc(&dq, n * 4); hipMalloc(&ds, n * 4);
  hipMemcpy(dx, x.data(), n * 4, hipMemcpyHostToDevice); hipMemcpy(dy, y.data(), n * 4, hipMemcpyHostToDevice);
  kdiv<<<n / 256, 256>>>(dx, dy, dq, ds, n);
  hipMemcpy(q.data(), dq, n * 4, hipMemcpyDeviceToHost); hipMemcpy(s.data(), ds, n * 4, hipMemcpyDeviceToHost);
  long bd = 0, bs = 0;
  for (int i = 0; i < n; ++i) { float qq = x[i] / y[i], ss = sqrtf(fabsf(x[i])); bd += memcmp(&qq, &q[i], 4) != 0; bs += memcmp(&ss, &s[i], 4) != 0; }
  printf("div mismatches %ld / %d, sqrt mismatches %ld / %d\n", bd, n, bs, n);
  return 0;
}
