// pst_device.h — device-side building blocks of libpst (gfx950 / CDNA4).
//
// 1. Canonical numerics. Every operation is a fixed sequence of IEEE-754 ops
//    (fmaf, +, *, /, sqrtf are correctly rounded on gfx950; compiled with -ffp-contract=off),
//    so results are bit-identical to any CPU implementation of the same sequence.
// 2. The wave tile: 32 columns (edges, nodes or tokens — one per lane&31) x 128 channels held
//    as four 32x32 f32 MFMA accumulators. Lane l = (col = l&31, half h = l>>5) owns channels
//    c = 32*M + (r&3) + 8*(r>>2) + 4*h of accumulator M, register r. An accumulator tile feeds
//    the next v_mfma_f32_32x32x2_f32 as its B operand register by register (k-step (M, r) =
//    channel pair (c, c+4)), so a chain of Linear layers never leaves registers; the dot
//    products are fmaf chains in the "pi8" k order 0,4,1,5,2,6,3,7 per block of 8 channels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pst {

typedef float f32x16 __attribute__((ext_vector_type(16)));

// ------------------------------------------------------------------ canonical f32 math
// p / q for tanh's operand range (q in [4.9e-3, 1], |p| <= 1, no denormals): hardware
// reciprocal + one FMA (Markstein) correction. tools/micro/div_variants.hip and div_check.hip
// verify on the GPU that this equals the IEEE quotient for ALL 2^32 float32 inputs of c_tanh,
// so c_tanh stays bit-identical to the CPU form that uses '/'.
__device__ __forceinline__ float div_tanh(float p, float q) {
  float r = __builtin_amdgcn_rcpf(q);
  float y = p * r;
  float e = __builtin_fmaf(-q, y, p);
  return __builtin_fmaf(e, r, y);
}

__device__ __forceinline__ float c_tanh(float a) {
  const float clamp = 7.99881172180175781f;
  float x = fminf(fmaxf(a, -clamp), clamp);
  float x2 = x * x;
  float p = __builtin_fmaf(x2, -2.76076847742355e-16f, 2.00018790482477e-13f);
  p = __builtin_fmaf(x2, p, -8.60467152213735e-11f);
  p = __builtin_fmaf(x2, p, 5.12229709037114e-08f);
  p = __builtin_fmaf(x2, p, 1.48572235717979e-05f);
  p = __builtin_fmaf(x2, p, 6.37261928875436e-04f);
  p = __builtin_fmaf(x2, p, 4.89352455891786e-03f);
  p = x * p;
  float q = __builtin_fmaf(x2, 1.19825839466702e-06f, 1.18534705686654e-04f);
  q = __builtin_fmaf(x2, q, 2.26843463243900e-03f);
  q = __builtin_fmaf(x2, q, 4.89352518554385e-03f);
  float r = div_tanh(p, q);
  return fabsf(a) < 0.0004f ? a : r;
}

// tanh's rational core without the |x| < 4e-4 shortcut (used inside GELU)
__device__ __forceinline__ float c_tanh_core(float a) {
  const float clamp = 7.99881172180175781f;
  float x = fminf(fmaxf(a, -clamp), clamp);
  float x2 = x * x;
  float p = __builtin_fmaf(x2, -2.76076847742355e-16f, 2.00018790482477e-13f);
  p = __builtin_fmaf(x2, p, -8.60467152213735e-11f);
  p = __builtin_fmaf(x2, p, 5.12229709037114e-08f);
  p = __builtin_fmaf(x2, p, 1.48572235717979e-05f);
  p = __builtin_fmaf(x2, p, 6.37261928875436e-04f);
  p = __builtin_fmaf(x2, p, 4.89352455891786e-03f);
  p = x * p;
  float q = __builtin_fmaf(x2, 1.19825839466702e-06f, 1.18534705686654e-04f);
  q = __builtin_fmaf(x2, q, 2.26843463243900e-03f);
  q = __builtin_fmaf(x2, q, 4.89352518554385e-03f);
  return div_tanh(p, q);
}

// GELU (tanh form), canonical sequence: u = x (k0 + k0k1 x^2),
// g = h + h tanh(u), h = x / 2
#define GELU_K0 0.797884583473205566f
#define GELU_K0K1 0.035677406936883926f
__device__ __forceinline__ float c_gelu(float x) {
  float u = x * __builtin_fmaf(x * x, GELU_K0K1, GELU_K0);
  float hx = 0.5f * x;
  return __builtin_fmaf(hx, c_tanh_core(u), hx);
}

typedef float f32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ f32x2 pk_fma(f32x2 a, f32x2 b, f32x2 c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ f32x2 splat2(float v) { return (f32x2){v, v}; }

// 2·GELU(x) with the same bits as 2 * c_gelu(x) for every |x| >= 2^-125 (tools/micro/
// gelu_double_check.c, exhaustive): x + x·tanh(u) in one fma instead of h = x/2, h + h·tanh(u).
// The encoder kernels feed it to weights pre-scaled by 0.5 on the host (pst_api.cpp, exact for
// normal weights), so every product (2g)·(w/2) equals g·w and the chains are the canonical ones:
// one packed multiply less per pair of GELUs. Below 2^-125 the two forms differ by an ulp of a
// subnormal, a product that cannot change a chain holding anything above ~1e-30.
__device__ __forceinline__ f32x2 c_gelu2x(f32x2 x) {
  f32x2 u = x * pk_fma(x * x, splat2(GELU_K0K1), splat2(GELU_K0));
  const f32x2 clampv = splat2(7.99881172180175781f);
  f32x2 xc = __builtin_elementwise_min(__builtin_elementwise_max(u, -clampv), clampv);
  f32x2 s = xc * xc;
  f32x2 p = pk_fma(s, splat2(-2.76076847742355e-16f), splat2(2.00018790482477e-13f));
  p = pk_fma(s, p, splat2(-8.60467152213735e-11f));
  p = pk_fma(s, p, splat2(5.12229709037114e-08f));
  p = pk_fma(s, p, splat2(1.48572235717979e-05f));
  p = pk_fma(s, p, splat2(6.37261928875436e-04f));
  p = pk_fma(s, p, splat2(4.89352455891786e-03f));
  p = xc * p;
  f32x2 q = pk_fma(s, splat2(1.19825839466702e-06f), splat2(1.18534705686654e-04f));
  q = pk_fma(s, q, splat2(2.26843463243900e-03f));
  q = pk_fma(s, q, splat2(4.89352518554385e-03f));
  f32x2 r = {__builtin_amdgcn_rcpf(q.x), __builtin_amdgcn_rcpf(q.y)};
  f32x2 y = p * r;
  f32x2 e = pk_fma(-q, y, p);
  f32x2 t = pk_fma(e, r, y);
  return pk_fma(x, t, x);
}

// c_gelu2x with every packed op pinned as v_pk_* by inline asm: the compiler's pre-emit peephole
// otherwise unpacks packed FP32 ops that sit in an MFMA's shadow into two scalar ops each, and on
// gfx950 that costs VALU issue cycles the MFMA pipe does not hide (A/B on the box: k_mpnn 1.8 %
// faster pinned; PMC SQ_VALU_MFMA_COEXEC_CYCLES = 0). Same op sequence as c_gelu2x, bit for bit.
// Constant operands: SGPR pairs holding the constant in both halves (sc2).
__device__ __forceinline__ uint64_t sc2(float c) { return (uint64_t)__float_as_uint(c) * 0x100000001ull; }
__device__ __forceinline__ f32x2 apk_mul(f32x2 a, f32x2 b) {
  f32x2 d;
  asm("v_pk_mul_f32 %0, %1, %2" : "=v"(d) : "v"(a), "v"(b));
  return d;
}
__device__ __forceinline__ f32x2 apk_mul_s(f32x2 a, uint64_t c) {
  f32x2 d;
  asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[1,0]" : "=v"(d) : "v"(a), "s"(c));
  return d;
}
// a*b + c, c an SGPR constant
__device__ __forceinline__ f32x2 apk_fma_vvs(f32x2 a, f32x2 b, uint64_t c) {
  f32x2 d;
  asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[1,1,0]" : "=v"(d) : "v"(a), "v"(b), "s"(c));
  return d;
}
// a*b + c, b an SGPR constant, c a VGPR pair
__device__ __forceinline__ f32x2 apk_fma_vsv(f32x2 a, uint64_t b, f32x2 c) {
  f32x2 d;
  asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[1,0,1]" : "=v"(d) : "v"(a), "s"(b), "v"(c));
  return d;
}
__device__ __forceinline__ f32x2 apk_fma(f32x2 a, f32x2 b, f32x2 c) {
  f32x2 d;
  asm("v_pk_fma_f32 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
  return d;
}
// -a*b + c
__device__ __forceinline__ f32x2 apk_fma_neg(f32x2 a, f32x2 b, f32x2 c) {
  f32x2 d;
  asm("v_pk_fma_f32 %0, %1, %2, %3 neg_lo:[1,0,0] neg_hi:[1,0,0]" : "=v"(d) : "v"(a), "v"(b), "v"(c));
  return d;
}
// FRESH: x may have been written by an MFMA only a few instructions ago. Only the compiler's
// hazard recognizer knows the wait states an MFMA-written VGPR needs before a VALU read (an asm
// read can see the accumulator before its last k-step), so then the first step stays in C.
// tile_gemm_f evaluates k-steps 0..3 right after the producing GEMM (FRESH); later k-steps read
// accumulators finished >= 4 MFMA groups earlier. The clamp and the reciprocal stay in C (no
// packed forms). Measured costs (A/B, 512 x 256 residues): the GELU is ~10 % of k_mpnn, since
// f32 MFMA and f32 VALU share the vector datapath (MI355X: f32 MFMA peak = vector peak).
// Returns 2·GELU(x) (c_gelu2x's doubled form, for the half-scaled consumer weights).
template <bool FRESH>
__device__ __forceinline__ f32x2 c_gelu2x_asm(f32x2 x) {
  const f32x2 c5 = splat2(2.00018790482477e-13f), q2 = splat2(1.18534705686654e-04f);
  f32x2 u;
  if (FRESH) {
    u = x * pk_fma(x * x, splat2(GELU_K0K1), splat2(GELU_K0));
  } else {
    const f32x2 k0 = splat2(GELU_K0);
    f32x2 t0;
    asm("v_pk_mul_f32 %1, %2, %2\n\t"
        "v_pk_fma_f32 %1, %1, %3, %4\n\t"
        "v_pk_mul_f32 %0, %2, %1"
        : "=&v"(u), "=&v"(t0)
        : "v"(x), "s"(sc2(GELU_K0K1)), "v"(k0));
  }
  const float cl = 7.99881172180175781f;
  f32x2 xc = {__builtin_amdgcn_fmed3f(u.x, -cl, cl), __builtin_amdgcn_fmed3f(u.y, -cl, cl)};
  f32x2 q, sq;
  asm("v_pk_mul_f32 %1, %2, %2\n\t"
      "v_pk_fma_f32 %0, %1, %3, %4\n\t"
      "v_pk_fma_f32 %0, %1, %0, %5\n\t"
      "v_pk_fma_f32 %0, %1, %0, %6"
      : "=&v"(q), "=&v"(sq)
      : "v"(xc), "s"(sc2(1.19825839466702e-06f)), "v"(q2), "s"(sc2(2.26843463243900e-03f)),
        "s"(sc2(4.89352518554385e-03f)));
  // the reciprocal issues here, 7 instructions before its first use in the next group: that
  // covers the one wait state a v_rcp (trans) result needs, which the hazard recognizer does
  // not check for asm operands
  f32x2 r = {__builtin_amdgcn_rcpf(q.x), __builtin_amdgcn_rcpf(q.y)};
  f32x2 p, y, e, t;
  asm("v_pk_fma_f32 %0, %5, %8, %9\n\t"
      "v_pk_fma_f32 %0, %5, %0, %10\n\t"
      "v_pk_fma_f32 %0, %5, %0, %11\n\t"
      "v_pk_fma_f32 %0, %5, %0, %12\n\t"
      "v_pk_fma_f32 %0, %5, %0, %13\n\t"
      "v_pk_fma_f32 %0, %5, %0, %14\n\t"
      "v_pk_mul_f32 %0, %4, %0\n\t"
      "v_pk_mul_f32 %1, %0, %6\n\t"
      "v_pk_fma_f32 %2, %7, %1, %0 neg_lo:[1,0,0] neg_hi:[1,0,0]\n\t"
      "v_pk_fma_f32 %3, %2, %6, %1"
      : "=&v"(p), "=&v"(y), "=&v"(e), "=&v"(t)
      : "v"(xc), "v"(sq), "v"(r), "v"(q), "s"(sc2(-2.76076847742355e-16f)), "v"(c5),
        "s"(sc2(-8.60467152213735e-11f)), "s"(sc2(5.12229709037114e-08f)), "s"(sc2(1.48572235717979e-05f)),
        "s"(sc2(6.37261928875436e-04f)), "s"(sc2(4.89352455891786e-03f)));
  // the last step in C: its output is the B operand of the next MFMAs, and an MFMA reading a VGPR
  // a VALU just wrote needs 2 wait states that hipcc inserts for its own code but not after inline
  // asm (round 5: with this fma inside the asm, k_mpnn_q<1,4> read stale operands — its MFMA
  // followed the fma one instruction later; tools/mfma_hazard_scan.py checks the code objects)
  return pk_fma(x, t, x);
}

__device__ __forceinline__ float c_ldexpf(float v, int n) {
  if (n < -126) {
    v = v * __uint_as_float((uint32_t)(-126 + 127) << 23);
    n += 126;
    if (n < -126) n = -126;
  }
  if (n > 127) n = 127;
  return v * __uint_as_float((uint32_t)(n + 127) << 23);
}

__device__ __forceinline__ float c_exp(float x) {
  if (x > 88.7228394f) return __builtin_inff();
  if (x < -103.972084f) return 0.0f;
  float n = rintf(x * 1.44269502f);
  float r = __builtin_fmaf(n, -0.693145752f, x);
  r = __builtin_fmaf(n, -1.42860677e-6f, r);
  float p = 1.98756912e-4f;
  p = __builtin_fmaf(p, r, 1.39819994e-3f);
  p = __builtin_fmaf(p, r, 8.33345205e-3f);
  p = __builtin_fmaf(p, r, 4.16657962e-2f);
  p = __builtin_fmaf(p, r, 1.66666655e-1f);
  p = __builtin_fmaf(p, r, 5.00000012e-1f);
  float y = __builtin_fmaf(p, r * r, r) + 1.0f;
  return c_ldexpf(y, (int)n);
}

__device__ __forceinline__ float c_sigmoid(float x) { return 1.0f / (1.0f + c_exp(-x)); }

// ------------------------------------------------------------------ canonical f64 math
__device__ __forceinline__ double c_ldexp64(double v, int n) {
  if (n < -1022) {
    v = v * __longlong_as_double((long long)(-1022 + 1023) << 52);
    n += 1022;
    if (n < -1022) n = -1022;
  }
  if (n > 1023) n = 1023;
  return v * __longlong_as_double((long long)(n + 1023) << 52);
}

__device__ __forceinline__ double c_exp64(double x) {
  if (x > 709.782712893384) return __builtin_inf();
  if (x < -745.2) return 0.0;
  double n = rint(x * 1.4426950408889634);
  double r = __builtin_fma(n, -6.93147180369123816490e-01, x);
  r = __builtin_fma(n, -1.90821492927058770002e-10, r);
  double p = 1.0 / 6227020800.0;
  p = __builtin_fma(p, r, 1.0 / 479001600.0);
  p = __builtin_fma(p, r, 1.0 / 39916800.0);
  p = __builtin_fma(p, r, 1.0 / 3628800.0);
  p = __builtin_fma(p, r, 1.0 / 362880.0);
  p = __builtin_fma(p, r, 1.0 / 40320.0);
  p = __builtin_fma(p, r, 1.0 / 5040.0);
  p = __builtin_fma(p, r, 1.0 / 720.0);
  p = __builtin_fma(p, r, 1.0 / 120.0);
  p = __builtin_fma(p, r, 1.0 / 24.0);
  p = __builtin_fma(p, r, 1.0 / 6.0);
  p = __builtin_fma(p, r, 0.5);
  double y = __builtin_fma(p, r * r, r) + 1.0;
  return c_ldexp64(y, (int)n);
}

// ------------------------------------------------------------------ wave tile
__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

// channel held by (half h, accumulator M, register r)
__host__ __device__ constexpr int tile_channel(int h, int M, int r) {
  return 32 * M + (r & 3) + 8 * (r >> 2) + 4 * h;
}

struct Tile {
  f32x16 m[4];
};

// Buffer-resource loads/stores: wave-uniform base in SGPRs, per-lane byte offset in one VGPR,
// per-instruction constant offset in an SGPR. Keeps unrolled fragment streams from
// materialising one 64-bit address per k-step (which spilled the first version).
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, 0x7fffffff, 0x00020000);
}
// a resource whose accesses are all out of range when p is null (stores dropped, loads read 0)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc_or_null(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, p ? 0x7fffffff : 0, 0x00020000);
}
__device__ __forceinline__ float4 buf_load4(__amdgpu_buffer_rsrc_t rs, int voff, int soff) {
  u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, voff, soff, 0);
  return make_float4(__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z), __uint_as_float(v.w));
}
__device__ __forceinline__ float buf_load1(__amdgpu_buffer_rsrc_t rs, int voff, int soff) {
  return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, voff, soff, 0));
}
#ifndef PST_E_STORE_AUX
#define PST_E_STORE_AUX 0
#endif
#ifndef PST_E_LOAD_AUX
#define PST_E_LOAD_AUX 0
#endif
__device__ __forceinline__ void buf_store4(__amdgpu_buffer_rsrc_t rs, int voff, int soff, float a, float b, float c,
                                           float d) {
  u32x4 v = {__float_as_uint(a), __float_as_uint(b), __float_as_uint(c), __float_as_uint(d)};
  __builtin_amdgcn_raw_buffer_store_b128(v, rs, voff, soff, PST_E_STORE_AUX);
}

__device__ __forceinline__ void tile_zero(Tile& t) {
#pragma unroll
  for (int M = 0; M < 4; ++M)
#pragma unroll
    for (int r = 0; r < 16; ++r) t.m[M][r] = 0.0f;
}

// Load a 128-channel row stored in "perm" order (perm[h*64 + M*16 + r] = v[tile_channel]).
// `row` is this lane's row base; the lane reads its 64 floats (256 B) contiguously.
__device__ __forceinline__ void tile_load_perm(Tile& t, const float* __restrict__ row) {
  const float4* p = reinterpret_cast<const float4*>(row + (lane_id() >> 5) * 64);
#pragma unroll
  for (int M = 0; M < 4; ++M)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float4 v = p[M * 4 + q];
      t.m[M][4 * q + 0] = v.x;
      t.m[M][4 * q + 1] = v.y;
      t.m[M][4 * q + 2] = v.z;
      t.m[M][4 * q + 3] = v.w;
    }
}

__device__ __forceinline__ void tile_store_perm(const Tile& t, float* __restrict__ row) {
  float4* p = reinterpret_cast<float4*>(row + (lane_id() >> 5) * 64);
#pragma unroll
  for (int M = 0; M < 4; ++M)
#pragma unroll
    for (int q = 0; q < 4; ++q)
      p[M * 4 + q] = make_float4(t.m[M][4 * q], t.m[M][4 * q + 1], t.m[M][4 * q + 2], t.m[M][4 * q + 3]);
}

// Blocked tile storage: [16 quads][64 lanes][4] floats (16 KB), fully coalesced.
// `blk` must be wave-uniform.
__device__ __forceinline__ void tile_load_blk(Tile& t, const float* __restrict__ blk) {
  __amdgpu_buffer_rsrc_t rs = make_rsrc(blk);
  const int vo = lane_id() * 16;
#pragma unroll
  for (int M = 0; M < 4; ++M)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      u32x4 u = __builtin_amdgcn_raw_buffer_load_b128(rs, vo, (M * 4 + q) * 1024, PST_E_LOAD_AUX);
      float4 v = make_float4(__uint_as_float(u.x), __uint_as_float(u.y), __uint_as_float(u.z), __uint_as_float(u.w));
      t.m[M][4 * q + 0] = v.x;
      t.m[M][4 * q + 1] = v.y;
      t.m[M][4 * q + 2] = v.z;
      t.m[M][4 * q + 3] = v.w;
    }
}

__device__ __forceinline__ void tile_store_blk(const Tile& t, float* __restrict__ blk) {
  __amdgpu_buffer_rsrc_t rs = make_rsrc(blk);
  const int vo = lane_id() * 16;
#pragma unroll
  for (int M = 0; M < 4; ++M)
#pragma unroll
    for (int q = 0; q < 4; ++q)
      buf_store4(rs, vo, (M * 4 + q) * 1024, t.m[M][4 * q], t.m[M][4 * q + 1], t.m[M][4 * q + 2], t.m[M][4 * q + 3]);
}

// acc += X · W over K = 128 channels (64 k-steps), four output accumulators.
// Wf: A fragments, [64 k-steps][64 lanes] float4 (one f32 per output accumulator).
// The fragment stream runs GEMM_DEPTH k-steps ahead in a register ring; a scheduling
// barrier per k-step keeps the compiler from hoisting the whole stream (register spills).
#ifndef GEMM_DEPTH
#define GEMM_DEPTH 4
#endif
// Generic form: the B operand of k-step t is f(t, X[t]) — the previous layer's activation
// (bias + GELU, bias + ReLU, ...) evaluated just in time, one element per k-step, so its VALU
// work issues in the shadow of the current k-step's four MFMAs instead of as a separate
// VALU phase between GEMMs. The schedule interleaves MFMA and VALU groups explicitly.
// ACT_GROUP k-steps form one scheduling group; the ACT_GROUP/2 activation pairs of the next group
// are evaluated during the current one (independent chains the scheduler can interleave).
#ifndef ACT_GROUP
#define ACT_GROUP 4
#endif
// ActGelu's non-FRESH asm form (k-steps t >= ACT_GROUP) reads accumulators without hazard checks:
// it relies on their MFMA group having finished at least 4 k-steps earlier, so ACT_GROUP >= 4
static_assert(ACT_GROUP >= 4 && ACT_GROUP % 2 == 0 && 64 % ACT_GROUP == 0, "ACT_GROUP: even divisor of 64, >= 4");
template <typename F>
__device__ __forceinline__ void tile_gemm_f(Tile& acc, const Tile& X, const float4* __restrict__ Wf, F&& f) {
  constexpr int G = ACT_GROUP, NP = G / 2;
  __amdgpu_buffer_rsrc_t rs = make_rsrc(Wf);
  const int vo = lane_id() * 16;
  float4 ring[GEMM_DEPTH];
#pragma unroll
  for (int i = 0; i < GEMM_DEPTH; ++i) ring[i] = buf_load4(rs, vo, i * 1024);
  // activations run one group of G k-steps ahead (G/2 packed pairs per group)
  f32x2 bq[NP], bn[NP];
#pragma unroll
  for (int j = 0; j < NP; ++j) bq[j] = f(2 * j, (f32x2){X.m[0][2 * j], X.m[0][2 * j + 1]});
#pragma unroll
  for (int g = 0; g < 64 / G; ++g) {
#pragma unroll
    for (int j = 0; j < G; ++j) {
      const int t = G * g + j;
      float4 a = ring[t % GEMM_DEPTH];
      if (t + GEMM_DEPTH < 64) ring[t % GEMM_DEPTH] = buf_load4(rs, vo, (t + GEMM_DEPTH) * 1024);
      if (g < 64 / G - 1 && (j & 1) == 0) {
        const int u = t + G;
        bn[j >> 1] = f(u, (f32x2){X.m[u / 16][u % 16], X.m[u / 16][u % 16 + 1]});
      }
      const float b = (j & 1) ? bq[j >> 1].y : bq[j >> 1].x;
      acc.m[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, b, acc.m[0], 0, 0, 0);
      acc.m[1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, b, acc.m[1], 0, 0, 0);
      acc.m[2] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.z, b, acc.m[2], 0, 0, 0);
      acc.m[3] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.w, b, acc.m[3], 0, 0, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int j = 0; j < NP; ++j) bq[j] = bn[j];
  }
}

// acc += X · W (tile_gemm) that also writes X out blocked (tile_store_blk layout) through `st`:
// quad i of X leaves at k-step 4i, the first k-step that reads it. On gfx9 the vector memory
// counter covers stores and loads in issue order, so a 16-store burst ahead of a GEMM makes the
// GEMM's first fragment loads wait for every store's write acknowledgement; spread one per group
// of four k-steps, each store is >= 4 k-steps older than the load whose wait would cover it.
// Same MFMA chain as tile_gemm: same bits. A null `st` (num_records 0) drops the stores.
__device__ __forceinline__ void tile_gemm_store(Tile& acc, const Tile& X, const float4* __restrict__ Wf,
                                                __amdgpu_buffer_rsrc_t st) {
  __amdgpu_buffer_rsrc_t rs = make_rsrc(Wf);
  const int vo = lane_id() * 16;
  float4 ring[GEMM_DEPTH];
#pragma unroll
  for (int i = 0; i < GEMM_DEPTH; ++i) ring[i] = buf_load4(rs, vo, i * 1024);
#pragma unroll
  for (int g = 0; g < 16; ++g) {
    buf_store4(st, vo, g * 1024, X.m[g / 4][4 * (g % 4)], X.m[g / 4][4 * (g % 4) + 1], X.m[g / 4][4 * (g % 4) + 2],
               X.m[g / 4][4 * (g % 4) + 3]);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int t = 4 * g + j;
      float4 a = ring[t % GEMM_DEPTH];
      if (t + GEMM_DEPTH < 64) ring[t % GEMM_DEPTH] = buf_load4(rs, vo, (t + GEMM_DEPTH) * 1024);
      const float b = X.m[t / 16][t % 16];
      acc.m[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, b, acc.m[0], 0, 0, 0);
      acc.m[1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, b, acc.m[1], 0, 0, 0);
      acc.m[2] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.z, b, acc.m[2], 0, 0, 0);
      acc.m[3] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.w, b, acc.m[3], 0, 0, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
}

// tile_gemm_f with the fragments of k-steps 0 .. KL-1 read from LDS (`Wl`, staged once per
// workgroup) and the rest streamed from `Wf` as usual: the same operands and MFMA chain, same bits.
template <int KL, typename F>
__device__ __forceinline__ void tile_gemm_mix_f(Tile& acc, const Tile& X, const float4* Wl,
                                                const float4* __restrict__ Wf, F&& f) {
  constexpr int G = ACT_GROUP, NP = G / 2;
  __amdgpu_buffer_rsrc_t rs = make_rsrc(Wf);
  const int lane = lane_id();
  const int vo = lane * 16;
  float4 lr[2], ring[GEMM_DEPTH];
  lr[0] = Wl[lane];
  lr[1] = Wl[64 + lane];
  f32x2 bq[NP], bn[NP];
#pragma unroll
  for (int j = 0; j < NP; ++j) bq[j] = f(2 * j, (f32x2){X.m[0][2 * j], X.m[0][2 * j + 1]});
#pragma unroll
  for (int g = 0; g < 64 / G; ++g) {
#pragma unroll
    for (int j = 0; j < G; ++j) {
      const int t = G * g + j;
      float4 a;
      if (t < KL) {
        a = lr[t % 2];
        if (t + 2 < KL) lr[t % 2] = Wl[(t + 2) * 64 + lane];
      } else {
        a = ring[(t - KL) % GEMM_DEPTH];
        if (t + GEMM_DEPTH < 64) ring[(t - KL) % GEMM_DEPTH] = buf_load4(rs, vo, (t + GEMM_DEPTH) * 1024);
      }
      // the global stream starts GEMM_DEPTH k-steps before the LDS part ends
      if (t == KL - GEMM_DEPTH) {
#pragma unroll
        for (int i = 0; i < GEMM_DEPTH; ++i)
          if (KL + i < 64) ring[i] = buf_load4(rs, vo, (KL + i) * 1024);
      }
      if (g < 64 / G - 1 && (j & 1) == 0) {
        const int u = t + G;
        bn[j >> 1] = f(u, (f32x2){X.m[u / 16][u % 16], X.m[u / 16][u % 16 + 1]});
      }
      const float b = (j & 1) ? bq[j >> 1].y : bq[j >> 1].x;
      acc.m[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, b, acc.m[0], 0, 0, 0);
      acc.m[1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, b, acc.m[1], 0, 0, 0);
      acc.m[2] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.z, b, acc.m[2], 0, 0, 0);
      acc.m[3] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.w, b, acc.m[3], 0, 0, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int j = 0; j < NP; ++j) bq[j] = bn[j];
  }
}

// acc = bias + X·W: the bias enters as an extra leading k-step (A = bias fragment, lane half 0
// holds b[32M + (lane&31)], half 1 zeros; B = 1 on half 0, 0 on half 1), so the chain starts
// from exactly b without a VALU add or a 64-register bias tile.
template <typename F>
__device__ __forceinline__ void tile_gemm_bf(Tile& acc, const Tile& X, const float4* __restrict__ Wf,
                                             const float4* __restrict__ Bf, F&& f) {
  __amdgpu_buffer_rsrc_t rs = make_rsrc(Bf);
  const float4 bb = buf_load4(rs, lane_id() * 16, 0);
  const float one = lane_id() < 32 ? 1.0f : 0.0f;
  const f32x16 z = {};
  acc.m[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(bb.x, one, z, 0, 0, 0);
  acc.m[1] = __builtin_amdgcn_mfma_f32_32x32x2f32(bb.y, one, z, 0, 0, 0);
  acc.m[2] = __builtin_amdgcn_mfma_f32_32x32x2f32(bb.z, one, z, 0, 0, 0);
  acc.m[3] = __builtin_amdgcn_mfma_f32_32x32x2f32(bb.w, one, z, 0, 0, 0);
  tile_gemm_f(acc, X, Wf, f);
}
template <int KL, typename F>
__device__ __forceinline__ void tile_gemm_mix_bf(Tile& acc, const Tile& X, const float4* Wl, const float4* __restrict__ Wf,
                                                 const float4* __restrict__ Bf, F&& f) {
  __amdgpu_buffer_rsrc_t rs = make_rsrc(Bf);
  const float4 bb = buf_load4(rs, lane_id() * 16, 0);
  const float one = lane_id() < 32 ? 1.0f : 0.0f;
  const f32x16 z = {};
  acc.m[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(bb.x, one, z, 0, 0, 0);
  acc.m[1] = __builtin_amdgcn_mfma_f32_32x32x2f32(bb.y, one, z, 0, 0, 0);
  acc.m[2] = __builtin_amdgcn_mfma_f32_32x32x2f32(bb.z, one, z, 0, 0, 0);
  acc.m[3] = __builtin_amdgcn_mfma_f32_32x32x2f32(bb.w, one, z, 0, 0, 0);
  tile_gemm_mix_f<KL>(acc, X, Wl, Wf, f);
}

// Activation functors: f(t, {x_t, x_t+1}) -> B operands of k-steps t, t+1.
struct ActId {
  __device__ __forceinline__ f32x2 operator()(int, f32x2 x) const { return x; }
};

// 2·GELU of the previous layer's output (its bias is already in the accumulator: chains start
// from the bias); the consuming weights are pre-scaled by 0.5 (c_gelu2x)
struct ActGelu2x {
  __device__ __forceinline__ f32x2 operator()(int t, f32x2 x) const {
    // the first group's pairs are evaluated right after the GEMM that produced them (FRESH)
    return t < ACT_GROUP ? c_gelu2x_asm<true>(x) : c_gelu2x_asm<false>(x);
  }
};

struct ActBiasRelu {
  const float* b;
  __device__ __forceinline__ f32x2 operator()(int t, f32x2 x) const {
    const float* bb = b + (lane_id() >> 5) * 64 + t;
    f32x2 v = x + (f32x2){bb[0], bb[1]};
    return (f32x2){v.x > 0.0f ? v.x : 0.0f, v.y > 0.0f ? v.y : 0.0f};
  }
};

__device__ __forceinline__ void tile_gemm(Tile& acc, const Tile& X, const float4* __restrict__ Wf) {
  tile_gemm_f(acc, X, Wf, ActId{});
}

// acc(one 32-output accumulator) += X · W, W: [64 k-steps][64 lanes] f32 (K = 128)
__device__ __forceinline__ void tile_gemm_narrow(f32x16& acc, const Tile& X, const float* __restrict__ Wf) {
  __amdgpu_buffer_rsrc_t rs = make_rsrc(Wf);
  const int vo = lane_id() * 4;
#pragma unroll
  for (int t = 0; t < 64; ++t) {
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(buf_load1(rs, vo, t * 256), X.m[t / 16][t % 16], acc, 0, 0, 0);
  }
}

// elementwise helpers on a perm-ordered vector held in LDS/global (this lane's 64 values)
__device__ __forceinline__ void tile_add_vec(Tile& t, const float* __restrict__ vperm) {
  const float4* p = reinterpret_cast<const float4*>(vperm + (lane_id() >> 5) * 64);
#pragma unroll
  for (int M = 0; M < 4; ++M)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      __builtin_amdgcn_sched_barrier(0);
      float4 v = p[M * 4 + q];
      t.m[M][4 * q + 0] = t.m[M][4 * q + 0] + v.x;
      t.m[M][4 * q + 1] = t.m[M][4 * q + 1] + v.y;
      t.m[M][4 * q + 2] = t.m[M][4 * q + 2] + v.z;
      t.m[M][4 * q + 3] = t.m[M][4 * q + 3] + v.w;
    }
}

__device__ __forceinline__ void tile_gelu(Tile& t) {
#pragma unroll
  for (int M = 0; M < 4; ++M)
#pragma unroll
    for (int r = 0; r < 16; ++r) t.m[M][r] = c_gelu(t.m[M][r]);
}

__device__ __forceinline__ void tile_relu(Tile& t) {
#pragma unroll
  for (int M = 0; M < 4; ++M)
#pragma unroll
    for (int r = 0; r < 16; ++r) t.m[M][r] = t.m[M][r] > 0.0f ? t.m[M][r] : 0.0f;
}

__device__ __forceinline__ void tile_add(Tile& a, const Tile& b) {
#pragma unroll
  for (int M = 0; M < 4; ++M)
#pragma unroll
    for (int r = 0; r < 16; ++r) a.m[M][r] = a.m[M][r] + b.m[M][r];
}

__device__ __forceinline__ float partner(float v) { return __shfl_xor(v, 32, 64); }

// split sum (canonical): this lane's 64 channels in order, plus the partner half's sum
__device__ __forceinline__ float tile_split_sum(const Tile& t) {
  float s = 0.0f;
#pragma unroll
  for (int M = 0; M < 4; ++M)
#pragma unroll
    for (int r = 0; r < 16; ++r) s = s + t.m[M][r];
  return s + partner(s);
}

// LayerNorm / MaskedLayerNorm (mask 1) over the 128 channels of each column, in place.
// scale/offset are perm-ordered 128-vectors.
// The elementwise steps run as pinned packed pairs (v_pk_add/mul_f32, as the GELU): d = x - mean
// is formed once and kept in place of x (the normalisation used to recompute it), d·d pairwise;
// only the variance sum stays a scalar chain (its order is canonical). Same operations, same
// bits as the scalar form: x - m == x + (-m) in IEEE arithmetic, products and sums unchanged.
__device__ __forceinline__ f32x2 apk_add(f32x2 a, f32x2 b) {
  f32x2 d;
  asm("v_pk_add_f32 %0, %1, %2" : "=v"(d) : "v"(a), "v"(b));
  return d;
}
__device__ __forceinline__ void tile_layer_norm(Tile& t, const float* __restrict__ scale,
                                                const float* __restrict__ offset) {
  float mean = tile_split_sum(t) / 128.0f;
  const f32x2 nm = {-mean, -mean};
  float s = 0.0f;
#pragma unroll
  for (int M = 0; M < 4; ++M)
#pragma unroll
    for (int r = 0; r < 16; r += 2) {
      const f32x2 d = apk_add((f32x2){t.m[M][r], t.m[M][r + 1]}, nm);
      const f32x2 dd = apk_mul(d, d);
      s = s + dd.x;
      s = s + dd.y;
      t.m[M][r] = d.x;
      t.m[M][r + 1] = d.y;
    }
  float var = (s + partner(s)) / 128.0f;
  float rs = 1.0f / sqrtf(var + 1e-5f);
  const f32x2 rr = {rs, rs};
  const float4* ps = reinterpret_cast<const float4*>(scale + (lane_id() >> 5) * 64);
  const float4* po = reinterpret_cast<const float4*>(offset + (lane_id() >> 5) * 64);
#pragma unroll
  for (int M = 0; M < 4; ++M)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      __builtin_amdgcn_sched_barrier(0);
      float4 sc = ps[M * 4 + q], of = po[M * 4 + q];
      const f32x2 inv0 = apk_mul((f32x2){sc.x, sc.y}, rr), inv1 = apk_mul((f32x2){sc.z, sc.w}, rr);
      const f32x2 y0 = apk_add(apk_mul(inv0, (f32x2){t.m[M][4 * q], t.m[M][4 * q + 1]}), (f32x2){of.x, of.y});
      const f32x2 y1 = apk_add(apk_mul(inv1, (f32x2){t.m[M][4 * q + 2], t.m[M][4 * q + 3]}), (f32x2){of.z, of.w});
      t.m[M][4 * q] = y0.x;
      t.m[M][4 * q + 1] = y0.y;
      t.m[M][4 * q + 2] = y1.x;
      t.m[M][4 * q + 3] = y1.y;
    }
}

}  // namespace pst
