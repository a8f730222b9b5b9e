/* Exhaustive characterisation of GELU forms over all 2^32 float32 inputs (NaN skipped): for each
 * form, 2g = x + x*t (the encoder kernels' doubled GELU) against the true value
 * x + x*tanh(sqrt(2/pi)(x + 0.044715 x^3)) in double, and bit-for-bit against the XLA form
 * (round 1-5 canonical: u in float32, Eigen/XLA's [13/6] rational tanh of u, clamp 7.99881).
 *   X54 — round 6 candidate: t = x P(x^2) / Q(x^2), (5, 4), |x| clamped to 4.9
 *   X64 — (6, 4), |x| clamped to 5.05
 * Reported per form: max / mean error in ulps of the true 2g (x >= 0), max absolute error (x < 0,
 * where x + x*t cancels), inputs whose bits differ from the XLA form.
 *     gcc -O2 -fopenmp -mfma tools/gelu/gelu_rational_check.c -lm && ./a.out      (all 2^32)
 *     -DSTRIDE=101 for a sample                                                       */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#ifndef STRIDE
#define STRIDE 1
#endif

static float t_xla(float x) {
  float a = x * fmaf(x * x, 0.035677406936883926f, 0.797884583473205566f);
  const float clamp = 7.99881172180175781f;
  float c = a > clamp ? clamp : (a < -clamp ? -clamp : a);
  float s = c * c;
  float p = fmaf(s, -2.76076847742355e-16f, 2.00018790482477e-13f);
  p = fmaf(s, p, -8.60467152213735e-11f);
  p = fmaf(s, p, 5.12229709037114e-08f);
  p = fmaf(s, p, 1.48572235717979e-05f);
  p = fmaf(s, p, 6.37261928875436e-04f);
  p = fmaf(s, p, 4.89352455891786e-03f);
  p = c * p;
  float q = fmaf(s, 1.19825839466702e-06f, 1.18534705686654e-04f);
  q = fmaf(s, q, 2.26843463243900e-03f);
  q = fmaf(s, q, 4.89352518554385e-03f);
  return p / q;
}

#include "gelu_rational_coeffs.h"

static float t_x54(float x) {
  float c = x > X54_CLAMP ? X54_CLAMP : (x < -X54_CLAMP ? -X54_CLAMP : x);
  float s = c * c;
  float q = fmaf(s, X54_Q4, X54_Q3);
  q = fmaf(s, q, X54_Q2);
  q = fmaf(s, q, X54_Q1);
  q = fmaf(s, q, 1.0f);
  float p = fmaf(s, X54_P5, X54_P4);
  p = fmaf(s, p, X54_P3);
  p = fmaf(s, p, X54_P2);
  p = fmaf(s, p, X54_P1);
  p = fmaf(s, p, X54_P0);
  p = c * p;
  return p / q;
}

static float t_x64(float x) {
  float c = x > X64_CLAMP ? X64_CLAMP : (x < -X64_CLAMP ? -X64_CLAMP : x);
  float s = c * c;
  float q = fmaf(s, X64_Q4, X64_Q3);
  q = fmaf(s, q, X64_Q2);
  q = fmaf(s, q, X64_Q1);
  q = fmaf(s, q, 1.0f);
  float p = fmaf(s, X64_P6, X64_P5);
  p = fmaf(s, p, X64_P4);
  p = fmaf(s, p, X64_P3);
  p = fmaf(s, p, X64_P2);
  p = fmaf(s, p, X64_P1);
  p = fmaf(s, p, X64_P0);
  p = c * p;
  return p / q;
}

static double ulp_of(double v) {
  float f = (float)fabs(v);
  if (f == 0.0f) return 1.401298464324817e-45;
  return (double)nextafterf(f, INFINITY) - (double)f;
}

typedef float (*tfun)(float);

int main(void) {
  tfun fs[3] = {t_xla, t_x54, t_x64};
  const char* names[3] = {"xla  ", "x54  ", "x64  "};
  for (int k = 0; k < 3; ++k) {
    double max_ulp = 0.0, sum_ulp = 0.0, max_abs_neg = 0.0, max_ulp_x = 0.0;
    long long n_pos = 0, differ = 0, over1 = 0;
#pragma omp parallel for reduction(max : max_ulp, max_abs_neg) reduction(+ : sum_ulp, n_pos, differ, over1) schedule(static, 1 << 20)
    for (long long i = 0; i < (1LL << 32); i += STRIDE) {
      uint32_t b = (uint32_t)i;
      float x;
      memcpy(&x, &b, 4);
      if (isnan(x) || isinf(x)) continue;
      const double xd = x;
      const double tt = tanh(0.7978845608028654 * (xd + 0.044715 * xd * xd * xd));
      const double g_true = xd + xd * tt;
      const float t = fs[k](x);
      const float g = fmaf(x, t, x);
      if (k > 0) {
        const float gx = fmaf(x, t_xla(x), x);
        uint32_t a1, a2;
        memcpy(&a1, &g, 4);
        memcpy(&a2, &gx, 4);
        if (a1 != a2) ++differ;
      }
      if (x >= 0.0f) {
        if (fabs(g_true) < 1e-37 || fabs(g_true) > 3e38) continue;
        const double e = fabs((double)g - g_true) / ulp_of(g_true);
        if (e > max_ulp) max_ulp = e;
        if (e > 1.0) ++over1;
        sum_ulp += e;
        ++n_pos;
      } else {
        const double e = fabs((double)g - g_true);
        if (e > max_abs_neg) max_abs_neg = e;
      }
    }
    printf("%s x>=0: max %.3f ulp, mean %.4f ulp, %lld inputs > 1 ulp (of %lld); x<0: max abs err %.3e; "
           "bits differing from xla: %lld\n",
           names[k], max_ulp, sum_ulp / (double)n_pos, over1, n_pos, max_abs_neg, differ);
    (void)max_ulp_x;
  }
  return 0;
}
