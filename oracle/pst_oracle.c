/*
 * pst_oracle.c — CPU restatement of the reference tokenize path. TEST INFRASTRUCTURE ONLY:
 * used by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg as the checker;
 * the product (libpst.so) never links or calls it.
 *
 * It restates, per protein, in plain C:
 *   - preprocess_sample's graph (structure_tokenizer/data/preprocessing.py:42-283):
 *     backbone filter (protein_structure_sample.py:64-70), frames
 *     (model/quat_affine.py:406-522), centroids / cdist / k-NN / RBF / p,q,k,t features
 *     (utils/protein_utils.py:257-281 RBFs, 325-438 graph) and the padding semantics of
 *     preprocessing.py:191-271 (incl. the < k residue branch), in float64 with the numpy
 *     operation order, rounded once to float32 (JAX's device transfer);
 *   - Vq3D.encode_and_quantize (model/model.py:357-479): positional encodings
 *     (positional_encoding_layer.py:49-150), init embeddings (structure_encoder.py:89-105),
 *     3 x MPNNLayer (gnn_layers.py:325-438, MaskedLayerNorm :79-164), the cross-attention
 *     downsampler (modules.py:199-262, 271-424, 427-636; local mask model.py:264-318),
 *     spherical norm + down_proj (model.py:148-192, 414-420) and FSQ (quantize.py:141-209).
 *
 * Numerics: the "canonical" float32 semantics documented in DESIGN.md §4 — every dot
 * product is an fmaf chain in the pi8 k-order (0,4,1,5,2,6,3,7 inside each block of 8; what
 * the MFMA register chaining of the GPU kernels produces), LayerNorm-style sums use two
 * interleaved partial sums (channels with bit 2 clear / set), segment sums are sequential in
 * slot order, and tanh/exp/sigmoid are fixed IEEE-operation sequences. Compiled with
 * -ffp-contract=off so the compiler never fuses what the spec keeps separate.
 */
#include "pst_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

#define H 128
#define KNN_MAX 64
#define NATOM 37
#define IDX_N 0
#define IDX_CA 1
#define IDX_C 2
#define IDX_O 4

/* ------------------------------------------------------------------ canonical math (f32) */
static float c_tanh(float a) {
  /* rational minimax (odd P(x^2)*x / even Q(x^2)), clamp, |x|<4e-4 -> x */
  const float clamp = 7.99881172180175781f;
  float x = a > clamp ? clamp : (a < -clamp ? -clamp : a);
  float x2 = x * x;
  float p = fmaf(x2, -2.76076847742355e-16f, 2.00018790482477e-13f);
  p = fmaf(x2, p, -8.60467152213735e-11f);
  p = fmaf(x2, p, 5.12229709037114e-08f);
  p = fmaf(x2, p, 1.48572235717979e-05f);
  p = fmaf(x2, p, 6.37261928875436e-04f);
  p = fmaf(x2, p, 4.89352455891786e-03f);
  p = x * p;
  float q = fmaf(x2, 1.19825839466702e-06f, 1.18534705686654e-04f);
  q = fmaf(x2, q, 2.26843463243900e-03f);
  q = fmaf(x2, q, 4.89352518554385e-03f);
  float r = p / q;
  return fabsf(a) < 0.0004f ? a : r;
}

/* tanh's rational core without the |x| < 4e-4 shortcut (used inside GELU) */
static float c_tanh_core(float a) {
  const float clamp = 7.99881172180175781f;
  float x = a > clamp ? clamp : (a < -clamp ? -clamp : a);
  float x2 = x * x;
  float p = fmaf(x2, -2.76076847742355e-16f, 2.00018790482477e-13f);
  p = fmaf(x2, p, -8.60467152213735e-11f);
  p = fmaf(x2, p, 5.12229709037114e-08f);
  p = fmaf(x2, p, 1.48572235717979e-05f);
  p = fmaf(x2, p, 6.37261928875436e-04f);
  p = fmaf(x2, p, 4.89352455891786e-03f);
  p = x * p;
  float q = fmaf(x2, 1.19825839466702e-06f, 1.18534705686654e-04f);
  q = fmaf(x2, q, 2.26843463243900e-03f);
  q = fmaf(x2, q, 4.89352518554385e-03f);
  return p / q;
}

/* GELU (tanh form, jax.nn.gelu approximate=True) in the canonical GPU-friendly sequence:
 * u = x * (k0 + k0k1 x^2), g = h + h * tanh(u), h = x/2. Within 2 ulp of
 * x * 0.5 * (1 + tanh(k0 (x + k1 x^3))). */
static float c_gelu(float x) {
  float u = x * fmaf(x * x, 0.035677406936883926f, 0.797884583473205566f);
  float hx = 0.5f * x;
  return fmaf(hx, c_tanh_core(u), hx);
}

static float c_ldexpf(float v, int n) {
  /* exact scaling by 2^n via exponent bits, two steps to reach the subnormal range */
  union { float f; uint32_t u; } s;
  if (n < -126) {
    s.u = (uint32_t)(-126 + 127) << 23;
    v = v * s.f;
    n += 126;
    if (n < -126) n = -126;
  }
  if (n > 127) n = 127;
  s.u = (uint32_t)(n + 127) << 23;
  return v * s.f;
}

static float c_exp(float x) {
  if (x > 88.7228394f) return INFINITY;
  if (x < -103.972084f) return 0.0f;
  float n = rintf(x * 1.44269502f);
  float r = fmaf(n, -0.693145752f, x);
  r = fmaf(n, -1.42860677e-6f, r);
  float p = 1.98756912e-4f;
  p = fmaf(p, r, 1.39819994e-3f);
  p = fmaf(p, r, 8.33345205e-3f);
  p = fmaf(p, r, 4.16657962e-2f);
  p = fmaf(p, r, 1.66666655e-1f);
  p = fmaf(p, r, 5.00000012e-1f);
  float y = fmaf(p, r * r, r) + 1.0f;
  return c_ldexpf(y, (int)n);
}

static float c_sigmoid(float x) { return 1.0f / (1.0f + c_exp(-x)); }

/* ------------------------------------------------------------------ canonical math (f64) */
static double c_ldexp64(double v, int n) {
  union { double f; uint64_t u; } s;
  if (n < -1022) {
    s.u = (uint64_t)(-1022 + 1023) << 52;
    v = v * s.f;
    n += 1022;
    if (n < -1022) n = -1022;
  }
  if (n > 1023) n = 1023;
  s.u = (uint64_t)(n + 1023) << 52;
  return v * s.f;
}

static double c_exp64(double x) {
  if (x > 709.782712893384) return INFINITY;
  if (x < -745.2) return 0.0;
  double n = rint(x * 1.4426950408889634);
  double r = fma(n, -6.93147180369123816490e-01, x);
  r = fma(n, -1.90821492927058770002e-10, r);
  /* Taylor/Horner to degree 13 on |r| <= 0.347 (error < 1 ulp) */
  double p = 1.0 / 6227020800.0;
  p = fma(p, r, 1.0 / 479001600.0);
  p = fma(p, r, 1.0 / 39916800.0);
  p = fma(p, r, 1.0 / 3628800.0);
  p = fma(p, r, 1.0 / 362880.0);
  p = fma(p, r, 1.0 / 40320.0);
  p = fma(p, r, 1.0 / 5040.0);
  p = fma(p, r, 1.0 / 720.0);
  p = fma(p, r, 1.0 / 120.0);
  p = fma(p, r, 1.0 / 24.0);
  p = fma(p, r, 1.0 / 6.0);
  p = fma(p, r, 0.5);
  double y = fma(p, r * r, r) + 1.0;
  return c_ldexp64(y, (int)n);
}

/* pi8 k-order: t -> k */
static inline int pi8(int t) { return (t & ~7) | ((t >> 1) & 3) | ((t & 1) << 2); }

/* y[o] = chain_{t<K} fmaf(x[pi8(t)], W[pi8(t)*ldw + o], init ? init[o] : 0) (+ b[o]) */
static void gemv(const float* x, int K, const float* W, int ldw, int O, const float* init,
                 const float* b, float* y) {
  float acc[1024];
  for (int o = 0; o < O; ++o) acc[o] = init ? init[o] : 0.0f;
  for (int t = 0; t < K; ++t) {
    int k = pi8(t);
    float xk = x[k];
    const float* w = W + (size_t)k * ldw;
    for (int o = 0; o < O; ++o) acc[o] = fmaf(xk, w[o], acc[o]);
  }
  for (int o = 0; o < O; ++o) y[o] = b ? acc[o] + b[o] : acc[o];
}

/* split sum over 128 channels: bit-2-clear channels ascending + bit-2-set channels ascending */
static float split_sum(const float* v) {
  float s0 = 0.0f, s1 = 0.0f;
  for (int c = 0; c < H; ++c) {
    if (c & 4) s1 = s1 + v[c];
    else s0 = s0 + v[c];
  }
  return s0 + s1;
}

/* LayerNorm / MaskedLayerNorm (mask = 1) over 128 channels */
static void layer_norm(const float* x, const float* scale, const float* offset, float* y) {
  float mean = split_sum(x) / 128.0f;
  float d[H];
  for (int c = 0; c < H; ++c) {
    float t = x[c] - mean;
    d[c] = t * t;
  }
  float var = split_sum(d) / 128.0f;
  float rs = 1.0f / sqrtf(var + 1e-5f);
  for (int c = 0; c < H; ++c) {
    float inv = scale[c] * rs;
    y[c] = inv * (x[c] - mean) + offset[c];
  }
}

/* ------------------------------------------------------------------ parameters */
typedef struct {
  const float *w, *b;
} lin_t;
typedef struct {
  lin_t msg[3], ff[2], edge[3];
  const float *ln_s[3], *ln_o[3];
} mpnn_t;
typedef struct {
  lin_t node_embed, edge_embed;
  mpnn_t L[3];
  const float *qn_s, *qn_o, *dn_s, *dn_o, *qw, *kw, *vw, *gw, *gb, *ow, *ob;
  const float *rt_ln_s, *rt_ln_o, *rt_w1, *rt_b1, *rt_w2, *rt_b2;
  const float *ot_ln_s, *ot_ln_o, *ot_w1, *ot_b1, *ot_w2, *ot_b2;
  lin_t down;
} params_t;

static const float* take(const float** p, size_t n) {
  const float* r = *p;
  *p += n;
  return r;
}

static size_t layout(const float* blob, int D, params_t* P) {
  const float* p = blob;
  P->node_embed.w = take(&p, H * H); P->node_embed.b = take(&p, H);
  P->edge_embed.w = take(&p, (H + 27) * H); P->edge_embed.b = take(&p, H);
  for (int l = 0; l < 3; ++l) {
    mpnn_t* m = &P->L[l];
    m->msg[0].w = take(&p, 3 * H * H); m->msg[0].b = take(&p, H);
    m->msg[1].w = take(&p, H * H); m->msg[1].b = take(&p, H);
    m->msg[2].w = take(&p, H * H); m->msg[2].b = take(&p, H);
    m->ff[0].w = take(&p, H * 4 * H); m->ff[0].b = take(&p, 4 * H);
    m->ff[1].w = take(&p, 4 * H * H); m->ff[1].b = take(&p, H);
    m->edge[0].w = take(&p, 3 * H * H); m->edge[0].b = take(&p, H);
    m->edge[1].w = take(&p, H * H); m->edge[1].b = take(&p, H);
    m->edge[2].w = take(&p, H * H); m->edge[2].b = take(&p, H);
    for (int i = 0; i < 3; ++i) { m->ln_s[i] = take(&p, H); m->ln_o[i] = take(&p, H); }
  }
  P->qn_s = take(&p, 3 * H); P->qn_o = take(&p, 3 * H);
  P->dn_s = take(&p, 3 * H); P->dn_o = take(&p, 3 * H);
  P->qw = take(&p, 3 * H * H); P->kw = take(&p, 3 * H * H); P->vw = take(&p, 3 * H * H);
  P->gw = take(&p, 3 * H * H); P->gb = take(&p, 3 * H);
  P->ow = take(&p, 3 * H * H); P->ob = take(&p, 3 * H);
  P->rt_ln_s = take(&p, 3 * H); P->rt_ln_o = take(&p, 3 * H);
  P->rt_w1 = take(&p, 3 * H * 2 * H); P->rt_b1 = take(&p, 3 * 2 * H);
  P->rt_w2 = take(&p, 3 * 2 * H * H); P->rt_b2 = take(&p, 3 * H);
  P->ot_ln_s = take(&p, 3 * H); P->ot_ln_o = take(&p, 3 * H);
  P->ot_w1 = take(&p, 3 * H * 2 * H); P->ot_b1 = take(&p, 3 * 2 * H);
  P->ot_w2 = take(&p, 3 * 2 * H * H); P->ot_b2 = take(&p, 3 * H);
  P->down.w = take(&p, (size_t)H * D); P->down.b = take(&p, D);
  return (size_t)(p - blob);
}

size_t pst_oracle_param_count(int D) {
  params_t P;
  return layout(NULL, D, &P);
}

/* ------------------------------------------------------------------ positional encodings */
/* positional_encoding_layer.py:49-66: odd k: cos(x*pi / n^(2(k-1)/d)), even k: sin(x*pi /
 * n^(2k/d)); float32 argument (x*f32(pi))/f32(pow), correctly rounded pow/cos/sin. */
static float pe_value(int x, int n, int k1) {
  int num = (k1 & 1) ? 2 * (k1 - 1) : 2 * k1;
  float e = (float)num / 128.0f;
  float pw = (float)pow((double)n, (double)e);
  float arg = ((float)x * 3.14159274101257324f) / pw;
  return (float)((k1 & 1) ? cos((double)arg) : sin((double)arg));
}

void pst_oracle_pe_row(int x, int n, float* out) {
  for (int k = 1; k <= H; ++k) out[k - 1] = pe_value(x, n, k);
}

/* ------------------------------------------------------------------ graph (float64) */
typedef struct {
  double n[3], u[3], v[3]; /* basis rows: M[2], M[0], M[1] */
} frame_t;

static void mat3_mul(const double a[3][3], const double b[3][3], double r[3][3]) {
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) r[i][j] = a[i][0] * b[0][j] + a[i][1] * b[1][j] + a[i][2] * b[2][j];
}

/* quat_affine.py:406-492 make_canonical_transform, then the row split of preprocessing.py:94 */
static void make_frame(const double* N, const double* CA, const double* C, frame_t* f) {
  double nx = N[0] + (-CA[0]), ny = N[1] + (-CA[1]), nz = N[2] + (-CA[2]);
  double cx = C[0] + (-CA[0]), cy = C[1] + (-CA[1]), cz = C[2] + (-CA[2]);
  double s1 = sqrt(1e-20 + cx * cx + cy * cy);
  double sin_c1 = -cy / s1, cos_c1 = cx / s1;
  double c1[3][3] = {{cos_c1, -sin_c1, 0.0}, {sin_c1, cos_c1, 0.0}, {0.0, 0.0, 1.0}};
  double s2 = sqrt(1e-20 + cx * cx + cy * cy + cz * cz);
  double sin_c2 = cz / s2, cos_c2 = sqrt(cx * cx + cy * cy) / s2;
  double c2[3][3] = {{cos_c2, 0.0, sin_c2}, {0.0, 1.0, 0.0}, {-sin_c2, 0.0, cos_c2}};
  double cr[3][3];
  mat3_mul(c2, c1, cr);
  double ry = cr[1][0] * nx + cr[1][1] * ny + cr[1][2] * nz;
  double rz = cr[2][0] * nx + cr[2][1] * ny + cr[2][2] * nz;
  double s3 = sqrt(1e-20 + ry * ry + rz * rz);
  double sin_n = -rz / s3, cos_n = ry / s3;
  double nr[3][3] = {{1.0, 0.0, 0.0}, {0.0, cos_n, -sin_n}, {0.0, sin_n, cos_n}};
  double M[3][3];
  mat3_mul(nr, cr, M);
  for (int k = 0; k < 3; ++k) { f->u[k] = M[0][k]; f->v[k] = M[1][k]; f->n[k] = M[2][k]; }
}

typedef struct {
  double d;
  int i;
} dk_t;

static int cmp_dk(const void* a, const void* b) {
  const dk_t* x = (const dk_t*)a;
  const dk_t* y = (const dk_t*)b;
  if (x->d < y->d) return -1;
  if (x->d > y->d) return 1;
  return (x->i > y->i) - (x->i < y->i);
}

/* numpy's einsum("ijk,nik->inj") / ("ijk,nk->inj") evaluates the 3-term contraction as
 * ((+0 + p0) + p2) + p1 (measured against numpy 2.2 in the build container; tests pin it) */
static double dot3(const double* b, const double* x) { return ((0.0 + b[0] * x[0]) + b[2] * x[2]) + b[1] * x[1]; }

/* 27 edge features of edge (receiver r, sender s), protein_utils.py:257-281 (RBF), 409-434 (p,q,k,t) */
static void edge_features(int r, int s, double dist, const double* ca, const frame_t* fr, float* out) {
  double d2 = dist * dist;
  double ls = 1.0;
  for (int j = 0; j < 15; ++j) {
    out[j] = (float)c_exp64(-d2 / ls);
    ls *= 1.5;
  }
  const frame_t* B = &fr[r];
  const double* rows[3] = {B->n, B->u, B->v};
  double diff[3] = {ca[3 * s] - ca[3 * r], ca[3 * s + 1] - ca[3 * r + 1], ca[3 * s + 2] - ca[3 * r + 2]};
  for (int j = 0; j < 3; ++j) {
    out[15 + j] = (float)dot3(rows[j], diff);
    out[18 + j] = (float)dot3(rows[j], fr[s].n);
    out[21 + j] = (float)dot3(rows[j], fr[s].u);
    out[24 + j] = (float)dot3(rows[j], fr[s].v);
  }
}

int pst_oracle_graph(const double* pos, const uint8_t* flags, int n_raw, int k,
                     int* n_out, int32_t* kept, int32_t* senders, int32_t* deg_out, float* feat) {
  if (k > KNN_MAX || n_raw <= 0) return -1;
  int n = 0;
  for (int i = 0; i < n_raw; ++i) {
    const uint8_t* fl = flags + (size_t)i * NATOM;
    if ((fl[IDX_N] & 1) && (fl[IDX_CA] & 1) && (fl[IDX_C] & 1) && (fl[IDX_O] & 1)) kept[n++] = i;
  }
  *n_out = n;
  if (n == 0) return 0;
  frame_t* fr = (frame_t*)malloc(sizeof(frame_t) * n);
  double* cen = (double*)malloc(sizeof(double) * 3 * n);
  double* ca = (double*)malloc(sizeof(double) * 3 * n);
  for (int i = 0; i < n; ++i) {
    const double* P = pos + (size_t)kept[i] * NATOM * 3;
    const uint8_t* fl = flags + (size_t)kept[i] * NATOM;
    make_frame(P + 3 * IDX_N, P + 3 * IDX_CA, P + 3 * IDX_C, &fr[i]);
    double sx = 0, sy = 0, sz = 0;
    int m = 0;
    for (int a = 0; a < NATOM; ++a)
      if ((fl[a] & 3) == 3) {
        if (m == 0) { sx = P[3 * a]; sy = P[3 * a + 1]; sz = P[3 * a + 2]; }
        else { sx += P[3 * a]; sy += P[3 * a + 1]; sz += P[3 * a + 2]; }
        ++m;
      }
    cen[3 * i] = sx / m; cen[3 * i + 1] = sy / m; cen[3 * i + 2] = sz / m;
    for (int c = 0; c < 3; ++c) ca[3 * i + c] = P[3 * IDX_CA + c];
  }
  /* sorted neighbour lists (distance, then index), self included at rank 0 */
  int keep = n <= k ? n : k + 1;
  int32_t* sorted = (int32_t*)malloc(sizeof(int32_t) * (size_t)n * keep);
  double* sdist = (double*)malloc(sizeof(double) * (size_t)n * keep);
  dk_t* row = (dk_t*)malloc(sizeof(dk_t) * n);
  for (int r = 0; r < n; ++r) {
    for (int s = 0; s < n; ++s) {
      double dx = cen[3 * r] - cen[3 * s], dy = cen[3 * r + 1] - cen[3 * s + 1], dz = cen[3 * r + 2] - cen[3 * s + 2];
      row[s].d = sqrt(dx * dx + dy * dy + dz * dz);
      row[s].i = s;
    }
    qsort(row, n, sizeof(dk_t), cmp_dk); /* ties: lower index first */
    for (int t = 0; t < keep; ++t) {
      sorted[(size_t)r * keep + t] = row[t].i;
      sdist[(size_t)r * keep + t] = row[t].d;
    }
  }
  free(row);
  int deg = n <= k ? n : k;
  int off = n <= k ? 0 : 1;
  for (int r = 0; r < n; ++r) {
    deg_out[r] = deg;
    for (int j = 0; j < k; ++j) {
      size_t slot = (size_t)r * k + j;
      float* out = feat + slot * 32;
      memset(out, 0, 32 * sizeof(float));
      if (n < k) { /* preprocessing.py:229-260: slots keep the n*n enumeration's features */
        senders[slot] = j < deg ? sorted[(size_t)r * keep + j] : -1;
        if (slot < (size_t)n * n) {
          int rr = (int)(slot / n), cc = (int)(slot % n);
          edge_features(rr, sorted[(size_t)rr * keep + cc], sdist[(size_t)rr * keep + cc], ca, fr, out);
        }
        continue;
      }
      senders[slot] = sorted[(size_t)r * keep + j + off];
      {
        edge_features(r, senders[slot], sdist[(size_t)r * keep + j + off], ca, fr, out);
      }
    }
  }
  free(fr); free(cen); free(ca); free(sorted); free(sdist);
  return 0;
}

/* ------------------------------------------------------------------ encoder */
typedef struct {
  int n, k, df, D;
  const int32_t* senders; /* [n*k] local, -1 = unused slot */
  const int32_t* deg;
  const float* feat;      /* [n*k*32] */
} graph_t;

/* Every Linear's fma chain starts from its bias ("bias-first"); the first layer of an edge
 * MLP starts from Ps[s] + Pr[r], where Pr's own chain started from that layer's bias. */
/* The message MLP up to its last (linear) layer: g = GELU(b1 + GELU(t1)·W1); the last layer
 * runs once per receiver on the ordered sum of the g rows (msg_agg), since
 * sum_j (g_j·W2 + b2) = (sum_j g_j)·W2 + deg·b2. */
static void msg_hidden(float* t1, const lin_t* L, float* g) {
  for (int c = 0; c < H; ++c) t1[c] = c_gelu(t1[c]);
  gemv(t1, H, L[1].w, H, H, L[1].b, NULL, g);
  for (int c = 0; c < H; ++c) g[c] = c_gelu(g[c]);
}

static void msg_agg(const float* G, int deg, const lin_t* L, float* agg) {
  float init[H];
  for (int c = 0; c < H; ++c) init[c] = (float)deg * L[2].b[c];
  gemv(G, H, L[2].w, H, H, init, NULL, agg);
}

static void mlp3_tail(float* t1, const lin_t* L, float* y) {
  float t2[H];
  for (int c = 0; c < H; ++c) t1[c] = c_gelu(t1[c]);
  gemv(t1, H, L[1].w, H, H, L[1].b, NULL, t2);
  for (int c = 0; c < H; ++c) t2[c] = c_gelu(t2[c]);
  gemv(t2, H, L[2].w, H, H, L[2].b, NULL, y);
}

static void mlp3(const float* Ps, const float* Pr, const float* e, const lin_t* L, float* y) {
  float init[H], t1[H];
  for (int c = 0; c < H; ++c) init[c] = Ps[c] + Pr[c];
  gemv(e, H, L[0].w + 2 * H * H, H, H, init, NULL, t1);
  mlp3_tail(t1, L, y);
}

/* Layer 0's message MLP through the factors of the edge embedding: with
 * e0 = T[s-r] + f·Wf, the first layer's e-part is U[s-r] + f·Wm, U = T·Wc, Wm = Wf·Wc (Wc = the
 * first layer's rows 256..383), each an fmaf chain in the canonical order; the chain starts from
 * (Ps[s] + Pr[r]) + U[s-r] and runs over the 32 (27 + zero pad) features. */
static void msg_hidden_l0(const float* Ps, const float* Pr, const float* U, const float* f32, const float* Wm,
                          const lin_t* L, float* g) {
  float init[H], t1[H];
  for (int c = 0; c < H; ++c) init[c] = (Ps[c] + Pr[c]) + U[c];
  gemv(f32, 32, Wm, H, H, init, NULL, t1);
  msg_hidden(t1, L, g);
}

static void msg_hidden_e(const float* Ps, const float* Pr, const float* e, const lin_t* L, float* g) {
  float init[H], t1[H];
  for (int c = 0; c < H; ++c) init[c] = Ps[c] + Pr[c];
  gemv(e, H, L[0].w + 2 * H * H, H, H, init, NULL, t1);
  msg_hidden(t1, L, g);
}

/* node projections of an MLP's first layer: Ps = h W[0:128] (from 0), Pr = b + h W[128:256] */
static void proj2(const float* h, const lin_t* L0, float* Ps, float* Pr) {
  gemv(h, H, L0->w, H, H, NULL, NULL, Ps);
  gemv(h, H, L0->w + H * H, H, H, L0->b, NULL, Pr);
}

int pst_oracle_encode(const float* blob, int D, const int32_t* levels, int df, int n, int k,
                      const int32_t* senders, const int32_t* deg, const float* feat,
                      float* h_layers /*[4][n][128] or NULL*/, float* pre_proj /*[T][128]*/,
                      float* z_out /*[T][D]*/, float* b_out /*[T][D]*/, float* q_out /*[T][D]*/,
                      uint32_t* tokens /*[T]*/) {
  params_t P;
  layout(blob, D, &P);
  size_t nk = (size_t)n * k;
  float* h = (float*)malloc(sizeof(float) * n * H);
  float* hn = (float*)malloc(sizeof(float) * n * H);
  float* e = (float*)malloc(sizeof(float) * nk * H);
  float* en = (float*)malloc(sizeof(float) * nk * H);
  float* Ps = (float*)malloc(sizeof(float) * n * H);
  float* Pr = (float*)malloc(sizeof(float) * n * H);
  float* Es = (float*)malloc(sizeof(float) * n * H);
  float* Er = (float*)malloc(sizeof(float) * n * H);
  float pe[H];
  /* init node embedding h0[i] = Linear(nodePE(i)) (structure_encoder.py:89-92) */
  for (int i = 0; i < n; ++i) {
    pst_oracle_pe_row(i, 512, pe);
    gemv(pe, H, P.node_embed.w, H, H, NULL, P.node_embed.b, h + (size_t)i * H);
  }
  if (h_layers) memcpy(h_layers, h, sizeof(float) * n * H);
  /* init edge embedding: T[x] = edgePE(x) W[0:128] (x = s - r), then the chain continues
   * over the 27 features (weights rows 128..154, zero-padded to 32) from T, + bias */
  float* Ttab = (float*)malloc(sizeof(float) * 1023 * H);
  for (int x = -511; x <= 511; ++x) {
    pst_oracle_pe_row(x, 512, pe);
    gemv(pe, H, P.edge_embed.w, H, H, P.edge_embed.b, NULL, Ttab + (size_t)(x + 511) * H);
  }
  float* Wf = (float*)calloc(32 * H, sizeof(float));
  memcpy(Wf, P.edge_embed.w + H * H, sizeof(float) * 27 * H);
  for (int r = 0; r < n; ++r)
    for (int j = 0; j < k; ++j) {
      size_t slot = (size_t)r * k + j;
      int s = senders[slot] < 0 ? r : senders[slot];
      float f32[32];
      memcpy(f32, feat + slot * 32, sizeof(f32));
      for (int c = 27; c < 32; ++c) f32[c] = 0.0f;
      gemv(f32, 32, Wf, H, H, Ttab + (size_t)(s - r + 511) * H, NULL, e + slot * H);
    }
  /* layer-0 message factors: U[x] = T[x]·Wc, Wm[f] = Wf[f]·Wc (rows 27..31 stay zero) */
  const float* Wc = P.L[0].msg[0].w + 2 * H * H;
  float* Utab = (float*)malloc(sizeof(float) * 1023 * H);
  for (int x = 0; x < 1023; ++x) gemv(Ttab + (size_t)x * H, H, Wc, H, H, NULL, NULL, Utab + (size_t)x * H);
  float* Wm = (float*)calloc(32 * H, sizeof(float));
  for (int f = 0; f < 27; ++f) gemv(Wf + (size_t)f * H, H, Wc, H, H, NULL, NULL, Wm + (size_t)f * H);
  free(Ttab);
  free(Wf);
  for (int l = 0; l < 3; ++l) {
    const mpnn_t* M = &P.L[l];
    if (l > 0) { /* edge update of layer l-1 with the node features it produced */
      const mpnn_t* Mp = &P.L[l - 1];
      for (int i = 0; i < n; ++i) proj2(h + (size_t)i * H, &Mp->edge[0], Es + (size_t)i * H, Er + (size_t)i * H);
      for (int r = 0; r < n; ++r)
        for (int j = 0; j < k; ++j) {
          size_t slot = (size_t)r * k + j;
          int s = senders[slot] < 0 ? r : senders[slot];
          float m[H], x[H];
          mlp3(Es + (size_t)s * H, Er + (size_t)r * H, e + slot * H, Mp->edge, m);
          for (int c = 0; c < H; ++c) x[c] = e[slot * H + c] + m[c];
          layer_norm(x, Mp->ln_s[2], Mp->ln_o[2], en + slot * H);
        }
      float* t = e; e = en; en = t;
    }
    for (int i = 0; i < n; ++i) proj2(h + (size_t)i * H, &M->msg[0], Ps + (size_t)i * H, Pr + (size_t)i * H);
    for (int r = 0; r < n; ++r) {
      float gsum[H], agg[H], m[H], x[H], h1[H], f1[4 * H], f2[H];
      for (int c = 0; c < H; ++c) gsum[c] = 0.0f;
      for (int j = 0; j < deg[r]; ++j) {
        size_t slot = (size_t)r * k + j;
        int s = senders[slot];
        if (l == 0) {
          float f32[32];
          memcpy(f32, feat + slot * 32, sizeof(f32));
          for (int c = 27; c < 32; ++c) f32[c] = 0.0f;
          msg_hidden_l0(Ps + (size_t)s * H, Pr + (size_t)r * H, Utab + (size_t)(s - r + 511) * H, f32, Wm, M->msg, m);
        } else {
          msg_hidden_e(Ps + (size_t)s * H, Pr + (size_t)r * H, e + slot * H, M->msg, m);
        }
        for (int c = 0; c < H; ++c) gsum[c] = gsum[c] + m[c];
      }
      msg_agg(gsum, deg[r], M->msg, agg);
      for (int c = 0; c < H; ++c) x[c] = h[(size_t)r * H + c] + agg[c] / 50.0f;
      layer_norm(x, M->ln_s[0], M->ln_o[0], h1);
      gemv(h1, H, M->ff[0].w, 4 * H, 4 * H, M->ff[0].b, NULL, f1);
      for (int c = 0; c < 4 * H; ++c) f1[c] = c_gelu(f1[c]);
      gemv(f1, 4 * H, M->ff[1].w, H, H, M->ff[1].b, NULL, f2);
      for (int c = 0; c < H; ++c) x[c] = h1[c] + f2[c];
      layer_norm(x, M->ln_s[1], M->ln_o[1], hn + (size_t)r * H);
    }
    float* t = h; h = hn; hn = t;
    if (h_layers) memcpy(h_layers + (size_t)(l + 1) * n * H, h, sizeof(float) * n * H);
  }
  /* ---------------- cross-attention downsampler (df local window), spherical norm, FSQ */
  int T = n / df;
  int max_out = 512 / df;
  float* o = h; /* original track [n][128] */
  float* ot = hn;
  for (int t = 0; t < T; ++t) {
    float r[H];
    pst_oracle_pe_row(t, max_out, r);
    for (int blk = 0; blk < 3; ++blk) {
      const float* qw = P.qw + (size_t)blk * H * H;
      const float* kw = P.kw + (size_t)blk * H * H;
      const float* vw = P.vw + (size_t)blk * H * H;
      const float* gw = P.gw + (size_t)blk * H * H;
      const float* ow = P.ow + (size_t)blk * H * H;
      float qn[H], q[H], g[H], wa[H], out[H], logit[4][4], v[4][H];
      layer_norm(r, P.qn_s + blk * H, P.qn_o + blk * H, qn);
      gemv(qn, H, qw, H, H, NULL, NULL, q);
      for (int c = 0; c < H; ++c) q[c] = q[c] * 0.176776692f;
      gemv(qn, H, gw, H, H, NULL, P.gb + blk * H, g);
      for (int c = 0; c < H; ++c) g[c] = c_sigmoid(g[c]);
      for (int p = 0; p < df; ++p) {
        int node = t * df + p;
        float dn[H], kk[H];
        layer_norm(o + (size_t)node * H, P.dn_s + blk * H, P.dn_o + blk * H, dn);
        gemv(dn, H, kw, H, H, NULL, NULL, kk);
        gemv(dn, H, vw, H, H, NULL, NULL, v[p]);
        for (int hd = 0; hd < 4; ++hd) {
          float acc = 0.0f;
          for (int tt = 0; tt < 32; ++tt) {
            int c = pi8(tt);
            acc = fmaf(q[hd * 32 + c], kk[hd * 32 + c], acc);
          }
          logit[hd][p] = acc;
        }
      }
      for (int hd = 0; hd < 4; ++hd) {
        float mx = logit[hd][0];
        for (int p = 1; p < df; ++p) mx = logit[hd][p] > mx ? logit[hd][p] : mx;
        float ex[4], sum = 0.0f;
        for (int p = 0; p < df; ++p) { ex[p] = c_exp(logit[hd][p] - mx); sum = sum + ex[p]; }
        for (int c = 0; c < 32; ++c) {
          float acc = 0.0f;
          for (int p = 0; p < df; ++p) acc = fmaf(ex[p] / sum, v[p][hd * 32 + c], acc);
          wa[hd * 32 + c] = acc * g[hd * 32 + c];
        }
      }
      gemv(wa, H, ow, H, H, NULL, P.ob + blk * H, out);
      for (int c = 0; c < H; ++c) r[c] = r[c] + out[c];
      /* resampled transition */
      float tn[H], t1[2 * H], t2[H];
      layer_norm(r, P.rt_ln_s + blk * H, P.rt_ln_o + blk * H, tn);
      gemv(tn, H, P.rt_w1 + (size_t)blk * H * 2 * H, 2 * H, 2 * H, NULL, P.rt_b1 + blk * 2 * H, t1);
      for (int c = 0; c < 2 * H; ++c) t1[c] = t1[c] > 0.0f ? t1[c] : 0.0f;
      gemv(t1, 2 * H, P.rt_w2 + (size_t)blk * 2 * H * H, H, H, NULL, P.rt_b2 + blk * H, t2);
      for (int c = 0; c < H; ++c) r[c] = r[c] + t2[c];
      /* original transition of this token's window (blocks 1,2 only feed later blocks) */
      if (blk < 2)
        for (int p = 0; p < df; ++p) {
          int node = t * df + p;
          const float* x = o + (size_t)node * H;
          layer_norm(x, P.ot_ln_s + blk * H, P.ot_ln_o + blk * H, tn);
          gemv(tn, H, P.ot_w1 + (size_t)blk * H * 2 * H, 2 * H, 2 * H, NULL, P.ot_b1 + blk * 2 * H, t1);
          for (int c = 0; c < 2 * H; ++c) t1[c] = t1[c] > 0.0f ? t1[c] : 0.0f;
          gemv(t1, 2 * H, P.ot_w2 + (size_t)blk * 2 * H * H, H, H, NULL, P.ot_b2 + blk * H, t2);
          for (int c = 0; c < H; ++c) ot[(size_t)node * H + c] = x[c] + t2[c];
        }
      if (blk < 2)
        for (int p = 0; p < df; ++p) memcpy(o + (size_t)(t * df + p) * H, ot + (size_t)(t * df + p) * H, sizeof(float) * H);
    }
    /* spherical norm (model.py:169-174) and down_proj */
    float sq[H], xs[H], z[8];
    for (int c = 0; c < H; ++c) sq[c] = r[c] * r[c];
    float nrm = sqrtf(split_sum(sq)) + 1e-6f;
    for (int c = 0; c < H; ++c) xs[c] = r[c] / nrm;
    if (pre_proj) memcpy(pre_proj + (size_t)t * H, xs, sizeof(xs));
    gemv(xs, H, P.down.w, D, D, NULL, P.down.b, z);
    /* FSQ (quantize.py:175-209) */
    uint32_t idx = 0, basis = 1;
    for (int d = 0; d < D; ++d) {
      int L = levels[d];
      float half_l = ((float)(L - 1) * 0.999f) / 2.0f;
      float offset = (L % 2 == 0) ? 0.5f : 0.0f;
      float shift = (float)tan((double)(offset / half_l));
      float b = c_tanh(z[d] + shift) * half_l - offset;
      float qv = rintf(b);
      if (z_out) z_out[(size_t)t * D + d] = z[d];
      if (b_out) b_out[(size_t)t * D + d] = b;
      if (q_out) q_out[(size_t)t * D + d] = qv;
      idx += (uint32_t)((int)qv + L / 2) * basis;
      basis *= (uint32_t)L;
    }
    tokens[t] = idx;
  }
  free(h); free(hn); free(e); free(en); free(Ps); free(Pr); free(Es); free(Er); free(Utab); free(Wm);
  return T;
}

int pst_oracle_tokenize(const float* blob, int D, const int32_t* levels, int df, int k,
                        const double* pos, const uint8_t* flags, int n_raw, uint32_t* tokens,
                        float* b_out, float* pre_proj, int* n_nodes) {
  int32_t* kept = (int32_t*)malloc(sizeof(int32_t) * n_raw);
  int32_t* senders = (int32_t*)malloc(sizeof(int32_t) * (size_t)n_raw * k);
  int32_t* deg = (int32_t*)malloc(sizeof(int32_t) * n_raw);
  float* feat = (float*)malloc(sizeof(float) * (size_t)n_raw * k * 32);
  int n = 0;
  int rc = pst_oracle_graph(pos, flags, n_raw, k, &n, kept, senders, deg, feat);
  if (rc == 0 && n > 0)
    rc = pst_oracle_encode(blob, D, levels, df, n, k, senders, deg, feat, NULL, pre_proj, NULL, b_out, NULL, tokens);
  else if (rc == 0)
    rc = 0;
  if (n_nodes) *n_nodes = n;
  free(kept); free(senders); free(deg); free(feat);
  return rc;
}

/* Ragged batch, proteins in parallel (OpenMP): the CPU-baseline entry. */
int pst_oracle_tokenize_batch(const float* blob, int D, const int32_t* levels, int df, int k,
                              const double* pos, const uint8_t* flags, const int64_t* offsets,
                              int n_prot, uint32_t* tokens, int32_t* n_tokens, int n_threads) {
  int err = 0;
#pragma omp parallel for schedule(dynamic, 1) num_threads(n_threads) reduction(| : err)
  for (int b = 0; b < n_prot; ++b) {
    int64_t o = offsets[b];
    int nn = 0;
    int T = pst_oracle_tokenize(blob, D, levels, df, k, pos + o * NATOM * 3, flags + o * NATOM,
                                (int)(offsets[b + 1] - o), tokens + o, NULL, NULL, &nn);
    if (T < 0) err |= 1;
    n_tokens[b] = T < 0 ? 0 : T;
  }
  return err ? -1 : 0;
}

/* exported canonical math, so tests can pin it (accuracy vs float64 libm) */
float pst_oracle_tanh(float x) { return c_tanh(x); }
float pst_oracle_gelu(float x) { return c_gelu(x); }
float pst_oracle_exp(float x) { return c_exp(x); }
float pst_oracle_sigmoid(float x) { return c_sigmoid(x); }
double pst_oracle_exp64(double x) { return c_exp64(x); }

/* ------------------------------------------------------------------ FSQ aux (quantize.py:205-239)
 * Mirrors libpst's k_fsq_aux operation for operation: per row, dims split into a low group
 * (0..2) and a high group (3..D-1); group tables A/B = sequential sums of (b_d - c)^2; EA/EB =
 * exp(table - max); group sums in the GPU's order (64 lane partials, each sequential over
 * i = lane, lane+64, ... from +0, then a xor butterfly 32..1); distance = A + B,
 * soft_proba = (EA*EB) * (1/(S_A*S_B)); argmin = per-dimension nearest level (lowest on ties). */
static float group_tables(const float* bv, const int32_t* L, int d0, int d1, float* S, float* E) {
  int n = 1;
  for (int d = d0; d < d1; ++d) n *= L[d];
  float mx = -INFINITY;
  for (int i = 0; i < n; ++i) {
    int rem = i;
    float s = 0.0f;
    for (int d = d0; d < d1; ++d) {
      int digit = rem % L[d];
      rem /= L[d];
      float diff = bv[d] - (float)(digit - L[d] / 2);
      float sq = diff * diff;
      s = d == d0 ? sq : s + sq;
    }
    S[i] = s;
    if (s > mx) mx = s;
  }
  float part[64];
  for (int l = 0; l < 64; ++l) part[l] = 0.0f;
  for (int i = 0; i < n; ++i) {
    E[i] = c_exp(S[i] - mx);
    part[i & 63] = part[i & 63] + E[i];
  }
  for (int m = 32; m >= 1; m >>= 1) {
    float nx[64];
    for (int l = 0; l < 64; ++l) nx[l] = part[l] + part[l ^ m];
    memcpy(part, nx, sizeof(part));
  }
  return part[0];
}

int pst_oracle_fsq_aux(const int32_t* levels, int D, const float* bounded, int64_t T, float* dist,
                       float* prob, uint32_t* argmin) {
  if (D < 4 || D > 8) return -1;
  int K_lo = levels[0] * levels[1] * levels[2], K_hi = 1;
  for (int d = 3; d < D; ++d) K_hi *= levels[d];
  int64_t K = (int64_t)K_lo * K_hi;
  float* A = (float*)malloc(sizeof(float) * K_lo * 2);
  float* B = (float*)malloc(sizeof(float) * K_hi * 2);
  for (int64_t r = 0; r < T; ++r) {
    const float* bv = bounded + r * D;
    float sa = group_tables(bv, levels, 0, 3, A, A + K_lo);
    float sb = group_tables(bv, levels, 3, D, B, B + K_hi);
    float inv_s = 1.0f / (sa * sb);
    for (int64_t k = 0; k < K; ++k) {
      int khi = (int)(k / K_lo), klo = (int)(k % K_lo);
      if (dist) dist[r * K + k] = A[klo] + B[khi];
      if (prob) prob[r * K + k] = (A[K_lo + klo] * B[K_hi + khi]) * inv_s;
    }
    if (argmin) {
      uint32_t k = 0, basis = 1;
      for (int d = 0; d < D; ++d) {
        int best = 0;
        float bd = INFINITY;
        for (int g = 0; g < levels[d]; ++g) {
          float diff = bv[d] - (float)(g - levels[d] / 2);
          float sq = diff * diff;
          if (sq < bd) { bd = sq; best = g; }
        }
        k += (uint32_t)best * basis;
        basis *= (uint32_t)levels[d];
      }
      argmin[r] = k;
    }
  }
  free(A);
  free(B);
  return 0;
}
