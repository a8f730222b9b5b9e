// pst_kernels.hip — HIP kernels of the tokenize path for gfx950 (MI355X).
//
// Pipeline per batch (one stream, 6 launches, all data resident in HBM):
//   k_prep       block/protein: backbone filter + compaction, frames, centroids, CA
//                (preprocessing.py:69-149, quat_affine.py:406-522)
//   k_knn        wave/receiver: float64 cdist row, ordered k-NN selection, 27 edge features
//                (protein_utils.py:325-438; padding semantics preprocessing.py:191-271)
//   k_mpnn<0..2> wave/32 receivers (1600 edge slots = 50 MFMA blocks of 32 edges): fused
//                edge update of layer l-1 + message MLP of layer l + ordered segment sum +
//                node update (masked LN, 128->512->128 FFN, masked LN) + the next layer's node
//                projections (gnn_layers.py:325-438). Edge features never leave registers
//                between Linear layers; e is stored once per layer in a coalesced blocked
//                layout.
//   k_down<DF>   wave/32 tokens: cross-attention downsampler (3 blocks), spherical norm,
//                down_proj and FSQ (modules.py:427-636, model.py:169-174, quantize.py:175-209)
// See pst_device.h for the wave-tile layout and DESIGN.md for the numerics contract.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pst_device.h"
#include <algorithm>
#include <utility>

#include "pst_kernels.h"

namespace pst {

#ifndef MPNN_MIN_BLOCKS
#define MPNN_MIN_BLOCKS 2
#endif
#define NATOM 37
#define KNN 50

// ---------------------------------------------------------------------------- k_prep
struct Frame {
  double u[3], v[3], n[3];
};

__device__ __forceinline__ void make_frame(const double* N, const double* CA, const double* C, double* out) {
  double nx = N[0] + (-CA[0]), ny = N[1] + (-CA[1]), nz = N[2] + (-CA[2]);
  double cx = C[0] + (-CA[0]), cy = C[1] + (-CA[1]), cz = C[2] + (-CA[2]);
  double s1 = sqrt(1e-20 + cx * cx + cy * cy);
  double sin_c1 = -cy / s1, cos_c1 = cx / s1;
  double c1[3][3] = {{cos_c1, -sin_c1, 0.0}, {sin_c1, cos_c1, 0.0}, {0.0, 0.0, 1.0}};
  double s2 = sqrt(1e-20 + cx * cx + cy * cy + cz * cz);
  double sin_c2 = cz / s2, cos_c2 = sqrt(cx * cx + cy * cy) / s2;
  double c2[3][3] = {{cos_c2, 0.0, sin_c2}, {0.0, 1.0, 0.0}, {-sin_c2, 0.0, cos_c2}};
  double cr[3][3];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) cr[i][j] = c2[i][0] * c1[0][j] + c2[i][1] * c1[1][j] + c2[i][2] * c1[2][j];
  double ry = cr[1][0] * nx + cr[1][1] * ny + cr[1][2] * nz;
  double rz = cr[2][0] * nx + cr[2][1] * ny + cr[2][2] * nz;
  double s3 = sqrt(1e-20 + ry * ry + rz * rz);
  double sin_n = -rz / s3, cos_n = ry / s3;
  double nr[3][3] = {{1.0, 0.0, 0.0}, {0.0, cos_n, -sin_n}, {0.0, sin_n, cos_n}};
  double M[3][3];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) M[i][j] = nr[i][0] * cr[0][j] + nr[i][1] * cr[1][j] + nr[i][2] * cr[2][j];
  // stored rows: [n | u | v] = [M2 | M0 | M1]  (basis_matrices order, protein_utils.py:406-408)
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    out[k] = M[2][k];
    out[3 + k] = M[0][k];
    out[6 + k] = M[1][k];
  }
}

// F32: float32 positions (pst_tokenize_f32) — a template parameter, so the coordinate loads carry
// no per-element branch between the two input formats
template <bool F32>
__global__ __launch_bounds__(512) void k_prep(PrepArgs a) {
  __shared__ int wave_cnt[8];
  const int b = a.prot0 + (int)blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int64_t off = a.offsets[b];
  const int Rb = (int)(a.offsets[b + 1] - off);
  bool keep = false;
  if (tid < Rb) {
    const uint8_t* fl = a.flags + (off + tid) * NATOM;
    keep = (fl[0] & 1) && (fl[1] & 1) && (fl[2] & 1) && (fl[4] & 1);  // N, CA, C, O gt_exists
  }
  unsigned long long m = __ballot(keep);
  if (lane == 0) wave_cnt[w] = __popcll(m);
  __syncthreads();
  int base = 0, total = 0;
  for (int i = 0; i < 8; ++i) {
    if (i < w) base += wave_cnt[i];
    total += wave_cnt[i];
  }
  const int loc = base + __popcll(m & ((1ull << lane) - 1ull));
  if (tid == 0) a.n_nodes[b] = total;
  if (keep) {
    const int64_t slot = off + loc;
    // positions widened to f64 on load: float32 inputs (pst_tokenize_f32) give the same doubles the
    // f64 path reads for float32-exact coordinates, so everything below is bitwise unchanged
    const int64_t p0 = (off + tid) * NATOM * 3;
    auto P = [&](int i) -> double { return F32 ? (double)a.pos32[p0 + i] : a.pos[p0 + i]; };
    const uint8_t* fl = a.flags + (off + tid) * NATOM;
    double bb[9];
#pragma unroll
    for (int i = 0; i < 9; ++i) bb[i] = P(i);
    make_frame(bb + 0, bb + 3, bb + 6, a.frame + slot * 9);
    // centroid over the atoms with gt_exists & atom_exists (preprocessing.py:72), summed in atom
    // order. The 37 flags are loaded together, then the present atoms' coordinates 8 atoms at a
    // time (exec-masked loads issued back to back, one wait per group): loading each atom's flag
    // and then its coordinates made ~37 dependent memory round trips per residue.
    uint8_t f[NATOM];
#pragma unroll
    for (int at = 0; at < NATOM; ++at) f[at] = fl[at];
    double sx = 0.0, sy = 0.0, sz = 0.0;
    int cnt = 0;
    constexpr int CH = 8;
#pragma unroll
    for (int a0 = 0; a0 < NATOM; a0 += CH) {
      double xs[CH][3];
#pragma unroll
      for (int k = 0; k < CH; ++k)
        if (a0 + k < NATOM && (f[a0 + k] & 3) == 3)
#pragma unroll
          for (int c = 0; c < 3; ++c) xs[k][c] = P(3 * (a0 + k) + c);
#pragma unroll
      for (int k = 0; k < CH; ++k)
        if (a0 + k < NATOM && (f[a0 + k] & 3) == 3) {
          if (cnt == 0) { sx = xs[k][0]; sy = xs[k][1]; sz = xs[k][2]; }
          else { sx += xs[k][0]; sy += xs[k][1]; sz += xs[k][2]; }
          ++cnt;
        }
    }
    a.cen[slot * 3 + 0] = sx / cnt;
    a.cen[slot * 3 + 1] = sy / cnt;
    a.cen[slot * 3 + 2] = sz / cnt;
    a.ca[slot * 3 + 0] = bb[3];
    a.ca[slot * 3 + 1] = bb[4];
    a.ca[slot * 3 + 2] = bb[5];
    a.node_local[slot] = loc;
    a.node_prot[slot] = b;
  }
  if (tid >= total && tid < Rb) {  // gap slots left by filtered residues
    a.node_local[off + tid] = -1;
    a.node_prot[off + tid] = b;
  }
}

// ---------------------------------------------------------------------------- k_knn
__device__ __forceinline__ double dot3(const double* b, const double* x) {
  // numpy einsum's evaluation order for the 3-term contraction (protein_utils.py:411-423)
  return ((0.0 + b[0] * x[0]) + b[2] * x[2]) + b[1] * x[1];
}

__device__ void edge_features(const double* fr_r, const double* fr_s, const double* ca_r,
                              const double* ca_s, double dist, float4* __restrict__ o) {
  float f[FEAT_USED];
  double d2 = dist * dist;
  double ls = 1.0;
#pragma unroll
  for (int j = 0; j < 15; ++j) {
    f[j] = (float)c_exp64(-d2 / ls);
    ls *= 1.5;
  }
  double diff[3] = {ca_s[0] - ca_r[0], ca_s[1] - ca_r[1], ca_s[2] - ca_r[2]};
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const double* row = fr_r + 3 * j;  // rows n, u, v of the receiver basis
    f[15 + j] = (float)dot3(row, diff);
    f[18 + j] = (float)dot3(row, fr_s + 0);
    f[21 + j] = (float)dot3(row, fr_s + 3);
    f[24 + j] = (float)dot3(row, fr_s + 6);
  }
  // stored in the feature GEMMs' slot order (feat_slot), padding slots +0 (picked per slot at
  // compile time: a second 32-float array here cost k_knn 24 VGPRs and three waves per SIMD)
  auto v = [&](int sl) { return slot_feat(sl) < 0 ? 0.0f : f[slot_feat(sl)]; };
#pragma unroll
  for (int q = 0; q < 8; ++q) o[feat_f4_q(q)] = make_float4(v(4 * q), v(4 * q + 1), v(4 * q + 2), v(4 * q + 3));
}

__device__ __forceinline__ bool lex_less(double d1, int s1, double d2, int s2) {
  return d1 < d2 || (d1 == d2 && s1 < s2);
}

__device__ __forceinline__ double cen_dist(const double* cen, int64_t r, int64_t s) {
  double dx = cen[r * 3] - cen[s * 3], dy = cen[r * 3 + 1] - cen[s * 3 + 1], dz = cen[r * 3 + 2] - cen[s * 3 + 2];
  return sqrt(dx * dx + dy * dy + dz * dz);
}

// rank-cc neighbour (self included) of local receiver rr, by counting (n < k branch only)
__device__ int rank_select(const double* cen, int64_t base, int n, int rr, int cc, double* dsel) {
  for (int s = 0; s < n; ++s) {
    double ds = cen_dist(cen, base + rr, base + s);
    int rank = 0;
    for (int q = 0; q < n; ++q) {
      double dq = cen_dist(cen, base + rr, base + q);
      rank += lex_less(dq, q, ds, s);
    }
    if (rank == cc) { *dsel = ds; return s; }
  }
  *dsel = 0.0;
  return rr;
}


// LDS of k_knn's radix select, one slice per wave
__shared__ unsigned knn_hist[4][256];
__shared__ double knn_sd[4][64];
__shared__ int knn_ss[4][64];

__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__global__ __launch_bounds__(256) void k_knn(KnnArgs a) {
  const int lane = threadIdx.x & 63;
  const int64_t g = a.slot0 + (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (g >= a.n_slots) return;
  const int loc = a.node_local[g];
  int32_t* snd = a.senders + g * KNN;
  // this lane's edge E = g * KNN + lane in the blocked layout: float4 q at o[feat_f4_q(q)]
  const int64_t E = g * KNN + lane;
  float4* o = reinterpret_cast<float4*>(a.feat) + feat_f4(E, 0);
  if (loc < 0) {  // gap / padding slot: self edges, zero features, degree 0
    if (lane < KNN) {
      snd[lane] = (int32_t)g;
      for (int q = 0; q < 8; ++q) o[feat_f4_q(q)] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    if (lane == 0) a.deg[g] = 0;
    return;
  }
  const int b = a.node_prot[g];
  const int64_t base = a.offsets[b];
  const int n = a.n_nodes[b];
  // candidate distances (float64, scipy cdist order), 8 per lane
  double d[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    int s = lane + 64 * i;
    d[i] = s < n ? cen_dist(a.cen, g, base + s) : __builtin_inf();
  }
  const int keep = n <= KNN ? n : KNN + 1;
  const int drop = n <= KNN ? 0 : 1;  // column 0 (self) dropped when n > k (protein_utils.py:385-389)
  int my_s = -1;
  double my_d = 0.0;
  {
    // Radix select of the keep smallest (distance, index) pairs: 8 passes of an 8-bit histogram
    // over the distance bits (non-negative doubles order like their bit patterns) find the exact
    // keep-th distance T; ties at T are taken in index order; the selected pairs are ranked by
    // counting (keep <= 51 entries) — the same order as the lexicographic argsort.
    const int w = threadIdx.x >> 6;
    unsigned* hist = knn_hist[w];
    unsigned long long key[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) key[i] = (unsigned long long)__double_as_longlong(d[i]);
    unsigned long long prefix = 0, mask = 0, lt_bound = 0;
    int rem = keep;
    for (int shift = 56; shift >= 0; shift -= 8) {
#pragma unroll
      for (int q = 0; q < 4; ++q) hist[lane * 4 + q] = 0u;
      wave_lds_sync();
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int si = lane + 64 * i;
        if (si < n && (key[i] & mask) == prefix) atomicAdd(&hist[(unsigned)(key[i] >> shift) & 255u], 1u);
      }
      wave_lds_sync();
      unsigned c[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) c[q] = hist[lane * 4 + q];
      const unsigned tot = c[0] + c[1] + c[2] + c[3];
      unsigned incl = tot;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const unsigned v = __shfl_up(incl, o, 64);
        if (lane >= o) incl += v;
      }
      unsigned run = incl - tot;  // buckets before this lane's four
      int found = -1;
      unsigned below = 0;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (found < 0 && run < (unsigned)rem && (unsigned)rem <= run + c[q]) {
          found = lane * 4 + q;
          below = run;
        }
        run += c[q];
      }
      const unsigned long long hit = __ballot(found >= 0);
      const int wl = __builtin_ctzll(hit);
      const unsigned cnt = (unsigned)__builtin_amdgcn_readlane((int)hist[found < 0 ? 0 : found], wl);
      found = __builtin_amdgcn_readlane(found, wl);
      below = (unsigned)__builtin_amdgcn_readlane((int)below, wl);
      prefix |= (unsigned long long)found << shift;
      mask |= 0xFFull << shift;
      rem -= (int)below;
      wave_lds_sync();  // the next pass rewrites the histogram
      if (cnt == (unsigned)rem) {
        // the crossing bucket is taken whole: every key up to the bucket's top is selected
        lt_bound = (prefix | ((1ull << shift) - 1ull)) + 1ull;
        rem = 0;
        break;
      }
    }
    if (rem) lt_bound = prefix;
    // take every key < lt_bound and, after a full 8-pass descent, the first `rem` keys == prefix
    // (the exact keep-th distance) in index order
    double* sd = knn_sd[w];
    int* ss = knn_ss[w];
    int pos = 0, eq_left = rem;
    const unsigned long long lt_lane = (1ull << lane) - 1ull;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int si = lane + 64 * i;
      const bool valid = si < n;
      const bool lt = valid && key[i] < lt_bound;
      const bool eq = valid && key[i] == prefix;
      const unsigned long long eqm = __ballot(eq);
      const int eq_rank = __popcll(eqm & lt_lane);
      const bool take_eq = eq && eq_rank < eq_left;
      const bool take = lt || take_eq;
      const unsigned long long tm = __ballot(take);
      if (take) {
        const int p = pos + __popcll(tm & lt_lane);
        sd[p] = d[i];
        ss[p] = si;
      }
      pos += __popcll(tm);
      eq_left -= min(eq_left, __popcll(eqm));
    }
    wave_lds_sync();
    double vd = 0.0;
    int vs = 0, rank = 0;
    if (lane < keep) {
      vd = sd[lane];
      vs = ss[lane];
      for (int m = 0; m < keep; ++m) rank += lex_less(sd[m], ss[m], vd, vs);
    }
    wave_lds_sync();
    if (lane < keep) {
      sd[rank] = vd;
      ss[rank] = vs;
    }
    wave_lds_sync();
    if (lane + drop < keep) {
      my_s = ss[lane + drop];
      my_d = sd[lane + drop];
    }
  }
  const int deg = n <= KNN ? n : KNN;
  if (lane == 0) a.deg[g] = deg;
  if (lane < KNN) {
    if (n >= KNN) {
      snd[lane] = (int32_t)(base + my_s);
      edge_features(a.frame + g * 9, a.frame + (base + my_s) * 9, a.ca + g * 3, a.ca + (base + my_s) * 3, my_d,
                    o);
    } else {
      // n < k (preprocessing.py:229-260): senders stay per-row, features keep the n*n order
      snd[lane] = lane < n ? (int32_t)(base + my_s) : (int32_t)g;
      int64_t f = (int64_t)loc * KNN + lane;
      if (f < (int64_t)n * n) {
        int rr = (int)(f / n), cc = (int)(f % n);
        double ds;
        int s = rank_select(a.cen, base, n, rr, cc, &ds);
        edge_features(a.frame + (base + rr) * 9, a.frame + (base + s) * 9, a.ca + (base + rr) * 3,
                      a.ca + (base + s) * 3, ds, o);
      } else {
        for (int q = 0; q < 8; ++q) o[feat_f4_q(q)] = make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
  }
}

// ---------------------------------------------------------------------------- k_mpnn
// perm position of channel c (inverse of tile_channel)
__device__ __forceinline__ int perm_pos(int c) {
  int h = (c >> 2) & 1, M = c >> 5, cc = c & 31;
  int r = (cc & 3) + 4 * (cc >> 3);
  return h * 64 + M * 16 + r;
}

// 1.0f if bit `ee` of the wave-uniform mask is set, else 0.0f, made on the scalar unit (an SGPR
// operand of the consuming FMA; a C select would be materialised per lane)
template <int EE>
__device__ __forceinline__ float umask(uint32_t bits) {
  float r;
  asm volatile("s_bitcmp1_b32 %1, %2\n\ts_cselect_b32 %0, 1.0, 0" : "=s"(r) : "s"(bits), "I"(EE) : "scc");
  return r;
}
// the two chains over the 32 edges of a block (v: this lane's channel row, edges in order)
#ifndef SEG_PACKED
#define SEG_PACKED 1
#endif
#if SEG_PACKED
// Both chains in ONE packed FMA per edge (round 6): (accA, accB) = (v_e, v_e)·(mA_e, mB_e) +
// (accA, accB), v_e broadcast from its register pair by op_sel, the mask pair from SGPRs — per
// half exactly the fmaf of the scalar form, so the same bits at half the VALU issue
template <int EE>
__device__ __forceinline__ void seg_step(f32x2& acc, f32x2 vp, uint32_t mA, uint32_t mB) {
  const f32x2 m = {umask<EE>(mA), umask<EE>(mB)};
  if (EE & 1)
    asm volatile("v_pk_fma_f32 %0, %1, %2, %0 op_sel:[1,0,0] op_sel_hi:[1,1,1]" : "+v"(acc) : "v"(vp), "s"(m));
  else
    asm volatile("v_pk_fma_f32 %0, %1, %2, %0 op_sel:[0,0,0] op_sel_hi:[0,1,1]" : "+v"(acc) : "v"(vp), "s"(m));
}
template <int... EE>
__device__ __forceinline__ void seg_chains(const float (&v)[32], uint32_t mA, uint32_t mB, float& accA, float& accB,
                                           std::integer_sequence<int, EE...>) {
  f32x2 acc = {accA, accB};
  (seg_step<EE>(acc, (f32x2){v[EE & ~1], v[EE | 1]}, mA, mB), ...);
  accA = acc.x;
  accB = acc.y;
}
#else
template <int... EE>
__device__ __forceinline__ void seg_chains(const float (&v)[32], uint32_t mA, uint32_t mB, float& accA, float& accB,
                                           std::integer_sequence<int, EE...>) {
  ((accA = __builtin_fmaf(v[EE], umask<EE>(mA), accA), accB = __builtin_fmaf(v[EE], umask<EE>(mB), accB)), ...);
}
#endif

// acc = a_row + b_row (perm rows); b is streamed 4 values at a time so the sum needs one tile
// of registers, not two
__device__ __forceinline__ void tile_add_rows(Tile& acc, const float* __restrict__ a_row, const float* __restrict__ b_row) {
  tile_load_perm(acc, a_row);
  const float4* p = reinterpret_cast<const float4*>(b_row + (lane_id() >> 5) * 64);
#pragma unroll
  for (int M = 0; M < 4; ++M)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float4 v = p[M * 4 + q];
      acc.m[M][4 * q + 0] = acc.m[M][4 * q + 0] + v.x;
      acc.m[M][4 * q + 1] = acc.m[M][4 * q + 1] + v.y;
      acc.m[M][4 * q + 2] = acc.m[M][4 * q + 2] + v.z;
      acc.m[M][4 * q + 3] = acc.m[M][4 * q + 3] + v.w;
    }
}

// acc += row (perm order), elementwise
__device__ __forceinline__ void tile_add_row(Tile& acc, const float* __restrict__ row) {
  const float4* p = reinterpret_cast<const float4*>(row + (lane_id() >> 5) * 64);
#pragma unroll
  for (int M = 0; M < 4; ++M)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float4 v = p[M * 4 + q];
      acc.m[M][4 * q + 0] = acc.m[M][4 * q + 0] + v.x;
      acc.m[M][4 * q + 1] = acc.m[M][4 * q + 1] + v.y;
      acc.m[M][4 * q + 2] = acc.m[M][4 * q + 2] + v.z;
      acc.m[M][4 * q + 3] = acc.m[M][4 * q + 3] + v.w;
    }
}

// 3-layer edge MLP starting from acc = init (Ps[s] + Pr[r], Pr's chain started from b0):
// acc <- MLP(init, X). Layers 2 and 3 chain from their biases; the GELU of layers 1 and 2 is
// applied just in time inside the next GEMM.
__device__ __forceinline__ void mlp3_tail(Tile& acc, const MlpW& W) {
  Tile a2;
  tile_gemm_bf(a2, acc, W.w1, W.bf1, ActGelu2x{});
  tile_gemm_bf(acc, a2, W.w2, W.bf2, ActGelu2x{});
}
__device__ __forceinline__ void mlp3(Tile& acc, const Tile& X, const MlpW& W) {
  tile_gemm(acc, X, W.w0);
  mlp3_tail(acc, W);
}

// The message MLP up to its last (linear) layer: acc <- GELU(b1 + GELU(acc)·W1). The last layer
// commutes with the segment sum, sum_j (g_j·W2 + b2) = (sum_j g_j)·W2 + deg·b2, so it runs once
// per receiver (agg_from_gsum) instead of once per edge.
// k-steps of the message MLP's W1 the fused kernels hold in LDS (fragments of k-steps 0 .. KL-1,
// 1 KB each, read by the workgroup's four waves instead of streamed from L2 every block): layer 0
// 40 (W1 is most of its weight stream), layers 1-2 32; 2 workgroups per CU still fit (36 KB of
// segment-sum scratch + 32 / 40 KB). Measured at 1 024 x 256 residues (profiles/r02_ab_w1_lds.txt):
// k_mpnn<0> 8.50-8.56 (none) -> 8.36-8.40 (32) -> 8.24-8.29 ms (40); layers 1-2 unchanged.
#ifndef W1_LDS_KSTEPS
#define W1_LDS_KSTEPS 32
#endif
#ifndef W1_LDS_KSTEPS_L0
#define W1_LDS_KSTEPS_L0 40
#endif
template <int LAYER>
constexpr int w1_lds_ksteps() { return LAYER == 0 ? W1_LDS_KSTEPS_L0 : W1_LDS_KSTEPS; }

template <int KL = 0>
__device__ __forceinline__ void msg_hidden(Tile& acc, const MlpW& W, const float4* w1_lds = nullptr) {
  Tile a2;
  if (KL > 0 && w1_lds)
    tile_gemm_mix_bf<(KL > 0 ? KL : 1)>(a2, acc, w1_lds, W.w1, W.bf1, ActGelu2x{});
  else
    tile_gemm_bf(a2, acc, W.w1, W.bf1, ActGelu2x{});
  __builtin_amdgcn_sched_barrier(0);
  // 20 wait states: the packed GELU's asm reads the accumulators the last MFMAs just wrote,
  // and only the compiler's hazard recognizer would otherwise space them
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3");
#pragma unroll
  for (int M = 0; M < 4; ++M)
#pragma unroll
    for (int r = 0; r < 16; r += 2) {
      const f32x2 v = c_gelu2x_asm<false>((f32x2){a2.m[M][r], a2.m[M][r + 1]});
      acc.m[M][r] = v.x;
      acc.m[M][r + 1] = v.y;
    }
}

// agg = deg·b2 + G·W2 for the 32 receivers of the tile (G = ordered sums of the hidden rows,
// perm rows at gsum; lane&31 = receiver with `deg` messages)
__device__ __forceinline__ void agg_from_gsum(Tile& ag, const float* __restrict__ gsum, int deg, const MlpW& W) {
  Tile G;
  tile_load_perm(G, gsum);
  const float* b2 = W.b2 + (lane_id() >> 5) * 64;
  const float fd = (float)deg;
#pragma unroll
  for (int M = 0; M < 4; ++M)
#pragma unroll
    for (int r = 0; r < 16; ++r) ag.m[M][r] = fd * b2[M * 16 + r];
  tile_gemm(ag, G, W.w2);
}

// acc += x[slots] · Wf over the 27 edge features in 32 slots (feat_slot, pst_kernels.h);
// x[r] holds slots (r&3) + 8(r>>2) + 4·half (the k order of the fragments)
// (fragments through a buffer resource with constant SGPR offsets and a FEAT_DEPTH-deep register
// ring, as tile_gemm_f: no per-k-step 64-bit addresses; k_mpnn<0> 8.60 -> 8.45 ms)
// k-steps 14 and 15 hold only zero padding (slots 26, 27, 30, 31; feat_slot packs the 27 features
// into k-steps 0..13), so they are skipped: their MFMAs would add +-0 products to the chains (no
// change to a nonzero sum). Round 2 skipped k-step 15 (8.36 -> 8.29 ms); round 5 moved features
// 25 and 26 into slots 28 and 25 (same chain order) so k-step 14 goes too.
#ifndef FEAT_DEPTH
#define FEAT_DEPTH 4
#endif
#ifndef FEAT_KSTEPS
#define FEAT_KSTEPS 14
#endif
// ST: also write tile E out blocked through `st`, quad r at k-step r (the rest after the loop),
// spread as in tile_gemm_store
template <bool ST>
__device__ __forceinline__ void feat_gemm_st(Tile& acc, const float (&x)[16], const float4* __restrict__ Wf,
                                             const Tile* E, __amdgpu_buffer_rsrc_t st) {
  __amdgpu_buffer_rsrc_t rs = make_rsrc(Wf);
  const int vo = lane_id() * 16;
  float4 ring[FEAT_DEPTH];
#pragma unroll
  for (int i = 0; i < FEAT_DEPTH; ++i) ring[i] = buf_load4(rs, vo, i * 1024);
#pragma unroll
  for (int r = 0; r < FEAT_KSTEPS; ++r) {
    if (ST)
      buf_store4(st, vo, r * 1024, E->m[r / 4][4 * (r % 4)], E->m[r / 4][4 * (r % 4) + 1], E->m[r / 4][4 * (r % 4) + 2],
                 E->m[r / 4][4 * (r % 4) + 3]);
    const float4 wa = ring[r % FEAT_DEPTH];
    if (r + FEAT_DEPTH < FEAT_KSTEPS) ring[r % FEAT_DEPTH] = buf_load4(rs, vo, (r + FEAT_DEPTH) * 1024);
    acc.m[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(wa.x, x[r], acc.m[0], 0, 0, 0);
    acc.m[1] = __builtin_amdgcn_mfma_f32_32x32x2f32(wa.y, x[r], acc.m[1], 0, 0, 0);
    acc.m[2] = __builtin_amdgcn_mfma_f32_32x32x2f32(wa.z, x[r], acc.m[2], 0, 0, 0);
    acc.m[3] = __builtin_amdgcn_mfma_f32_32x32x2f32(wa.w, x[r], acc.m[3], 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
  }
  if (ST)
#pragma unroll
    for (int r = FEAT_KSTEPS; r < 16; ++r)
      buf_store4(st, vo, r * 1024, E->m[r / 4][4 * (r % 4)], E->m[r / 4][4 * (r % 4) + 1], E->m[r / 4][4 * (r % 4) + 2],
                 E->m[r / 4][4 * (r % 4) + 3]);
}
__device__ __forceinline__ void feat_gemm(Tile& acc, const float (&x)[16], const float4* __restrict__ Wf) {
  feat_gemm_st<false>(acc, x, Wf, nullptr, make_rsrc(Wf));
}

// One 32-edge block `blk` of task `task` (receivers g0 .. g0+31): for LAYER >= 1 the edge
// update of layer LAYER-1, e = LN(e + MLP([h_s | h_r | e])), stored back blocked; for LAYER 0
// the edge embedding. Then the message MLP of layer LAYER -> m.
// Sender of this lane's edge in 32-edge block `blk` of the task starting at receiver g0. The
// callers load it one block ahead: the sender index heads a chain of dependent loads (index →
// projection rows), so fetching it during the previous block's GEMMs takes one memory latency
// off every block.
__device__ __forceinline__ int32_t edge_sender(const MpnnArgs& a, int64_t g0, int lane, int blk) {
  return a.senders[g0 * KNN + 32 * blk + (lane & 31)];
}

#ifndef L0_PAIR_TABLE
#define L0_PAIR_TABLE 1
#endif
#ifndef E_STORE_SPREAD
#define E_STORE_SPREAD 1
#endif
// Layer 0: this lane's edge features of block `blk` (edges g0·50 + 32·blk + e: a task's edges are
// consecutive), x[r] = slots (r&3) + 8(r>>2) + 4·half as feat_gemm reads them: float4 2i + half of
// its edge, which the blocked layout (feat_f4) holds at lane-linear position i·64 + lane
__device__ __forceinline__ void edge_feat(const MpnnArgs& a, int64_t g0, int lane, int blk, float (&x)[16]) {
  const float4* fp = reinterpret_cast<const float4*>(a.feat) + ((g0 / 32) * KNN + blk) * 256 + lane;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float4 v = fp[64 * i];
    x[4 * i] = v.x; x[4 * i + 1] = v.y; x[4 * i + 2] = v.z; x[4 * i + 3] = v.w;
  }
}

template <int LAYER, int KL = w1_lds_ksteps<LAYER>()>
__device__ __forceinline__ void edge_block(const MpnnArgs& a, int64_t task, int64_t g0, int lane, int blk,
                                           int32_t s_pre, Tile& m, const float4* w1_lds = nullptr) {
  const int te = 32 * blk + (lane & 31);
  const int rl = te / 50;
  const int64_t g = g0 + rl;
  const int64_t s = s_pre;
  const int64_t eblk = (task * 50 + blk) * 4096;
  Tile e;
  float x[16];  // layer 0: this lane's edge features
  int lr0 = 0, ls0 = 0;
  if (LAYER == 0) {
    // init_edge_embed: chain from T[s-r] (= b + edgePE(s-r) W[0:128]) over the 27 features.
    // A protein's nodes sit in consecutive slots (slot = protein base + local index, k_prep), so
    // ls - lr = s - g without reading node_local[s]; gap/padding receivers have self edges
    // (s = g) and lr clamped to 0, hence ls = 0 as before. The T row then needs no load at all.
    const int d = (int)(s - g);
    int lr = a.node_local[g];
    lr = lr < 0 ? 0 : lr;
    lr0 = lr;
    ls0 = lr + d;
    tile_load_perm(e, a.Ttab + (int64_t)(d + 511) * 128);
    edge_feat(a, g0, lane, blk, x);
    feat_gemm(e, x, a.W_embed);
  } else {
    // edge update of layer LAYER-1: e = LN(e + MLP([h_s | h_r | e]))
    Tile ein;
    tile_load_blk(ein, a.e_in + eblk);
    Tile acc;
    tile_add_rows(acc, a.P_in + s * 512 + 0, a.P_in + g * 512 + 128);
    mlp3(acc, ein, a.edge);
    tile_load_blk(e, a.e_in + eblk);
    tile_add(e, acc);
    tile_layer_norm(e, a.edge_ln_s, a.edge_ln_o);
  }
  if (a.e_out && !E_STORE_SPREAD) tile_store_blk(e, a.e_out + eblk);
  // message MLP of layer LAYER
  if (LAYER == 0) {
    // first layer through the embedding's factors: e0·W = T[s-r]·W + f·(Wf·W),
    // so the chain starts from (h_s·W_s + (b + h_r·W_r)) + U[s-r] and runs over the 32
    // features: 16 k-steps instead of 64
    if (L0_PAIR_TABLE) {  // the same sums, precomputed per (lr, ls): one gathered row, no adds
      tile_load_perm(m, a.V0 + ((int64_t)lr0 * 512 + ls0) * 128);
    } else {
      tile_add_rows(m, a.PM0 + (int64_t)ls0 * 256 + 0, a.PM0 + (int64_t)lr0 * 256 + 128);
      tile_add_row(m, a.Utab + (int64_t)(ls0 - lr0 + 511) * 128);
    }
    if (E_STORE_SPREAD)  // e leaves during this GEMM, after the gathers above (tile_gemm_store)
      feat_gemm_st<true>(m, x, a.W_msg0f, &e, make_rsrc_or_null(a.e_out ? a.e_out + eblk : nullptr));
    else
      feat_gemm(m, x, a.W_msg0f);
    msg_hidden<KL>(m, a.msg, w1_lds);
  } else {
    tile_add_rows(m, a.P_in + s * 512 + 256, a.P_in + g * 512 + 384);
    if (E_STORE_SPREAD)  // e leaves during the GEMM that reads it (tile_gemm_store)
      tile_gemm_store(m, e, a.msg.w0, make_rsrc_or_null(a.e_out ? a.e_out + eblk : nullptr));
    else
      tile_gemm(m, e, a.msg.w0);
    msg_hidden<KL>(m, a.msg, w1_lds);
  }
}

// Node update of the 32 receivers g0 .. g0+31 (lane&31 = receiver): x = h + agg/50, where
// aggl holds the 32 ordered segment sums (perm rows); h = LN(x); h = LN(h + FFN(h)); then the
// next layer's 4 node projections.
template <int LAYER>
__device__ __forceinline__ void node_update(const MpnnArgs& a, int lane, int64_t g0, const float* aggl) {
  const int64_t gl = g0 + (lane & 31);
  Tile x;
  {
    Tile ag;
    agg_from_gsum(ag, aggl + (lane & 31) * 128, a.deg[gl], a.msg);
    if (LAYER == 0) {
      int lr = a.node_local[gl];
      tile_load_perm(x, a.h0tab + (int64_t)(lr < 0 ? 0 : lr) * 128);
    } else {
      tile_load_perm(x, a.h_in + gl * 128);
    }
#pragma unroll
    for (int M = 0; M < 4; ++M)
#pragma unroll
      for (int r = 0; r < 16; ++r) x.m[M][r] = x.m[M][r] + ag.m[M][r] / 50.0f;
  }
  tile_layer_norm(x, a.ln0_s, a.ln0_o);  // V_i_0
  Tile out;
  for (int ck = 0; ck < 4; ++ck) {
    Tile hid;
    tile_gemm_bf(hid, x, a.ff_w1 + ck * 64 * 64, a.ff_bf1 + ck * 64, ActId{});
    if (ck == 0)
      tile_gemm_bf(out, hid, a.ff_w2, a.ff_bf2, ActGelu2x{});
    else
      tile_gemm_f(out, hid, a.ff_w2 + ck * 64 * 64, ActGelu2x{});
  }
  tile_add(x, out);
  tile_layer_norm(x, a.ln1_s, a.ln1_o);  // V_i_1
  tile_store_perm(x, a.h_out + gl * 128);
  if (a.P_out) {
#pragma unroll 1
    for (int p = 0; p < 4; ++p) {
      Tile pr;
      if (p & 1) {  // receiver parts chain from the layer's first-layer bias
        tile_gemm_bf(pr, x, a.proj_w + p * 64 * 64, a.proj_bf[p >> 1], ActId{});
      } else {
        tile_zero(pr);
        tile_gemm(pr, x, a.proj_w + p * 64 * 64);
      }
      tile_store_perm(pr, a.P_out + gl * 512 + p * 128);
    }
  }
}


// Wave priority from the edge blocks a wave still has to run (s_setprio 3 / 2 / 1 / 0 while at
// least 10 / 5 / 2 / 0 blocks of a 25-block half remain, `scale` x that for 50-block tasks). A
// SIMD's two waves otherwise issue oldest-first: the older ran ahead and the younger finished the
// launch alone at the one-wave rate. With the wave that has more left winning issue, the two end
// together (same instructions, same bits; round 5, profiles/r05_ab_wave_priority.txt).
__device__ __forceinline__ void tail_prio(int rem, int scale) {
  if (rem >= 10 * scale) __builtin_amdgcn_s_setprio(3);
  else if (rem >= 5 * scale) __builtin_amdgcn_s_setprio(2);
  else if (rem >= 2 * scale) __builtin_amdgcn_s_setprio(1);
  else __builtin_amdgcn_s_setprio(0);
}

// The edge phase of one fused-layer task (receivers task*32 .. task*32+31), edge blocks blk_lo ..
// blk_hi-1 in order: edge update / embedding, message MLP, and the ordered segment sums of the
// receivers these blocks complete, stored to agg (perm rows). lds_scratch[w]: this wave's LDS tile.
template <int LAYER, int KL, int NW>
__device__ __forceinline__ void mpnn_edge_blocks(const MpnnArgs& a, int64_t task, int lane, int blk_lo, int blk_hi,
                                                 const float4* w1_lds, float (&lds_scratch)[NW][64 * 36], int w) {
  const int64_t g0 = task * 32;
  float* scratch = lds_scratch[w];
  float* aggl = a.agg + task * 32 * 128;
  float carry[2] = {0.f, 0.f};  // running sums of the receiver continuing into the next block

  int32_t s_next = edge_sender(a, g0, lane, blk_lo);
  for (int blk = blk_lo; blk < blk_hi; ++blk) {
    const int32_t s_cur = s_next;
    tail_prio(blk_hi - blk, 1);
    if (blk < blk_hi - 1) s_next = edge_sender(a, g0, lane, blk + 1);
    Tile m;
    edge_block<LAYER, KL>(a, task, g0, lane, blk, s_cur, m, w1_lds);
    // ordered segment sum over the 50 slots of each receiver (jax.ops.segment_sum order). The
    // block holds edges of two receivers: rA (block edges 0..lastA) and rA+1 (the rest).
    // Transpose through LDS two accumulator blocks at a time, so that lane l owns channel
    // 64·p + l of pass p and runs both receivers' sequential chains over the block's edges
    // itself. The chain bounds are wave-uniform (no divergence, no data-dependent loops): edge
    // ee enters chain A iff ee <= hiA and chain B iff loB <= ee <= hiB, as fmaf(v, 1, acc)
    // (= acc + v, one rounding) or fmaf(v, 0, acc) (= acc exactly: a chain never holds -0, and
    // messages are finite GELU outputs).
    const int rA = (32 * blk) / 50;                    // wave-uniform
    const int lastA = 50 * (rA + 1) - 1 - 32 * blk;    // block-local index of rA's last edge
    const int j0 = 32 * blk - 50 * rA;                 // slot of the block's edge 0 within rA
    const int degA = a.deg[g0 + rA];
    const int degB = rA + 1 < 32 ? a.deg[g0 + rA + 1] : 0;
    const int hiA = min(min(lastA, 31), degA - 1 - j0);  // chain A sums edges [0, hiA]
    const int loB = lastA + 1;                           // chain B sums edges [loB, hiB]
    const int hiB = min(31, lastA + degB);
    // wave-uniform edge masks of the two chains (bit ee set = edge ee enters the chain)
    const uint32_t mA = (uint32_t)__builtin_amdgcn_readfirstlane(
        hiA < 0 ? 0u : (hiA >= 31 ? 0xffffffffu : (1u << (hiA + 1)) - 1u));
    const uint32_t mB = (uint32_t)__builtin_amdgcn_readfirstlane(
        loB > hiB ? 0u : ((hiB >= 31 ? 0xffffffffu : (1u << (hiB + 1)) - 1u) & ~((1u << loB) - 1u)));
#pragma unroll
    for (int p = 0; p < 2; ++p) {
#pragma unroll
      for (int Mh = 0; Mh < 2; ++Mh)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int lc = 32 * Mh + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
          scratch[lc * 36 + (lane & 31)] = m.m[2 * p + Mh][r];
        }
      __builtin_amdgcn_wave_barrier();
      const float4* srow = reinterpret_cast<const float4*>(scratch + lane * 36);
      float v[32];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const float4 t = srow[q];
        v[4 * q] = t.x; v[4 * q + 1] = t.y; v[4 * q + 2] = t.z; v[4 * q + 3] = t.w;
      }
      float accA = carry[p], accB = 0.0f;
      seg_chains(v, mA, mB, accA, accB, std::make_integer_sequence<int, 32>{});
      __builtin_amdgcn_wave_barrier();
      if (lastA <= 31) {
        aggl[rA * 128 + perm_pos(64 * p + lane)] = accA;
        carry[p] = lastA < 31 ? accB : 0.0f;
      } else {
        carry[p] = accA;
      }
    }
  }
}

// The node phase of one fused-layer task (lane&31 = receiver of g0 .. g0+31), the sums at aggl: the
// body node_update had, forced inline into the kernels (calling node_update from k_mpnn made the
// compiler spill 45 VGPRs in k_mpnn<1,2>).
template <int LAYER>
__device__ __forceinline__ void mpnn_node_tile(const MpnnArgs& a, int64_t g0, int lane, const float* aggl) {
  const int64_t gl = g0 + (lane & 31);
  Tile x;
  {
    Tile ag;
    agg_from_gsum(ag, aggl + (lane & 31) * 128, a.deg[gl], a.msg);
    if (LAYER == 0) {
      int lr = a.node_local[gl];
      tile_load_perm(x, a.h0tab + (int64_t)(lr < 0 ? 0 : lr) * 128);
    } else {
      tile_load_perm(x, a.h_in + gl * 128);
    }
#pragma unroll
    for (int M = 0; M < 4; ++M)
#pragma unroll
      for (int r = 0; r < 16; ++r) x.m[M][r] = x.m[M][r] + ag.m[M][r] / 50.0f;
  }
  tile_layer_norm(x, a.ln0_s, a.ln0_o);  // V_i_0
  Tile out;
  for (int ck = 0; ck < 4; ++ck) {
    Tile hid;
    tile_gemm_bf(hid, x, a.ff_w1 + ck * 64 * 64, a.ff_bf1 + ck * 64, ActId{});
    if (ck == 0)
      tile_gemm_bf(out, hid, a.ff_w2, a.ff_bf2, ActGelu2x{});
    else
      tile_gemm_f(out, hid, a.ff_w2 + ck * 64 * 64, ActGelu2x{});
  }
  tile_add(x, out);
  tile_layer_norm(x, a.ln1_s, a.ln1_o);  // V_i_1
  tile_store_perm(x, a.h_out + gl * 128);
  if (a.P_out) {
#pragma unroll 1
    for (int p = 0; p < 4; ++p) {
      Tile pr;
      if (p & 1) {  // receiver parts chain from the layer's first-layer bias
        tile_gemm_bf(pr, x, a.proj_w + p * 64 * 64, a.proj_bf[p >> 1], ActId{});
      } else {
        tile_zero(pr);
        tile_gemm(pr, x, a.proj_w + p * 64 * 64);
      }
      tile_store_perm(pr, a.P_out + gl * 512 + p * 128);
    }
  }
}

// Clock stamps of a fused MPNN launch (measurement, MpnnArgs::clk, 8 u64 per layer): the first
// wave of workgroup 0 adds its s_memtime (shader clock) and s_memrealtime (100 MHz) deltas to
// clk[0..1] — clock = d(memtime) / d(memrealtime) x 100 MHz, over the launch for the persistent
// k_mpnn_q whose waves live as long as it does; every wave adds its lifetime (100 MHz ticks) to
// clk[2], lowers clk[3] to its start, raises clk[4] to its end and counts itself in clk[5], so
// the launch's wave-slot occupancy is clk[2] / (slots x (clk[4] - clk[3])). One lane, vector
// atomics, twice per wave.
struct ClockStamp {
  uint64_t t0 = 0, r0 = 0;
  __device__ __forceinline__ void start(unsigned long long* clk) {
    if (clk) {
      t0 = __builtin_amdgcn_s_memtime();
      r0 = __builtin_amdgcn_s_memrealtime();
    }
  }
  __device__ __forceinline__ void stop(unsigned long long* clk) {
    if (clk) {
      const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
      if ((threadIdx.x & 63) == 0) {
        if (blockIdx.x == 0 && threadIdx.x == 0) {
          atomicAdd(clk, (unsigned long long)(t1 - t0));
          atomicAdd(clk + 1, (unsigned long long)(r1 - r0));
        }
        atomicAdd(clk + 2, (unsigned long long)(r1 - r0));
        atomicMin(clk + 3, (unsigned long long)r0);
        atomicMax(clk + 4, (unsigned long long)r1);
        atomicAdd(clk + 5, 1ull);
      }
    }
  }
};

// Fused layer (large batches): one wave per task runs its 50 edge blocks in order, carrying the
// ordered segment sums in registers/LDS, then the node update. No per-edge message traffic.
// HALF (batches of at most one round of tasks): two waves per task, wave 2t+h running edge
// blocks 25h .. 25h+24 — exactly receivers 16h .. 16h+15 (800 = 16 x 50 edges), so each half's
// segment sums are complete on their own; the wave that finishes its half second runs the
// task's node update alone (an LDS counter per task; the first leaves). The same operations in
// the same order: identical bits. Every SIMD then holds two waves where a one-wave-per-task round
// would hold one.
template <int LAYER, bool HALF>
__global__ __launch_bounds__(256, MPNN_MIN_BLOCKS) void k_mpnn(MpnnArgs a) {
  __shared__ float lds_scratch[4][64 * 36];
  ClockStamp cs;
  cs.start(a.clk);
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform (no waterfalls)
  const int64_t task = HALF ? (int64_t)blockIdx.x * 2 + (w >> 1) : (int64_t)blockIdx.x * 4 + w;
  const int hh = w & 1;  // HALF: which half of the task's edge blocks
  // the first KL k-steps of the message MLP's W1 fragments (msg_hidden), read by every block of
  // the workgroup's four waves from LDS instead of L2; filled before any wave may leave
  constexpr int KL = w1_lds_ksteps<LAYER>();
  __shared__ float4 w1_lds_buf[(KL > 0 ? KL : 1) * 64];
  const float4* w1_lds = KL > 0 ? w1_lds_buf : nullptr;
  __shared__ int s_done[2];  // HALF: halves of each of the workgroup's two tasks finished
  if (HALF && threadIdx.x < 2) s_done[threadIdx.x] = 0;
  if (KL > 0) {
    for (int i = threadIdx.x; i < KL * 64; i += 256) w1_lds_buf[i] = a.msg.w1[i];
  }
  if (KL > 0 || HALF) __syncthreads();
  // HALF grids hold exactly n_tasks / 2 workgroups (n_tasks is a multiple of 4)
  if (!HALF && task >= a.n_tasks) return;
  const int blk_lo = HALF ? 25 * hh : 0, blk_hi = HALF ? blk_lo + 25 : 50;
  const int64_t g0 = task * 32;
  float* scratch = lds_scratch[w];
  float* aggl = a.agg + task * 32 * 128;
  float carry[2] = {0.f, 0.f};  // running sums of the receiver continuing into the next block

  int32_t s_next = edge_sender(a, g0, lane, blk_lo);
  for (int blk = blk_lo; blk < blk_hi; ++blk) {
    const int32_t s_cur = s_next;
    if (HALF) tail_prio(blk_hi - blk, 1);
    else tail_prio(blk_hi - blk, 2);
    if (blk < blk_hi - 1) s_next = edge_sender(a, g0, lane, blk + 1);
    Tile m;
    edge_block<LAYER>(a, task, g0, lane, blk, s_cur, m, w1_lds);
    // ordered segment sum over the 50 slots of each receiver (jax.ops.segment_sum order). The
    // block holds edges of two receivers: rA (block edges 0..lastA) and rA+1 (the rest).
    // Transpose through LDS two accumulator blocks at a time, so that lane l owns channel
    // 64·p + l of pass p and runs both receivers' sequential chains over the block's edges
    // itself. The chain bounds are wave-uniform (no divergence, no data-dependent loops): edge
    // ee enters chain A iff ee <= hiA and chain B iff loB <= ee <= hiB, as fmaf(v, 1, acc)
    // (= acc + v, one rounding) or fmaf(v, 0, acc) (= acc exactly: a chain never holds -0, and
    // messages are finite GELU outputs).
    const int rA = (32 * blk) / 50;                    // wave-uniform
    const int lastA = 50 * (rA + 1) - 1 - 32 * blk;    // block-local index of rA's last edge
    const int j0 = 32 * blk - 50 * rA;                 // slot of the block's edge 0 within rA
    const int degA = a.deg[g0 + rA];
    const int degB = rA + 1 < 32 ? a.deg[g0 + rA + 1] : 0;
    const int hiA = min(min(lastA, 31), degA - 1 - j0);  // chain A sums edges [0, hiA]
    const int loB = lastA + 1;                           // chain B sums edges [loB, hiB]
    const int hiB = min(31, lastA + degB);
    // wave-uniform edge masks of the two chains (bit ee set = edge ee enters the chain)
    const uint32_t mA = (uint32_t)__builtin_amdgcn_readfirstlane(
        hiA < 0 ? 0u : (hiA >= 31 ? 0xffffffffu : (1u << (hiA + 1)) - 1u));
    const uint32_t mB = (uint32_t)__builtin_amdgcn_readfirstlane(
        loB > hiB ? 0u : ((hiB >= 31 ? 0xffffffffu : (1u << (hiB + 1)) - 1u) & ~((1u << loB) - 1u)));
#pragma unroll
    for (int p = 0; p < 2; ++p) {
#pragma unroll
      for (int Mh = 0; Mh < 2; ++Mh)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int lc = 32 * Mh + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
          scratch[lc * 36 + (lane & 31)] = m.m[2 * p + Mh][r];
        }
      __builtin_amdgcn_wave_barrier();
      const float4* srow = reinterpret_cast<const float4*>(scratch + lane * 36);
      float v[32];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const float4 t = srow[q];
        v[4 * q] = t.x; v[4 * q + 1] = t.y; v[4 * q + 2] = t.z; v[4 * q + 3] = t.w;
      }
      float accA = carry[p], accB = 0.0f;
      seg_chains(v, mA, mB, accA, accB, std::make_integer_sequence<int, 32>{});
      __builtin_amdgcn_wave_barrier();
      if (lastA <= 31) {
        aggl[rA * 128 + perm_pos(64 * p + lane)] = accA;
        carry[p] = lastA < 31 ? accB : 0.0f;
      } else {
        carry[p] = accA;
      }
    }
  }
  // the sums were stored by other lanes of this wave (HALF: and by the partner wave): drain
  // stores, then read back
  if (HALF) {
    // hand-off inside the workgroup: the wave that finishes its half FIRST leaves (its SIMD slot
    // goes to the other workgroup's waves); the second runs the task's node update alone, the
    // one-wave form below — so the later workgroup of a CU does not end the launch with node
    // updates split over pairs of waves (round 5, per-wave stamps: those ran at half the MFMA
    // rate, one wave per SIMD, after everything else)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_s_waitcnt(0);
    int prev = 0;
    if (lane == 0) prev = __hip_atomic_fetch_add(&s_done[w >> 1], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    prev = __builtin_amdgcn_readfirstlane(prev);
    if (prev == 0) {
      cs.stop(a.clk);
      return;
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    __builtin_amdgcn_s_waitcnt(0);
  } else {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  }
  // ---------------- node update for the 32 receivers (lane&31 = receiver): the body of
  // node_update, kept inline here — calling the helper makes the compiler spill 45 VGPRs
  // in k_mpnn<1,2> (2 inline).
  const int64_t gl = g0 + (lane & 31);
  Tile x;
  {
    Tile ag;
    agg_from_gsum(ag, aggl + (lane & 31) * 128, a.deg[gl], a.msg);
    if (LAYER == 0) {
      int lr = a.node_local[gl];
      tile_load_perm(x, a.h0tab + (int64_t)(lr < 0 ? 0 : lr) * 128);
    } else {
      tile_load_perm(x, a.h_in + gl * 128);
    }
#pragma unroll
    for (int M = 0; M < 4; ++M)
#pragma unroll
      for (int r = 0; r < 16; ++r) x.m[M][r] = x.m[M][r] + ag.m[M][r] / 50.0f;
  }
  tile_layer_norm(x, a.ln0_s, a.ln0_o);  // V_i_0
  Tile out;
  for (int ck = 0; ck < 4; ++ck) {
    Tile hid;
    tile_gemm_bf(hid, x, a.ff_w1 + ck * 64 * 64, a.ff_bf1 + ck * 64, ActId{});
    if (ck == 0)
      tile_gemm_bf(out, hid, a.ff_w2, a.ff_bf2, ActGelu2x{});
    else
      tile_gemm_f(out, hid, a.ff_w2 + ck * 64 * 64, ActGelu2x{});
  }
  tile_add(x, out);
  tile_layer_norm(x, a.ln1_s, a.ln1_o);  // V_i_1
  tile_store_perm(x, a.h_out + gl * 128);
  if (a.P_out) {
#pragma unroll 1
    for (int p = 0; p < 4; ++p) {
      Tile pr;
      if (p & 1) {  // receiver parts chain from the layer's first-layer bias
        tile_gemm_bf(pr, x, a.proj_w + p * 64 * 64, a.proj_bf[p >> 1], ActId{});
      } else {
        tile_zero(pr);
        tile_gemm(pr, x, a.proj_w + p * 64 * 64);
      }
      tile_store_perm(pr, a.P_out + gl * 512 + p * 128);
    }
  }
  cs.stop(a.clk);
}

// Fused layer as a persistent work queue (batches of more than one round of tasks). The unit of
// work is HALF a task — edge blocks 25h .. 25h+24, exactly receivers 16h .. 16h+15 (as in
// k_mpnn<L, true>) — so the last units of a launch are half as long as whole tasks and the
// layer's tail shrinks with them; every wave slot pulls units until the queues are empty. The
// wave that completes the SECOND half of a task (told by the value its add on the task's counter
// returns) runs the task's node update alone, as k_mpnn<L, false> does. Same operations in the
// same order as the other fused forms: identical bits.
// Queues: one per XCD (tasks split into 8 contiguous ranges of units). Unit order: groups of
// q_group tasks (the wave slots of one XCD), the group's first halves, then its second halves —
// so a launch of exactly one wave per task-slot runs like k_mpnn<L, false> (each wave: two halves,
// then the node update), where adjacent halves (q_group 0: units 2t, 2t+1 = the halves of task
// t) ran both halves at once and left the node updates of one half of the waves in series with
// the next units of the other half. A wave pulls from its own XCD's queue (s_getreg XCC_ID; locality only) and, once that is
// empty, from the next ones in turn; it leaves after finding all eight empty (every exit path is
// bounded: one failed pull per queue). The halves of a task may run on different XCDs, so the
// segment-sum hand-off is the agent-scope release / acquire pair (MI355X_MICROARCH.md,
// inter-workgroup visibility): the producer's stores drained, release, then the counter add;
// the consumer's acquire after its add returned. q_head / q_done are zeroed before each launch.
// The kernel arguments are re-read through an opaque pointer to the kernarg segment at every unit
// (scalar loads), so the compiler does not keep ~70 argument registers live across the queue
// loop (carried, they spilled 43 VGPRs and 149 SGPRs).
typedef const MpnnArgs __attribute__((address_space(4)))* MpnnArgsK;

// NW: waves per workgroup — 4 (two workgroups per CU, the first w1_lds_ksteps k-steps of W1 in
// LDS) or 8 (one workgroup per CU sharing ALL 64 W1 k-steps through LDS: a persistent grid has no
// tail for the larger workgroup to lengthen)
template <int LAYER, int NW>
__global__ __launch_bounds__(64 * NW, 8 / NW) void k_mpnn_q(MpnnArgs a_in) {
  const MpnnArgsK a_k = (MpnnArgsK)__builtin_amdgcn_kernarg_segment_ptr();
  ClockStamp cs;
  cs.start(a_in.clk);
  __shared__ float lds_scratch[NW][64 * 36];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  constexpr int KL = NW == 8 ? 64 : w1_lds_ksteps<LAYER>();
  __shared__ float4 w1_lds_buf[(KL > 0 ? KL : 1) * 64];
  const float4* w1_lds = KL > 0 ? w1_lds_buf : nullptr;
  if (KL > 0) {
    for (int i = threadIdx.x; i < KL * 64; i += 64 * NW) w1_lds_buf[i] = a_k->msg.w1[i];
    __syncthreads();
  }
  // HW_REG_XCC_ID (hwreg 20): bits 0-3 = this wave's XCD
  int q = __builtin_amdgcn_readfirstlane((int)(__builtin_amdgcn_s_getreg(0xf814) & 7));
  int empty = 0;
  while (empty < 8) {
    MpnnArgsK ap = a_k;
    asm volatile("" : "+s"(ap));
    const MpnnArgs& a = *(const MpnnArgs*)ap;
    int j = 0;
    if (lane == 0) j = __hip_atomic_fetch_add(a.q_head + 16 * q, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    j = __builtin_amdgcn_readfirstlane(j);
    const int64_t t0 = a.n_tasks * q / 8, t1 = a.n_tasks * (q + 1) / 8;
    if (j >= 2 * (t1 - t0)) {
      ++empty;
      q = (q + 1) & 7;
      continue;
    }
    int64_t task;
    int hh;
    const int G = a.q_group;
    if (G > 0) {  // group g: tasks gG .. gG+gs-1, their first halves, then their second halves
      const int g = j / (2 * G), r = j - 2 * G * g;
      const int64_t rest = t1 - t0 - (int64_t)g * G;
      const int gs = rest < G ? (int)rest : G;
      hh = r >= gs;
      task = t0 + (int64_t)g * G + (r - hh * gs);
    } else {
      task = t0 + (j >> 1);
      hh = j & 1;
    }
    // the lane index re-made opaque per unit: nothing lane-derived is hoisted out of the loop
    int ln = lane;
    asm volatile("" : "+v"(ln));
    mpnn_edge_blocks<LAYER, KL, NW>(a, task, ln, 25 * hh, 25 * hh + 25, w1_lds, lds_scratch, w);
    // hand-off of this half's segment sums: stores drained, agent release, then the counter
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    int prev = 0;
    if (lane == 0) prev = __hip_atomic_fetch_add(a.q_done + task, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    prev = __builtin_amdgcn_readfirstlane(prev);
    if (prev == 1) {  // both halves done: this wave runs the node update
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      mpnn_node_tile<LAYER>(a, task * 32, ln, a.agg + task * 32 * 128);
    }
  }
  cs.stop(a_k->clk);
}

// Split layer (small batches, where one wave per 32 receivers cannot fill the GPU): the edge
// blocks of all tasks run in parallel, `blocks_per_wave` consecutive blocks per wave, and store
// their messages as rows `msg_rows[E][128]` (perm order); k_seg_sum forms each receiver's
// ordered segment sum from those rows — the same additions in the same order as k_mpnn, so
// both modes give identical bits — and k_mpnn_node runs the node update on the sums.
__device__ __forceinline__ int64_t gb_edge(int64_t gb, int lane) { return gb * 32 + (lane & 31); }

template <int LAYER>
__global__ __launch_bounds__(256, MPNN_MIN_BLOCKS) void k_mpnn_edge(MpnnArgs a) {
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t nb = a.n_tasks * 50;
  const int64_t b0 = ((int64_t)blockIdx.x * 4 + w) * a.blocks_per_wave;
  if (b0 >= nb) return;
  const int64_t b1 = min(b0 + (int64_t)a.blocks_per_wave, nb);
  // edge block gb covers edges 32*gb .. 32*gb+31 (E = task*1600 + 32*blk + col)
  int32_t s_next = a.senders[gb_edge(b0, lane)];
  for (int64_t gb = b0; gb < b1; ++gb) {
    const int64_t task = gb / 50;
    const int blk = (int)(gb - task * 50);
    const int32_t s_cur = s_next;
    if (gb + 1 < b1) s_next = a.senders[gb_edge(gb + 1, lane)];
    Tile m;
    edge_block<LAYER>(a, task, task * 32, lane, blk, s_cur, m);
    tile_store_perm(m, a.msg_rows + (gb * 32 + (lane & 31)) * 128);  // row E = task*1600 + 32*blk + col
  }
}

// Ordered segment sums of the split schedule, one wave per receiver: lane l sums channels
// (2l, 2l+1) of the perm-ordered message rows over the receiver's slots in order,
// agg = ((0 + m_0) + m_1) + ... + m_{deg-1} — the fused kernel's additions in its order. Reads
// are whole 512-byte rows per step; thousands of waves keep HBM busy where the 32-receiver node
// tiles alone could not.
__global__ __launch_bounds__(256) void k_seg_sum(const float* __restrict__ msg_rows, const int32_t* __restrict__ deg,
                                                 float* __restrict__ agg, int64_t n_rows) {
  const int lane = threadIdx.x & 63;
  const int64_t g = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (g >= n_rows) return;
  const int d = deg[g];
  const float2* row = reinterpret_cast<const float2*>(msg_rows + g * KNN * 128) + lane;
  float2 acc = make_float2(0.0f, 0.0f);
  // rows are loaded 10 at a time ahead of their (ordered) additions: one memory round trip per
  // 10 slots instead of one per slot; the sums are the same chain in slot order
  int j = 0;
  for (; j + 10 <= d; j += 10) {
    float2 v[10];
#pragma unroll
    for (int u = 0; u < 10; ++u) v[u] = row[(j + u) * 64];
#pragma unroll
    for (int u = 0; u < 10; ++u) {
      acc.x = acc.x + v[u].x;
      acc.y = acc.y + v[u].y;
    }
  }
  for (; j < d; ++j) {
    const float2 v = row[j * 64];
    acc.x = acc.x + v.x;
    acc.y = acc.y + v.y;
  }
  reinterpret_cast<float2*>(agg + g * 128)[lane] = acc;
}

template <int LAYER>
__global__ __launch_bounds__(256, MPNN_MIN_BLOCKS) void k_mpnn_node(MpnnArgs a) {
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t task = (int64_t)blockIdx.x * 4 + w;
  if (task >= a.n_tasks) return;
  const int64_t g0 = task * 32;
  node_update<LAYER>(a, lane, g0, a.agg + task * 32 * 128);  // sums from k_seg_sum
}

// ---------------------------------------------------------------------------- k_down
template <int DF>
// df 1 fits 2 waves/SIMD in 256 registers (3 spilled); df 2/4 keep the attention state of DF
// keys and need the 512-register, 1 wave/SIMD form
__global__ __launch_bounds__(256, DF == 1 ? 2 : 1) void k_down(DownArgs a) {
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int tile_id = blockIdx.x * 4 + w;
  if (tile_id >= a.n_tiles) return;
  const int b = a.tile_prot[tile_id];
  const int t0 = a.tile_t0[tile_id];
  const int64_t base = a.offsets[b];
  const int T = a.n_nodes[b] / DF;
  const int t = t0 + (lane & 31);
  const bool valid = t < T;
  const int tc = valid ? t : (T > 0 ? T - 1 : 0);  // clamp: invalid lanes recompute a real row
  float* rrow = a.r_buf + (base + tc) * 128;
  // resampled track init: sinusoidal PE of the token index (modules.py:488-500)
  {
    Tile r;
    tile_load_perm(r, a.RPE + (int64_t)tc * 128);
    if (valid) tile_store_perm(r, rrow);
  }
  for (int blk = 0; blk < 3; ++blk) {
    const DownBlockW& W = a.blk[blk];
    // ---- cross attention: v (and logits for DF > 1) from the original track
    Tile wa;
    if (DF == 1) {
      Tile x;
      tile_load_perm(x, a.o_buf + (base + tc) * 128);
      tile_layer_norm(x, W.dn_s, W.dn_o);
      tile_zero(wa);
      tile_gemm(wa, x, W.wv);
#pragma unroll
      for (int M = 0; M < 4; ++M)
#pragma unroll
        for (int r = 0; r < 16; ++r) wa.m[M][r] = wa.m[M][r] + 0.0f;  // fmaf(1, v, 0)
    } else {
      // q for the logits
      Tile q;
      tile_load_perm(q, rrow);
      tile_layer_norm(q, W.qn_s, W.qn_o);
      Tile qq;
      tile_zero(qq);
      tile_gemm(qq, q, W.wq);
#pragma unroll
      for (int M = 0; M < 4; ++M)
#pragma unroll
        for (int r = 0; r < 16; ++r) qq.m[M][r] = qq.m[M][r] * 0.176776692f;
      float logit[4][DF];
      for (int p = 0; p < DF; ++p) {
        Tile x;
        tile_load_perm(x, a.o_buf + (base + (int64_t)tc * DF + p) * 128);
        tile_layer_norm(x, W.dn_s, W.dn_o);
        Tile kk;
        tile_zero(kk);
        tile_gemm(kk, x, W.wk);
        Tile vv;
        tile_zero(vv);
        tile_gemm(vv, x, W.wv);
        tile_store_perm(vv, a.v_buf + (base + (int64_t)tc * DF + p) * 128);
#pragma unroll
        for (int hd = 0; hd < 4; ++hd) {
          float accl = 0.0f;
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            float q0 = qq.m[hd][r], k0 = kk.m[hd][r];
            float q1 = __shfl_xor(q0, 32, 64), k1 = __shfl_xor(k0, 32, 64);
            if (lane >= 32) { float tq = q0; q0 = q1; q1 = tq; float tk = k0; k0 = k1; k1 = tk; }
            accl = __builtin_fmaf(q0, k0, accl);  // channel f(r)      (half 0)
            accl = __builtin_fmaf(q1, k1, accl);  // channel f(r) + 4  (half 1)
          }
          logit[hd][p] = accl;
        }
      }
      float wgt[4][DF];
#pragma unroll
      for (int hd = 0; hd < 4; ++hd) {
        float mx = logit[hd][0];
        for (int p = 1; p < DF; ++p) mx = logit[hd][p] > mx ? logit[hd][p] : mx;
        float ex[DF], sum = 0.0f;
        for (int p = 0; p < DF; ++p) { ex[p] = c_exp(logit[hd][p] - mx); sum = sum + ex[p]; }
        for (int p = 0; p < DF; ++p) wgt[hd][p] = ex[p] / sum;
      }
      tile_zero(wa);
      for (int p = 0; p < DF; ++p) {
        Tile vv;
        tile_load_perm(vv, a.v_buf + (base + (int64_t)tc * DF + p) * 128);
#pragma unroll
        for (int M = 0; M < 4; ++M)
#pragma unroll
          for (int r = 0; r < 16; ++r) wa.m[M][r] = __builtin_fmaf(wgt[M][p], vv.m[M][r], wa.m[M][r]);
      }
    }
    {  // gating: sigmoid(LN_q(r) Wg + bg)
      Tile q;
      tile_load_perm(q, rrow);
      tile_layer_norm(q, W.qn_s, W.qn_o);
      Tile gt;
      tile_zero(gt);
      tile_gemm(gt, q, W.wg);
      tile_add_vec(gt, W.gb);
#pragma unroll
      for (int M = 0; M < 4; ++M)
#pragma unroll
        for (int r = 0; r < 16; ++r) wa.m[M][r] = wa.m[M][r] * c_sigmoid(gt.m[M][r]);
    }
    {  // output projection + residual
      Tile o;
      tile_zero(o);
      tile_gemm(o, wa, W.wo);
      tile_add_vec(o, W.ob);
      Tile r;
      tile_load_perm(r, rrow);
      tile_add(r, o);
      if (valid) tile_store_perm(r, rrow);
      // resampled transition: r += T(LN(r))
      Tile x = r;
      tile_layer_norm(x, W.rt_ln_s, W.rt_ln_o);
      Tile acc;
      tile_zero(acc);
      for (int ck = 0; ck < 2; ++ck) {
        Tile hid;
        tile_zero(hid);
        tile_gemm(hid, x, W.rt_w1 + ck * 64 * 64);
        tile_gemm_f(acc, hid, W.rt_w2 + ck * 64 * 64, ActBiasRelu{W.rt_b1 + ck * 128});
      }
      tile_add_vec(acc, W.rt_b2);
      tile_load_perm(r, rrow);
      tile_add(r, acc);
      if (valid) tile_store_perm(r, rrow);
    }
    if (blk < 2) {  // original transition (block 3's is dead: only "resampled" is returned)
      for (int p = 0; p < DF; ++p) {
        float* orow = a.o_buf + (base + (int64_t)tc * DF + p) * 128;
        Tile x;
        tile_load_perm(x, orow);
        tile_layer_norm(x, W.ot_ln_s, W.ot_ln_o);
        Tile acc;
        tile_zero(acc);
        for (int ck = 0; ck < 2; ++ck) {
          Tile hid;
          tile_zero(hid);
          tile_gemm(hid, x, W.ot_w1 + ck * 64 * 64);
          tile_add_vec(hid, W.ot_b1 + ck * 128);
          tile_relu(hid);
          tile_gemm(acc, hid, W.ot_w2 + ck * 64 * 64);
        }
        tile_add_vec(acc, W.ot_b2);
        tile_load_perm(x, orow);
        tile_add(x, acc);
        if (valid) tile_store_perm(x, orow);
      }
    }
  }
  // ---- spherical norm, down_proj, FSQ
  Tile r;
  tile_load_perm(r, rrow);
  float s = 0.0f;
#pragma unroll
  for (int M = 0; M < 4; ++M)
#pragma unroll
    for (int q = 0; q < 16; ++q) s = s + r.m[M][q] * r.m[M][q];
  float nrm = sqrtf(s + __shfl_xor(s, 32, 64)) + 1e-6f;
#pragma unroll
  for (int M = 0; M < 4; ++M)
#pragma unroll
    for (int q = 0; q < 16; ++q) r.m[M][q] = r.m[M][q] / nrm;
  f32x16 z;
#pragma unroll
  for (int q = 0; q < 16; ++q) z[q] = 0.0f;
  tile_gemm_narrow(z, r, a.down_w);
  // output o = (q&3) + 8*(q>>2) + 4*half: d<4 in half 0 regs 0..3, d = 4..7 in half 1 regs 0..3
  uint32_t part_idx = 0;
  const int h = lane >> 5;
  const int64_t orow_i = base + t;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    int d = q + 4 * h;
    if (d < a.D) {
      float zz = z[q] + a.down_b[d];
      float bnd = c_tanh(zz + a.fsq_shift[d]) * a.fsq_half[d] - a.fsq_off[d];
      float qv = rintf(bnd);
      part_idx += (uint32_t)((int)qv + a.fsq_L[d] / 2) * (uint32_t)a.fsq_basis[d];
      if (valid) {
        a.bounded_out[orow_i * 8 + d] = bnd;
        a.quant_out[orow_i * 8 + d] = qv;
      }
    }
  }
  uint32_t idx = part_idx + (uint32_t)__shfl_xor((int)part_idx, 32, 64);
  if (valid) {
    if (h == 0) a.tokens_out[orow_i] = idx;
    // continuous_embedding_pre_proj in natural channel order
    float4* pp = reinterpret_cast<float4*>(a.pre_proj_out + orow_i * 128);
#pragma unroll
    for (int M = 0; M < 4; ++M)
#pragma unroll
      for (int q = 0; q < 4; ++q)
        pp[(32 * M + 8 * q + 4 * h) / 4] = make_float4(r.m[M][4 * q], r.m[M][4 * q + 1], r.m[M][4 * q + 2], r.m[M][4 * q + 3]);
  }
}

// ------------------------------------------------------------------- k_down_pair
// k_down<1> with the two tracks of a tile on two waves, for batches of at most one round of tiles
// (the N = 8 share of config 3: 1 024 tiles, where k_down<1> leaves every SIMD's second wave slot
// empty). Per block b, the original-track wave ("o") computes v_b = LN(o_b)·Wv, hands it over
// through LDS (double buffered, one workgroup barrier per block) and then runs the original
// transition o_{b+1} = o_b + T(LN(o_b)); the resampled-track wave ("r") computes the gate from
// LN(r), waits for v_b, and runs gating, output projection and the resampled transition. The r
// wave's chain per block is 384 k-steps instead of 704. Every value is computed by the same
// operations in the same order as in k_down<1> — only which wave runs them changes — so the bits
// are identical (test_down_coop_and_one_wave_identical forces all three forms). Workgroup = 4
// waves = 2 tiles (waves 2i, 2i+1 = tile i's r and o waves); every wave passes the same three
// barriers, tiles past the end included.
__global__ __launch_bounds__(256, 2) void k_down_pair(DownArgs a) {
  __shared__ float vx[2][2][64 * 64];  // [tile in workgroup][buffer][register][lane]
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int tw = w >> 1, role_o = w & 1;
  const int tile_id = blockIdx.x * 2 + tw;
  const bool live = tile_id < a.n_tiles;
  int b = 0, t0 = 0, T = 0;
  int64_t base = 0;
  if (live) {
    b = a.tile_prot[tile_id];
    t0 = a.tile_t0[tile_id];
    base = a.offsets[b];
    T = a.n_nodes[b];
  }
  const int t = t0 + (lane & 31);
  const bool valid = live && t < T;
  const int tc = valid ? t : (T > 0 ? T - 1 : 0);
  if (!role_o) {
    // ---- the resampled-track wave
    float* rrow = a.r_buf + (base + tc) * 128;
    if (live) {
      Tile r;
      tile_load_perm(r, a.RPE + (int64_t)tc * 128);
      if (valid) tile_store_perm(r, rrow);
    }
    for (int blk = 0; blk < 3; ++blk) {
      const DownBlockW& W = a.blk[blk];
      const float* xs = vx[tw][blk & 1];
      Tile wa;
      if (live) {  // gating logits LN_q(r) Wg + bg; after the handover, v · sigmoid(logits)
        Tile q;
        tile_load_perm(q, rrow);
        tile_layer_norm(q, W.qn_s, W.qn_o);
        tile_zero(wa);
        tile_gemm(wa, q, W.wg);
        tile_add_vec(wa, W.gb);
      }
      __syncthreads();
      if (!live) continue;
#pragma unroll
      for (int M = 0; M < 4; ++M)
#pragma unroll
        for (int r = 0; r < 16; ++r) wa.m[M][r] = xs[(M * 16 + r) * 64 + lane] * c_sigmoid(wa.m[M][r]);
      Tile o;
      tile_zero(o);
      tile_gemm(o, wa, W.wo);
      tile_add_vec(o, W.ob);
      Tile r;
      tile_load_perm(r, rrow);
      tile_add(r, o);
      if (valid) tile_store_perm(r, rrow);
      Tile x = r;
      tile_layer_norm(x, W.rt_ln_s, W.rt_ln_o);
      Tile acc;
      tile_zero(acc);
      for (int ck = 0; ck < 2; ++ck) {
        Tile hid;
        tile_zero(hid);
        tile_gemm(hid, x, W.rt_w1 + ck * 64 * 64);
        tile_gemm_f(acc, hid, W.rt_w2 + ck * 64 * 64, ActBiasRelu{W.rt_b1 + ck * 128});
      }
      tile_add_vec(acc, W.rt_b2);
      tile_load_perm(r, rrow);
      tile_add(r, acc);
      if (valid) tile_store_perm(r, rrow);
    }
    if (!live) return;
    // spherical norm, down_proj, FSQ (as k_down<1>)
    Tile r;
    tile_load_perm(r, rrow);
    float s = 0.0f;
#pragma unroll
    for (int M = 0; M < 4; ++M)
#pragma unroll
      for (int q = 0; q < 16; ++q) s = s + r.m[M][q] * r.m[M][q];
    float nrm = sqrtf(s + __shfl_xor(s, 32, 64)) + 1e-6f;
#pragma unroll
    for (int M = 0; M < 4; ++M)
#pragma unroll
      for (int q = 0; q < 16; ++q) r.m[M][q] = r.m[M][q] / nrm;
    f32x16 z;
#pragma unroll
    for (int q = 0; q < 16; ++q) z[q] = 0.0f;
    tile_gemm_narrow(z, r, a.down_w);
    uint32_t part_idx = 0;
    const int h = lane >> 5;
    const int64_t orow_i = base + t;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      int d = q + 4 * h;
      if (d < a.D) {
        float zz = z[q] + a.down_b[d];
        float bnd = c_tanh(zz + a.fsq_shift[d]) * a.fsq_half[d] - a.fsq_off[d];
        float qv = rintf(bnd);
        part_idx += (uint32_t)((int)qv + a.fsq_L[d] / 2) * (uint32_t)a.fsq_basis[d];
        if (valid) {
          a.bounded_out[orow_i * 8 + d] = bnd;
          a.quant_out[orow_i * 8 + d] = qv;
        }
      }
    }
    uint32_t idx = part_idx + (uint32_t)__shfl_xor((int)part_idx, 32, 64);
    if (valid) {
      if (h == 0) a.tokens_out[orow_i] = idx;
      float4* pp = reinterpret_cast<float4*>(a.pre_proj_out + orow_i * 128);
#pragma unroll
      for (int M = 0; M < 4; ++M)
#pragma unroll
        for (int q = 0; q < 4; ++q)
          pp[(32 * M + 8 * q + 4 * h) / 4] =
              make_float4(r.m[M][4 * q], r.m[M][4 * q + 1], r.m[M][4 * q + 2], r.m[M][4 * q + 3]);
    }
    return;
  }
  // ---- the original-track wave: v_b for the r wave, then the original transition
  float* orow = a.o_buf + (base + tc) * 128;
  for (int blk = 0; blk < 3; ++blk) {
    const DownBlockW& W = a.blk[blk];
    float* xs = vx[tw][blk & 1];
    if (live) {  // v_b = LN(o_b)·Wv (+0.0f: fmaf(1, v, 0), as k_down<1>)
      Tile x;
      tile_load_perm(x, orow);
      tile_layer_norm(x, W.dn_s, W.dn_o);
      Tile wa;
      tile_zero(wa);
      tile_gemm(wa, x, W.wv);
#pragma unroll
      for (int M = 0; M < 4; ++M)
#pragma unroll
        for (int r = 0; r < 16; ++r) xs[(M * 16 + r) * 64 + lane] = wa.m[M][r] + 0.0f;
    }
    __syncthreads();
    if (live && blk < 2) {  // original transition (block 3's is dead)
      Tile x;
      tile_load_perm(x, orow);
      tile_layer_norm(x, W.ot_ln_s, W.ot_ln_o);
      Tile acc;
      tile_zero(acc);
      for (int ck = 0; ck < 2; ++ck) {
        Tile hid;
        tile_zero(hid);
        tile_gemm(hid, x, W.ot_w1 + ck * 64 * 64);
        tile_add_vec(hid, W.ot_b1 + ck * 128);
        tile_relu(hid);
        tile_gemm(acc, hid, W.ot_w2 + ck * 64 * 64);
      }
      tile_add_vec(acc, W.ot_b2);
      tile_load_perm(x, orow);
      tile_add(x, acc);
      if (valid) tile_store_perm(x, orow);
    }
  }
}

// ------------------------------------------------------------------- k_down_coop
// Small-batch form of k_down<1>: one workgroup per 32-token tile, wave w computes output
// block w (channels 32w … 32w+31) of every GEMM, so a tile's 20 sequential 128x128 GEMMs take
// a quarter of the MFMA chain latency. Each output channel's fmaf chain is the same one the
// one-wave kernel runs (same k order, same activation on the B operand), so the bits are equal;
// full tiles (LayerNorm inputs, next-GEMM operands) are assembled through LDS, double buffered
// so each exchange costs one barrier. The tracks stay in registers (r_buf / o_buf unused).

// acc (block w) += f(X) · W over K = 128; W fragments as in tile_gemm_f, component w, streamed
// 16 k-steps ahead (64 ahead measured the same)
#ifndef PST_COOP_DEPTH
#define PST_COOP_DEPTH 16
#endif
template <typename F>
__device__ __forceinline__ void blk_gemm_f(f32x16& acc, const Tile& X, const float4* __restrict__ Wf, int w, F&& f) {
  __amdgpu_buffer_rsrc_t rs = make_rsrc(Wf);
  const int vo = lane_id() * 16 + 4 * w;
  constexpr int D = PST_COOP_DEPTH;
  float ring[D];
#pragma unroll
  for (int i = 0; i < D; ++i) ring[i] = buf_load1(rs, vo, i * 1024);
#pragma unroll
  for (int t = 0; t < 64; t += 2) {
    const f32x2 b = f(t, (f32x2){X.m[t / 16][t % 16], X.m[t / 16][t % 16 + 1]});
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const float a = ring[(t + j) % D];
      if (t + j + D < 64) ring[(t + j) % D] = buf_load1(rs, vo, (t + j + D) * 1024);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, j ? b.y : b.x, acc, 0, 0, 0);
    }
  }
}
__device__ __forceinline__ void blk_gemm(f32x16& acc, const Tile& X, const float4* __restrict__ Wf, int w) {
  blk_gemm_f(acc, X, Wf, w, ActId{});
}
__device__ __forceinline__ f32x16 blk_pick(const Tile& t, int w) {
  return w == 0 ? t.m[0] : w == 1 ? t.m[1] : w == 2 ? t.m[2] : t.m[3];
}
// v (block w) += vperm (block w)
__device__ __forceinline__ void blk_add_vec(f32x16& v, const float* __restrict__ vperm, int w) {
  const float4* p = reinterpret_cast<const float4*>(vperm + (lane_id() >> 5) * 64 + w * 16);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    float4 x = p[q];
    v[4 * q] = v[4 * q] + x.x;
    v[4 * q + 1] = v[4 * q + 1] + x.y;
    v[4 * q + 2] = v[4 * q + 2] + x.z;
    v[4 * q + 3] = v[4 * q + 3] + x.w;
  }
}
// every wave contributes its block; all waves get the full tile
__device__ __forceinline__ void blk_exchange(Tile& t, const f32x16& part, float* xs, int& xb, int w) {
  float* buf = xs + xb * (4 * 16 * 64);
  xb ^= 1;
  const int lane = lane_id();
#pragma unroll
  for (int r = 0; r < 16; ++r) buf[(w * 16 + r) * 64 + lane] = part[r];
  __syncthreads();
#pragma unroll
  for (int M = 0; M < 4; ++M)
#pragma unroll
    for (int r = 0; r < 16; ++r) t.m[M][r] = buf[(M * 16 + r) * 64 + lane];
}

__global__ __launch_bounds__(256, 1) void k_down_coop(DownArgs a) {
  __shared__ float xs[2 * 4 * 16 * 64];
  int xb = 0;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int tile_id = blockIdx.x;
  if (tile_id >= a.n_tiles) return;  // whole workgroup
  const int b = a.tile_prot[tile_id];
  const int t0 = a.tile_t0[tile_id];
  const int64_t base = a.offsets[b];
  const int T = a.n_nodes[b];
  const int t = t0 + (lane & 31);
  const bool valid = t < T;
  const int tc = valid ? t : (T > 0 ? T - 1 : 0);
  Tile r, o;
  tile_load_perm(r, a.RPE + (int64_t)tc * 128);
  tile_load_perm(o, a.o_buf + (base + tc) * 128);
  for (int blk = 0; blk < 3; ++blk) {
    const DownBlockW& W = a.blk[blk];
    f32x16 wa = {};
    {
      Tile x = o;
      tile_layer_norm(x, W.dn_s, W.dn_o);
      blk_gemm(wa, x, W.wv, w);
#pragma unroll
      for (int i = 0; i < 16; ++i) wa[i] = wa[i] + 0.0f;  // fmaf(1, v, 0)
    }
    {
      Tile q = r;
      tile_layer_norm(q, W.qn_s, W.qn_o);
      f32x16 gt = {};
      blk_gemm(gt, q, W.wg, w);
      blk_add_vec(gt, W.gb, w);
#pragma unroll
      for (int i = 0; i < 16; ++i) wa[i] = wa[i] * c_sigmoid(gt[i]);
    }
    {
      Tile waf;
      blk_exchange(waf, wa, xs, xb, w);
      f32x16 oo = {};
      blk_gemm(oo, waf, W.wo, w);
      blk_add_vec(oo, W.ob, w);
      f32x16 rp = blk_pick(r, w);
#pragma unroll
      for (int i = 0; i < 16; ++i) rp[i] = rp[i] + oo[i];
      blk_exchange(r, rp, xs, xb, w);
    }
    {  // resampled transition
      Tile x = r;
      tile_layer_norm(x, W.rt_ln_s, W.rt_ln_o);
      f32x16 acc = {};
      for (int ck = 0; ck < 2; ++ck) {
        f32x16 h1 = {};
        blk_gemm(h1, x, W.rt_w1 + ck * 64 * 64, w);
        Tile hid;
        blk_exchange(hid, h1, xs, xb, w);
        blk_gemm_f(acc, hid, W.rt_w2 + ck * 64 * 64, w, ActBiasRelu{W.rt_b1 + ck * 128});
      }
      blk_add_vec(acc, W.rt_b2, w);
      f32x16 rp = blk_pick(r, w);
#pragma unroll
      for (int i = 0; i < 16; ++i) rp[i] = rp[i] + acc[i];
      blk_exchange(r, rp, xs, xb, w);
    }
    if (blk < 2) {  // original transition
      Tile x = o;
      tile_layer_norm(x, W.ot_ln_s, W.ot_ln_o);
      f32x16 acc = {};
      for (int ck = 0; ck < 2; ++ck) {
        f32x16 h1 = {};
        blk_gemm(h1, x, W.ot_w1 + ck * 64 * 64, w);
        // bias + ReLU on the B operand after the exchange (the same two ops as k_down's add_vec
        // + relu): applying them to the wave's block before the exchange, or loading biases
        // ahead of the GEMMs, measured 20-100 % slower
        Tile hid;
        blk_exchange(hid, h1, xs, xb, w);
        blk_gemm_f(acc, hid, W.ot_w2 + ck * 64 * 64, w, ActBiasRelu{W.ot_b1 + ck * 128});
      }
      blk_add_vec(acc, W.ot_b2, w);
      f32x16 op = blk_pick(o, w);
#pragma unroll
      for (int i = 0; i < 16; ++i) op[i] = op[i] + acc[i];
      blk_exchange(o, op, xs, xb, w);
    }
  }
  // spherical norm (every wave, full tile, canonical order)
  float s = 0.0f;
#pragma unroll
  for (int M = 0; M < 4; ++M)
#pragma unroll
    for (int q = 0; q < 16; ++q) s = s + r.m[M][q] * r.m[M][q];
  const float nrm = sqrtf(s + __shfl_xor(s, 32, 64)) + 1e-6f;
  const int h = lane >> 5;
  const int64_t orow_i = base + t;
  if (valid) {  // continuous_embedding_pre_proj, block w, natural channel order
    f32x16 rn = blk_pick(r, w);
    float4* pp = reinterpret_cast<float4*>(a.pre_proj_out + orow_i * 128);
#pragma unroll
    for (int q = 0; q < 4; ++q)
      pp[(32 * w + 8 * q + 4 * h) / 4] =
          make_float4(rn[4 * q] / nrm, rn[4 * q + 1] / nrm, rn[4 * q + 2] / nrm, rn[4 * q + 3] / nrm);
  }
  if (w != 0) return;
#pragma unroll
  for (int M = 0; M < 4; ++M)
#pragma unroll
    for (int q = 0; q < 16; ++q) r.m[M][q] = r.m[M][q] / nrm;
  f32x16 z;
#pragma unroll
  for (int q = 0; q < 16; ++q) z[q] = 0.0f;
  tile_gemm_narrow(z, r, a.down_w);
  uint32_t part_idx = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    int d = q + 4 * h;
    if (d < a.D) {
      float zz = z[q] + a.down_b[d];
      float bnd = c_tanh(zz + a.fsq_shift[d]) * a.fsq_half[d] - a.fsq_off[d];
      float qv = rintf(bnd);
      part_idx += (uint32_t)((int)qv + a.fsq_L[d] / 2) * (uint32_t)a.fsq_basis[d];
      if (valid) {
        a.bounded_out[orow_i * 8 + d] = bnd;
        a.quant_out[orow_i * 8 + d] = qv;
      }
    }
  }
  uint32_t idx = part_idx + (uint32_t)__shfl_xor((int)part_idx, 32, 64);
  if (valid && h == 0) a.tokens_out[orow_i] = idx;
}

// ------------------------------------------------------------- k_mpnn_node_coop
// Small-batch node update (split schedule): one workgroup per 32 receivers, wave w owns output
// channels 32w … 32w+31 of each of the 13 GEMMs (node_update's chains, same order), full tiles
// assembled through LDS as in k_down_coop. The FFN's GELU is applied to a wave's own block
// before the exchange (elementwise, same function), so it is not evaluated four times.

// acc (block w) = bias + f(X)·W (tile_gemm_bf for one output block)
template <typename F>
__device__ __forceinline__ void blk_gemm_bf(f32x16& acc, const Tile& X, const float4* __restrict__ Wf,
                                            const float4* __restrict__ Bf, int w, F&& f) {
  __amdgpu_buffer_rsrc_t rs = make_rsrc(Bf);
  const float bb = buf_load1(rs, lane_id() * 16 + 4 * w, 0);
  const float one = lane_id() < 32 ? 1.0f : 0.0f;
  const f32x16 z = {};
  acc = __builtin_amdgcn_mfma_f32_32x32x2f32(bb, one, z, 0, 0, 0);
  blk_gemm_f(acc, X, Wf, w, f);
}
// this lane's block-w values of a perm row
__device__ __forceinline__ f32x16 blk_load_row(const float* __restrict__ row, int w) {
  const float4* p = reinterpret_cast<const float4*>(row + (lane_id() >> 5) * 64 + w * 16);
  f32x16 v;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float4 x = p[q];
    v[4 * q] = x.x;
    v[4 * q + 1] = x.y;
    v[4 * q + 2] = x.z;
    v[4 * q + 3] = x.w;
  }
  return v;
}
__device__ __forceinline__ void blk_store_row(const f32x16& v, float* __restrict__ row, int w) {
  float4* p = reinterpret_cast<float4*>(row + (lane_id() >> 5) * 64 + w * 16);
#pragma unroll
  for (int q = 0; q < 4; ++q) p[q] = make_float4(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
}

template <int LAYER>
__global__ __launch_bounds__(256, 1) void k_mpnn_node_coop(MpnnArgs a) {
  __shared__ float xs[2 * 4 * 16 * 64];
  int xb = 0;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t task = blockIdx.x;
  if (task >= a.n_tasks) return;  // whole workgroup
  const int64_t gl = task * 32 + (lane & 31);
  Tile x;
  {
    // agg = deg·b2 + G·W2 (agg_from_gsum), block w
    f32x16 ag;
    const float* b2 = a.msg.b2 + (lane >> 5) * 64 + w * 16;
    const float fd = (float)a.deg[gl];
#pragma unroll
    for (int r = 0; r < 16; ++r) ag[r] = fd * b2[r];
    Tile G;
    tile_load_perm(G, a.agg + gl * 128);
    blk_gemm(ag, G, a.msg.w2, w);
    const float* hrow;
    if (LAYER == 0) {
      const int lr = a.node_local[gl];
      hrow = a.h0tab + (int64_t)(lr < 0 ? 0 : lr) * 128;
    } else {
      hrow = a.h_in + gl * 128;
    }
    f32x16 xp = blk_load_row(hrow, w);
#pragma unroll
    for (int r = 0; r < 16; ++r) xp[r] = xp[r] + ag[r] / 50.0f;
    blk_exchange(x, xp, xs, xb, w);
  }
  tile_layer_norm(x, a.ln0_s, a.ln0_o);  // V_i_0
  f32x16 out;
  for (int ck = 0; ck < 4; ++ck) {
    f32x16 h1;
    blk_gemm_bf(h1, x, a.ff_w1 + ck * 64 * 64, a.ff_bf1 + ck * 64, w, ActId{});
#pragma unroll
    for (int r = 0; r < 16; r += 2) {
      const f32x2 v = c_gelu2x((f32x2){h1[r], h1[r + 1]});
      h1[r] = v.x;
      h1[r + 1] = v.y;
    }
    Tile hid;
    blk_exchange(hid, h1, xs, xb, w);
    if (ck == 0)
      blk_gemm_bf(out, hid, a.ff_w2, a.ff_bf2, w, ActId{});
    else
      blk_gemm(out, hid, a.ff_w2 + ck * 64 * 64, w);
  }
  {
    f32x16 xp = blk_pick(x, w);
#pragma unroll
    for (int r = 0; r < 16; ++r) xp[r] = xp[r] + out[r];
    blk_exchange(x, xp, xs, xb, w);
  }
  tile_layer_norm(x, a.ln1_s, a.ln1_o);  // V_i_1
  blk_store_row(blk_pick(x, w), a.h_out + gl * 128, w);
  if (a.P_out) {
#pragma unroll 1
    for (int p = 0; p < 4; ++p) {
      f32x16 pr;
      if (p & 1) {
        blk_gemm_bf(pr, x, a.proj_w + p * 64 * 64, a.proj_bf[p >> 1], w, ActId{});
      } else {
#pragma unroll
        for (int r = 0; r < 16; ++r) pr[r] = 0.0f;
        blk_gemm(pr, x, a.proj_w + p * 64 * 64, w);
      }
      blk_store_row(pr, a.P_out + gl * 512 + p * 128, w);
    }
  }
}

// ---------------------------------------------------------------------------- tables
// Y[row] = X[row] · W (+ b); rows of X and Y in perm order, 32 rows per wave.
__global__ __launch_bounds__(256) void k_table_gemm(const float* __restrict__ X, int n_rows,
                                                    const float4* __restrict__ Wf, const float* __restrict__ b,
                                                    const float* __restrict__ init, float* __restrict__ Y, int ldy) {
  const int lane = threadIdx.x & 63;
  const int wtile = blockIdx.x * 4 + (threadIdx.x >> 6);
  int row = wtile * 32 + (lane & 31);
  if (wtile * 32 >= n_rows) return;
  int rc = row < n_rows ? row : n_rows - 1;
  Tile x, acc;
  tile_load_perm(x, X + (int64_t)rc * 128);
  if (init)
    tile_load_perm(acc, init);
  else
    tile_zero(acc);
  tile_gemm(acc, x, Wf);
  if (b) tile_add_vec(acc, b);
  if (row < n_rows) tile_store_perm(acc, Y + (int64_t)row * ldy);
}

// V0[lr][ls] = (PM0_s[ls] + PM0_r[lr]) + U[ls - lr] for lr, ls < 512 (perm rows): layer 0's message
// chain start as one gathered row per edge, the same two additions in the same order as edge_block
// does them from the three tables (L0_PAIR_TABLE).
__global__ __launch_bounds__(256) void k_pair_table(const float4* __restrict__ PM0, const float4* __restrict__ U,
                                                    float4* __restrict__ V) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;  // float4 of V
  const int c = (int)(i & 31), ls = (int)((i >> 5) & 511), lr = (int)(i >> 14);
  const float4 a = PM0[ls * 64 + c], b = PM0[lr * 64 + 32 + c], u = U[(ls - lr + 511) * 32 + c];
  float4 v;
  v.x = (a.x + b.x) + u.x;
  v.y = (a.y + b.y) + u.y;
  v.z = (a.z + b.z) + u.z;
  v.w = (a.w + b.w) + u.w;
  V[i] = v;
}

// --------------------------------------------------------------------------- launchers
void launch_pair_table(const float* PM0, const float* U, float* V, hipStream_t st) {
  hipLaunchKernelGGL(k_pair_table, dim3(512 * 512 * 32 / 256), dim3(256), 0, st,
                     reinterpret_cast<const float4*>(PM0), reinterpret_cast<const float4*>(U),
                     reinterpret_cast<float4*>(V));
}

void launch_prep(const PrepArgs& a, int n_prot, hipStream_t st) {
  if (n_prot <= 0) return;
  if (a.pos32) hipLaunchKernelGGL(k_prep<true>, dim3(n_prot), dim3(512), 0, st, a);
  else hipLaunchKernelGGL(k_prep<false>, dim3(n_prot), dim3(512), 0, st, a);
}
void launch_knn(const KnnArgs& a, hipStream_t st) {
  if (a.n_slots > a.slot0) hipLaunchKernelGGL(k_knn, dim3((unsigned)((a.n_slots - a.slot0 + 3) / 4)), dim3(256), 0, st, a);
}
void launch_mpnn(int layer, const MpnnArgs& a, bool node_coop, hipStream_t st) {
  dim3 grid((unsigned)((a.n_tasks + 3) / 4));
  if (a.msg_rows) {  // split mode
    const int64_t waves = (a.n_tasks * 50 + a.blocks_per_wave - 1) / a.blocks_per_wave;
    dim3 egrid((unsigned)((waves + 3) / 4));
    if (layer == 0) hipLaunchKernelGGL(k_mpnn_edge<0>, egrid, dim3(256), 0, st, a);
    else if (layer == 1) hipLaunchKernelGGL(k_mpnn_edge<1>, egrid, dim3(256), 0, st, a);
    else hipLaunchKernelGGL(k_mpnn_edge<2>, egrid, dim3(256), 0, st, a);
    const int64_t rows = a.n_tasks * 32;
    hipLaunchKernelGGL(k_seg_sum, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, st, a.msg_rows, a.deg, a.agg, rows);
    const dim3 cgrid((unsigned)a.n_tasks);
    if (node_coop && layer == 0) hipLaunchKernelGGL(k_mpnn_node_coop<0>, cgrid, dim3(256), 0, st, a);
    else if (node_coop && layer == 1) hipLaunchKernelGGL(k_mpnn_node_coop<1>, cgrid, dim3(256), 0, st, a);
    else if (node_coop) hipLaunchKernelGGL(k_mpnn_node_coop<2>, cgrid, dim3(256), 0, st, a);
    else if (layer == 0) hipLaunchKernelGGL(k_mpnn_node<0>, grid, dim3(256), 0, st, a);
    else if (layer == 1) hipLaunchKernelGGL(k_mpnn_node<1>, grid, dim3(256), 0, st, a);
    else hipLaunchKernelGGL(k_mpnn_node<2>, grid, dim3(256), 0, st, a);
    return;
  }
  if (a.q_head) {  // persistent half-task queue: every wave slot, at most one unit per wave
    const int64_t units = 2 * a.n_tasks;
    if (a.q_waves == 8) {  // q_grid counts 4-wave workgroups: half as many 8-wave ones
      const dim3 qgrid((unsigned)std::min<int64_t>((units + 7) / 8, a.q_grid / 2));
      if (layer == 0) hipLaunchKernelGGL((k_mpnn_q<0, 8>), qgrid, dim3(512), 0, st, a);
      else if (layer == 1) hipLaunchKernelGGL((k_mpnn_q<1, 8>), qgrid, dim3(512), 0, st, a);
      else hipLaunchKernelGGL((k_mpnn_q<2, 8>), qgrid, dim3(512), 0, st, a);
      return;
    }
    const dim3 qgrid((unsigned)std::min<int64_t>((units + 3) / 4, a.q_grid));
    if (layer == 0) hipLaunchKernelGGL((k_mpnn_q<0, 4>), qgrid, dim3(256), 0, st, a);
    else if (layer == 1) hipLaunchKernelGGL((k_mpnn_q<1, 4>), qgrid, dim3(256), 0, st, a);
    else hipLaunchKernelGGL((k_mpnn_q<2, 4>), qgrid, dim3(256), 0, st, a);
    return;
  }
  if (a.half_tasks) {  // two waves per task (n_tasks % 4 == 0: run() pads slots to 128)
    const dim3 hgrid((unsigned)(a.n_tasks / 2));
    if (layer == 0) hipLaunchKernelGGL((k_mpnn<0, true>), hgrid, dim3(256), 0, st, a);
    else if (layer == 1) hipLaunchKernelGGL((k_mpnn<1, true>), hgrid, dim3(256), 0, st, a);
    else hipLaunchKernelGGL((k_mpnn<2, true>), hgrid, dim3(256), 0, st, a);
    return;
  }
  if (layer == 0) hipLaunchKernelGGL((k_mpnn<0, false>), grid, dim3(256), 0, st, a);
  else if (layer == 1) hipLaunchKernelGGL((k_mpnn<1, false>), grid, dim3(256), 0, st, a);
  else hipLaunchKernelGGL((k_mpnn<2, false>), grid, dim3(256), 0, st, a);
}
void launch_down(int df, const DownArgs& a, int form, hipStream_t st) {
  dim3 grid((unsigned)((a.n_tiles + 3) / 4));
  if (df == 1 && form == DOWN_COOP) hipLaunchKernelGGL(k_down_coop, dim3((unsigned)a.n_tiles), dim3(256), 0, st, a);
  else if (df == 1 && form == DOWN_PAIR)
    hipLaunchKernelGGL(k_down_pair, dim3((unsigned)((a.n_tiles + 1) / 2)), dim3(256), 0, st, a);
  else if (df == 1) hipLaunchKernelGGL(k_down<1>, grid, dim3(256), 0, st, a);
  else if (df == 2) hipLaunchKernelGGL(k_down<2>, grid, dim3(256), 0, st, a);
  else hipLaunchKernelGGL(k_down<4>, grid, dim3(256), 0, st, a);
}
void launch_table_gemm(const float* X, int n_rows, const float4* Wf, const float* b, const float* init, float* Y,
                       int ldy, hipStream_t st) {
  int tiles = (n_rows + 31) / 32;
  hipLaunchKernelGGL(k_table_gemm, dim3((tiles + 3) / 4), dim3(256), 0, st, X, n_rows, Wf, b, init, Y, ldy);
}

}  // namespace pst

