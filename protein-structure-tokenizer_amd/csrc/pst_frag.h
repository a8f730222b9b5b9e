// pst_frag.h — host-side packing of weights into the wave-tile layout of pst_device.h
// (MFMA A-fragments, bias fragments, perm-ordered vectors). Shared by the encoder (pst_api.cpp)
// and the decoder's fused pair kernel (pst_decode.hip).
#pragma once
#include <vector>

namespace pst_host {

inline int tile_channel(int h, int M, int r) { return 32 * M + (r & 3) + 8 * (r >> 2) + 4 * h; }

// canonical k order of every fmaf chain (0,4,1,5,2,6,3,7 per block of 8; oracle/pst_oracle.c pi8)
inline int pi8(int t) { return (t & ~7) | ((t >> 1) & 3) | ((t & 1) << 2); }

// A fragments of a GEMM over K input channels [k0, k0+Kc) (Kc = 128 -> 64 k-steps, 32 -> 16)
// and outputs [o0, o0+128): frag[t][lane][M] = W[k0 + c(t,h)][o0 + 32 M + (lane&31)].
inline std::vector<float> frag(const float* W, int ldw, int k0, int Kvalid, int Kc, int o0, int Ovalid) {
  int steps = Kc / 2;
  std::vector<float> f((size_t)steps * 64 * 4, 0.0f);
  for (int t = 0; t < steps; ++t)
    for (int lane = 0; lane < 64; ++lane) {
      int c = tile_channel(lane >> 5, t / 16, t % 16);
      for (int M = 0; M < 4; ++M) {
        int o = 32 * M + (lane & 31);
        float v = 0.0f;
        if (c < Kvalid && o < Ovalid) v = W[(size_t)(k0 + c) * ldw + o0 + o];
        f[((size_t)t * 64 + lane) * 4 + M] = v;
      }
    }
  return f;
}

inline std::vector<float> frag_narrow(const float* W, int ldw, int O) {  // K = 128, outputs < O
  std::vector<float> f(64 * 64, 0.0f);
  for (int t = 0; t < 64; ++t)
    for (int lane = 0; lane < 64; ++lane) {
      int c = tile_channel(lane >> 5, t / 16, t % 16);
      int o = lane & 31;
      if (o < O) f[t * 64 + lane] = W[(size_t)c * ldw + o];
    }
  return f;
}

// bias fragment for tile_gemm_bf: [64 lanes] float4, lane l < 32 holds b[32M + l] in
// component M, lanes 32..63 zeros
inline std::vector<float> bfrag(const float* b) {
  std::vector<float> f(64 * 4, 0.0f);
  for (int lane = 0; lane < 32; ++lane)
    for (int M = 0; M < 4; ++M) f[lane * 4 + M] = b[32 * M + lane];
  return f;
}

inline std::vector<float> perm(const float* v) {  // 128-vector → perm order
  std::vector<float> p(128);
  for (int h = 0; h < 2; ++h)
    for (int M = 0; M < 4; ++M)
      for (int r = 0; r < 16; ++r) p[h * 64 + M * 16 + r] = v[tile_channel(h, M, r)];
  return p;
}

inline std::vector<float> perm_rows(const std::vector<float>& nat, int rows) {
  std::vector<float> out((size_t)rows * 128);
  for (int i = 0; i < rows; ++i) {
    auto p = perm(nat.data() + (size_t)i * 128);
    std::copy(p.begin(), p.end(), out.begin() + (size_t)i * 128);
  }
  return out;
}

}  // namespace pst_host
