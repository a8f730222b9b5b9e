// pst_pe.h — sinusoidal positional encoding on the host (positional_encoding_layer.py:49-88):
// component k = 1..128 of PE(x; n): odd k → cos(x·π / n^(2(k−1)/d)), even k → sin(x·π / n^(2k/d)),
// argument in float32 as JAX computes it, cos/sin correctly rounded via double.
#pragma once
#include <cmath>
#include <vector>

namespace pst {

inline float pe_value(int x, int n, int k1) {
  int num = (k1 & 1) ? 2 * (k1 - 1) : 2 * k1;
  float e = (float)num / 128.0f;
  float pw = (float)std::pow((double)n, (double)e);
  float arg = ((float)x * 3.14159274101257324f) / pw;
  return (float)((k1 & 1) ? std::cos((double)arg) : std::sin((double)arg));
}

// rows x0 .. x0+count-1 of PE(.; n), natural channel order, [count][128]
inline std::vector<float> pe_rows(int x0, int count, int n) {
  std::vector<float> out((size_t)count * 128);
  for (int i = 0; i < count; ++i)
    for (int k = 1; k <= 128; ++k) out[(size_t)i * 128 + k - 1] = pe_value(x0 + i, n, k);
  return out;
}

}  // namespace pst
