/* sanitize_harness.c — TEST INFRASTRUCTURE: drives the C oracle under AddressSanitizer +
 * UndefinedBehaviorSanitizer (`make -C oracle asan`; tests/test_sanitize.py writes the input).
 *
 * usage: oracle_harness_asan IN.bin OUT.bin
 * IN.bin (little-endian): int32 D, df, n_prot; int32 levels[D]; int64 offsets[n_prot+1];
 *   float blob[pst_oracle_param_count(D)]; double pos[R*111]; uint8 flags[R*37]  (R = offsets[n_prot])
 * OUT.bin: uint32 tokens[R], int32 n_tokens[n_prot]  (pst_oracle_tokenize_batch, one thread)
 * Also runs pst_oracle_fsq_aux on the first protein's latents. */
#include <stdio.h>
#include <stdlib.h>

#include "pst_oracle.h"

static void* read_n(FILE* f, size_t bytes) {
  void* p = malloc(bytes ? bytes : 1);
  if (!p || fread(p, 1, bytes, f) != bytes) {
    fprintf(stderr, "short read (%zu bytes)\n", bytes);
    exit(2);
  }
  return p;
}

int main(int argc, char** argv) {
  if (argc != 3) {
    fprintf(stderr, "usage: %s IN.bin OUT.bin\n", argv[0]);
    return 2;
  }
  FILE* f = fopen(argv[1], "rb");
  if (!f) return 2;
  int32_t* hdr = (int32_t*)read_n(f, 3 * sizeof(int32_t));
  const int D = hdr[0], df = hdr[1], B = hdr[2];
  int32_t* levels = (int32_t*)read_n(f, sizeof(int32_t) * (size_t)D);
  int64_t* off = (int64_t*)read_n(f, sizeof(int64_t) * (size_t)(B + 1));
  const size_t np = pst_oracle_param_count(D);
  float* blob = (float*)read_n(f, sizeof(float) * np);
  const int64_t R = off[B];
  double* pos = (double*)read_n(f, sizeof(double) * 111 * (size_t)R);
  uint8_t* flags = (uint8_t*)read_n(f, 37 * (size_t)R);
  fclose(f);
  uint32_t* tok = (uint32_t*)calloc((size_t)R + 1, sizeof(uint32_t));
  int32_t* nt = (int32_t*)calloc((size_t)B + 1, sizeof(int32_t));
  int rc = pst_oracle_tokenize_batch(blob, D, levels, df, 50, pos, flags, off, B, tok, nt, 1);
  if (rc != 0) {
    fprintf(stderr, "tokenize_batch failed: %d\n", rc);
    return 3;
  }
  /* FSQ aux over the first protein's bounded latents */
  const int n0 = (int)(off[1] - off[0]);
  uint32_t* t0 = (uint32_t*)calloc((size_t)n0 + 1, sizeof(uint32_t));
  float* b0 = (float*)calloc((size_t)n0 * D + 1, sizeof(float));
  float* pre = (float*)calloc((size_t)n0 * 128 + 1, sizeof(float));
  int nn = 0;
  int T = pst_oracle_tokenize(blob, D, levels, df, 50, pos, flags, n0, t0, b0, pre, &nn);
  if (T > 0) {
    int64_t K = 1;
    for (int d = 0; d < D; ++d) K *= levels[d];
    float* dist = (float*)malloc(sizeof(float) * (size_t)(T * K));
    float* prob = (float*)malloc(sizeof(float) * (size_t)(T * K));
    uint32_t* am = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)T);
    pst_oracle_fsq_aux(levels, D, b0, T, dist, prob, am);
    for (int t = 0; t < T; ++t)
      if (am[t] != t0[t]) {
        fprintf(stderr, "fsq argmin %u != token %u at %d\n", am[t], t0[t], t);
        return 4;
      }
    free(dist);
    free(prob);
    free(am);
  }
  FILE* g = fopen(argv[2], "wb");
  if (!g) return 2;
  fwrite(tok, sizeof(uint32_t), (size_t)R, g);
  fwrite(nt, sizeof(int32_t), (size_t)B, g);
  fclose(g);
  printf("oracle_harness: %d proteins, %lld residues, first protein %d tokens\n", B, (long long)R, T);
  free(hdr); free(levels); free(off); free(blob); free(pos); free(flags); free(tok); free(nt);
  free(t0); free(b0); free(pre);
  return 0;
}
