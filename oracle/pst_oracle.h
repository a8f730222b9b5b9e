/* pst_oracle.h — CPU restatement of the tokenize path (TEST INFRASTRUCTURE ONLY; see
 * pst_oracle.c). Per-protein entry points; inputs are one protein's raw atom37 arrays. */
#ifndef PST_ORACLE_H_
#define PST_ORACLE_H_
#include <stddef.h>
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif
size_t pst_oracle_param_count(int D);
void pst_oracle_pe_row(int x, int n, float* out);
/* graph: kept[n_raw] (kept residue indices), senders/deg/feat per slot (k slots per node) */
int pst_oracle_graph(const double* pos, const uint8_t* flags, int n_raw, int k, int* n_out,
                     int32_t* kept, int32_t* senders, int32_t* deg, float* feat);
int pst_oracle_encode(const float* blob, int D, const int32_t* levels, int df, int n, int k,
                      const int32_t* senders, const int32_t* deg, const float* feat,
                      float* h_layers, float* pre_proj, float* z_out, float* b_out, float* q_out,
                      uint32_t* tokens);
int pst_oracle_tokenize(const float* blob, int D, const int32_t* levels, int df, int k,
                        const double* pos, const uint8_t* flags, int n_raw, uint32_t* tokens,
                        float* b_out, float* pre_proj, int* n_nodes);
int pst_oracle_tokenize_batch(const float* blob, int D, const int32_t* levels, int df, int k,
                              const double* pos, const uint8_t* flags, const int64_t* offsets,
                              int n_prot, uint32_t* tokens, int32_t* n_tokens, int n_threads);
int pst_oracle_fsq_aux(const int32_t* levels, int D, const float* bounded, int64_t T, float* dist,
                       float* prob, uint32_t* argmin);
float pst_oracle_tanh(float x);
float pst_oracle_gelu(float x);
float pst_oracle_exp(float x);
float pst_oracle_sigmoid(float x);
double pst_oracle_exp64(double x);
#ifdef __cplusplus
}
#endif
#endif
