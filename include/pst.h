/*
 * pst.h — C ABI of libpst, the MI355X-native structure-tokenization path
 * (PDB atom37 arrays → residue k-NN graph → MPNN encoder → cross-attention downsampler →
 * FSQ token ids). Plain pointers and sizes; no torch types.
 *
 * What each entry point replaces in the reference (xwang112358/protein-structure-tokenizer):
 *   pst_create       InferenceRunner.prepare_tokenize_fn + load_params/device_put_replicated
 *                    (scripts/inference_runner.py:180-191, 237-248): one context per GPU holding
 *                    the encoder-half parameters and precomputed input-independent tables.
 *   pst_tokenize     make_graph_from_pdb → preprocess_sample (structure_tokenizer/data/
 *                    preprocessing.py:42-283; graph build: utils/protein_utils.py:325-438,
 *                    model/quat_affine.py:406-522) + the pmap'd Vq3D.encode_and_quantize
 *                    (model/model.py:453-479) + tokens D2H (scripts/inference_runner.py:303-306).
 *                    Host buffers in, host token ids out (synchronous).
 *   pst_tokenize_device  the same on device-resident buffers, asynchronous on the context's
 *                    stream (what a pipelined runner or bench uses: inputs already in HBM).
 *   pst_aux          the non-token QuantizerOutput fields (quantize, continuous_embedding,
 *                    continuous_embedding_pre_proj; model/quantize.py:183-242).
 *   pst_codebook_aux(_device)  FSQ distances / soft_proba / argmin / histogram / perplexity over
 *                    the implicit codebook (model/quantize.py:205-239).
 *   pst_device_count jax.local_device_count (scripts/inference_runner.py:169-177).
 *   pst_sync / pst_last_error / pst_destroy   runtime plumbing (block_until_ready, errors).
 *
 * Errors: every call returns PST_OK (0) or a negative PST_E* code; pst_last_error(ctx) gives
 * the message. The Python layer maps PST_E_TOO_LARGE / PST_E_TOO_SMALL to NotImplementedError
 * and PST_E_INVALID to ValueError, the reference's exception types.
 *
 * Threading: one context per GPU; contexts are independent and may be driven from different
 * host threads; a single context is not thread-safe.
 */
#ifndef PST_H_
#define PST_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PST_ABI_VERSION 1

enum {
  PST_OK = 0,
  PST_E_INVALID = -1,    /* bad argument / shape (ValueError) */
  PST_E_TOO_LARGE = -2,  /* protein > seq_max_size residues (NotImplementedError) */
  PST_E_TOO_SMALL = -3,  /* protein < graph_max_neighbor residues (NotImplementedError) */
  PST_E_HIP = -4,        /* HIP runtime error */
  PST_E_NOMEM = -5,
};

/* Model hyper-parameters (config/structure_tokenizer/model/gnn/ablation_*_df_*.yaml). */
typedef struct {
  int32_t abi_version;        /* = PST_ABI_VERSION */
  int32_t codebook_size;      /* 432 | 1728 | 4096 | 64000 (= prod(levels)) */
  int32_t downsampling_ratio; /* df: 1 | 2 | 4 */
  int32_t n_levels;           /* D = codes_dimension (5 or 6) */
  int32_t levels[8];          /* FSQ levels, e.g. {4,4,4,4,4,4} or {8,8,8,5,5,5} */
  int32_t seq_max_size;       /* 512: proteins above it are rejected */
  int32_t graph_max_neighbor; /* k = 50 */
} pst_model_desc;

/*
 * Parameter blob: float32, the encoder-half tensors of Vq3D in haiku shapes, row-major,
 * concatenated in this order (names after params_keys_conversion; "ENC" =
 * vq3_d/~/structure_encoder, "L" = ENC/~/graph_neural_network/~/mpnn_layer{,_1,_2},
 * "DS" = vq3_d/~/cross_attn_downsampling/cross_attn_scaler_iteration):
 *   ENC/init_node_embed w[128,128] b[128];  ENC/init_edge_embed w[155,128] b[128]
 *   3 x { L/node_mlp_0/~/linear_{0,1,2} w[384|128|128,128] b[128];
 *         L/node_mlp_1/~/linear_0 w[128,512] b[512]; L/node_mlp_1/~/linear_1 w[512,128] b[128];
 *         L/edge_mlp/~/linear_{0,1,2} (as node_mlp_0);
 *         L/norm_msg{,_1,_2} scale[128] offset[128] }
 *   DS/cross_attention/{query_norm,data_norm} scale[3,128] offset[3,128]
 *   DS/cross_attention/attention query_w key_w value_w gating_w [3,128,4,32]
 *                                gating_b[3,4,32] output_w[3,4,32,128] output_b[3,128]
 *   DS/{resampled,original}_transition: input_layer_norm scale[3,128] offset[3,128],
 *        transition1 weights[3,128,256] bias[3,256], transition2 weights[3,256,128] bias[3,128]
 *   vq3_d/down_proj w[128,D] b[D]
 * (pst_amd/params.py:param_spec is the same list.)
 */
size_t pst_param_count(int32_t n_levels);

typedef struct pst_ctx pst_ctx;

int pst_create(int32_t device, const pst_model_desc* desc, const float* params, size_t n_params,
               pst_ctx** out);
int pst_destroy(pst_ctx* ctx);
const char* pst_last_error(const pst_ctx* ctx);
/* Last error of a failed pst_create (no context exists yet). */
const char* pst_create_error(void);

/* Number of visible HIP devices (0 when none); replaces jax.local_device_count(backend="gpu")
 * in InferenceRunner.prepare_devices (scripts/inference_runner.py:169-177). */
int pst_device_count(int32_t* n);

/*
 * Tokenize a ragged batch of B proteins (host buffers, synchronous).
 *   atom_pos     [R,37,3] float64   atom37 coordinates (R = prot_offsets[B])
 *   atom_flags   [R,37]   uint8     bit0 = atom37_gt_exists, bit1 = atom37_atom_exists
 *   prot_offsets [B+1]    int64     residue offsets of each protein in the arrays above
 *   tokens_out   [R]      uint32    protein b's ids at tokens_out[prot_offsets[b] ...]
 *   n_tokens_out [B]      int32     floor(n_b / df), n_b = residues with N, CA, C and O
 *   n_nodes_out  [B]      int32     n_b (may be NULL)
 * Each protein must have graph_max_neighbor <= R_b <= seq_max_size residues
 * (scripts/inference_runner.py:52-62), else PST_E_TOO_SMALL / PST_E_TOO_LARGE.
 */
int pst_tokenize(pst_ctx* ctx, const double* atom_pos, const uint8_t* atom_flags,
                 const int64_t* prot_offsets, int32_t n_prot, uint32_t* tokens_out,
                 int32_t* n_tokens_out, int32_t* n_nodes_out);

/*
 * pst_tokenize with float32 atom positions [R,37,3]: the PDB path's coordinates are float32
 * values (Biopython's atom.coord; protein_structure_sample.py:166-248 stores them in float64
 * arrays), so this is the same input in half the H2D bytes. k_prep widens each value to
 * float64 on load: for float32-exact coordinates the results are bit-identical to
 * pst_tokenize's. Same arguments, errors and outputs otherwise.
 */
int pst_tokenize_f32(pst_ctx* ctx, const float* atom_pos, const uint8_t* atom_flags,
                     const int64_t* prot_offsets, int32_t n_prot, uint32_t* tokens_out,
                     int32_t* n_tokens_out, int32_t* n_nodes_out);

/*
 * Same on device buffers (d_* in HBM of ctx's device), asynchronous on ctx's stream.
 * prot_offsets stays a HOST array (it sizes the launch). Outputs are device buffers with the
 * layout of pst_tokenize; d_n_nodes_out is required (the graph build writes it), d_n_tokens_out
 * may be NULL. Call pst_sync before reading them.
 */
int pst_tokenize_device(pst_ctx* ctx, const double* d_atom_pos, const uint8_t* d_atom_flags,
                        const int64_t* prot_offsets, int32_t n_prot, uint32_t* d_tokens_out,
                        int32_t* d_n_tokens_out, int32_t* d_n_nodes_out);

/*
 * The residue graph alone (replaces the graph part of preprocessing.py:42-283
 * preprocess_sample, i.e. protein_utils.py:325-438 compute_nearest_neighbors_graph on the
 * residues with N, CA, C and O): runs the graph kernels of pst_tokenize and copies back, per
 * residue row g of the packed inputs (protein b's node i at row prot_offsets[b] + i, i < n_b;
 * rows n_b.. of a protein are zero / -1):
 *   senders_out       [R, 50]     int32  neighbour node index within the protein, nearest first
 *                                        (for n_b <= 50: all n_b nodes, self first; -1 after)
 *   edge_features_out [R, 50, 27] f32    [rbf15, p3, q3, k3, t3]; for n_b <= 50 row-major over
 *                                        the reference's n_b x n_b enumeration
 *   ca_out            [R, 3]      f64    C-alpha coordinates (the graph's node_features)
 *   n_nodes_out       [B]         int32  n_b
 * Size gates as pst_tokenize. Invalidates pst_aux / pst_codebook_aux of an earlier call.
 * Python: pst_amd.graph.build_protein_graphs pads these into the reference's ProteinGraph.
 */
int pst_build_graph(pst_ctx* ctx, const double* atom_pos, const uint8_t* atom_flags,
                    const int64_t* prot_offsets, int32_t n_prot, int32_t* senders_out,
                    float* edge_features_out, double* ca_out, int32_t* n_nodes_out);

/*
 * Non-token QuantizerOutput fields of the LAST tokenize call, copied to host:
 *   bounded  [R, D]   continuous_embedding (tanh-bounded latents, masked)
 *   quantize [R, D]   quantize (rounded codes)
 *   pre_proj [R, 128] continuous_embedding_pre_proj (spherical-normalised)
 * Rows are laid out like tokens_out. Any pointer may be NULL.
 */
int pst_aux(pst_ctx* ctx, float* bounded, float* quantize, float* pre_proj);

/*
 * FSQ aux over the implicit codebook for the LAST tokenize call (model/quantize.py:205-239),
 * one row per real token, rows compact in protein order (protein b's token t at row
 * sum_{b'<b} n_tokens_out[b'] + t):
 *   distances  [T, K] f32  sum_d (b_d - c_kd)^2   (QuantizerOutput.distances)
 *   soft_proba [T, K] f32  softmax_k(distances)   (QuantizerOutput.soft_proba, + sign as reference)
 *   argmin     [T]   u32   nearest code (per-dimension nearest level, lowest on ties)
 *   histogram  [K]   u32   token-id counts over the T rows (one-hot sum, quantize.py:211-221)
 *   perplexity [1]   f32   exp(-sum p log(p + 1e-10)), p = histogram / T (quantize.py:222-224)
 * Host buffers; any pointer may be NULL. `rows` = rows the caller's [T,...] buffers hold
 * (T = sum of n_tokens_out). Synchronous. K = 64000 → 256 KB per row per tensor.
 */
int pst_codebook_aux(pst_ctx* ctx, float* distances, float* soft_proba, uint32_t* argmin,
                     uint32_t* histogram, float* perplexity, int64_t rows);

/*
 * Same on device buffers, asynchronous on ctx's stream (the kernel is a streaming HBM write of
 * 4·K bytes per row per tensor). row_capacity must be >= sum_b floor(R_b / df) of the last call
 * (rows used = sum of n_tokens). The last call's device outputs must still be alive.
 */
int pst_codebook_aux_device(pst_ctx* ctx, float* d_distances, float* d_soft_proba,
                            uint32_t* d_argmin, uint32_t* d_histogram, int64_t row_capacity);

int pst_sync(pst_ctx* ctx);

/*
 * Decode path (token ids → backbone structure): replaces InferenceRunner.prepare_decode_fn /
 * prepare_token_to_code_fn / decode_and_save_pdbs (scripts/inference_runner.py:193-233, 326-437),
 * i.e. Vq3D.indexes_to_codes + decode + structure_module (model/model.py:261-262, 481-569).
 * The decoder-half parameter blob is every tensor of pst_amd.params.decoder_param_spec, row-major,
 * concatenated in that order (up_proj, cross_attn_upsampling, sequence_decoder, structure_module).
 */
typedef struct pst_decoder pst_decoder;
size_t pst_decoder_param_count(int32_t n_levels);
int pst_decoder_create(int32_t device, const pst_model_desc* desc, const float* params, size_t n_params,
                       pst_decoder** out);
int pst_decoder_destroy(pst_decoder* dec);
const char* pst_decoder_last_error(const pst_decoder* dec);
const char* pst_decoder_create_error(void);
/* Decode B proteins (host buffers, synchronous). Protein b's token ids are
 * tokens[token_offsets[b] .. token_offsets[b+1]) (at most 512/df, ids < codebook size); it gets
 * N_b = df · T_b residues. atom37_out [sum N_b, 37, 3] f32 receives final_atom_positions (N, CA,
 * C and O set, every other atom 0 — the reference's dummy-ALA mask, model.py:547-568);
 * n_nodes_out [B] (may be NULL) receives N_b. */
int pst_decoder_decode(pst_decoder* dec, const uint32_t* tokens, const int64_t* token_offsets,
                       int32_t n_prot, float* atom37_out, int32_t* n_nodes_out);
/* pst_decoder_decode for the autoencoder pass (Vq3D.__call__, model/model.py:194-259, which
 * InferenceRunner.prepare_ae_fn pmaps, scripts/inference_runner.py:209-222): there the decoder's
 * nodes_mask is the graph's, so protein b decodes n_nodes_in[b] residues, df·T_b <= n < df·(T_b+1)
 * (the node count its T_b = floor(n / df) tokens came from, preprocessing.py:212-216); NULL gives
 * df·T_b as pst_decoder_decode. up_proj_out [sum T_b, 128] (may be NULL) receives
 * quantize_post_proj = up_proj(codes) of every token, rows laid out like `tokens`. */
int pst_decoder_decode_ex(pst_decoder* dec, const uint32_t* tokens, const int64_t* token_offsets,
                          int32_t n_prot, const int32_t* n_nodes_in, float* atom37_out,
                          int32_t* n_nodes_out, float* up_proj_out);
/* Intermediates of the last decode call (needs PST_DEBUG=1): which = 0 single [sum N,128],
 * 1 pair [sum N², 128], 2 affine trajectory [per protein 8, N, 7], 3 torsion sin/cos
 * [per protein 8, N, 3, 2], 4 atom14 [sum N, 14, 3]. */
int pst_decoder_debug(pst_decoder* dec, int32_t which, float* out, size_t n_floats);

/* Decoder stage timing (measurement; tools/bench_decode.py's roofline): while enabled, every
 * group is launched directly (no graph replay) with HIP events around its stages, and
 * pst_decoder_get_timing returns ms[0..3] summed over the groups since enabling: upsampler,
 * pair-chain inputs (LayerNorm + left/right/init GEMMs), k_pair_fused, the 8 fold iterations. */
#define PST_DECODER_N_STAGES 4
int pst_decoder_set_timing(pst_decoder* dec, int32_t enable);
int pst_decoder_get_timing(pst_decoder* dec, float* ms);

/*
 * Native PDB parsing (host, no GPU): replaces protein_structure_from_pdb_string
 * (structure_tokenizer/data/protein_structure_sample.py:166-248, Biopython PDBParser semantics,
 * restated in pst_amd/pdb.py) for make_graph_from_pdb (scripts/inference_runner.py:47-50).
 * n inputs are parsed on n_threads host threads into a batch handle; chain_id = 0 parses all
 * chains, else only that chain. A failing input (multi-model, insertion code, malformed
 * record, unreadable file) gets status PST_E_INVALID and 0 residues; the others are unaffected.
 */
typedef struct pst_pdb_batch pst_pdb_batch;
int pst_pdb_parse_files(const char* const* paths, int32_t n, char chain_id, int32_t n_threads,
                        pst_pdb_batch** out);
int pst_pdb_parse_strings(const char* const* texts, const size_t* lens, int32_t n, char chain_id,
                          int32_t n_threads, pst_pdb_batch** out);
/* number of inputs and total residues kept */
int pst_pdb_batch_sizes(const pst_pdb_batch* b, int32_t* n, int64_t* n_residues);
/* Copy out the packed batch (any pointer may be NULL):
 *   positions [R,37,3] f64, flags [R,37] u8 (bit0 gt_exists, bit1 atom_exists),
 *   aatype [R] u8 (restype index, 20 = UNK), offsets [n+1] i64, status [n] i32 */
int pst_pdb_batch_copy(const pst_pdb_batch* b, double* positions, uint8_t* flags, uint8_t* aatype,
                       int64_t* offsets, int32_t* status);
/* The same with positions as float32 [R,37,3]: exact (the parser rounds every coordinate to
 * float32 as Bio stores atom.coord), half the bytes — the input pst_tokenize_f32 takes. */
int pst_pdb_batch_copy_f32(const pst_pdb_batch* b, float* positions, uint8_t* flags, uint8_t* aatype,
                           int64_t* offsets, int32_t* status);
const char* pst_pdb_batch_error(const pst_pdb_batch* b, int32_t i);
void pst_pdb_batch_free(pst_pdb_batch* b);
/* Tokenize a parsed batch as it stands (the CLI's parse -> tokenize step without a copy through
 * the caller): the parser's float32 atom37 arrays are packed into the context's page-locked
 * staging on the host pool and tokenized as pst_tokenize_f32 (same results). Every input must
 * have parsed: otherwise PST_E_INVALID with that input's parser message (pst_last_error).
 * tokens_out [R] (R from pst_pdb_batch_sizes), n_tokens_out / n_nodes_out [n] (may be NULL). */
int pst_tokenize_pdb_batch(pst_ctx* ctx, const pst_pdb_batch* b, uint32_t* tokens_out, int32_t* n_tokens_out,
                           int32_t* n_nodes_out);
/* The CLI's read -> parse -> tokenize step with the parse on the GPU: the n files are read into
 * page-locked memory on n_threads host threads, their text copied to HBM once, and one workgroup
 * per file turns it into atom37 rows in the tokenizer's input buffers (pst_pdb_gpu.hip): the
 * positions never return to the host. Files outside the GPU fast path (MODEL records, altlocs,
 * insertion codes, unusual columns or bytes, residues that are not contiguous; pst_pdb_gpu.hip)
 * are parsed by the native host parser instead, with its results and its errors (PST_E_INVALID +
 * the parser's message). Same rows as pst_pdb_parse_files + pst_tokenize_f32, bit for bit.
 * tokens_out [tokens_cap] receives R token slots (raw-offset layout, R = offsets_out[n]; a
 * residue needs >= 55 bytes of file, so sum(file sizes) / 54 + n always suffices; when tokens_cap
 * is smaller than R the call fails with PST_E_INVALID "token buffer too small" and, if offsets_out
 * is given, offsets_out[n] = R so the caller can retry with a buffer of that size),
 * n_tokens_out / n_nodes_out [n] and offsets_out [n+1] may be NULL. */
int pst_tokenize_pdb_files(pst_ctx* ctx, const char* const* paths, int32_t n, int32_t n_threads,
                           uint32_t* tokens_out, int64_t tokens_cap, int32_t* n_tokens_out, int32_t* n_nodes_out,
                           int64_t* offsets_out);
/* files of the last pst_tokenize_pdb_files call that the host parser took (-1: no context) */
int32_t pst_pdb_files_host_parsed(const pst_ctx* ctx);

/* Token-file output of the tokenize loop (scripts/inference_runner.py:313-321 writes one
 * np.save per protein): n whole files written (created / truncated) from host buffers on
 * n_threads threads of libpst's host pool; the caller builds the .npy bytes. PST_E_INVALID if
 * any file could not be written. */
int pst_write_files(int32_t n, const char* const* paths, const void* const* data, const size_t* lens,
                    int32_t n_threads);

/* Per-stage timing of the last tokenize call (HIP events on the context's stream):
 * ms[0..5] = prep, knn, mpnn layer 0, mpnn layer 1, mpnn layer 2, downsampler+FSQ. */
#define PST_N_STAGES 6
int pst_set_timing(pst_ctx* ctx, int32_t enable);
int pst_get_timing(pst_ctx* ctx, float* ms);

/* Clock and occupancy counters of the fused MPNN launches (measurement; bench.py reports them).
 * out[8l + i] for layer l = 0..2, over the calls since the last reset (waits for the context's
 * stream): i = 0, 1: s_memtime (shader clock) and s_memrealtime (100 MHz) deltas of the first wave
 * of workgroup 0 (clock = out[0] / out[1] x 100 MHz; the persistent queue form's waves live as
 * long as the launch); 2: Σ wave lifetimes (100 MHz ticks); 3 / 4: earliest wave start / latest
 * wave end; 5: waves (occupancy = out[2] / (wave slots x (out[4] - out[3]))); 6, 7: 0. reset != 0
 * restarts them after the read. Split-schedule layers (small batches) add nothing. The stamps run
 * only while enabled (pst_set_clock_counters); a context starts with them off, so production
 * launches carry no measurement code path. */
int pst_clock_counters(pst_ctx* ctx, uint64_t* out, int32_t reset);
int pst_set_clock_counters(pst_ctx* ctx, int32_t enable);

/* Stream the context launches on (hipStream_t), for event timing by callers. */
void* pst_stream(pst_ctx* ctx);

/* Debug: copy an intermediate of the LAST call to host.
 *   which = 0..3: node features after init embed / MPNN layer 1..3, [R,128] (raw slot rows)
 *   which = 10:   edge features [R*k, 32] float (27 used), which = 11: senders [R*k] int32
 *   which = 13:   input positions [R,37,3] float32 of the last float32-input call (pst_tokenize_f32,
 *                 pst_tokenize_pdb_batch, pst_tokenize_pdb_files), which = 14: its flags [R,37] u8
 *   which = 20:   int32[20] plan of the last pst_tokenize(_f32) call: [0] copy ranges of its first
 *                 chunk (0 = one copy, the range branch not taken), [1] pipeline chunks C,
 *                 [2 .. 2+C] the chunks' first proteins (and n_prot), [11 .. 11+C-1] each chunk's
 *                 layer schedule (0 fused one wave per task, 1 fused two waves per task, 2 split,
 *                 3 fused as the persistent half-task queue),
 *                 [19] the last chunk's downsampler form (0 one wave per tile, 1 four waves per
 *                 tile, 2 two waves per tile) */
int pst_debug_fetch(pst_ctx* ctx, int32_t which, void* out, size_t bytes);

#ifdef __cplusplus
}
#endif
#endif /* PST_H_ */
