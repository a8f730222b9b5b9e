// pst_kernels.h — kernel argument blocks and launchers (host <-> device contract of libpst).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pst {

// Storage slot of edge feature f (0..26) in the 32-float feature rows k_knn writes. The feature
// GEMMs read slot (r&3) + 8(r>>2) + 4h at k-step r, lane half h (the MFMA k order, half 0 first),
// so the chain visits the real features in the order f0, f4, f1, f5, …, f23 (k-steps 0..11), then
// f24, f25 (k-step 12) and f26 (k-step 13, slot 25; its partner slot 29 is +0): the same order the
// identity layout visited them in, with its zero padding interleaved there. Padding adds +-0
// products, which leave a nonzero chain unchanged, so k-steps 14 and 15 (only padding) are
// skipped with identical results. Slots 26, 27, 29, 30 and 31 hold +0.
__host__ __device__ constexpr int feat_slot(int f) { return f == 25 ? 28 : f == 26 ? 25 : f; }
// the inverse: feature held by slot s, -1 for the zero padding slots
__host__ __device__ constexpr int slot_feat(int s) {
  return s < 25 ? s : s == 25 ? 26 : s == 28 ? 25 : -1;
}
constexpr int FEAT_USED = 27;
// Edge features in HBM, blocked by 32 edges (edge E = receiver slot · 50 + neighbour; a task's
// 50 blocks are consecutive): float4 q of edge E (slots 4q .. 4q+3) sits at float4 index
// feat_f4(E, q) — per block 4 KB as [q >> 1][q & 1][E & 31] — so layer 0's lane (half h, edge e),
// which needs float4s 2i + h (i = 0..3), reads each i as one lane-linear 1 KB load
__host__ __device__ constexpr int feat_f4_q(int q) { return (q >> 1) * 64 + (q & 1) * 32; }
__host__ __device__ constexpr int64_t feat_f4(int64_t E, int q) { return (E >> 5) * 256 + (E & 31) + feat_f4_q(q); }

struct PrepArgs {
  const double* pos;       // [R,37,3]
  const uint8_t* flags;    // [R,37]
  const int64_t* offsets;  // [B+1]
  int32_t* n_nodes;        // [B]
  int32_t* node_local;     // [R_pad] (-1 = gap / padding)
  int32_t* node_prot;      // [R_pad]
  double* frame;           // [R_pad,9] rows n,u,v
  double* cen;             // [R_pad,3]
  double* ca;              // [R_pad,3]
  const float* pos32;      // [R,37,3] float32 positions (pst_tokenize_f32); when set, read instead of pos
  int32_t prot0;           // first protein of this launch (one block per protein from prot0)
};

struct KnnArgs {
  int64_t n_slots;  // R_pad
  const int64_t* offsets;
  const int32_t* n_nodes;
  const int32_t* node_local;
  const int32_t* node_prot;
  const double* frame;
  const double* cen;
  const double* ca;
  int32_t* senders;  // [R_pad*50] global slot of the sender
  int32_t* deg;      // [R_pad] valid slots per receiver
  float* feat;       // [R_pad*50, 32]
  int64_t slot0;     // first slot of this launch (slots slot0 .. n_slots-1, one wave each)
};

struct MlpW {  // one 3-layer MLP on the edge tile; w*: A fragments [64][64] float4, b*: perm
  const float4* w0;  // rows 256..383 of the [384,128] first layer (the edge part)
  const float* b0;
  const float4* w1;
  const float* b1;
  const float4* w2;
  const float* b2;
  const float4* bf1;  // bias fragments [64 lanes] float4 (see tile_gemm_bf)
  const float4* bf2;
};

struct MpnnArgs {
  int64_t n_tasks;  // R_pad / 32
  const int32_t* senders;
  const int32_t* deg;
  const int32_t* node_local;
  // layer 0 only
  const float* feat;       // graph edge features
  const float* Ttab;       // [1023][128] perm: edge PE projection
  const float4* W_embed;   // [16][64] float4: init_edge_embed rows 128..154 (+zero pad)
  const float* b_embed;    // perm (folded into Ttab: unused by the kernel)
  const float* PM0;        // [512][256] perm: h0 · msg0 W[0:128] | W[128:256]
  const float* Utab;       // [1023][128] perm: T · msg0 W[256:384] (layer-0 message)
  const float* V0;         // [512][512][128] perm: (PM0_s[ls] + PM0_r[lr]) + Utab[ls - lr] (k_pair_table)
  const float4* W_msg0f;   // [16][64] float4: init_edge_embed rows 128..154 · msg0 W[256:384]
  const float* h0tab;      // [512][128] perm: init_node_embed(node PE)
  // layers >= 1
  const float* e_in;       // blocked edge features of the previous layer
  const float* P_in;       // [R_pad][512] perm projections [E_s | E_r | M_s | M_r]
  const float* h_in;       // [R_pad][128] perm
  MlpW edge;               // edge MLP of layer-1
  const float* edge_ln_s;
  const float* edge_ln_o;
  // this layer
  MlpW msg;
  const float* ln0_s;
  const float* ln0_o;
  const float* ln1_s;
  const float* ln1_o;
  const float4* ff_w1;  // [4 chunks][64][64]
  const float* ff_b1;   // [4][128] perm
  const float4* ff_w2;  // [4 chunks][64][64]
  const float* ff_b2;
  const float4* proj_w;  // [4][64][64]: next kernel's E_s, E_r, M_s, M_r projections (or null)
  const float4* proj_bf[2];  // bias fragments: first-layer biases the E_r / M_r chains start from
  const float4* ff_bf1;      // [4 chunks][64 lanes] float4 bias fragments
  const float4* ff_bf2;
  float* agg;  // [n_tasks][32][128] scratch: segment sums (perm order)
  // split mode (k_mpnn_edge + k_mpnn_node) when non-null: per-edge messages [E][128] (perm rows)
  float* msg_rows;
  int32_t blocks_per_wave;  // edge blocks of 32 per k_mpnn_edge wave
  int32_t half_tasks;       // fused mode: two waves per task (k_mpnn<L, true>; n_tasks % 4 == 0)
  // fused mode as a persistent half-task queue (k_mpnn_q<L>) when non-null: per-XCD queue heads
  // (8, 64 B apart) and per-task half counters [n_tasks], zeroed before the launch; q_grid =
  // the workgroups the device holds at once
  int32_t* q_head;
  int32_t* q_done;
  int64_t q_grid;
  int32_t q_waves;  // 4 or 8 waves per queue workgroup (k_mpnn_q<L, NW>)
  // unit order within an XCD's queue: groups of q_group tasks, first halves of the group before
  // its second halves (0 = halves of a task adjacent: units 2t, 2t+1)
  int32_t q_group;
  // clock / occupancy stamps (measurement, 8 u64, see ClockStamp and pst_clock_counters); null = off
  unsigned long long* clk;
  // outputs
  float* e_out;  // blocked (null for the last layer)
  float* h_out;
  float* P_out;  // null for the last layer
};

struct DownBlockW {
  const float *qn_s, *qn_o, *dn_s, *dn_o;
  const float4 *wq, *wk, *wv, *wg, *wo;
  const float *gb, *ob;
  const float *rt_ln_s, *rt_ln_o;
  const float4* rt_w1;  // [2][64][64]
  const float* rt_b1;   // [2][128]
  const float4* rt_w2;  // [2][64][64]
  const float* rt_b2;
  const float *ot_ln_s, *ot_ln_o;
  const float4* ot_w1;
  const float* ot_b1;
  const float4* ot_w2;
  const float* ot_b2;
};

struct DownArgs {
  int32_t n_tiles;
  const int32_t* tile_prot;
  const int32_t* tile_t0;
  const int64_t* offsets;
  const int32_t* n_nodes;
  const float* RPE;  // [max_out][128] perm
  float* o_buf;      // [R_pad][128] perm: original track (h3, updated in place)
  float* r_buf;      // [R_pad][128] perm: resampled track
  float* v_buf;      // [R_pad][128] perm: values (DF > 1)
  DownBlockW blk[3];
  const float* down_w;  // [64][64] f32 narrow fragments
  const float* down_b;  // [8]
  int32_t D;
  float fsq_half[8], fsq_off[8], fsq_shift[8];
  int32_t fsq_L[8], fsq_basis[8];
  uint32_t* tokens_out;  // [R] (raw-offset layout)
  float* bounded_out;    // [R,8]
  float* quant_out;      // [R,8]
  float* pre_proj_out;   // [R,128]
};

#define FSQ_AUX_MAX_LO 512  // codes of dims 0..2 (8*8*8 for the 64000 codebook)
#define FSQ_AUX_MAX_HI 128  // codes of dims 3..D-1 (5*5*5)

struct FsqAuxArgs {
  int32_t n_rows_grid;  // n_tiles * 32 (one workgroup per potential token row)
  const int32_t* tile_prot;
  const int32_t* tile_t0;
  const int64_t* offsets;
  const int32_t* n_nodes;
  const int64_t* row_start;  // [B+1] compact output row of each protein's token 0 (k_row_start)
  const float* bounded;      // [Rpad, 8] continuous_embedding, raw-offset rows
  const uint32_t* tokens;    // [R] raw-offset token ids
  int32_t df, D, K, K_lo, K_hi;
  int32_t L[8];
  int32_t basis[8];
  float* dist;         // [T, K] or null
  float* prob;         // [T, K] or null
  uint32_t* argmin;    // [T] or null
  uint32_t* hist;      // [K] (zeroed by the caller) or null
};

// PDB text -> atom37 rows on the GPU (pst_pdb_gpu.hip, pst_tokenize_pdb_files)
struct PdbTables {
  uint32_t atom_key[37];  // atom37 names packed little-endian (stripped, <= 4 characters)
  uint32_t res_key[20];   // the 20 standard residue names, packed
  uint32_t hoh, wat;
  uint8_t exists[21][37];  // residue type x atom37: the atom belongs to the residue (UNK: none)
};
struct PdbScanArgs {
  const char* text;          // all files back to back
  const int64_t* file_off;   // [n+1] byte offsets
  const int64_t* rec_base;   // [n+1] record / residue-run scratch base per file (>= len/54 + 1 each)
  int32_t* line_start;       // [total bytes + n] line starts, file f from file_off[f] + f
  uint8_t* line_kind;        // same indexing
  // records (ATOM / HETATM lines), file f from rec_base[f]
  uint8_t* rec_chain;
  uint8_t* rec_het;          // 0 ATOM, 1 water, 2 other HETATM
  int8_t* rec_atom;          // atom37 index or -1
  int32_t* rec_resseq;
  uint32_t* rec_name;        // residue name, packed
  float* rec_xyz;            // [records][3]
  int32_t* rec_run;          // residue run of the record
  int32_t* run_first;        // first record of each run
  int32_t* run_out;          // kept-residue ordinal of each run (-1: no atom37 atom)
  int8_t* run_type;          // residue type of each run (0..19 the standard ones, 20 UNK)
  int32_t* slot;             // [runs][37] first record of each atom37 name
  int32_t* n_res;            // [n] kept residues
  int32_t* n_run;            // [n]
  int32_t* host_path;        // [n] 1 = outside the fast path: parsed on the host instead
  const int64_t* res_off;    // [n+1] output row of each file's first residue (k_pdb_write)
  float* pos;                // [R,37,3] float32 positions (the tokenizer's input)
  uint8_t* flags;            // [R,37]
  PdbTables tab;
};
void launch_pdb_scan(const PdbScanArgs& a, int n_files, hipStream_t st);
void launch_pdb_write(const PdbScanArgs& a, int n_files, hipStream_t st);

void launch_prep(const PrepArgs& a, int n_prot, hipStream_t st);
void launch_knn(const KnnArgs& a, hipStream_t st);
// node_coop (split schedule only): node update as k_mpnn_node_coop, four waves per 32 receivers
void launch_mpnn(int layer, const MpnnArgs& a, bool node_coop, hipStream_t st);
// coop (df 1 only): one workgroup per tile, the GEMMs split over its four waves (small batches)
// downsampler forms (df 1; df 2/4 always run k_down<df>): one wave per tile (k_down<1>), four
// waves per tile (k_down_coop), two waves per tile, one track each (k_down_pair). Identical bits.
enum { DOWN_ONE_WAVE = 0, DOWN_COOP = 1, DOWN_PAIR = 2 };
void launch_down(int df, const DownArgs& a, int form, hipStream_t st);
void launch_fsq_aux(const FsqAuxArgs& a, int n_prot, hipStream_t st);
// Y = (init or 0) + X·W (+ b): init / b perm-ordered 128-vectors (either may be null)
void launch_pair_table(const float* PM0, const float* U, float* V, hipStream_t st);
void launch_table_gemm(const float* X, int n_rows, const float4* Wf, const float* b, const float* init, float* Y,
                       int ldy, hipStream_t st);

}  // namespace pst
