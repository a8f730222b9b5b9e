// pst_api.cpp — C ABI of libpst (include/pst.h): contexts, weight re-layout, workspace,
// launch sequence. Host code only; kernels live in pst_kernels.hip.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>

#include "../../include/pst.h"
#include "pst_pe.h"
#include "pst_kernels.h"
#include "pst_frag.h"
#include "pst_pool.h"
#include "pst_residue_tables.h"

namespace {
using namespace pst_host;

constexpr int H = 128;
constexpr int KNN = 50;
// MPNN schedule choice (measured on MI355X with tools/split_ab.sh). The fused
// kernel runs one wave per 32-receiver task at 2 waves/SIMD, so its time steps with
// k = ceil(tasks / SIMDs): about k·SIMDs task-units for k >= 2 and 1.1·SIMDs for k = 1 (one
// wave per SIMD runs alone). The split schedule costs about 1.1 units per task (message rows
// through HBM). Split wins below ~1 000 tasks and in the half-empty rounds above.
// 1.05 measured below ~1 000 tasks (tools/policy_check.sh); at 7 680 tasks (960 proteins, the
// last fused round 3/4 full) the split layers ran 49.98 ms against 48.2 ms for the fused layers
// of 8 192 tasks — 1.10 per task (profiles/r02_tail_and_policy.txt) — so 1.1
constexpr double SPLIT_COST_PER_TASK = 1.1;
constexpr double FUSED_SINGLE_ROUND = 1.1;
// A single round more than half full runs the fused layers with two waves per task
// (use_half_tasks): both wave slots of every SIMD busy, about one round of full-size cost plus
// the node update on one wave.
constexpr double FUSED_HALF_ROUND = 1.02;
// Fused layers of more than one round run as a persistent queue of half tasks (k_mpnn_q): the
// unit is 25 edge blocks, so a layer's last units are half as long and its tail half as deep.
constexpr bool MPNN_QUEUE_DEFAULT = true;
// Layers that run as the queue (bit l = layer l) when the queue is on. Round 4 kept layer 0 as
// k_mpnn<0, false> (1 024 / 512 / 256 proteins 8.24-8.30 / 4.15-4.21 / 2.08-2.09 ms against 8.42 /
// 4.34-4.37 / 2.12 ms as the queue, profiles/r04_ab_qgroup.txt); with the wave priorities of round 5
// in both forms the queue wins for layer 0 too: host to host 1 024 proteins 51.99 vs 52.19 ms, 512
// 26.79 vs 26.89, 256 13.96 vs 13.99 (8 interleaved rounds, identical tokens;
// profiles/r06_ab_layer0_queue.txt).
constexpr int64_t MPNN_QUEUE_LAYERS = 7;
bool use_half_tasks(int64_t n_tasks, int64_t n_simds) { return 2 * n_tasks > n_simds && n_tasks <= n_simds; }
bool use_split_schedule(int64_t n_tasks, int64_t n_simds) {
  const int64_t k = (n_tasks + n_simds - 1) / n_simds;
  const double single = use_half_tasks(n_tasks, n_simds) ? FUSED_HALF_ROUND : FUSED_SINGLE_ROUND;
  const double fused = k <= 1 ? single * (double)n_simds : (double)(k * n_simds);
  return SPLIT_COST_PER_TASK * (double)n_tasks < fused;
}

// Downsampler (df 1): a batch of at most this many tiles per SIMD runs k_down_coop (four waves
// per 32-token tile, one wave per SIMD: up to SIMDs/4 tiles in one round) instead of k_down (one
// wave per tile): below that the one-wave kernel leaves most SIMDs idle and its latency is the 20
// sequential GEMMs of one wave. Above it, up to one round of tiles, k_down_pair (two waves per
// tile). Measured (tools/r03_down_forms.sh, profiles/r03_down_forms.jsonl, ms one-wave / coop /
// pair): 128 tiles 0.405 / 0.203 / 0.278; 384 tiles 0.410 / 0.354 / 0.288; 512 0.417 / 0.354 /
// 0.295; 768 0.433 / 0.508 / 0.332; 1024 0.447 / 0.656 / 0.357; 2048 0.626 / 1.253 / 0.726.
constexpr double DOWN_COOP_SIMD_FRACTION = 0.25;
// Split-schedule node update: k_mpnn_node_coop (four waves per 32 receivers) up to this many
// tasks per SIMD, k_mpnn_node (one wave) above.
constexpr double NODE_COOP_SIMD_FRACTION = 0.375;
// Split schedule: one 32-edge block per wave by default. Waves run in rounds of (2 per SIMD)
// slots, so b blocks per wave cost ceil(ceil(B/b)/slots)·b block times — minimal at b = 1
// (measured: 32 proteins 2.75 -> 2.41 ms, CASP14 1.82 -> 1.78 ms vs ~4096 waves of 2-4 blocks;
// tools/edge_waves_sizes.sh). PST_EDGE_WAVES=n targets about n waves instead.
constexpr int64_t SPLIT_EDGE_WAVES = 0;
// Host-buffer calls (pst_tokenize) pipeline the atom37 H2D (≈925 B per residue, ~55 GB/s) with the
// compute (~5 M residues/s) in protein chunks. The fused layers' time steps with
// k = ceil(tasks / SIMDs) (use_split_schedule), so every chunk but the last holds a whole number
// of those rounds — cutting anywhere else adds a round per chunk (bench, 8 192 tasks: an even
// 1:4 split cost 59.2 vs 52.3 ms device-resident). The first chunk is H2D_FIRST_ROUNDS rounds
// (its copy is the only exposed one; one round runs two waves per task, use_half_tasks); each
// next chunk is at most H2D_GROWTH times the previous (the copy runs ~12x faster than the
// compute, so chunk k+1's copy hides under chunk k). No pipeline below H2D_MIN_ROUNDS rounds in
// all. Measured at 8 rounds (tools/r02_first.sh): chunks of 1+7 rounds 54.0-54.2 ms, 2+6
// 54.9-55.0, 3+5 56.1-56.8, 1+3+4 54.9-55.3, 1+2+4+1 55.2-55.8.
constexpr int H2D_MAX_CHUNKS = 8;
// The first chunk's copy is the exposed one: it is issued as H2D_GRAPH_RANGES protein ranges of
// about equal residues, and each range's k_prep + k_knn start when that range has landed
// (GraphRanges), so the graph of the first ranges runs under the copy of the later ones.
constexpr int64_t H2D_GRAPH_RANGES = 4;
constexpr int64_t H2D_FIRST_ROUNDS = 1;
constexpr int64_t H2D_GROWTH = 8;
// With float64 positions 2 / 3 rounds gained from the pipeline (15.2-15.3 -> 14.9-15.0 / 22.4-22.7 ->
// 21.2-21.4 ms); with the float32 wire format and graph ranges 2 rounds run better unpipelined
// (256 proteins 14.56 -> 14.31-14.40 ms), 4 rounds still gain (512: 28.09-28.16 -> 27.95-28.05 ms,
// 1024: 54.8 -> 53.8 ms; profiles/r02_h2d_policy_f32.txt)
constexpr int64_t H2D_MIN_ROUNDS = 3;

// Schedule thresholds from the environment, read once per context: -2 = not read yet, -1 = unset
// (use the cost model), >= 0 = the override.
void env_threshold(int64_t& v, const char* name) {
  if (v != -2) return;
  const char* e = getenv(name);
  v = e ? std::max<int64_t>(0, atoll(e)) : -1;
}

thread_local std::string g_create_error;


// float index of slot `slot` of edge e in the blocked feature layout (pst::feat_f4), and the floats
// that n_edges edges occupy (whole 32-edge blocks)
inline size_t feat_float(size_t e, int slot) { return (size_t)pst::feat_f4((int64_t)e, slot >> 2) * 4 + (slot & 3); }
inline size_t feat_floats(size_t n_edges) { return (n_edges + 31) / 32 * 32 * 32; }

// ------------------------------------------------------------------ parameter views
struct Lin {
  const float* w;
  const float* b;
};
struct Layer {
  Lin msg[3], ff[2], edge[3];
  const float *ln_s[3], *ln_o[3];
};
struct HostParams {
  Lin node_embed, edge_embed;
  Layer L[3];
  const float *qn_s, *qn_o, *dn_s, *dn_o, *qw, *kw, *vw, *gw, *gb, *ow, *ob;
  const float *rt_ln_s, *rt_ln_o, *rt_w1, *rt_b1, *rt_w2, *rt_b2;
  const float *ot_ln_s, *ot_ln_o, *ot_w1, *ot_b1, *ot_w2, *ot_b2;
  Lin down;
};

size_t walk(const float* base, int D, HostParams* P) {
  size_t o = 0;
  auto take = [&](size_t n) {
    const float* r = base ? base + o : nullptr;
    o += n;
    return r;
  };
  P->node_embed = {take(H * H), take(H)};
  P->edge_embed = {take((H + 27) * H), take(H)};
  for (int l = 0; l < 3; ++l) {
    Layer& m = P->L[l];
    m.msg[0] = {take(3 * H * H), take(H)};
    m.msg[1] = {take(H * H), take(H)};
    m.msg[2] = {take(H * H), take(H)};
    m.ff[0] = {take(H * 4 * H), take(4 * H)};
    m.ff[1] = {take(4 * H * H), take(H)};
    m.edge[0] = {take(3 * H * H), take(H)};
    m.edge[1] = {take(H * H), take(H)};
    m.edge[2] = {take(H * H), take(H)};
    for (int i = 0; i < 3; ++i) {
      m.ln_s[i] = take(H);
      m.ln_o[i] = take(H);
    }
  }
  P->qn_s = take(3 * H); P->qn_o = take(3 * H);
  P->dn_s = take(3 * H); P->dn_o = take(3 * H);
  P->qw = take(3 * H * H); P->kw = take(3 * H * H); P->vw = take(3 * H * H);
  P->gw = take(3 * H * H); P->gb = take(3 * H);
  P->ow = take(3 * H * H); P->ob = take(3 * H);
  P->rt_ln_s = take(3 * H); P->rt_ln_o = take(3 * H);
  P->rt_w1 = take(3 * H * 2 * H); P->rt_b1 = take(3 * 2 * H);
  P->rt_w2 = take(3 * 2 * H * H); P->rt_b2 = take(3 * H);
  P->ot_ln_s = take(3 * H); P->ot_ln_o = take(3 * H);
  P->ot_w1 = take(3 * H * 2 * H); P->ot_b1 = take(3 * 2 * H);
  P->ot_w2 = take(3 * 2 * H * H); P->ot_b2 = take(3 * H);
  P->down = {take((size_t)H * D), take(D)};
  return o;
}

// ------------------------------------------------------------------ device re-layout
// Everything device-side lives in one arena; builders append and return element offsets.
struct Arena {
  std::vector<float> h;
  size_t add(const std::vector<float>& v) {
    size_t o = h.size();
    h.insert(h.end(), v.begin(), v.end());
    while (h.size() % 64) h.push_back(0.0f);  // 256-B alignment for every array
    return o;
  }
};






std::vector<float> cat(std::initializer_list<std::vector<float>> parts) {
  std::vector<float> out;
  for (auto& p : parts) out.insert(out.end(), p.begin(), p.end());
  return out;
}

// positional_encoding_layer.py:49-66 with a float32 argument
struct MlpOff {
  size_t w0, b0, w1, b1, w2, b2, bf0, bf1, bf2;
};
struct LayerOff {
  MlpOff msg, edge;
  size_t ff_w1, ff_b1, ff_w2, ff_b2, ff_bf1, ff_bf2, proj;  // proj: filled per kernel
  size_t ln_s[3], ln_o[3];
};
struct BlockOff {
  size_t qn_s, qn_o, dn_s, dn_o, wq, wk, wv, wg, wo, gb, ob;
  size_t rt_ln_s, rt_ln_o, rt_w1, rt_b1, rt_w2, rt_b2;
  size_t ot_ln_s, ot_ln_o, ot_w1, ot_b1, ot_w2, ot_b2;
};

}  // namespace

// ------------------------------------------------------------------ context
struct pst_ctx {
  int device = 0;
  pst_model_desc desc{};
  int D = 6, df = 1, max_out = 512;
  hipStream_t stream = nullptr;
  std::string err;
  // weights arena (device) + offsets
  float* d_arena = nullptr;
  size_t emb_w = 0, emb_b = 0, w_msg0f = 0;
  LayerOff L[3]{};
  size_t proj[2]{};
  BlockOff B[3]{};
  size_t down_w = 0, down_b = 0;
  // tables (device, separate allocations)
  float *d_h0 = nullptr, *d_PM0 = nullptr, *d_T = nullptr, *d_U = nullptr, *d_RPE = nullptr;
  float* d_V0 = nullptr;  // [512][512][128]: layer 0's per-(receiver, sender) message chain start
  float fsq_half[8]{}, fsq_off[8]{}, fsq_shift[8]{};
  int fsq_L[8]{}, fsq_basis[8]{};
  // workspace (grow-only)
  int64_t cap_R = 0;
  int cap_B = 0;
  void* ws = nullptr;
  size_t ws_bytes = 0;
  // per-call layout
  int64_t last_R = 0, last_Rpad = 0;
  int last_B = 0;
  struct {
    int64_t* offsets;
    int32_t *n_nodes, *node_local, *node_prot, *senders, *deg, *tile_prot, *tile_t0;
    double *frame, *cen, *ca;
    float *feat, *e0, *e1, *h0, *h1, *P0, *P1, *agg, *r_buf, *v_buf, *bounded, *quant, *pre_proj;
    double* pos;
    uint8_t* flags;
    uint32_t* tokens;
    int32_t* n_tok;
    int64_t* row_start;
    int32_t* qctr;  // k_mpnn_q's counters, per layer: [8 heads x 16] + [n_tasks]
  } w{};
  // last call's outputs the aux kernels read (device; the caller's buffers for pst_tokenize_device)
  const uint32_t* last_tokens = nullptr;
  const int32_t* last_nnodes = nullptr;
  int32_t last_ntiles = 0;
  // grow-only scratch of pst_codebook_aux (host variant)
  void* aux = nullptr;
  size_t aux_bytes = 0;
  // grow-only per-edge message rows of the split MPNN mode (small batches only)
  float* msg = nullptr;
  size_t msg_bytes = 0;
  int64_t split_tasks = -2;  // PST_SPLIT_TASKS: split iff n_tasks <= this; -1 = cost model; -2 = not read yet
  int64_t n_simds = 1024;    // 4 x compute units of the device
  int64_t edge_waves = -2;   // PST_EDGE_WAVES: split-schedule edge waves target; -1 = SPLIT_EDGE_WAVES
  int64_t node_coop = -2;    // PST_NODE_COOP: k_mpnn_node_coop iff split and n_tasks <= this; -1 = default
  int64_t down_coop = -2;    // PST_DOWN_COOP: k_down_coop iff n_tiles <= this; -1 = default; -2 = not read yet
  int64_t down_pair = -2;    // PST_DOWN_PAIR: 1 = k_down_pair whenever not coop (df 1), 0 = never; -1 = one round of tiles
  int32_t* h_counts = nullptr;  // pinned host copy of [n_tok | n_nodes] (cap_B each)
  uint32_t* h_tokens = nullptr;  // pinned landing buffer of the token D2H (cap_R)
  int32_t last_down_form = 0;  // pst::DOWN_* of the last run (pst_debug_fetch 20, plan[19])
  int64_t half_tasks = -2;   // PST_HALF_TASKS: 1 = fused layers always two waves per task, 0 = never; -1 = policy
  int64_t mpnn_qwaves = -2;  // PST_MPNN_QWAVES: 4 = two 4-wave queue workgroups per CU; else one 8-wave workgroup
                             // per CU with all of W1 in LDS (k_mpnn<0..2> -1.0..-2.8 %, profiles/r04_ab_qwaves.txt)
  int64_t pdb_gpu_max_file = -2;  // PST_PDB_GPU_MAX_FILE: bytes; a file this large sends the call to the host parser
  int64_t mpnn_qgroup = -2;  // PST_MPNN_QGROUP: queue unit order, tasks per group (0 = halves adjacent); -1 = wave slots per XCD
  int64_t mpnn_queue_layers = -2;  // PST_MPNN_QUEUE_LAYERS: layer mask of the queue form; -1 = MPNN_QUEUE_LAYERS
  int64_t mpnn_queue = -2;   // PST_MPNN_QUEUE: 1 = fused layers as the half-task queue (k_mpnn_q) whenever not
                             // k_mpnn<L, true>, 0 = never (k_mpnn<L, false>); -1 = policy
  std::vector<int64_t> h_offsets;
  // pst_tokenize's H2D pipeline: proteins copied in chunks on copy_stream, chunk k+1's copy
  // overlapping chunk k's compute on `stream` (H2D_MAX_CHUNKS events)
  hipStream_t copy_stream = nullptr;
  hipStream_t copy_stream2 = nullptr;  // odd graph ranges of the first chunk (PST_H2D_COPY_STREAMS=2)
  int64_t h2d_streams = -2;            // PST_H2D_COPY_STREAMS: copy streams for the graph ranges (1 or 2)
  hipEvent_t copy_ev[8] = {};
  int64_t h2d_chunks = -2;  // PST_H2D_CHUNKS: force the chunk count (1 = no pipeline); -1 = policy
  int64_t h2d_first = -2;   // PST_H2D_FIRST_ROUNDS: rounds in the first pipelined chunk; -1 = H2D_FIRST_ROUNDS
  int64_t h2d_growth = -2;  // PST_H2D_GROWTH: chunk-size growth factor; -1 = H2D_GROWTH
  int64_t h2d_min = -2;     // PST_H2D_MIN_ROUNDS: no pipeline below this many rounds; -1 = H2D_MIN_ROUNDS
  int64_t h2d_ranges = -2;  // PST_H2D_GRAPH_RANGES: copy ranges of the first chunk (1 = one copy); -1 = H2D_GRAPH_RANGES
  hipEvent_t range_ev[8] = {};  // one per copy range of the first chunk (GraphRanges)
  hipEvent_t idle_ev = nullptr; // recorded on `stream` before copy_stream overwrites the inputs
  bool chunked_last = false; // last call was pipelined: per-layer debug intermediates hold its last chunk only
  // last host call's plan (pst_debug_fetch 20): [0] copy ranges of its first chunk (0 = one copy),
  // [1] chunks, [2..10] protein cuts of the chunks, [11..18] each chunk's layer schedule
  // (0 fused one wave per task, 1 fused two waves per task, 2 split), [19] the last chunk's
  // downsampler form (pst::DOWN_*)
  int32_t last_plan[20] = {};
  int32_t last_sched = 0;  // schedule of the last run()
  float* dbg[3] = {nullptr, nullptr, nullptr};  // PST_DEBUG=1: node features after each layer
  // optional per-stage timing (HIP events on ctx->stream)
  bool timing = false;
  hipEvent_t ev[PST_N_STAGES + 1] = {};
  int64_t dbg_cap = 0;
  // clock stamps of the fused MPNN launches (pst_clock_counters): per layer 8 u64 — [shader cycles,
  // 100 MHz ticks] of the stamping wave, Σ wave lifetimes, min wave start, max wave end, waves —
  // summed over calls (min / max over calls)
  unsigned long long* d_clk = nullptr;
  // page-locked staging of pst_tokenize_pdb_batch (grow-only): positions [R,37,3] f32, flags [R,37]
  float* h_stage_pos = nullptr;
  uint8_t* h_stage_flags = nullptr;
  int64_t h_stage_cap = 0;
  // pst_tokenize_pdb_files (grow-only): page-locked file text, device scratch of the GPU parse,
  // page-locked per-file counts
  char* h_text = nullptr;
  size_t h_text_cap = 0;
  void* d_pdb = nullptr;
  size_t d_pdb_cap = 0;
  int32_t* h_pdb_counts = nullptr;
  int64_t h_pdb_counts_cap = 0;
  int32_t last_pdb_host_files = 0;  // files of the last pst_tokenize_pdb_files the host parser took
  bool clock_on = false;  // pst_set_clock_counters: stamp the fused MPNN launches (off by default)
};

namespace {
int reset_clock_counters(pst_ctx* ctx);  // below (pst_clock_counters)

inline void mark(pst_ctx* ctx, int i) {
  if (ctx->timing) (void)hipEventRecord(ctx->ev[i], ctx->stream);
}

#define HIPCHK(x)                                                                   \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      ctx->err = std::string(#x) + ": " + hipGetErrorString(e_);                    \
      return PST_E_HIP;                                                             \
    }                                                                               \
  } while (0)

int fail(pst_ctx* ctx, int code, const std::string& msg) {
  ctx->err = msg;
  return code;
}

int build_weights(pst_ctx* ctx, const float* blob) {
  HostParams P;
  walk(blob, ctx->D, &P);
  Arena A;
  // the feature rows of the edge embedding and of layer 0's message factor in the slot order of
  // the features k_knn writes (pst::feat_slot; unused slots zero)
  auto slot_rows = [&](const float* W) {
    std::vector<float> S((size_t)32 * H, 0.0f);
    for (int f = 0; f < pst::FEAT_USED; ++f)
      std::copy(W + (size_t)f * H, W + (size_t)(f + 1) * H, S.begin() + (size_t)pst::feat_slot(f) * H);
    return S;
  };
  ctx->emb_w = A.add(frag(slot_rows(P.edge_embed.w + (size_t)128 * H).data(), H, 0, 32, 32, 0, 128));
  ctx->emb_b = A.add(perm(P.edge_embed.b));
  {
    // layer-0 message over the embedding's feature factor: Wm[f] = Wf[f] · msg0
    // W[256:384], each output an fmaf chain over the 128 channels in the canonical k order (the
    // oracle computes the same chain)
    const float* Wc = P.L[0].msg[0].w + (size_t)256 * H;
    std::vector<float> Wm((size_t)32 * H, 0.0f);
    for (int f = 0; f < 27; ++f) {
      const float* wf = P.edge_embed.w + (size_t)(128 + f) * H;
      for (int o = 0; o < H; ++o) {
        float acc = 0.0f;
        for (int t = 0; t < H; ++t) {
          const int k = pi8(t);
          acc = std::fmaf(wf[k], Wc[(size_t)k * H + o], acc);
        }
        Wm[(size_t)f * H + o] = acc;
      }
    }
    ctx->w_msg0f = A.add(frag(slot_rows(Wm.data()).data(), H, 0, 32, 32, 0, 128));
  }
  for (int l = 0; l < 3; ++l) {
    const Layer& S = P.L[l];
    LayerOff& O = ctx->L[l];
    // The GEMMs that consume a GELU output (MLP layers 1 and 2 — for the message MLP, layer 2
    // runs on the segment sums of GELU outputs — and the FFN's second layer) get their weights
    // scaled by 0.5: the kernels evaluate 2·GELU in one fma less (c_gelu2x, pst_device.h), and
    // (2g)·(w/2) = g·w exactly, so every chain is the canonical one the oracle computes
    auto half = [](std::vector<float> v) {
      for (float& x : v) x *= 0.5f;
      return v;
    };
    auto mlp = [&](const Lin* m, MlpOff& o) {
      o.w0 = A.add(frag(m[0].w, H, 256, 128, 128, 0, 128));
      o.b0 = A.add(perm(m[0].b));
      o.w1 = A.add(half(frag(m[1].w, H, 0, 128, 128, 0, 128)));
      o.b1 = A.add(perm(m[1].b));
      o.w2 = A.add(half(frag(m[2].w, H, 0, 128, 128, 0, 128)));
      o.b2 = A.add(perm(m[2].b));
      o.bf0 = A.add(bfrag(m[0].b));
      o.bf1 = A.add(bfrag(m[1].b));
      o.bf2 = A.add(bfrag(m[2].b));
    };
    mlp(S.msg, O.msg);
    mlp(S.edge, O.edge);
    std::vector<float> w1, b1, w2, bf1;
    for (int ck = 0; ck < 4; ++ck) {
      auto bfr = bfrag(S.ff[0].b + 128 * ck);
      bf1.insert(bf1.end(), bfr.begin(), bfr.end());
      auto f = frag(S.ff[0].w, 4 * H, 0, 128, 128, 128 * ck, 128);
      w1.insert(w1.end(), f.begin(), f.end());
      auto bp = perm(S.ff[0].b + 128 * ck);
      b1.insert(b1.end(), bp.begin(), bp.end());
      auto g = half(frag(S.ff[1].w, H, 128 * ck, 128, 128, 0, 128));
      w2.insert(w2.end(), g.begin(), g.end());
    }
    O.ff_w1 = A.add(w1);
    O.ff_b1 = A.add(b1);
    O.ff_w2 = A.add(w2);
    O.ff_b2 = A.add(perm(S.ff[1].b));
    O.ff_bf1 = A.add(bf1);
    O.ff_bf2 = A.add(bfrag(S.ff[1].b));
    for (int i = 0; i < 3; ++i) {
      O.ln_s[i] = A.add(perm(S.ln_s[i]));
      O.ln_o[i] = A.add(perm(S.ln_o[i]));
    }
  }
  // projections produced by kernel l for kernel l+1: [E_s, E_r] (edge MLP of layer l),
  // [M_s, M_r] (message MLP of layer l+1): first-layer rows 0..127 / 128..255; the receiver
  // parts chain from the first-layer bias (k_mpnn node phase)
  for (int l = 0; l < 2; ++l) {
    const Layer& S = P.L[l];
    const Layer& N = P.L[l + 1];
    ctx->proj[l] = A.add(cat({frag(S.edge[0].w, H, 0, 128, 128, 0, 128), frag(S.edge[0].w, H, 128, 128, 128, 0, 128),
                              frag(N.msg[0].w, H, 0, 128, 128, 0, 128), frag(N.msg[0].w, H, 128, 128, 128, 0, 128)}));
  }
  for (int b = 0; b < 3; ++b) {
    BlockOff& O = ctx->B[b];
    const size_t v = (size_t)b * H, m = (size_t)b * H * H;
    O.qn_s = A.add(perm(P.qn_s + v)); O.qn_o = A.add(perm(P.qn_o + v));
    O.dn_s = A.add(perm(P.dn_s + v)); O.dn_o = A.add(perm(P.dn_o + v));
    O.wq = A.add(frag(P.qw + m, H, 0, 128, 128, 0, 128));
    O.wk = A.add(frag(P.kw + m, H, 0, 128, 128, 0, 128));
    O.wv = A.add(frag(P.vw + m, H, 0, 128, 128, 0, 128));
    O.wg = A.add(frag(P.gw + m, H, 0, 128, 128, 0, 128));
    O.gb = A.add(perm(P.gb + v));
    O.wo = A.add(frag(P.ow + m, H, 0, 128, 128, 0, 128));
    O.ob = A.add(perm(P.ob + v));
    auto trans = [&](const float* ln_s, const float* ln_o, const float* w1, const float* b1, const float* w2,
                     const float* b2, size_t& s, size_t& o, size_t& W1, size_t& B1, size_t& W2, size_t& B2) {
      s = A.add(perm(ln_s + v));
      o = A.add(perm(ln_o + v));
      const float* w1b = w1 + (size_t)b * H * 2 * H;
      const float* w2b = w2 + (size_t)b * 2 * H * H;
      W1 = A.add(cat({frag(w1b, 2 * H, 0, 128, 128, 0, 128), frag(w1b, 2 * H, 0, 128, 128, 128, 128)}));
      B1 = A.add(cat({perm(b1 + (size_t)b * 2 * H), perm(b1 + (size_t)b * 2 * H + 128)}));
      W2 = A.add(cat({frag(w2b, H, 0, 128, 128, 0, 128), frag(w2b, H, 128, 128, 128, 0, 128)}));
      B2 = A.add(perm(b2 + v));
    };
    trans(P.rt_ln_s, P.rt_ln_o, P.rt_w1, P.rt_b1, P.rt_w2, P.rt_b2, O.rt_ln_s, O.rt_ln_o, O.rt_w1, O.rt_b1, O.rt_w2,
          O.rt_b2);
    trans(P.ot_ln_s, P.ot_ln_o, P.ot_w1, P.ot_b1, P.ot_w2, P.ot_b2, O.ot_ln_s, O.ot_ln_o, O.ot_w1, O.ot_b1, O.ot_w2,
          O.ot_b2);
  }
  ctx->down_w = A.add(frag_narrow(P.down.w, ctx->D, ctx->D));
  std::vector<float> db(64, 0.0f);
  for (int d = 0; d < ctx->D; ++d) db[d] = P.down.b[d];
  ctx->down_b = A.add(db);
  // staging inputs for the table GEMMs
  auto nodePE = perm_rows(pst::pe_rows(0, 512, 512), 512);
  auto edgePE = perm_rows(pst::pe_rows(-511, 1023, 512), 1023);
  auto rpe = perm_rows(pst::pe_rows(0, ctx->max_out, ctx->max_out), ctx->max_out);
  size_t o_npe = A.add(nodePE), o_epe = A.add(edgePE);
  size_t o_ne_w = A.add(frag(P.node_embed.w, H, 0, 128, 128, 0, 128)), o_ne_b = A.add(perm(P.node_embed.b));
  size_t o_ee_w = A.add(frag(P.edge_embed.w, H, 0, 128, 128, 0, 128));
  size_t o_m0s = A.add(frag(P.L[0].msg[0].w, H, 0, 128, 128, 0, 128));
  size_t o_m0r = A.add(frag(P.L[0].msg[0].w, H, 128, 128, 128, 0, 128));

  HIPCHK(hipMalloc(&ctx->d_arena, A.h.size() * sizeof(float)));
  HIPCHK(hipMemcpy(ctx->d_arena, A.h.data(), A.h.size() * sizeof(float), hipMemcpyHostToDevice));
  HIPCHK(hipMalloc(&ctx->d_h0, 512 * 128 * sizeof(float)));
  HIPCHK(hipMalloc(&ctx->d_PM0, 512 * 256 * sizeof(float)));
  HIPCHK(hipMalloc(&ctx->d_T, 1023 * 128 * sizeof(float)));
  HIPCHK(hipMalloc(&ctx->d_U, 1023 * 128 * sizeof(float)));
  HIPCHK(hipMalloc(&ctx->d_V0, (size_t)512 * 512 * 128 * sizeof(float)));
  HIPCHK(hipMalloc(&ctx->d_RPE, (size_t)ctx->max_out * 128 * sizeof(float)));
  HIPCHK(hipMemcpy(ctx->d_RPE, rpe.data(), rpe.size() * sizeof(float), hipMemcpyHostToDevice));
  HIPCHK(hipMalloc(&ctx->d_clk, 24 * sizeof(unsigned long long)));
  if (int rc = reset_clock_counters(ctx)) return rc;
  float* a = ctx->d_arena;
  auto F4 = [&](size_t o) { return reinterpret_cast<const float4*>(a + o); };
  // h0 = nodePE·W + b; PM0 = [h0·W0[0:128] | b0 + h0·W0[128:256]] (message MLP of layer 0);
  // T = b + edgePE·W[0:128] (the edge embedding's bias is folded into its table)
  pst::launch_table_gemm(a + o_npe, 512, F4(o_ne_w), a + o_ne_b, nullptr, ctx->d_h0, 128, ctx->stream);
  pst::launch_table_gemm(ctx->d_h0, 512, F4(o_m0s), nullptr, nullptr, ctx->d_PM0, 256, ctx->stream);
  pst::launch_table_gemm(ctx->d_h0, 512, F4(o_m0r), nullptr, a + ctx->L[0].msg.b0, ctx->d_PM0 + 128, 256, ctx->stream);
  pst::launch_table_gemm(a + o_epe, 1023, F4(o_ee_w), nullptr, a + ctx->emb_b, ctx->d_T, 128, ctx->stream);
  // U = T · msg0 W[256:384]: the edge-PE half of layer 0's message first layer
  pst::launch_table_gemm(ctx->d_T, 1023, F4(ctx->L[0].msg.w0), nullptr, nullptr, ctx->d_U, 128, ctx->stream);
  // V0 = (PM0_s[ls] + PM0_r[lr]) + U[ls - lr] per (lr, ls): 128 MB, one row per layer-0 edge
  pst::launch_pair_table(ctx->d_PM0, ctx->d_U, ctx->d_V0, ctx->stream);
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(ctx->stream));
  // FSQ constants (quantize.py:175-181, computed in float32 as JAX does)
  uint32_t basis = 1;
  for (int d = 0; d < ctx->D; ++d) {
    int L = ctx->desc.levels[d];
    float half_l = ((float)(L - 1) * 0.999f) / 2.0f;
    float off = (L % 2 == 0) ? 0.5f : 0.0f;
    ctx->fsq_half[d] = half_l;
    ctx->fsq_off[d] = off;
    ctx->fsq_shift[d] = (float)std::tan((double)(off / half_l));
    ctx->fsq_L[d] = L;
    ctx->fsq_basis[d] = (int)basis;
    basis *= (uint32_t)L;
  }
  return PST_OK;
}

int ensure_workspace(pst_ctx* ctx, int64_t R, int B) {
  int64_t Rpad = (R + 127) / 128 * 128;
  if (Rpad <= ctx->cap_R && B <= ctx->cap_B) return PST_OK;
  Rpad = std::max<int64_t>(Rpad, ctx->cap_R);
  B = std::max(B, ctx->cap_B);
  if (ctx->ws) (void)hipFree(ctx->ws);
  ctx->ws = nullptr;
  size_t E = (size_t)Rpad * KNN;
  struct Item {
    void** p;
    size_t bytes;
  };
  auto& w = ctx->w;
  std::vector<Item> items = {
      {(void**)&w.offsets, sizeof(int64_t) * (B + 1)},   {(void**)&w.n_tok, sizeof(int32_t) * 2 * B},
      {(void**)&w.tile_prot, sizeof(int32_t) * (Rpad / 32 + B)},
      {(void**)&w.tile_t0, sizeof(int32_t) * (Rpad / 32 + B)},
      {(void**)&w.node_local, sizeof(int32_t) * Rpad}, {(void**)&w.node_prot, sizeof(int32_t) * Rpad},
      {(void**)&w.senders, sizeof(int32_t) * E},        {(void**)&w.deg, sizeof(int32_t) * Rpad},
      {(void**)&w.frame, sizeof(double) * 9 * Rpad},    {(void**)&w.cen, sizeof(double) * 3 * Rpad},
      {(void**)&w.ca, sizeof(double) * 3 * Rpad},       {(void**)&w.feat, sizeof(float) * 32 * E},
      {(void**)&w.e0, sizeof(float) * 128 * E},         {(void**)&w.e1, sizeof(float) * 128 * E},
      {(void**)&w.h0, sizeof(float) * 128 * Rpad},      {(void**)&w.agg, sizeof(float) * 128 * Rpad},      {(void**)&w.h1, sizeof(float) * 128 * Rpad},
      {(void**)&w.P0, sizeof(float) * 512 * Rpad},      {(void**)&w.P1, sizeof(float) * 512 * Rpad},
      {(void**)&w.r_buf, sizeof(float) * 128 * Rpad},   {(void**)&w.v_buf, sizeof(float) * 128 * Rpad},
      {(void**)&w.bounded, sizeof(float) * 8 * Rpad},   {(void**)&w.quant, sizeof(float) * 8 * Rpad},
      {(void**)&w.pre_proj, sizeof(float) * 128 * Rpad}, {(void**)&w.pos, sizeof(double) * 37 * 3 * Rpad},
      {(void**)&w.flags, sizeof(uint8_t) * 37 * Rpad},  {(void**)&w.tokens, sizeof(uint32_t) * Rpad},
      {(void**)&w.row_start, sizeof(int64_t) * (B + 1)},
      {(void**)&w.qctr, sizeof(int32_t) * 3 * (128 + Rpad / 32)},
  };
  size_t total = 0;
  for (auto& it : items) total += (it.bytes + 4095) / 4096 * 4096;
  hipError_t e = hipMalloc(&ctx->ws, total);
  if (e != hipSuccess) {
    ctx->ws = nullptr;
    ctx->cap_R = 0;
    ctx->cap_B = 0;
    return fail(ctx, PST_E_NOMEM, std::string("workspace allocation failed: ") + hipGetErrorString(e));
  }
  char* p = (char*)ctx->ws;
  for (auto& it : items) {
    *it.p = p;
    p += (it.bytes + 4095) / 4096 * 4096;
  }
  // the per-protein counts side by side, [n_tok (B) | n_nodes (B)]: one D2H for both
  w.n_nodes = w.n_tok + B;
  if (ctx->h_counts) (void)hipHostFree(ctx->h_counts);
  ctx->h_counts = nullptr;
  if (hipHostMalloc((void**)&ctx->h_counts, sizeof(int32_t) * 2 * B) != hipSuccess) ctx->h_counts = nullptr;
  if (ctx->h_tokens) (void)hipHostFree(ctx->h_tokens);
  ctx->h_tokens = nullptr;
  if (hipHostMalloc((void**)&ctx->h_tokens, sizeof(uint32_t) * Rpad) != hipSuccess) ctx->h_tokens = nullptr;
  ctx->ws_bytes = total;
  const char* dbg = getenv("PST_DEBUG");
  if (dbg && dbg[0] == '1') {
    for (int l = 0; l < 3; ++l) {
      if (ctx->dbg[l]) (void)hipFree(ctx->dbg[l]);
      if (hipMalloc(&ctx->dbg[l], sizeof(float) * 128 * Rpad) != hipSuccess) ctx->dbg[l] = nullptr;
    }
  }
  ctx->cap_R = Rpad;
  ctx->cap_B = B;
  return PST_OK;
}

// clock / occupancy counters (pst_clock_counters) to their start values: sums 0, min start ~0
int reset_clock_counters(pst_ctx* ctx) {
  uint64_t init[24] = {};
  for (int l = 0; l < 3; ++l) init[8 * l + 3] = ~0ull;
  HIPCHK(hipMemcpyAsync(ctx->d_clk, init, sizeof(init), hipMemcpyHostToDevice, ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  return PST_OK;
}

int validate(pst_ctx* ctx, const int64_t* offsets, int32_t n_prot) {
  if (n_prot <= 0 || !offsets) return fail(ctx, PST_E_INVALID, "empty batch");
  if (offsets[0] != 0) return fail(ctx, PST_E_INVALID, "prot_offsets[0] must be 0");
  for (int b = 0; b < n_prot; ++b) {
    int64_t r = offsets[b + 1] - offsets[b];
    if (r < 0) return fail(ctx, PST_E_INVALID, "prot_offsets must be non-decreasing");
    if (r > ctx->desc.seq_max_size)
      return fail(ctx, PST_E_TOO_LARGE,
                  "We currently don't support protein with more than " + std::to_string(ctx->desc.seq_max_size) +
                      " residues given: " + std::to_string(r));
    if (r < ctx->desc.graph_max_neighbor)
      return fail(ctx, PST_E_TOO_SMALL,
                  "We currently don't support protein with less than " +
                      std::to_string(ctx->desc.graph_max_neighbor) + " residues given: " + std::to_string(r));
  }
  return PST_OK;
}

// Per-protein token tiles of 32 (upper bound from the raw residue counts) → w.tile_prot/tile_t0,
// and the batch offsets → w.offsets (stream-ordered uploads)
int upload_batch_meta(pst_ctx* ctx, const int64_t* offsets, int32_t n_prot, int32_t* n_tiles) {
  auto& w = ctx->w;
  hipStream_t st = ctx->stream;
  std::vector<int32_t> tp, tt;
  for (int b = 0; b < n_prot; ++b) {
    int64_t Tmax = (offsets[b + 1] - offsets[b]) / ctx->df;
    for (int64_t t0 = 0; t0 < Tmax; t0 += 32) {
      tp.push_back(b);
      tt.push_back((int32_t)t0);
    }
  }
  ctx->h_offsets.assign(offsets, offsets + n_prot + 1);
  HIPCHK(hipMemcpyAsync(w.offsets, ctx->h_offsets.data(), sizeof(int64_t) * (n_prot + 1), hipMemcpyHostToDevice, st));
  if (!tp.empty()) {
    HIPCHK(hipMemcpyAsync(w.tile_prot, tp.data(), sizeof(int32_t) * tp.size(), hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(w.tile_t0, tt.data(), sizeof(int32_t) * tt.size(), hipMemcpyHostToDevice, st));
  }
  *n_tiles = (int32_t)tp.size();
  return PST_OK;
}

// One batch (or one chunk of a pipelined batch) through graph → encoder → downsampler/FSQ on
// ctx->stream. `out_row0`: raw residue row of offsets[0] in the caller's batch, where the
// raw-layout aux outputs (bounded, quantize, pre_proj) of this batch go.
// Protein sub-ranges of one run() whose inputs land separately (pst_tokenize's H2D pipeline):
// the graph kernels of range k (proteins cut[k] .. cut[k+1]-1) wait for ev[k] only, so they run
// while the copies of the later ranges are still in flight.
struct GraphRanges {
  int n;
  const int32_t* cut;  // [n+1], cut[0] = 0, cut[n] = n_prot
  const hipEvent_t* ev;
};

// `d_pos32`: float32 positions (pst_tokenize_f32), read by k_prep instead of d_pos when set.
int run(pst_ctx* ctx, const double* d_pos, const uint8_t* d_flags, const int64_t* offsets, int32_t n_prot,
        uint32_t* d_tokens, int32_t* d_ntok, int32_t* d_nnodes, bool graph_only = false, int64_t out_row0 = 0,
        const float* d_pos32 = nullptr, const GraphRanges* ranges = nullptr) {
  const int64_t R = offsets[n_prot];
  int rc = ensure_workspace(ctx, R, n_prot);
  if (rc) return rc;
  auto& w = ctx->w;
  const int64_t Rpad = (R + 127) / 128 * 128;
  hipStream_t st = ctx->stream;
  int32_t n_tiles = 0;
  rc = upload_batch_meta(ctx, offsets, n_prot, &n_tiles);
  if (rc) return rc;
  ctx->chunked_last = false;
  HIPCHK(hipMemsetAsync(w.node_local, 0xff, sizeof(int32_t) * Rpad, st));
  HIPCHK(hipMemsetAsync(w.node_prot, 0, sizeof(int32_t) * Rpad, st));

  mark(ctx, 0);
  // the graph per protein range (one range unless the caller pipelines the copy): k_prep over the
  // range's proteins, then k_knn over its slots (the last range also takes the padding slots)
  const int n_ranges = ranges ? ranges->n : 1;
  for (int k = 0; k < n_ranges; ++k) {
    const int32_t p0 = ranges ? ranges->cut[k] : 0, p1 = ranges ? ranges->cut[k + 1] : n_prot;
    if (ranges) HIPCHK(hipStreamWaitEvent(st, ranges->ev[k], 0));
    pst::PrepArgs pa{d_pos, d_flags, w.offsets, d_nnodes, w.node_local, w.node_prot, w.frame, w.cen, w.ca, d_pos32, p0};
    pst::launch_prep(pa, p1 - p0, st);
    if (k == 0) mark(ctx, 1);
    const int64_t s1 = p1 == n_prot ? Rpad : offsets[p1];
    pst::KnnArgs ka{s1, w.offsets, d_nnodes, w.node_local, w.node_prot, w.frame, w.cen, w.ca, w.senders, w.deg,
                    w.feat, offsets[p0]};
    pst::launch_knn(ka, st);
  }
  mark(ctx, 2);
  if (graph_only) {  // pst_build_graph: the encoder's outputs of an earlier call are gone
    HIPCHK(hipGetLastError());
    ctx->last_R = 0;
    ctx->last_Rpad = Rpad;
    return PST_OK;
  }

  const float* A = ctx->d_arena;
  auto F4 = [&](size_t o) { return reinterpret_cast<const float4*>(A + o); };
  auto mlp = [&](const MlpOff& o) {
    return pst::MlpW{F4(o.w0), A + o.b0, F4(o.w1), A + o.b1, F4(o.w2), A + o.b2, F4(o.bf1), F4(o.bf2)};
  };
  // Batches whose 32-receiver tasks leave fused rounds half empty (use_split_schedule) run each
  // layer split: one edge block per wave, messages through HBM, ordered sums in
  // k_seg_sum, node update; bit-identical results.
  const int64_t n_tasks = Rpad / 32;
  env_threshold(ctx->split_tasks, "PST_SPLIT_TASKS");
  const bool split = ctx->split_tasks >= 0 ? n_tasks <= ctx->split_tasks : use_split_schedule(n_tasks, ctx->n_simds);
  env_threshold(ctx->node_coop, "PST_NODE_COOP");
  const bool node_coop =
      split && n_tasks <= (ctx->node_coop >= 0 ? ctx->node_coop : (int64_t)(NODE_COOP_SIMD_FRACTION * ctx->n_simds));
  env_threshold(ctx->half_tasks, "PST_HALF_TASKS");
  const bool half = !split && (ctx->half_tasks >= 0 ? ctx->half_tasks != 0 : use_half_tasks(n_tasks, ctx->n_simds));
  env_threshold(ctx->mpnn_queue, "PST_MPNN_QUEUE");
  const bool queue = !split && !half && (ctx->mpnn_queue >= 0 ? ctx->mpnn_queue != 0 : MPNN_QUEUE_DEFAULT);
  ctx->last_sched = split ? 2 : half ? 1 : queue ? 3 : 0;
  env_threshold(ctx->mpnn_queue_layers, "PST_MPNN_QUEUE_LAYERS");
  const int64_t queue_layers = ctx->mpnn_queue_layers >= 0 ? ctx->mpnn_queue_layers : MPNN_QUEUE_LAYERS;
  if (queue) HIPCHK(hipMemsetAsync(w.qctr, 0, sizeof(int32_t) * 3 * (128 + n_tasks), st));
  float* msg_rows = nullptr;
  int32_t bpw = 1;
  if (split) {
    const size_t need = (size_t)n_tasks * 32 * KNN * 128 * sizeof(float);
    if (need > ctx->msg_bytes) {
      if (ctx->msg) (void)hipFree(ctx->msg);
      ctx->msg = nullptr;
      ctx->msg_bytes = 0;
      hipError_t e = hipMalloc(&ctx->msg, need);
      if (e != hipSuccess) {
        ctx->msg = nullptr;
        return fail(ctx, PST_E_NOMEM, std::string("message buffer allocation failed: ") + hipGetErrorString(e));
      }
      ctx->msg_bytes = need;
    }
    msg_rows = ctx->msg;
    env_threshold(ctx->edge_waves, "PST_EDGE_WAVES");
    const int64_t target = ctx->edge_waves > 0 ? ctx->edge_waves : SPLIT_EDGE_WAVES;
    bpw = target > 0 ? (int32_t)std::max<int64_t>(1, (n_tasks * 50 + target - 1) / target) : 1;
  }
  float* hbuf[4] = {nullptr, w.h0, w.h1, w.h0};
  float* ebuf[3] = {w.e0, w.e1, nullptr};
  float* pbuf[3] = {w.P0, w.P1, nullptr};
  for (int l = 0; l < 3; ++l) {
    pst::MpnnArgs m{};
    m.n_tasks = n_tasks;
    m.msg_rows = msg_rows;
    m.blocks_per_wave = bpw;
    m.half_tasks = half ? 1 : 0;
    m.clk = ctx->clock_on ? ctx->d_clk + 8 * l : nullptr;
    if (queue && ((queue_layers >> l) & 1)) {
      m.q_head = w.qctr + l * (128 + n_tasks);
      m.q_done = m.q_head + 128;
      m.q_grid = 2 * (ctx->n_simds / 4);  // two 4-wave workgroups per CU (MPNN_MIN_BLOCKS)
      env_threshold(ctx->mpnn_qwaves, "PST_MPNN_QWAVES");
      m.q_waves = ctx->mpnn_qwaves == 4 ? 4 : 8;
      env_threshold(ctx->mpnn_qgroup, "PST_MPNN_QGROUP");
      // wave slots of one XCD: q_grid x 4 waves over 8 XCDs (both workgroup sizes hold that many)
      m.q_group = (int32_t)(ctx->mpnn_qgroup >= 0 ? ctx->mpnn_qgroup : m.q_grid * 4 / 8);
    }
    m.senders = w.senders;
    m.deg = w.deg;
    m.node_local = w.node_local;
    m.agg = w.agg;
    m.feat = w.feat;
    m.Ttab = ctx->d_T;
    m.W_embed = F4(ctx->emb_w);
    m.b_embed = A + ctx->emb_b;
    m.PM0 = ctx->d_PM0;
    m.Utab = ctx->d_U;
    m.V0 = ctx->d_V0;
    m.W_msg0f = F4(ctx->w_msg0f);
    m.h0tab = ctx->d_h0;
    if (l > 0) {
      m.e_in = ebuf[l - 1];
      m.P_in = pbuf[l - 1];
      m.h_in = hbuf[l];
      m.edge = mlp(ctx->L[l - 1].edge);
      m.edge_ln_s = A + ctx->L[l - 1].ln_s[2];
      m.edge_ln_o = A + ctx->L[l - 1].ln_o[2];
    }
    const LayerOff& L = ctx->L[l];
    m.msg = mlp(L.msg);
    m.ln0_s = A + L.ln_s[0];
    m.ln0_o = A + L.ln_o[0];
    m.ln1_s = A + L.ln_s[1];
    m.ln1_o = A + L.ln_o[1];
    m.ff_w1 = F4(L.ff_w1);
    m.ff_b1 = A + L.ff_b1;
    m.ff_w2 = F4(L.ff_w2);
    m.ff_b2 = A + L.ff_b2;
    m.proj_w = l < 2 ? F4(ctx->proj[l]) : nullptr;
    if (l < 2) {
      m.proj_bf[0] = F4(ctx->L[l].edge.bf0);     // E_r: edge MLP of layer l
      m.proj_bf[1] = F4(ctx->L[l + 1].msg.bf0);  // M_r: message MLP of layer l+1
    }
    m.ff_bf1 = F4(L.ff_bf1);
    m.ff_bf2 = F4(L.ff_bf2);
    m.e_out = ebuf[l];
    m.h_out = hbuf[l + 1];
    m.P_out = pbuf[l];
    pst::launch_mpnn(l, m, node_coop, st);
    mark(ctx, 3 + l);
    if (ctx->dbg[l]) HIPCHK(hipMemcpyAsync(ctx->dbg[l], m.h_out, sizeof(float) * 128 * Rpad, hipMemcpyDeviceToDevice, st));
  }
  // k_down updates the original track in place, so it works on a copy of h3 (h3 stays available
  // to pst_debug_fetch); k_down_coop (df 1, small batches) keeps the track in registers and
  // reads h3 directly
  env_threshold(ctx->down_coop, "PST_DOWN_COOP");
  const int64_t coop_max = ctx->down_coop >= 0 ? ctx->down_coop : (int64_t)(DOWN_COOP_SIMD_FRACTION * ctx->n_simds);
  const bool down_coop = ctx->df == 1 && (int64_t)n_tiles <= coop_max;
  // above the coop threshold but at most one round of tiles, k_down_pair puts the two tracks of
  // a tile on two waves (k_down<1> would leave every SIMD's second wave slot empty)
  env_threshold(ctx->down_pair, "PST_DOWN_PAIR");
  const bool down_pair = ctx->df == 1 && !down_coop &&
                         (ctx->down_pair >= 0 ? ctx->down_pair != 0 : (int64_t)n_tiles <= ctx->n_simds);
  ctx->last_down_form = down_coop ? pst::DOWN_COOP : down_pair ? pst::DOWN_PAIR : pst::DOWN_ONE_WAVE;
  if (!down_coop) HIPCHK(hipMemcpyAsync(w.h1, hbuf[3], sizeof(float) * 128 * Rpad, hipMemcpyDeviceToDevice, st));
  pst::DownArgs d{};
  d.n_tiles = n_tiles;
  d.tile_prot = w.tile_prot;
  d.tile_t0 = w.tile_t0;
  d.offsets = w.offsets;
  d.n_nodes = d_nnodes;
  d.RPE = ctx->d_RPE;
  d.o_buf = down_coop ? hbuf[3] : w.h1;
  d.r_buf = w.r_buf;
  d.v_buf = w.v_buf;
  for (int b = 0; b < 3; ++b) {
    const BlockOff& O = ctx->B[b];
    pst::DownBlockW& W = d.blk[b];
    W.qn_s = A + O.qn_s; W.qn_o = A + O.qn_o; W.dn_s = A + O.dn_s; W.dn_o = A + O.dn_o;
    W.wq = F4(O.wq); W.wk = F4(O.wk); W.wv = F4(O.wv); W.wg = F4(O.wg); W.wo = F4(O.wo);
    W.gb = A + O.gb; W.ob = A + O.ob;
    W.rt_ln_s = A + O.rt_ln_s; W.rt_ln_o = A + O.rt_ln_o; W.rt_w1 = F4(O.rt_w1); W.rt_b1 = A + O.rt_b1;
    W.rt_w2 = F4(O.rt_w2); W.rt_b2 = A + O.rt_b2;
    W.ot_ln_s = A + O.ot_ln_s; W.ot_ln_o = A + O.ot_ln_o; W.ot_w1 = F4(O.ot_w1); W.ot_b1 = A + O.ot_b1;
    W.ot_w2 = F4(O.ot_w2); W.ot_b2 = A + O.ot_b2;
  }
  d.down_w = A + ctx->down_w;
  d.down_b = A + ctx->down_b;
  d.D = ctx->D;
  for (int i = 0; i < 8; ++i) {
    d.fsq_half[i] = ctx->fsq_half[i];
    d.fsq_off[i] = ctx->fsq_off[i];
    d.fsq_shift[i] = ctx->fsq_shift[i];
    d.fsq_L[i] = ctx->fsq_L[i] ? ctx->fsq_L[i] : 1;
    d.fsq_basis[i] = ctx->fsq_basis[i];
  }
  d.tokens_out = d_tokens;
  d.bounded_out = w.bounded + 8 * out_row0;
  d.quant_out = w.quant + 8 * out_row0;
  d.pre_proj_out = w.pre_proj + 128 * out_row0;
  if (d.n_tiles > 0) pst::launch_down(ctx->df, d, ctx->last_down_form, st);
  mark(ctx, 6);
  HIPCHK(hipGetLastError());
  ctx->last_R = R;
  ctx->last_Rpad = Rpad;
  ctx->last_B = n_prot;
  ctx->last_tokens = d_tokens;
  ctx->last_nnodes = d_nnodes;
  ctx->last_ntiles = n_tiles;
  (void)d_ntok;
  return PST_OK;
}

__global__ void k_ntok(const int32_t* n_nodes, int32_t* n_tok, int B, int df) {
  int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b < B) n_tok[b] = n_nodes[b] / df;
}

}  // namespace

extern "C" {

int pst_set_timing(pst_ctx* ctx, int32_t enable) {
  if (!ctx) return PST_E_INVALID;
  HIPCHK(hipSetDevice(ctx->device));
  if (enable && !ctx->ev[0])
    for (int i = 0; i <= PST_N_STAGES; ++i) HIPCHK(hipEventCreate(&ctx->ev[i]));
  ctx->timing = enable != 0;
  return PST_OK;
}

int pst_get_timing(pst_ctx* ctx, float* ms) {
  if (!ctx || !ctx->timing || !ms) return PST_E_INVALID;
  HIPCHK(hipEventSynchronize(ctx->ev[PST_N_STAGES]));
  for (int i = 0; i < PST_N_STAGES; ++i) HIPCHK(hipEventElapsedTime(&ms[i], ctx->ev[i], ctx->ev[i + 1]));
  return PST_OK;
}

int pst_set_clock_counters(pst_ctx* ctx, int32_t enable) {
  if (!ctx) return PST_E_INVALID;
  ctx->clock_on = enable != 0;
  return PST_OK;
}

int pst_clock_counters(pst_ctx* ctx, uint64_t* out, int32_t reset) {
  if (!ctx) return PST_E_INVALID;
  HIPCHK(hipSetDevice(ctx->device));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  if (out) HIPCHK(hipMemcpy(out, ctx->d_clk, 24 * sizeof(uint64_t), hipMemcpyDeviceToHost));
  return reset ? reset_clock_counters(ctx) : PST_OK;
}

size_t pst_param_count(int32_t n_levels) {
  HostParams P;
  return walk(nullptr, n_levels, &P);
}

const char* pst_create_error(void) { return g_create_error.c_str(); }

int pst_device_count(int32_t* n) {
  if (!n) return PST_E_INVALID;
  int c = 0;
  if (hipGetDeviceCount(&c) != hipSuccess) c = 0;
  *n = c;
  return PST_OK;
}

int pst_create(int32_t device, const pst_model_desc* desc, const float* params, size_t n_params, pst_ctx** out) {
  g_create_error.clear();
  if (!desc || !params || !out) {
    g_create_error = "null argument";
    return PST_E_INVALID;
  }
  if (desc->abi_version != PST_ABI_VERSION) {
    g_create_error = "ABI version mismatch";
    return PST_E_INVALID;
  }
  int D = desc->n_levels;
  int df = desc->downsampling_ratio;
  if (D < 1 || D > 8 || (df != 1 && df != 2 && df != 4) || desc->graph_max_neighbor != KNN ||
      desc->seq_max_size != 512) {
    g_create_error = "unsupported model description (need 1<=D<=8, df in {1,2,4}, k=50, seq_max_size=512)";
    return PST_E_INVALID;
  }
  int64_t K = 1;
  for (int d = 0; d < D; ++d) K *= desc->levels[d];
  if (K != desc->codebook_size) {
    g_create_error = "codebook_size != prod(levels)";
    return PST_E_INVALID;
  }
  if (n_params != pst_param_count(D)) {
    g_create_error = "parameter blob has " + std::to_string(n_params) + " floats, expected " +
                     std::to_string(pst_param_count(D));
    return PST_E_INVALID;
  }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) {
    g_create_error = "no such HIP device: " + std::to_string(device);
    return PST_E_HIP;
  }
  pst_ctx* ctx = new pst_ctx();
  ctx->device = device;
  ctx->desc = *desc;
  ctx->D = D;
  ctx->df = df;
  ctx->max_out = desc->seq_max_size / df;
  if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess) {
    g_create_error = "hip stream creation failed";
    delete ctx;
    return PST_E_HIP;
  }
  {
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0)
      ctx->n_simds = 4 * (int64_t)prop.multiProcessorCount;
  }

  int rc = build_weights(ctx, params);
  if (rc) {
    g_create_error = ctx->err;
    pst_destroy(ctx);
    return rc;
  }
  *out = ctx;
  return PST_OK;
}

int pst_destroy(pst_ctx* ctx) {
  if (!ctx) return PST_OK;
  (void)hipSetDevice(ctx->device);
  if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
  for (int l = 0; l < 3; ++l)
    if (ctx->dbg[l]) (void)hipFree(ctx->dbg[l]);
  for (int i = 0; i <= PST_N_STAGES; ++i)
    if (ctx->ev[i]) (void)hipEventDestroy(ctx->ev[i]);
  if (ctx->aux) (void)hipFree(ctx->aux);
  if (ctx->msg) (void)hipFree(ctx->msg);
  for (void* p : {(void*)ctx->d_arena, (void*)ctx->d_h0, (void*)ctx->d_PM0, (void*)ctx->d_T, (void*)ctx->d_U, (void*)ctx->d_V0, (void*)ctx->d_RPE, ctx->ws})
    if (p) (void)hipFree(p);
  if (ctx->h_counts) (void)hipHostFree(ctx->h_counts);
  if (ctx->h_tokens) (void)hipHostFree(ctx->h_tokens);
  if (ctx->h_stage_pos) (void)hipHostFree(ctx->h_stage_pos);
  if (ctx->h_stage_flags) (void)hipHostFree(ctx->h_stage_flags);
  if (ctx->h_text) (void)hipHostFree(ctx->h_text);
  if (ctx->h_pdb_counts) (void)hipHostFree(ctx->h_pdb_counts);
  if (ctx->d_pdb) (void)hipFree(ctx->d_pdb);
  for (hipStream_t cs : {ctx->copy_stream, ctx->copy_stream2})
    if (cs) {
      (void)hipStreamSynchronize(cs);
      (void)hipStreamDestroy(cs);
    }
  for (hipEvent_t e : ctx->copy_ev)
    if (e) (void)hipEventDestroy(e);
  for (hipEvent_t e : ctx->range_ev)
    if (e) (void)hipEventDestroy(e);
  if (ctx->idle_ev) (void)hipEventDestroy(ctx->idle_ev);
  if (ctx->d_clk) (void)hipFree(ctx->d_clk);
  if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
  delete ctx;
  return PST_OK;
}

const char* pst_last_error(const pst_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

void* pst_stream(pst_ctx* ctx) { return ctx ? (void*)ctx->stream : nullptr; }

int pst_sync(pst_ctx* ctx) {
  if (!ctx) return PST_E_INVALID;
  HIPCHK(hipSetDevice(ctx->device));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  return PST_OK;
}

int pst_tokenize_device(pst_ctx* ctx, const double* d_pos, const uint8_t* d_flags, const int64_t* offsets,
                        int32_t n_prot, uint32_t* d_tokens, int32_t* d_ntok, int32_t* d_nnodes) {
  if (!ctx) return PST_E_INVALID;
  ctx->err.clear();
  if (!d_pos || !d_flags || !d_tokens || !d_nnodes)
    return fail(ctx, PST_E_INVALID, "null device buffer (positions, flags, tokens and n_nodes are required)");
  int rc = validate(ctx, offsets, n_prot);
  if (rc) return rc;
  HIPCHK(hipSetDevice(ctx->device));
  rc = run(ctx, d_pos, d_flags, offsets, n_prot, d_tokens, d_ntok, d_nnodes);
  if (rc) return rc;
  if (d_ntok) hipLaunchKernelGGL(k_ntok, dim3((n_prot + 255) / 256), dim3(256), 0, ctx->stream, d_nnodes, d_ntok, n_prot, ctx->df);
  HIPCHK(hipGetLastError());
  return PST_OK;
}

}  // extern "C"

namespace {

// Protein-boundary chunk starts [0 = c_0 < c_1 < ... < c_n = n_prot] of a pipelined host call.
// Policy: whole fused rounds per chunk (see H2D_FIRST_ROUNDS). PST_H2D_CHUNKS=n forces n chunks
// of about equal residues (the first a quarter of the others; tests of the pipeline's bits).
std::vector<int32_t> plan_chunks(pst_ctx* ctx, const int64_t* offsets, int32_t n_prot) {
  const int64_t R = offsets[n_prot];
  // run() launches Rpad / 32 tasks, Rpad = R rounded up to 128 residues
  auto tasks_of = [](int64_t r) { return (r + 127) / 128 * 4; };
  const int64_t tasks = tasks_of(R);
  env_threshold(ctx->h2d_chunks, "PST_H2D_CHUNKS");
  std::vector<int32_t> cut{0};
  if (ctx->h2d_chunks >= 1) {
    const int n = std::max(1, std::min({(int)std::min<int64_t>(ctx->h2d_chunks, H2D_MAX_CHUNKS), (int)n_prot}));
    if (n > 1) {
      const double unit = (double)R / (0.25 + (n - 1));
      double target = 0.25 * unit;
      for (int32_t b = 1; b < n_prot && (int)cut.size() < n; ++b)
        if ((double)offsets[b] >= target) {
          cut.push_back(b);
          target += unit;
        }
    }
    cut.push_back(n_prot);
    return cut;
  }
  const int64_t round = std::max<int64_t>(1, ctx->n_simds);
  env_threshold(ctx->h2d_min, "PST_H2D_MIN_ROUNDS");
  if (tasks >= (ctx->h2d_min > 0 ? ctx->h2d_min : H2D_MIN_ROUNDS) * round) {
    env_threshold(ctx->h2d_first, "PST_H2D_FIRST_ROUNDS");
    env_threshold(ctx->h2d_growth, "PST_H2D_GROWTH");
    int64_t want = ctx->h2d_first > 0 ? ctx->h2d_first : H2D_FIRST_ROUNDS;  // rounds in the next chunk
    int32_t b = 0;
    while ((int)cut.size() < H2D_MAX_CHUNKS) {
      const int64_t r0 = offsets[b];
      if (tasks_of(R - r0) <= want * round) break;  // the rest fits in this chunk: last chunk
      // last protein boundary at which the chunk's tasks stay within `want` rounds
      int32_t e = b;
      while (e < n_prot && tasks_of(offsets[e + 1] - r0) <= want * round) ++e;
      if (e == b) break;
      cut.push_back(e);
      b = e;
      want *= ctx->h2d_growth > 0 ? ctx->h2d_growth : H2D_GROWTH;
    }
  }
  cut.push_back(n_prot);
  return cut;
}

// pst_tokenize / pst_tokenize_f32: `atom_pos` holds [R,37,3] doubles, or floats when `f32`
// (copied as they are — half the H2D bytes — and widened to f64 on load in k_prep).
// Token ids and per-protein counts of the last run() to the caller's (pageable) host buffers:
// one DMA each into the context's page-locked buffers, one stream sync, then host copies (the
// token rows on the host pool above 256 KB) — a D2H into pageable memory is staged and blocks the
// host per copy.
int results_to_host(pst_ctx* ctx, int64_t R, int32_t n_prot, uint32_t* tokens_out, int32_t* n_tokens_out,
                    int32_t* n_nodes_out) {
  auto& w = ctx->w;
  hipStream_t st = ctx->stream;
  uint32_t* tok_land = ctx->h_tokens && R <= ctx->cap_R ? ctx->h_tokens : tokens_out;
  HIPCHK(hipMemcpyAsync(tok_land, w.tokens, sizeof(uint32_t) * R, hipMemcpyDeviceToHost, st));
  // both count arrays in one copy into pinned memory (one DMA instead of two staged ones)
  const bool counts = n_tokens_out || n_nodes_out;
  const int64_t capB = ctx->cap_B;
  if (counts && ctx->h_counts) {
    HIPCHK(hipMemcpyAsync(ctx->h_counts, w.n_tok, sizeof(int32_t) * (capB + n_prot), hipMemcpyDeviceToHost, st));
  } else if (counts) {
    if (n_tokens_out) HIPCHK(hipMemcpyAsync(n_tokens_out, w.n_tok, sizeof(int32_t) * n_prot, hipMemcpyDeviceToHost, st));
    if (n_nodes_out) HIPCHK(hipMemcpyAsync(n_nodes_out, w.n_nodes, sizeof(int32_t) * n_prot, hipMemcpyDeviceToHost, st));
  }
  HIPCHK(hipStreamSynchronize(st));
  if (tok_land != tokens_out) {
    constexpr int64_t PART = 1 << 16;  // tokens per host copy task (256 KB)
    const int parts = (int)((R + PART - 1) / PART);
    pst::HostPool::get().run(parts, std::min(parts, 8), [&](int i) {
      const int64_t a = (int64_t)i * PART, b = std::min<int64_t>(R, a + PART);
      std::memcpy(tokens_out + a, tok_land + a, sizeof(uint32_t) * (b - a));
    });
  }
  if (counts && ctx->h_counts) {
    if (n_tokens_out) std::memcpy(n_tokens_out, ctx->h_counts, sizeof(int32_t) * n_prot);
    if (n_nodes_out) std::memcpy(n_nodes_out, ctx->h_counts + capB, sizeof(int32_t) * n_prot);
  }
  return PST_OK;
}

int tokenize_host(pst_ctx* ctx, const void* atom_pos, bool f32, const uint8_t* atom_flags, const int64_t* offsets,
                  int32_t n_prot, uint32_t* tokens_out, int32_t* n_tokens_out, int32_t* n_nodes_out) {
  if (!ctx) return PST_E_INVALID;
  ctx->err.clear();
  if (!atom_pos || !atom_flags || !tokens_out) return fail(ctx, PST_E_INVALID, "null host buffer");
  int rc = validate(ctx, offsets, n_prot);
  if (rc) return rc;
  HIPCHK(hipSetDevice(ctx->device));
  const int64_t R = offsets[n_prot];
  rc = ensure_workspace(ctx, R, n_prot);
  if (rc) return rc;
  auto& w = ctx->w;
  // device copy of the positions: w.pos (sized for doubles) holds the floats in its first half
  const size_t es = f32 ? sizeof(float) : sizeof(double);
  char* d_pos_bytes = reinterpret_cast<char*>(w.pos);
  const char* h_pos_bytes = static_cast<const char*>(atom_pos);
  auto pos64 = [&](int64_t r0) { return f32 ? nullptr : w.pos + 111 * r0; };
  auto pos32 = [&](int64_t r0) { return f32 ? reinterpret_cast<const float*>(d_pos_bytes) + 111 * r0 : nullptr; };
  const std::vector<int32_t> cut = plan_chunks(ctx, offsets, n_prot);
  const int n_chunks = (int)cut.size() - 1;
  env_threshold(ctx->h2d_ranges, "PST_H2D_GRAPH_RANGES");
  const int want_ranges = (int)std::min<int64_t>(8, ctx->h2d_ranges >= 0 ? std::max<int64_t>(1, ctx->h2d_ranges)
                                                                         : H2D_GRAPH_RANGES);
  if (!ctx->copy_stream) {
    HIPCHK(hipStreamCreateWithFlags(&ctx->copy_stream, hipStreamNonBlocking));
    HIPCHK(hipStreamCreateWithFlags(&ctx->copy_stream2, hipStreamNonBlocking));
    for (int k = 0; k < H2D_MAX_CHUNKS; ++k) HIPCHK(hipEventCreateWithFlags(&ctx->copy_ev[k], hipEventDisableTiming));
    for (int k = 0; k < 8; ++k) HIPCHK(hipEventCreateWithFlags(&ctx->range_ev[k], hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&ctx->idle_ev, hipEventDisableTiming));
  }
  // inputs are overwritten on copy_stream only after everything queued on `stream` so far
  HIPCHK(hipEventRecord(ctx->idle_ev, ctx->stream));
  HIPCHK(hipStreamWaitEvent(ctx->copy_stream, ctx->idle_ev, 0));
  env_threshold(ctx->h2d_streams, "PST_H2D_COPY_STREAMS");
  const bool two_streams = ctx->h2d_streams == 2;
  if (two_streams) HIPCHK(hipStreamWaitEvent(ctx->copy_stream2, ctx->idle_ev, 0));
  auto copy_rows = [&](int64_t r0, int64_t r1, hipStream_t cs) -> int {
    HIPCHK(hipMemcpyAsync(d_pos_bytes + es * 111 * r0, h_pos_bytes + es * 111 * r0, es * 111 * (r1 - r0),
                          hipMemcpyHostToDevice, cs));
    HIPCHK(hipMemcpyAsync(w.flags + 37 * r0, atom_flags + 37 * r0, 37 * (r1 - r0), hipMemcpyHostToDevice, cs));
    return PST_OK;
  };
  // chunk k: copied on copy_stream, its compute queued on `stream` behind the copy's event(s); the
  // host issues copy k+1 after compute k is queued. The first chunk is copied in protein ranges.
  std::vector<int64_t> loc;
  std::vector<int32_t> rcut;
  for (int k = 0; k < n_chunks; ++k) {
    const int32_t b0 = cut[k], b1 = cut[k + 1];
    const int64_t r0 = offsets[b0], r1 = offsets[b1];
    loc.assign(offsets + b0, offsets + b1 + 1);
    for (auto& o : loc) o -= r0;
    GraphRanges gr{0, nullptr, ctx->range_ev};
    // ranges only for a first chunk of at least half a round of tasks: below that the copy is
    // short and the extra (pageable-staged) copies and launches cost more than they hide
    // (CASP14, 176 tasks: tokenize 2.07 -> 2.49 ms with 4 ranges). An explicit
    // PST_H2D_GRAPH_RANGES > 1 applies at any size (tests reach the range branch with it).
    const bool big = (r1 - r0 + 127) / 128 * 4 >= std::max<int64_t>(1, ctx->n_simds / 2) || ctx->h2d_ranges > 1;
    const int nr = k == 0 && big ? std::min(want_ranges, (int)(b1 - b0)) : 1;
    if (nr > 1) {
      // range cuts at protein boundaries, about equal residues each
      rcut.assign(1, 0);
      for (int32_t b = 1; b < b1 - b0 && (int)rcut.size() < nr; ++b)
        if (loc[b] * nr >= (int64_t)rcut.size() * loc[b1 - b0]) rcut.push_back(b);
      rcut.push_back(b1 - b0);
      gr.n = (int)rcut.size() - 1;
      gr.cut = rcut.data();
      for (int q = 0; q < gr.n; ++q) {
        hipStream_t cs = two_streams && (q & 1) ? ctx->copy_stream2 : ctx->copy_stream;
        rc = copy_rows(r0 + loc[rcut[q]], r0 + loc[rcut[q + 1]], cs);
        if (rc) return rc;
        HIPCHK(hipEventRecord(ctx->range_ev[q], cs));
      }
    } else {
      rc = copy_rows(r0, r1, ctx->copy_stream);
      if (rc) return rc;
      HIPCHK(hipEventRecord(ctx->copy_ev[k], ctx->copy_stream));
      HIPCHK(hipStreamWaitEvent(ctx->stream, ctx->copy_ev[k], 0));
    }
    if (k == 0) {
      std::fill(std::begin(ctx->last_plan), std::end(ctx->last_plan), 0);
      ctx->last_plan[0] = nr > 1 ? gr.n : 0;  // 0: one copy, no range branch
      ctx->last_plan[1] = n_chunks;
      for (int q = 0; q <= n_chunks; ++q) ctx->last_plan[2 + q] = cut[q];
    }
    if (n_chunks == 1) {
      rc = run(ctx, pos64(0), w.flags, offsets, n_prot, w.tokens, w.n_tok, w.n_nodes, false, 0, pos32(0),
               gr.n > 0 ? &gr : nullptr);
      if (rc) return rc;
      ctx->last_plan[11] = ctx->last_sched;
      ctx->last_plan[19] = ctx->last_down_form;
      break;
    }
    rc = run(ctx, pos64(r0), w.flags + 37 * r0, loc.data(), b1 - b0, w.tokens + r0, w.n_tok + b0, w.n_nodes + b0,
             false, r0, pos32(r0), gr.n > 0 ? &gr : nullptr);
    if (rc) return rc;
    ctx->last_plan[11 + k] = ctx->last_sched;
    ctx->last_plan[19] = ctx->last_down_form;
  }
  if (n_chunks > 1) {
    // the batch as a whole for pst_aux / pst_codebook_aux: offsets, token tiles and last_* of all
    // chunks (the chunks' own metadata uploads were stream-ordered before this one)
    int32_t n_tiles = 0;
    rc = upload_batch_meta(ctx, offsets, n_prot, &n_tiles);
    if (rc) return rc;
    ctx->last_R = R;
    ctx->last_Rpad = (R + 127) / 128 * 128;
    ctx->last_B = n_prot;
    ctx->last_tokens = w.tokens;
    ctx->last_nnodes = w.n_nodes;
    ctx->last_ntiles = n_tiles;
    ctx->chunked_last = true;
  }
  hipLaunchKernelGGL(k_ntok, dim3((n_prot + 255) / 256), dim3(256), 0, ctx->stream, w.n_nodes, w.n_tok, n_prot, ctx->df);
  return results_to_host(ctx, R, n_prot, tokens_out, n_tokens_out, n_nodes_out);
}

}  // namespace

extern "C" {

int pst_tokenize(pst_ctx* ctx, const double* atom_pos, const uint8_t* atom_flags, const int64_t* offsets,
                 int32_t n_prot, uint32_t* tokens_out, int32_t* n_tokens_out, int32_t* n_nodes_out) {
  return tokenize_host(ctx, atom_pos, false, atom_flags, offsets, n_prot, tokens_out, n_tokens_out, n_nodes_out);
}

int pst_tokenize_f32(pst_ctx* ctx, const float* atom_pos, const uint8_t* atom_flags, const int64_t* offsets,
                     int32_t n_prot, uint32_t* tokens_out, int32_t* n_tokens_out, int32_t* n_nodes_out) {
  return tokenize_host(ctx, atom_pos, true, atom_flags, offsets, n_prot, tokens_out, n_tokens_out, n_nodes_out);
}

int pst_tokenize_pdb_batch(pst_ctx* ctx, const pst_pdb_batch* b, uint32_t* tokens_out, int32_t* n_tokens_out,
                           int32_t* n_nodes_out) {
  if (!ctx) return PST_E_INVALID;
  ctx->err.clear();
  if (!b || !tokens_out) return fail(ctx, PST_E_INVALID, "null batch or token buffer");
  int32_t n = 0;
  int64_t R = 0;
  if (pst_pdb_batch_sizes(b, &n, &R) != PST_OK) return fail(ctx, PST_E_INVALID, "invalid batch");
  HIPCHK(hipSetDevice(ctx->device));
  if (R > ctx->h_stage_cap) {
    if (ctx->h_stage_pos) (void)hipHostFree(ctx->h_stage_pos);
    if (ctx->h_stage_flags) (void)hipHostFree(ctx->h_stage_flags);
    ctx->h_stage_pos = nullptr;
    ctx->h_stage_flags = nullptr;
    ctx->h_stage_cap = 0;
    const int64_t cap = std::max<int64_t>(R, 4096);
    HIPCHK(hipHostMalloc((void**)&ctx->h_stage_pos, sizeof(float) * 111 * cap));
    HIPCHK(hipHostMalloc((void**)&ctx->h_stage_flags, 37 * cap));
    ctx->h_stage_cap = cap;
  }
  std::vector<int64_t> off(n + 1);
  std::vector<int32_t> st(n);
  pst_pdb_batch_copy_f32(b, ctx->h_stage_pos, ctx->h_stage_flags, nullptr, off.data(), st.data());
  for (int32_t i = 0; i < n; ++i)
    if (st[i] != PST_OK) return fail(ctx, PST_E_INVALID, pst_pdb_batch_error(b, i));
  return tokenize_host(ctx, ctx->h_stage_pos, true, ctx->h_stage_flags, off.data(), n, tokens_out, n_tokens_out,
                       n_nodes_out);
}

int pst_tokenize_pdb_files(pst_ctx* ctx, const char* const* paths, int32_t n, int32_t n_threads,
                           uint32_t* tokens_out, int64_t tokens_cap, int32_t* n_tokens_out, int32_t* n_nodes_out,
                           int64_t* offsets_out) {
  if (!ctx) return PST_E_INVALID;
  ctx->err.clear();
  if (n <= 0 || !paths || !tokens_out) return fail(ctx, PST_E_INVALID, "empty batch or null buffer");
  HIPCHK(hipSetDevice(ctx->device));
  const int threads = std::max(1, n_threads);
  auto& pool = pst::HostPool::get();
  // ---- files opened and sized, then their texts read straight into page-locked memory
  std::vector<int64_t> fsz(n, 0);
  std::vector<int> fds(n, -1);
  struct FdClose {
    std::vector<int>& f;
    ~FdClose() {
      for (int& d : f)
        if (d >= 0) ::close(d), d = -1;
    }
  } fd_close{fds};
  std::atomic<int> bad_file(-1);
  pool.run(n, threads, [&](int i) {
    const int fd = ::open(paths[i], O_RDONLY | O_CLOEXEC);
    struct stat st;
    if (fd < 0 || fstat(fd, &st) != 0) {
      if (fd >= 0) ::close(fd);
      bad_file.store(i);
      return;
    }
    fds[i] = fd;
    fsz[i] = (int64_t)st.st_size;
  });
  if (bad_file.load() >= 0) return fail(ctx, PST_E_INVALID, std::string("cannot open ") + paths[bad_file.load()]);
  std::vector<int64_t> foff(n + 1, 0), rbase(n + 1, 0);
  for (int i = 0; i < n; ++i) {
    foff[i + 1] = foff[i] + fsz[i];
    rbase[i + 1] = rbase[i] + fsz[i] / 54 + 1;  // an ATOM/HETATM record spans >= 54 columns + a separator
  }
  const int64_t T = foff[n], RB = rbase[n];
  if (T + 1 > (int64_t)ctx->h_text_cap) {
    if (ctx->h_text) (void)hipHostFree(ctx->h_text);
    ctx->h_text = nullptr;
    ctx->h_text_cap = 0;
    const size_t cap = (size_t)std::max<int64_t>(T + 1, 1 << 20);
    HIPCHK(hipHostMalloc((void**)&ctx->h_text, cap));
    ctx->h_text_cap = cap;
  }
  pool.run(n, threads, [&](int i) {
    int64_t got = 0;
    while (got < fsz[i]) {
      const ssize_t r = ::pread(fds[i], ctx->h_text + foff[i] + got, (size_t)(fsz[i] - got), (off_t)got);
      if (r <= 0) break;
      got += r;
    }
    ::close(fds[i]);
    fds[i] = -1;
    if (got != fsz[i]) bad_file.store(i);
  });
  if (bad_file.load() >= 0) return fail(ctx, PST_E_INVALID, std::string("cannot read ") + paths[bad_file.load()]);
  // Files of 1 GB and more (offsets inside a file are 32-bit on the GPU path) send the whole
  // call to the native host parser; PST_PDB_GPU_MAX_FILE lowers that bound (the GPU tests force
  // the all-host route with it)
  env_threshold(ctx->pdb_gpu_max_file, "PST_PDB_GPU_MAX_FILE");
  const int64_t gpu_max = ctx->pdb_gpu_max_file >= 0 ? ctx->pdb_gpu_max_file : (int64_t)1 << 30;
  bool all_host = *std::max_element(fsz.begin(), fsz.end()) >= gpu_max;
  // ---- device scratch of the GPU parse (one grow-only allocation, about 10x the text: when it
  // cannot be had, the whole call takes the native host parser instead of failing)
  pst::PdbScanArgs a{};
  if (!all_host) {
    struct Item {
      void** p;
      size_t bytes;
    };
    const size_t L = (size_t)(T + n);
    Item items[] = {{(void**)&a.text, (size_t)T + 1},
                    {(void**)&a.file_off, sizeof(int64_t) * (n + 1)},
                    {(void**)&a.rec_base, sizeof(int64_t) * (n + 1)},
                    {(void**)&a.res_off, sizeof(int64_t) * (n + 1)},
                    {(void**)&a.line_start, sizeof(int32_t) * L},
                    {(void**)&a.line_kind, L},
                    {(void**)&a.rec_chain, (size_t)RB},
                    {(void**)&a.rec_het, (size_t)RB},
                    {(void**)&a.rec_atom, (size_t)RB},
                    {(void**)&a.rec_resseq, sizeof(int32_t) * RB},
                    {(void**)&a.rec_name, sizeof(uint32_t) * RB},
                    {(void**)&a.rec_xyz, sizeof(float) * 3 * RB},
                    {(void**)&a.rec_run, sizeof(int32_t) * RB},
                    {(void**)&a.run_first, sizeof(int32_t) * RB},
                    {(void**)&a.run_out, sizeof(int32_t) * RB},
                    {(void**)&a.run_type, (size_t)RB},
                    {(void**)&a.slot, sizeof(int32_t) * 37 * RB},
                    {(void**)&a.n_res, sizeof(int32_t) * 3 * n}};
    size_t total = 0;
    for (const auto& it : items) total += (it.bytes + 255) / 256 * 256;
    if (total > ctx->d_pdb_cap) {
      if (ctx->d_pdb) (void)hipFree(ctx->d_pdb);
      ctx->d_pdb = nullptr;
      ctx->d_pdb_cap = 0;
      if (hipMalloc(&ctx->d_pdb, total) != hipSuccess) {
        (void)hipGetLastError();  // clear the sticky error: the host route follows
        ctx->d_pdb = nullptr;
        all_host = true;
      } else {
        ctx->d_pdb_cap = total;
      }
    }
    if (!all_host) {
      char* q = (char*)ctx->d_pdb;
      for (const auto& it : items) {
        *it.p = q;
        q += (it.bytes + 255) / 256 * 256;
      }
      a.n_run = a.n_res + n;
      a.host_path = a.n_res + 2 * n;
    }
  }
  if (3 * (int64_t)n > ctx->h_pdb_counts_cap) {
    if (ctx->h_pdb_counts) (void)hipHostFree(ctx->h_pdb_counts);
    ctx->h_pdb_counts = nullptr;
    ctx->h_pdb_counts_cap = 0;
    HIPCHK(hipHostMalloc((void**)&ctx->h_pdb_counts, sizeof(int32_t) * 3 * std::max(n, 64)));
    ctx->h_pdb_counts_cap = 3 * std::max(n, 64);
  }
  for (int q = 0; q < 37; ++q) {
    const char* nm = pst::kAtomNames[q];
    uint32_t k = 0;
    std::memcpy(&k, nm, std::min<size_t>(4, strlen(nm)));
    a.tab.atom_key[q] = k;
  }
  for (int r = 0; r < 20; ++r) {
    uint32_t k = 0;
    std::memcpy(&k, pst::kResName3[r], 3);
    a.tab.res_key[r] = k;
  }
  std::memcpy(&a.tab.hoh, "HOH\0", 4);
  std::memcpy(&a.tab.wat, "WAT\0", 4);
  for (int r = 0; r < 21; ++r)
    for (int q = 0; q < 37; ++q) a.tab.exists[r][q] = pst::kResAtomExists[r][q];
  hipStream_t st = ctx->stream;
  if (all_host) {
    for (int i = 0; i < n; ++i) {
      ctx->h_pdb_counts[i] = 0;
      ctx->h_pdb_counts[n + i] = 0;
      ctx->h_pdb_counts[2 * n + i] = 1;
    }
  } else {
    HIPCHK(hipMemcpyAsync((void*)a.text, ctx->h_text, (size_t)T, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync((void*)a.file_off, foff.data(), sizeof(int64_t) * (n + 1), hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync((void*)a.rec_base, rbase.data(), sizeof(int64_t) * (n + 1), hipMemcpyHostToDevice, st));
    pst::launch_pdb_scan(a, n, st);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(ctx->h_pdb_counts, a.n_res, sizeof(int32_t) * 3 * n, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
  }
  const int32_t* g_res = ctx->h_pdb_counts;
  const int32_t* g_host = ctx->h_pdb_counts + 2 * n;
  // ---- the files outside the fast path: the native host parser (its results and its errors)
  std::vector<int32_t> host_ids;
  for (int i = 0; i < n; ++i)
    if (g_host[i]) host_ids.push_back(i);
  pst_pdb_batch* hb = nullptr;
  std::vector<int64_t> hoff(host_ids.size() + 1, 0);
  struct BatchFree {
    pst_pdb_batch** b;
    ~BatchFree() {
      if (*b) pst_pdb_batch_free(*b);
    }
  } hb_free{&hb};
  if (!host_ids.empty()) {
    std::vector<const char*> tp;
    std::vector<size_t> tl;
    for (int i : host_ids) {
      tp.push_back(ctx->h_text + foff[i]);
      tl.push_back((size_t)fsz[i]);
    }
    pst_pdb_parse_strings(tp.data(), tl.data(), (int32_t)host_ids.size(), 0, threads, &hb);
    std::vector<int32_t> hst(host_ids.size());
    pst_pdb_batch_copy_f32(hb, nullptr, nullptr, nullptr, hoff.data(), hst.data());
    for (size_t j = 0; j < host_ids.size(); ++j)
      if (hst[j] != PST_OK) return fail(ctx, PST_E_INVALID, pst_pdb_batch_error(hb, (int32_t)j));
  }
  std::vector<int64_t> off(n + 1, 0);
  {
    size_t j = 0;
    for (int i = 0; i < n; ++i) {
      const int64_t ri = g_host[i] ? hoff[j + 1] - hoff[j] : g_res[i];
      if (g_host[i]) ++j;
      off[i + 1] = off[i] + ri;
    }
  }
  int rc = validate(ctx, off.data(), n);
  if (rc) return rc;
  const int64_t R = off[n];
  if (R > tokens_cap) {
    if (offsets_out) offsets_out[n] = R;
    return fail(ctx, PST_E_INVALID, "token buffer too small");
  }
  rc = ensure_workspace(ctx, R, n);
  if (rc) return rc;
  auto& w = ctx->w;
  a.pos = reinterpret_cast<float*>(w.pos);
  a.flags = w.flags;
  if (!all_host) {
    HIPCHK(hipMemcpyAsync((void*)a.res_off, off.data(), sizeof(int64_t) * (n + 1), hipMemcpyHostToDevice, st));
    pst::launch_pdb_write(a, n, st);
    HIPCHK(hipGetLastError());
  }
  if (!host_ids.empty()) {  // host-parsed rows into their places (through the page-locked staging)
    const int64_t HR = hoff.back();
    if (HR > ctx->h_stage_cap) {
      if (ctx->h_stage_pos) (void)hipHostFree(ctx->h_stage_pos);
      if (ctx->h_stage_flags) (void)hipHostFree(ctx->h_stage_flags);
      ctx->h_stage_pos = nullptr;
      ctx->h_stage_flags = nullptr;
      ctx->h_stage_cap = 0;
      const int64_t cap = std::max<int64_t>(HR, 4096);
      HIPCHK(hipHostMalloc((void**)&ctx->h_stage_pos, sizeof(float) * 111 * cap));
      HIPCHK(hipHostMalloc((void**)&ctx->h_stage_flags, 37 * cap));
      ctx->h_stage_cap = cap;
    }
    pst_pdb_batch_copy_f32(hb, ctx->h_stage_pos, ctx->h_stage_flags, nullptr, nullptr, nullptr);
    for (size_t j = 0; j < host_ids.size(); ++j) {
      const int64_t r0 = off[host_ids[j]], nr = hoff[j + 1] - hoff[j];
      if (!nr) continue;
      HIPCHK(hipMemcpyAsync(a.pos + 111 * r0, ctx->h_stage_pos + 111 * hoff[j], sizeof(float) * 111 * nr,
                            hipMemcpyHostToDevice, st));
      HIPCHK(hipMemcpyAsync(w.flags + 37 * r0, ctx->h_stage_flags + 37 * hoff[j], 37 * nr, hipMemcpyHostToDevice, st));
    }
  }
  ctx->last_pdb_host_files = (int32_t)host_ids.size();
  rc = run(ctx, nullptr, w.flags, off.data(), n, w.tokens, w.n_tok, w.n_nodes, false, 0, a.pos);
  if (rc) return rc;
  hipLaunchKernelGGL(k_ntok, dim3((n + 255) / 256), dim3(256), 0, st, w.n_nodes, w.n_tok, n, ctx->df);
  rc = results_to_host(ctx, R, n, tokens_out, n_tokens_out, n_nodes_out);
  if (rc) return rc;
  if (offsets_out) std::memcpy(offsets_out, off.data(), sizeof(int64_t) * (n + 1));
  return PST_OK;
}

int32_t pst_pdb_files_host_parsed(const pst_ctx* ctx) { return ctx ? ctx->last_pdb_host_files : -1; }

int pst_build_graph(pst_ctx* ctx, const double* atom_pos, const uint8_t* atom_flags, const int64_t* offsets,
                    int32_t n_prot, int32_t* senders_out, float* edge_features_out, double* ca_out,
                    int32_t* n_nodes_out) {
  if (!ctx) return PST_E_INVALID;
  ctx->err.clear();
  if (!atom_pos || !atom_flags || !senders_out || !edge_features_out || !ca_out || !n_nodes_out)
    return fail(ctx, PST_E_INVALID, "null host buffer");
  int rc = validate(ctx, offsets, n_prot);
  if (rc) return rc;
  HIPCHK(hipSetDevice(ctx->device));
  const int64_t R = offsets[n_prot];
  rc = ensure_workspace(ctx, R, n_prot);
  if (rc) return rc;
  auto& w = ctx->w;
  HIPCHK(hipMemcpyAsync(w.pos, atom_pos, sizeof(double) * 111 * R, hipMemcpyHostToDevice, ctx->stream));
  HIPCHK(hipMemcpyAsync(w.flags, atom_flags, 37 * R, hipMemcpyHostToDevice, ctx->stream));
  rc = run(ctx, w.pos, w.flags, offsets, n_prot, w.tokens, w.n_tok, w.n_nodes, /*graph_only=*/true);
  if (rc) return rc;
  std::vector<int32_t> snd((size_t)R * KNN);
  std::vector<float> feat(feat_floats((size_t)R * KNN));
  HIPCHK(hipMemcpyAsync(snd.data(), w.senders, sizeof(int32_t) * snd.size(), hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(hipMemcpyAsync(feat.data(), w.feat, sizeof(float) * feat.size(), hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(hipMemcpyAsync(ca_out, w.ca, sizeof(double) * 3 * R, hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(hipMemcpyAsync(n_nodes_out, w.n_nodes, sizeof(int32_t) * n_prot, hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  // global residue slots → per-protein node indices; the 27 features of the 32-wide rows
  for (int b = 0; b < n_prot; ++b) {
    const int64_t base = offsets[b], end = offsets[b + 1];
    for (int64_t g = base; g < end; ++g) {
      const bool real = g - base < n_nodes_out[b];
      for (int j = 0; j < KNN; ++j) {
        const size_t e = (size_t)g * KNN + j;
        senders_out[e] = real && snd[e] >= 0 ? (int32_t)(snd[e] - base) : -1;
        for (int c = 0; c < 27; ++c) edge_features_out[e * 27 + c] = real ? feat[feat_float(e, pst::feat_slot(c))] : 0.0f;
      }
      if (!real) ca_out[3 * g] = ca_out[3 * g + 1] = ca_out[3 * g + 2] = 0.0;
    }
  }
  return PST_OK;
}

int pst_aux(pst_ctx* ctx, float* bounded, float* quantize, float* pre_proj) {
  if (!ctx || ctx->last_R == 0) return PST_E_INVALID;
  HIPCHK(hipSetDevice(ctx->device));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  const int64_t R = ctx->last_R;
  const int D = ctx->D;
  if (bounded || quantize) {
    std::vector<float> b8((size_t)R * 8), q8((size_t)R * 8);
    HIPCHK(hipMemcpy(b8.data(), ctx->w.bounded, sizeof(float) * 8 * R, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(q8.data(), ctx->w.quant, sizeof(float) * 8 * R, hipMemcpyDeviceToHost));
    for (int64_t i = 0; i < R; ++i)
      for (int d = 0; d < D; ++d) {
        if (bounded) bounded[i * D + d] = b8[i * 8 + d];
        if (quantize) quantize[i * D + d] = q8[i * 8 + d];
      }
  }
  if (pre_proj) HIPCHK(hipMemcpy(pre_proj, ctx->w.pre_proj, sizeof(float) * 128 * R, hipMemcpyDeviceToHost));
  return PST_OK;
}

}  // extern "C"

namespace {

// upper bound of the last call's token rows (from the raw residue counts)
int64_t token_rows_upper(const pst_ctx* ctx) {
  int64_t t = 0;
  for (int b = 0; b < ctx->last_B; ++b) t += (ctx->h_offsets[b + 1] - ctx->h_offsets[b]) / ctx->df;
  return t;
}

int launch_codebook_aux(pst_ctx* ctx, float* d_dist, float* d_prob, uint32_t* d_argmin, uint32_t* d_hist) {
  const int D = ctx->D;
  int K_lo = 1, K_hi = 1;
  for (int d = 0; d < D; ++d) (d < 3 ? K_lo : K_hi) *= ctx->fsq_L[d];
  const int K = K_lo * K_hi;
  if (D < 4 || K_lo > FSQ_AUX_MAX_LO || K_hi > FSQ_AUX_MAX_HI || (K_lo & 3))
    return fail(ctx, PST_E_INVALID, "codebook aux supports D >= 4, prod(L[0:3]) <= 512 (multiple of 4), "
                                    "prod(L[3:]) <= 128");
  pst::FsqAuxArgs a{};
  a.n_rows_grid = ctx->last_ntiles * 32;
  a.tile_prot = ctx->w.tile_prot;
  a.tile_t0 = ctx->w.tile_t0;
  a.offsets = ctx->w.offsets;
  a.n_nodes = ctx->last_nnodes;
  a.row_start = ctx->w.row_start;
  a.bounded = ctx->w.bounded;
  a.tokens = ctx->last_tokens;
  a.df = ctx->df;
  a.D = D;
  a.K = K;
  a.K_lo = K_lo;
  a.K_hi = K_hi;
  for (int d = 0; d < 8; ++d) {
    a.L[d] = d < D ? ctx->fsq_L[d] : 1;
    a.basis[d] = d < D ? ctx->fsq_basis[d] : 0;
  }
  a.dist = d_dist;
  a.prob = d_prob;
  a.argmin = d_argmin;
  a.hist = d_hist;
  if (d_hist) HIPCHK(hipMemsetAsync(d_hist, 0, sizeof(uint32_t) * K, ctx->stream));
  pst::launch_fsq_aux(a, ctx->last_B, ctx->stream);
  HIPCHK(hipGetLastError());
  return PST_OK;
}

}  // namespace

extern "C" {

int pst_codebook_aux_device(pst_ctx* ctx, float* d_distances, float* d_soft_proba, uint32_t* d_argmin,
                            uint32_t* d_histogram, int64_t row_capacity) {
  if (!ctx) return PST_E_INVALID;
  if (ctx->last_R == 0 || !ctx->last_tokens) return fail(ctx, PST_E_INVALID, "no tokenize call yet");
  if ((d_distances || d_soft_proba || d_argmin) && row_capacity < token_rows_upper(ctx))
    return fail(ctx, PST_E_INVALID, "row_capacity below the token-row bound of the last call (sum floor(R_b/df))");
  HIPCHK(hipSetDevice(ctx->device));
  return launch_codebook_aux(ctx, d_distances, d_soft_proba, d_argmin, d_histogram);
}

int pst_codebook_aux(pst_ctx* ctx, float* distances, float* soft_proba, uint32_t* argmin, uint32_t* histogram,
                     float* perplexity, int64_t rows) {
  if (!ctx) return PST_E_INVALID;
  if (ctx->last_R == 0 || !ctx->last_tokens) return fail(ctx, PST_E_INVALID, "no tokenize call yet");
  HIPCHK(hipSetDevice(ctx->device));
  const int B = ctx->last_B;
  std::vector<int32_t> nn(B);
  HIPCHK(hipMemcpyAsync(nn.data(), ctx->last_nnodes, sizeof(int32_t) * B, hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  int64_t T = 0;
  for (int b = 0; b < B; ++b) T += nn[b] / ctx->df;
  if ((distances || soft_proba || argmin) && rows < T)
    return fail(ctx, PST_E_INVALID, "output buffers hold " + std::to_string(rows) + " rows, need " + std::to_string(T));
  int64_t K = 1;
  for (int d = 0; d < ctx->D; ++d) K *= ctx->fsq_L[d];
  const size_t tk = (size_t)T * (size_t)K * sizeof(float);
  auto al = [](size_t x) { return (x + 4095) / 4096 * 4096; };
  const size_t need = (distances ? al(tk) : 0) + (soft_proba ? al(tk) : 0) + al(sizeof(uint32_t) * (T + 1)) +
                      al(sizeof(uint32_t) * K);
  if (need > ctx->aux_bytes) {
    if (ctx->aux) (void)hipFree(ctx->aux);
    ctx->aux = nullptr;
    ctx->aux_bytes = 0;
    hipError_t e = hipMalloc(&ctx->aux, need);
    if (e != hipSuccess) return fail(ctx, PST_E_NOMEM, std::string("aux allocation failed: ") + hipGetErrorString(e));
    ctx->aux_bytes = need;
  }
  char* p = (char*)ctx->aux;
  float* d_dist = distances ? (float*)p : nullptr;
  p += distances ? al(tk) : 0;
  float* d_prob = soft_proba ? (float*)p : nullptr;
  p += soft_proba ? al(tk) : 0;
  uint32_t* d_arg = (uint32_t*)p;
  p += al(sizeof(uint32_t) * (T + 1));
  uint32_t* d_hist = (uint32_t*)p;
  int rc = launch_codebook_aux(ctx, d_dist, d_prob, argmin ? d_arg : nullptr, d_hist);
  if (rc) return rc;
  if (distances && T) HIPCHK(hipMemcpyAsync(distances, d_dist, tk, hipMemcpyDeviceToHost, ctx->stream));
  if (soft_proba && T) HIPCHK(hipMemcpyAsync(soft_proba, d_prob, tk, hipMemcpyDeviceToHost, ctx->stream));
  if (argmin && T) HIPCHK(hipMemcpyAsync(argmin, d_arg, sizeof(uint32_t) * T, hipMemcpyDeviceToHost, ctx->stream));
  std::vector<uint32_t> hist(K);
  HIPCHK(hipMemcpyAsync(hist.data(), d_hist, sizeof(uint32_t) * K, hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  if (histogram) std::copy(hist.begin(), hist.end(), histogram);
  if (perplexity) {  // quantize.py:222-224 (avg_probs = hist / total; exp(-sum p log(p + 1e-10)))
    double total = 0.0, h = 0.0;
    for (uint32_t c : hist) total += c;
    for (uint32_t c : hist) {
      double pr = total > 0 ? c / total : 0.0;
      h += pr * std::log(pr + 1e-10);
    }
    *perplexity = (float)std::exp(-h);
  }
  return PST_OK;
}

int pst_debug_fetch(pst_ctx* ctx, int32_t which, void* out, size_t bytes) {
  if (!ctx || ctx->last_R == 0) return PST_E_INVALID;
  if (which == 20) {  // the last host call's plan (see pst_ctx::last_plan)
    if (bytes < sizeof(ctx->last_plan)) return fail(ctx, PST_E_INVALID, "debug buffer too small");
    std::memcpy(out, ctx->last_plan, sizeof(ctx->last_plan));
    return PST_OK;
  }
  if (ctx->chunked_last)
    return fail(ctx, PST_E_INVALID, "the last call was pipelined in chunks (PST_H2D_CHUNKS=1 keeps intermediates)");
  HIPCHK(hipSetDevice(ctx->device));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  const int64_t Rp = ctx->last_Rpad;
  const void* src = nullptr;
  size_t need = 0;
  std::vector<float> tmp;
  if (which >= 0 && which <= 3) {  // node features after init embed / layer `which` (perm → natural)
    if (which == 0) return fail(ctx, PST_E_INVALID, "init embedding is a table (not kept per call)");
    const float* d = which == 3 ? ctx->w.h0 : ctx->dbg[which - 1];
    if (!d) return fail(ctx, PST_E_INVALID, "intermediate layers need PST_DEBUG=1 at context creation");
    tmp.resize((size_t)Rp * 128);
    HIPCHK(hipMemcpy(tmp.data(), d, tmp.size() * sizeof(float), hipMemcpyDeviceToHost));
    need = (size_t)ctx->last_R * 128 * sizeof(float);
    if (bytes < need) return fail(ctx, PST_E_INVALID, "debug buffer too small");
    float* o = (float*)out;
    for (int64_t i = 0; i < ctx->last_R; ++i)
      for (int h = 0; h < 2; ++h)
        for (int M = 0; M < 4; ++M)
          for (int r = 0; r < 16; ++r) o[i * 128 + tile_channel(h, M, r)] = tmp[i * 128 + h * 64 + M * 16 + r];
    return PST_OK;
  }
  if (which == 10) {  // 32-float rows in feature order (features 0..26, then +0), from feat_slot's
    need = (size_t)ctx->last_R * KNN * 32 * sizeof(float);
    if (bytes < need) return fail(ctx, PST_E_INVALID, "debug buffer too small");
    tmp.resize(feat_floats((size_t)ctx->last_R * KNN));
    HIPCHK(hipMemcpy(tmp.data(), ctx->w.feat, tmp.size() * sizeof(float), hipMemcpyDeviceToHost));
    float* o = (float*)out;
    for (size_t e = 0; e < (size_t)ctx->last_R * KNN; ++e)
      for (int f = 0; f < 32; ++f) o[e * 32 + f] = f < pst::FEAT_USED ? tmp[feat_float(e, pst::feat_slot(f))] : 0.0f;
    return PST_OK;
  } else if (which == 13 || which == 14) {  // the last call's input rows: positions f32 (pst_tokenize_f32 /
    // pst_tokenize_pdb_batch / pst_tokenize_pdb_files) [R,37,3], flags [R,37]
    need = (size_t)ctx->last_R * (which == 13 ? 111 * sizeof(float) : 37);
    src = which == 13 ? (const void*)ctx->w.pos : (const void*)ctx->w.flags;
  } else if (which == 11) {
    src = ctx->w.senders;
    need = (size_t)ctx->last_R * KNN * sizeof(int32_t);
  } else if (which == 12) {
    src = ctx->w.deg;
    need = (size_t)ctx->last_R * sizeof(int32_t);
  } else {
    return fail(ctx, PST_E_INVALID, "unknown debug id");
  }
  if (bytes < need) return fail(ctx, PST_E_INVALID, "debug buffer too small");
  HIPCHK(hipMemcpy(out, src, need, hipMemcpyDeviceToHost));
  return PST_OK;
}

}  // extern "C"
