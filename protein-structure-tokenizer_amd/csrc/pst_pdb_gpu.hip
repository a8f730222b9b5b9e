// pst_pdb_gpu.hip — PDB text → atom37 rows on the GPU: the parse half of pst_tokenize_pdb_files.
//
// The host reads the files into one page-locked buffer and copies the text to HBM (3.9 MB for
// the 31 CASP14 structures); one workgroup per file then does what the native parser's two
// passes do (pst_pdb.cpp, the restatement of Bio's PDBParser in pst_amd/pdb.py), and a second
// launch writes each kept residue's atom37 row straight into the tokenizer's input buffers —
// the positions never travel back to the host. The fast path covers the files PDB writers
// emit; anything else is flagged per file and parsed by the native host parser instead, so the
// product's semantics stay those of pst_pdb.cpp file for file:
//   * bytes: printable ASCII, '\n' and '\r' (a '\r' ends a line, as in pst_pdb.cpp; the empty
//     line between "\r\n" is not a record) — a tab or any other byte: host path;
//   * records: the header ends at the first ATOM / HETATM / MODEL line, the coordinates at the
//     first "END   " / "CONECT" line after it; a MODEL or ENDMDL record in between: host path
//     (single-model files with MODEL lines, and every multi-model error, stay there);
//   * ATOM / HETATM: at least 54 columns, altloc and insertion code blank, resseq an integer,
//     x / y / z in the fixed "%8.3f" form (m / 1000.0 as one IEEE division: the double strtod
//     gives, then rounded to float32 as Bio stores atom.coord), occupancy blank or decimal;
//     anything else: host path (which parses it or raises the reference's error);
//   * residues: keyed by (chain, het flag, resseq, resname when the het flag is "H_<resname>"),
//     contiguous in the file: each chain one block of lines, and within a chain the keys strictly
//     increasing in (ATOM before HETATM, resseq) — so a residue never reappears and Bio's
//     order of first appearance is the file order; otherwise: host path;
//   * atoms: the first record of an atom37 name in its residue (no altlocs on this path); names
//     outside atom37 are dropped; residues without an atom37 atom are skipped; the residue type
//     is the first record's resname among the 20 standard ones, else UNK.
// Every choice above is checked against the host parser bit for bit on the GPU
// (tests/test_gpu_pdb_parse.py: positions and flags of every CASP14 file and of handcrafted files
// covering each host-path trigger).
#include "pst_kernels.h"

namespace pst {

namespace {

constexpr int PDB_THREADS = 1024;
constexpr int PDB_INT_MAX = 0x7fffffff;

enum : uint8_t { K_OTHER = 0, K_ATOM = 1, K_HETATM = 2, K_MODEL = 3, K_ENDMDL = 4, K_STOP = 5 };

// exclusive prefix sum over the workgroup (PDB_THREADS threads); *total = the sum
__device__ int block_scan(int v, int* total) {
  __shared__ int wsum[PDB_THREADS / 64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int x = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int y = __shfl_up(x, d);
    if (lane >= d) x += y;
  }
  if (lane == 63) wsum[w] = x;
  __syncthreads();
  int base = 0, tot = 0;
  for (int i = 0; i < PDB_THREADS / 64; ++i) {
    const int s = wsum[i];
    if (i < w) base += s;
    tot += s;
  }
  __syncthreads();  // wsum is reused by the next call
  *total = tot;
  return base + x - v;
}

constexpr int TILE_BYTES = 64 * PDB_THREADS;  // the lines pass's tile

// 0x80 in each byte of x equal to the byte of c (c: one byte value replicated), exact
__device__ __forceinline__ uint32_t swar_eq(uint32_t x, uint32_t c) {
  const uint32_t y = x ^ c;
  return ~(((y & 0x7f7f7f7fu) + 0x7f7f7f7fu) | y) & 0x80808080u;
}
// the four 0x80 flags of a SWAR mask as bits 0..3 (byte order)
__device__ __forceinline__ uint32_t swar_bits(uint32_t m) {
  return ((m >> 7) & 1u) | ((m >> 14) & 2u) | ((m >> 21) & 4u) | ((m >> 28) & 8u);
}

__device__ __forceinline__ bool is6(const char* p, const char* s) {
  return p[0] == s[0] && p[1] == s[1] && p[2] == s[2] && p[3] == s[3] && p[4] == s[4] && p[5] == s[5];
}

// stripped field [a, b) of a line of length ll (spaces only: tabs never reach this path)
__device__ __forceinline__ void field(const char* line, int ll, int a, int b, int* s, int* n) {
  if (b > ll) b = ll;
  while (a < b && line[a] == ' ') ++a;
  while (b > a && line[b - 1] == ' ') --b;
  *s = a;
  *n = b > a ? b - a : 0;
}

__device__ __forceinline__ uint32_t pack4(const char* p, int n) {
  uint32_t k = 0;
  for (int i = 0; i < n && i < 4; ++i) k |= (uint32_t)(uint8_t)p[i] << (8 * i);
  return k;
}

// "%8.3f" field at column a (pst_pdb.cpp coord_fixed): false = not that form
__device__ __forceinline__ bool coord_fixed(const char* p, double* v) {
  if (p[4] != '.') return false;
  const unsigned d5 = (unsigned)(p[5] - '0'), d6 = (unsigned)(p[6] - '0'), d7 = (unsigned)(p[7] - '0');
  if (d5 > 9 || d6 > 9 || d7 > 9) return false;
  int i = 0;
  while (i < 4 && p[i] == ' ') ++i;
  bool neg = false;
  if (i < 4 && (p[i] == '-' || p[i] == '+')) {
    neg = p[i] == '-';
    ++i;
  }
  if (i == 4) return false;
  int64_t m = 0;
  for (; i < 4; ++i) {
    const unsigned d = (unsigned)(p[i] - '0');
    if (d > 9) return false;
    m = m * 10 + d;
  }
  m = (m * 10 + d5) * 100 + d6 * 10 + d7;
  const double r = (double)m / 1000.0;
  *v = neg ? -r : r;
  return true;
}

__device__ __forceinline__ int line_end(const PdbScanArgs& a, int64_t lb, int i, int n_lines, int len) {
  return i + 1 < n_lines ? a.line_start[lb + i + 1] - 1 : len;
}

}  // namespace

// One workgroup per file: lines, records, residues, atom slots; per-file kept-residue counts and
// the host-path flag. Scratch per file f: lines at line_base = file_off[f] + f, records and
// residue runs at rec_base[f] (rec_base[f+1] - rec_base[f] >= len / 54 + 1 records fit).
__global__ __launch_bounds__(PDB_THREADS) void k_pdb_scan(PdbScanArgs a) {
  const int f = blockIdx.x, tid = threadIdx.x;
  const int64_t f0 = a.file_off[f];
  const int len = (int)(a.file_off[f + 1] - f0);
  const char* tx = a.text + f0;
  const int64_t lb = f0 + f, rb = a.rec_base[f];
  const int rec_cap = (int)(a.rec_base[f + 1] - rb);
  __shared__ int s_bad, s_start, s_stop, s_chain_seg[256];
  // LDS: the text tile of the lines pass (64 KB), then each record's first 64 bytes per thread
  // (stride 17 dwords: no bank conflicts)
  __shared__ uint32_t s_buf[PDB_THREADS * 17];
  uint32_t(*s_line)[17] = reinterpret_cast<uint32_t(*)[17]>(s_buf);
  const char* s_tile = reinterpret_cast<const char*>(s_buf);
  if (tid == 0) {
    s_bad = 0;
    s_start = PDB_INT_MAX;
    s_stop = PDB_INT_MAX;
  }
  for (int c = tid; c < 256; c += PDB_THREADS) s_chain_seg[c] = 0;
  __syncthreads();
  // ---- lines and their record kinds: the file's bytes as 16-byte words of the (256-aligned)
  // text buffer, 64 contiguous bytes per thread per 64 KB tile (the next tile's words loaded
  // during this one's scan): separators '\n' / '\r' counted, scanned, and at each one the line
  // start it opens and that line's kind written. The header ends at the first ATOM / HETATM /
  // MODEL line. A kind needs its 6 bytes inside the file (a match never holds a separator, so it
  // lies inside the line).
  // tile_lo: the file position of the LDS tile's byte 0 (the tile holds TILE_BYTES bytes)
  auto kind_at = [&](int st, int64_t tile_lo) -> uint8_t {
    if (st + 6 > len) return K_OTHER;
    const int64_t o = f0 + st - tile_lo;
    const char* p = o >= 0 && o + 6 <= TILE_BYTES ? s_tile + o : tx + st;
    if (is6(p, "ATOM  ")) return K_ATOM;
    if (is6(p, "HETATM")) return K_HETATM;
    if (is6(p, "MODEL ")) return K_MODEL;
    if (is6(p, "ENDMDL")) return K_ENDMDL;
    if (is6(p, "END   ") || is6(p, "CONECT")) return K_STOP;
    return K_OTHER;
  };
  auto note_kind = [&](int i, int st, int64_t tile_lo) {
    const uint8_t k = kind_at(st, tile_lo);
    a.line_kind[lb + i] = k;
    // s_start only falls: past the header no atomic is issued
    if ((k == K_ATOM || k == K_HETATM || k == K_MODEL) && i < *(volatile int*)&s_start) atomicMin(&s_start, i);
  };
  const int64_t w0 = f0 >> 4, w1 = (f0 + len + 15) >> 4;
  const uint4* tw = reinterpret_cast<const uint4*>(a.text);
  constexpr int TW = 4 * PDB_THREADS;  // words per tile
  if (tid == 0) {
    a.line_start[lb] = 0;
    note_kind(0, 0, -TILE_BYTES);  // (not in the tile: read from HBM)
  }
  int at = 1;
  bool bad = false;
  uint4 cur[4], nxt[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int64_t wi = w0 + 4 * tid + q;
    cur[q] = wi < w1 ? tw[wi] : make_uint4(0u, 0u, 0u, 0u);
  }
  for (int64_t t0 = w0; t0 < w1; t0 += TW) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int64_t wi = t0 + TW + 4 * tid + q;
      nxt[q] = wi < w1 ? tw[wi] : make_uint4(0u, 0u, 0u, 0u);
    }
    const int64_t pb = (t0 + 4 * tid) * 16;  // absolute position of this thread's byte 0
    // this thread's 64 bytes into the LDS tile (read by the kinds below after the scan's barrier)
    uint4* tl = reinterpret_cast<uint4*>(s_buf) + 4 * tid;
#pragma unroll
    for (int q = 0; q < 4; ++q) tl[q] = cur[q];
    // bytes of the file within this thread's 64: [lo, hi)
    const int lo = (int)max<int64_t>(0, min<int64_t>(64, f0 - pb));
    const int hi = (int)max<int64_t>(0, min<int64_t>(64, f0 + len - pb));
    const uint64_t in = hi <= lo ? 0ull : ((hi >= 64 ? ~0ull : (1ull << hi) - 1ull) & ~((1ull << lo) - 1ull));
    // per-byte flags four bytes at a time (exact SWAR tests): separators, and bytes outside
    // printable ASCII other than them
    uint64_t sep = 0, bad_m = 0;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const uint4& v = cur[j >> 2];
      const uint32_t x = (j & 3) == 0 ? v.x : (j & 3) == 1 ? v.y : (j & 3) == 2 ? v.z : v.w;
      const uint32_t s_m = swar_eq(x, 0x0a0a0a0au) | swar_eq(x, 0x0d0d0d0du);
      const uint32_t lo7 = x & 0x7f7f7f7fu;
      const uint32_t lt20 = ~(lo7 + 0x60606060u) & ~x & 0x80808080u;  // byte < 0x20
      const uint32_t ge7f = (x & 0x80808080u) | swar_eq(x, 0x7f7f7f7fu);  // byte > 0x7e
      sep |= (uint64_t)swar_bits(s_m) << (4 * j);
      bad_m |= (uint64_t)swar_bits((lt20 | ge7f) & ~s_m) << (4 * j);
    }
    sep &= in;
    if (bad_m & in) bad = true;
    const int cnt = __builtin_popcountll(sep);
    int tile = 0;
    int q = at + block_scan(cnt, &tile);
    while (sep) {
      const int b = __builtin_ctzll(sep);
      sep &= sep - 1;
      const int st = (int)(pb + b - f0) + 1;
      a.line_start[lb + q] = st;
      note_kind(q, st, t0 * 16);
      ++q;
    }
    at += tile;
#pragma unroll
    for (int q2 = 0; q2 < 4; ++q2) cur[q2] = nxt[q2];
    __syncthreads();  // the LDS tile is rewritten next
  }
  if (bad) s_bad = 1;
  const int n_lines = at;  // separators + 1 (the last line may be empty)
  __syncthreads();
  const int start = s_start;
  if (start == PDB_INT_MAX) {
    // no ATOM / HETATM / MODEL line (empty, header-only or REMARK/TER-only file): the native
    // parser raises the reference's error for it (pst_pdb.cpp, "Found 0 models"). Uniform exit:
    // start is the same LDS value in every thread and no barrier follows.
    if (tid == 0) {
      a.n_res[f] = 0;
      a.n_run[f] = 0;
      a.host_path[f] = 1;
    }
    return;
  }
  for (int i = tid; i < n_lines; i += PDB_THREADS)
    if (i > start && a.line_kind[lb + i] == K_STOP) atomicMin(&s_stop, i);
  __syncthreads();
  const int stop = min(s_stop, n_lines);
  // ---- ATOM / HETATM records of [start, stop) in line order, fields parsed
  int n_rec = 0;
  // each line's kind / start / end loaded one iteration ahead
  auto line_info = [&](int i, uint8_t& k, int& st, int& en) {
    k = K_OTHER;
    st = en = 0;
    if (i < stop) {
      k = a.line_kind[lb + i];
      st = a.line_start[lb + i];
      en = line_end(a, lb, i, n_lines, len);
    }
  };
  uint8_t k_nx;
  int s_nx, e_nx;
  line_info(start + tid, k_nx, s_nx, e_nx);
  for (int t0 = start; t0 < stop; t0 += PDB_THREADS) {
    const uint8_t k = k_nx;
    const int s = s_nx, ll = e_nx - s_nx;
    line_info(t0 + PDB_THREADS + tid, k_nx, s_nx, e_nx);
    if (k == K_MODEL || k == K_ENDMDL) s_bad = 1;
    const bool rec = k == K_ATOM || k == K_HETATM;
    int tile = 0;
    const int r = n_rec + block_scan(rec ? 1 : 0, &tile);
    n_rec += tile;
    if (!rec) continue;
    if (r >= rec_cap) {  // cannot happen for >= 54-column records; guards the scratch bounds
      s_bad = 1;
      continue;
    }
    // the record's first 64 bytes into this thread's LDS row (17 independent dword loads, byte-
    // aligned with alignbyte; reads past the line stay inside the scratch allocation and are never
    // used: every column read below is < 54 <= ll or clipped to ll)
    {
      const int64_t pa = f0 + s;
      const uint32_t* t32 = reinterpret_cast<const uint32_t*>(a.text) + (pa >> 2);
      const uint32_t sh = (uint32_t)(pa & 3);
      uint32_t dw[17];
#pragma unroll
      for (int j = 0; j < 17; ++j) dw[j] = t32[j];
#pragma unroll
      for (int j = 0; j < 16; ++j) s_line[tid][j] = __builtin_amdgcn_alignbyte(dw[j + 1], dw[j], sh);
    }
    const char* L = reinterpret_cast<const char*>(s_line[tid]);
    bool ok = ll >= 54 && L[16] == ' ' && L[26] == ' ';
    double x = 0.0, y = 0.0, z = 0.0;
    int rs = 0;
    if (ok) ok = coord_fixed(L + 30, &x) && coord_fixed(L + 38, &y) && coord_fixed(L + 46, &z);
    if (ok) {  // resseq: optional sign, 1-4 digits
      int fs, fn;
      field(L, ll, 22, 26, &fs, &fn);
      int j = fs, sg = 1;
      if (fn > 0 && (L[j] == '-' || L[j] == '+')) {
        sg = L[j] == '-' ? -1 : 1;
        ++j;
      }
      ok = j < fs + fn;
      for (; ok && j < fs + fn; ++j) {
        const unsigned d = (unsigned)(L[j] - '0');
        if (d > 9) ok = false;
        rs = rs * 10 + (int)d;
      }
      rs *= sg;
    }
    if (ok && ll > 54) {  // occupancy blank or [sign] digits [. digits]
      int fs, fn;
      field(L, ll, 54, 60, &fs, &fn);
      int j = fs, digits = 0, dots = 0;
      if (fn > 0 && (L[j] == '-' || L[j] == '+')) ++j;
      for (; ok && j < fs + fn; ++j) {
        if (L[j] >= '0' && L[j] <= '9') ++digits;
        else if (L[j] == '.' && dots == 0) ++dots;
        else ok = false;
      }
      if (fn > 0 && digits == 0) ok = false;
    }
    if (!ok) {
      s_bad = 1;
      continue;
    }
    int ns, nn, rsn, rsl;
    field(L, ll, 12, 16, &ns, &nn);
    field(L, ll, 17, 20, &rsn, &rsl);
    const uint32_t name = pack4(L + ns, nn), resname = pack4(L + rsn, rsl);
    int atom = -1;
    if (nn >= 1 && nn <= 4)
      for (int q = 0; q < 37; ++q)
        if (a.tab.atom_key[q] == name) atom = q;
    const bool water = rsl == 3 && (resname == a.tab.hoh || resname == a.tab.wat);
    const int64_t o = rb + r;
    a.rec_chain[o] = (uint8_t)L[21];
    a.rec_het[o] = k == K_ATOM ? 0 : water ? 1 : 2;
    a.rec_atom[o] = (int8_t)atom;
    a.rec_resseq[o] = rs;
    a.rec_name[o] = rsl <= 4 ? resname : 0xffffffffu;  // a 4+ character name is never standard
    a.rec_xyz[3 * o + 0] = (float)x;
    a.rec_xyz[3 * o + 1] = (float)y;
    a.rec_xyz[3 * o + 2] = (float)z;
  }
  __syncthreads();
  n_rec = min(n_rec, rec_cap);
  // ---- residue runs: a record opens one when its key differs from the previous record's
  auto same = [&](int64_t p, int64_t q) {
    return a.rec_chain[p] == a.rec_chain[q] && a.rec_het[p] == a.rec_het[q] && a.rec_resseq[p] == a.rec_resseq[q] &&
           (a.rec_het[p] != 2 || a.rec_name[p] == a.rec_name[q]);
  };
  int n_run = 0;
  for (int t0 = 0; t0 < n_rec; t0 += PDB_THREADS) {
    const int k = t0 + tid;
    const bool opens = k < n_rec && (k == 0 || !same(rb + k, rb + k - 1));
    int tile = 0;
    const int r = n_run + block_scan(opens ? 1 : 0, &tile);
    if (opens) a.run_first[rb + r] = k;
    n_run += tile;
  }
  __syncthreads();
  // run of each record (the last run opened at or before it), and the contiguity checks
  for (int r = tid; r < n_run; r += PDB_THREADS) {
    const int k0 = a.run_first[rb + r], k1 = r + 1 < n_run ? a.run_first[rb + r + 1] : n_rec;
    for (int k = k0; k < k1; ++k) a.rec_run[rb + k] = r;
    a.run_out[rb + r] = 0;  // set to 1 below by any record of an atom37 name
    {  // residue type: the first record's name among the 20 standard ones, else UNK
      const uint32_t rn = a.rec_name[rb + k0];
      int rt = 20;
      for (int q = 0; q < 20; ++q)
        if (a.tab.res_key[q] == rn) rt = q;
      a.run_type[rb + r] = (int8_t)rt;
    }
    const uint8_t ch = a.rec_chain[rb + k0];
    if (r == 0 || a.rec_chain[rb + a.run_first[rb + r - 1]] != ch) {
      atomicAdd(&s_chain_seg[ch], 1);
    } else {  // same chain: keys strictly increasing in (ATOM before HETATM, resseq)
      const int64_t p = rb + a.run_first[rb + r - 1], q = rb + k0;
      const int hp = a.rec_het[p] ? 1 : 0, hq = a.rec_het[q] ? 1 : 0;
      if (!(hq > hp || (hq == hp && a.rec_resseq[q] > a.rec_resseq[p]))) s_bad = 1;
    }
  }
  for (int r = tid; r < n_run * 37; r += PDB_THREADS) a.slot[37 * rb + r] = PDB_INT_MAX;
  __syncthreads();
  for (int c = tid; c < 256; c += PDB_THREADS)
    if (s_chain_seg[c] > 1) s_bad = 1;  // a chain that reappears after another one
  // ---- atom slots: the first record of each atom37 name in its residue
  for (int k = tid; k < n_rec; k += PDB_THREADS) {
    const int at = a.rec_atom[rb + k];
    if (at >= 0) {
      const int r = a.rec_run[rb + k];
      atomicMin(&a.slot[37 * (rb + r) + at], k);
      a.run_out[rb + r] = 1;
    }
  }
  __syncthreads();
  // ---- kept residues (at least one atom37 atom), numbered in file order
  int n_keep = 0;
  for (int t0 = 0; t0 < n_run; t0 += PDB_THREADS) {
    const int r = t0 + tid;
    const bool keep = r < n_run && a.run_out[rb + r] != 0;
    int tile = 0;
    const int o = n_keep + block_scan(keep ? 1 : 0, &tile);
    if (r < n_run) a.run_out[rb + r] = keep ? o : -1;
    n_keep += tile;
  }
  if (tid == 0) {
    a.n_res[f] = n_keep;
    a.n_run[f] = n_run;
    a.host_path[f] = s_bad;
  }
}

// Kept residue rows of the fast-path files into the tokenizer's inputs: positions float32
// [R,37,3] (absent atoms 0) and flags [R,37] (bit0 present, bit1 atom37 atom of the residue type).
__global__ __launch_bounds__(256) void k_pdb_write(PdbScanArgs a) {
  const int f = blockIdx.x;
  if (a.host_path[f]) return;
  const int64_t rb = a.rec_base[f], row0 = a.res_off[f];
  const int n_el = a.n_run[f] * 37;
  for (int e = blockIdx.y * 256 + threadIdx.x; e < n_el; e += gridDim.y * 256) {
    const int r = e / 37, at = e - 37 * r;
    const int o = a.run_out[rb + r];
    if (o < 0) continue;
    const int rt = a.run_type[rb + r];
    const int k = a.slot[37 * (rb + r) + at];
    const int64_t row = row0 + o;
    float* p = a.pos + (row * 37 + at) * 3;
    if (k != PDB_INT_MAX) {
      p[0] = a.rec_xyz[3 * (rb + k) + 0];
      p[1] = a.rec_xyz[3 * (rb + k) + 1];
      p[2] = a.rec_xyz[3 * (rb + k) + 2];
    } else {
      p[0] = 0.0f;
      p[1] = 0.0f;
      p[2] = 0.0f;
    }
    a.flags[row * 37 + at] = (uint8_t)((k != PDB_INT_MAX ? 1 : 0) | (a.tab.exists[rt][at] << 1));
  }
}

// k_pdb_write: workgroups per file (each a strided share of the file's residue-atom slots)
constexpr int PDB_WRITE_SPLIT = 8;

void launch_pdb_scan(const PdbScanArgs& a, int n_files, hipStream_t st) {
  hipLaunchKernelGGL(k_pdb_scan, dim3(n_files), dim3(PDB_THREADS), 0, st, a);
}

void launch_pdb_write(const PdbScanArgs& a, int n_files, hipStream_t st) {
  hipLaunchKernelGGL(k_pdb_write, dim3(n_files, PDB_WRITE_SPLIT), dim3(256), 0, st, a);
}

}  // namespace pst
