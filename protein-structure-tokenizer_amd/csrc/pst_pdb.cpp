// pst_pdb.cpp — native PDB → atom37 parser (host side of the tokenize path, C ABI in include/pst.h).
//
// Semantics follow the reference's `protein_structure_from_pdb_string`
// (structure_tokenizer/data/protein_structure_sample.py:166-248) on top of Biopython's
// PDBParser(QUIET=True), exactly as restated in pst_amd/pdb.py (the readable spec; the tests
// compare both parsers record for record):
//   * MODEL/ENDMDL: only the first model is read; more than one model (or none) is an error;
//   * ATOM and HETATM records build residues keyed by (hetero flag, resseq, icode), grouped per
//     chain in order of first appearance (a chain that reappears is continued);
//   * hetero flag: "W" for HOH/WAT, "H_<resname>" for other HETATM, " " for ATOM;
//   * coordinates are float32 (double parse, then rounded to float, as Bio stores them);
//   * a repeated atom name keeps the first record unless an altloc record has a strictly higher
//     occupancy (highest occupancy wins, first on ties);
//   * insertion codes are an error; residue names outside the 20 standard types become UNK;
//     atoms outside atom37 are ignored; residues without any atom37 atom are skipped.
// Inputs are parsed in parallel (one std::thread pool per call); outputs are packed ragged
// arrays in input order, the layout pst_tokenize takes.
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>

#include <algorithm>
#include <atomic>
#include <memory>
#include <cerrno>
#include <functional>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/pst.h"
#include "pst_pool.h"
#include "pst_residue_tables.h"

namespace {

struct Parsed {
  int status = PST_OK;
  std::string error;
  std::vector<float> pos;      // [n,37,3] (Bio's float32 atom.coord)
  std::vector<uint8_t> flags;  // [n,37]
  std::vector<uint8_t> aatype; // [n]
  int64_t n = 0;
};

// Python str.strip() of a fixed-width field [a, b) of a line (spaces past the end), no allocation
struct Field {
  const char* p;
  int n;
  bool empty() const { return n == 0; }
  bool eq(const char* s) const { return (int)strlen(s) == n && !memcmp(p, s, n); }
};

inline Field field(const char* line, int len, int a, int b) {
  if (b > len) b = len;
  while (a < b && (line[a] == ' ' || line[a] == '\t')) ++a;
  while (b > a && (line[b - 1] == ' ' || line[b - 1] == '\t')) --b;
  return Field{line + a, a < b ? b - a : 0};
}

// Python int() of a field (optional sign, decimal digits); false if malformed
inline bool parse_int(Field f, int* v) {
  if (f.empty() || f.n > 15) return false;
  int i = 0;
  bool neg = false;
  if (f.p[0] == '-' || f.p[0] == '+') {
    neg = f.p[0] == '-';
    i = 1;
  }
  if (i >= f.n) return false;
  long r = 0;
  for (; i < f.n; ++i) {
    const char c = f.p[i];
    if (c < '0' || c > '9') {
      // anything else (e.g. digit-group underscores) through strtol's stricter reading
      char buf[16];
      memcpy(buf, f.p, f.n);
      buf[f.n] = 0;
      errno = 0;
      char* end = nullptr;
      long x = strtol(buf, &end, 10);
      if (errno || *end) return false;
      *v = (int)x;
      return true;
    }
    r = r * 10 + (c - '0');
  }
  *v = (int)(neg ? -r : r);
  return true;
}

// Python float() of a field. Fast path for the fixed-point form PDB writers emit ("-12.345"):
// mantissa and 10^k are exact doubles, so one IEEE division is the correctly rounded value —
// the same double strtod returns. Anything else goes through strtod.
inline bool parse_double(Field f, double* v) {
  if (f.empty() || f.n > 31) return false;
  {
    int i = 0;
    bool neg = false;
    if (f.p[0] == '-' || f.p[0] == '+') {
      neg = f.p[0] == '-';
      i = 1;
    }
    int64_t m = 0;
    int digits = 0, frac = -1;
    bool ok = i < f.n;
    for (; i < f.n && ok; ++i) {
      const char c = f.p[i];
      if (c >= '0' && c <= '9') {
        m = m * 10 + (c - '0');
        ++digits;
        if (frac >= 0) ++frac;
      } else if (c == '.' && frac < 0) {
        frac = 0;
      } else {
        ok = false;
      }
    }
    if (ok && digits > 0 && digits <= 15) {
      static const double p10[16] = {1e0, 1e1, 1e2, 1e3, 1e4, 1e5, 1e6, 1e7, 1e8, 1e9, 1e10, 1e11, 1e12, 1e13, 1e14, 1e15};
      double r = frac > 0 ? (double)m / p10[frac] : (double)m;
      *v = neg ? -r : r;
      return true;
    }
  }
  char buf[32];
  memcpy(buf, f.p, f.n);
  buf[f.n] = 0;
  char* end = nullptr;
  double r = strtod(buf, &end);
  if (*end) return false;
  *v = r;
  return true;
}

// Coordinate field [a, a+8) in the fixed "%8.3f" form PDB writers emit (right-aligned, '.' at
// a+4, three decimals, e.g. "  -12.345"): the integer m = value x 1000 and one IEEE division —
// the correctly rounded double, as parse_double's generic path and strtod give. false = not that
// form (the caller falls back to field() + parse_double, which also handles every other form).
inline bool coord_fixed(const char* line, int len, int a, double* v) {
  if (a + 8 > len || line[a + 4] != '.') return false;
  const char* p = line + a;
  const unsigned d5 = (unsigned)(p[5] - '0'), d6 = (unsigned)(p[6] - '0'), d7 = (unsigned)(p[7] - '0');
  if (d5 > 9 || d6 > 9 || d7 > 9) return false;
  int i = 0;
  while (i < 4 && p[i] == ' ') ++i;
  bool neg = false;
  if (i < 4 && (p[i] == '-' || p[i] == '+')) {
    neg = p[i] == '-';
    ++i;
  }
  if (i == 4) return false;  // no integer digit (".123", "-.123": the generic path)
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

// ---- atom37 name lookup: the stripped 1-4 character name packed little-endian into a uint32,
// found in a 128-entry open-addressing table built once
inline uint32_t pack_name(const char* p, int n) {
  uint32_t k = 0;
  memcpy(&k, p, n < 4 ? n : 4);
  return k;
}
struct AtomTable {
  uint32_t key[128];
  int8_t idx[128];
  AtomTable() {
    memset(key, 0, sizeof(key));
    memset(idx, -1, sizeof(idx));
    for (int a = 0; a < pst::kAtomTypes; ++a) {
      const uint32_t k = pack_name(pst::kAtomNames[a], (int)strlen(pst::kAtomNames[a]));
      uint32_t h = (k * 2654435761u) >> 25;
      while (idx[h] >= 0) h = (h + 1) & 127;
      key[h] = k;
      idx[h] = (int8_t)a;
    }
  }
  int find(uint32_t k) const {
    for (uint32_t h = (k * 2654435761u) >> 25;; h = (h + 1) & 127) {
      if (idx[h] < 0) return -1;
      if (key[h] == k) return idx[h];
    }
  }
};
const AtomTable& atom_table() {
  static const AtomTable t;
  return t;
}

// residue type of a stripped residue name: its packed little-endian bytes (pack_name) against the
// 20 standard names packed once (a name of 4+ characters never matches: pack_name keeps 4 bytes,
// and a 3-letter name packs with a zero 4th byte)
int restype_index(Field resname) {
  struct Names {
    uint32_t k[20];
    Names() {
      for (int r = 0; r < 20; ++r) k[r] = pack_name(pst::kResName3[r], 3);
    }
  };
  static const Names N;
  if (resname.n != 3) return 20;
  const uint32_t key = pack_name(resname.p, 3);
  for (int r = 0; r < 20; ++r)
    if (N.k[r] == key) return r;
  return 20;
}

// One residue as Bio builds it, reduced to what the output keeps: its atom37 slots. A repeated
// atom name keeps the first record unless an altloc record has a strictly higher occupancy;
// atoms outside atom37 never reach the output, so they are not stored at all.
struct Res {
  int resseq;
  char icode;
  uint8_t restype;
  uint64_t present;  // bit a: atom37 slot a filled (xyz / occ of slot a are set only then)
  float xyz[pst::kAtomTypes][3];
  double occ[pst::kAtomTypes];
  Res() {}  // no zero fill of the 740-byte slot arrays: only the present slots are ever read
};

struct Chain {
  char id;
  uint64_t last_key;
  int last_res;
  std::vector<int> residues;                // residue ids in order of first appearance
  std::unordered_map<uint64_t, int> index;  // key -> residue id
};

// Residue keys (het flag, resseq, icode[, resname]) are packed into 64 bits in assemble():
// het 0 = ATOM " ", 1 = water "W", 2 = "H_<resname>" (resname in bits 34..57).

// ---- pass 1 (parallel over line-aligned chunks of a file): each line's record, fields parsed
enum RecKind : uint8_t { R_ATOM, R_HETATM, R_MODEL, R_ENDMDL, R_STOP, R_BAD_COORD, R_BAD_OCC };

struct Rec {
  uint8_t kind;
  char altloc, chain, icode;
  int8_t atom;      // atom37 index or -1
  uint8_t restype;  // 0..20
  uint8_t het;      // 0 ATOM, 1 water, 2 other HETATM
  int32_t resseq;
  uint32_t resname;  // packed (het == 2 keys only)
  float xyz[3];
  double occ;
  uint32_t line;     // byte offset of the line (error messages)
};

inline int line_len_at(const char* text, size_t len, size_t p, size_t* next) {
  const char* line = text + p;
  const char* nl = (const char*)memchr(line, '\n', len - p);
  size_t q = nl ? (size_t)(nl - text) : len;
  const char* cr = (const char*)memchr(line, '\r', q - p);  // a lone '\r' ends a line too
  if (cr) q = (size_t)(cr - text);
  *next = (q + 1 < len && text[q] == '\r' && text[q + 1] == '\n') ? q + 2 : q + 1;  // \n, \r\n or \r
  return (int)(q - p);
}

// Records of the lines starting in [p0, p1) (p0 at a line start). Only the records Bio's reader
// acts on are kept: ATOM/HETATM (fields parsed; a malformed one becomes R_BAD_* and raises only if
// pass 2 reaches it), MODEL, ENDMDL and the CONECT / "END   " stop records.
void scan_chunk(const char* text, size_t len, size_t p0, size_t p1, std::vector<Rec>* out) {
  const AtomTable& T = atom_table();
  out->reserve(out->size() + (p1 - p0) / 80 + 4);
  size_t p = p0;
  while (p < p1) {
    size_t next;
    const char* line = text + p;
    const int ll = line_len_at(text, len, p, &next);
    const uint32_t at = (uint32_t)p;
    p = next;
    if (ll < 6) continue;  // no 6-column record name (a bare "END" is not Bio's "END   ")
    Rec r;
    r.line = at;
    const bool is_atom = !memcmp(line, "ATOM  ", 6), is_het = !is_atom && !memcmp(line, "HETATM", 6);
    if (!is_atom && !is_het) {
      if (!memcmp(line, "MODEL ", 6)) r.kind = R_MODEL;
      else if (!memcmp(line, "ENDMDL", 6)) r.kind = R_ENDMDL;
      else if (!memcmp(line, "CONECT", 6) || !memcmp(line, "END   ", 6)) r.kind = R_STOP;
      else continue;  // any other record: Bio skips it
      out->push_back(r);
      continue;
    }
    r.kind = is_atom ? R_ATOM : R_HETATM;
    const Field name = field(line, ll, 12, 16);
    r.altloc = 16 < ll ? line[16] : ' ';
    const Field resname = field(line, ll, 17, 20);
    r.chain = 21 < ll ? line[21] : ' ';
    r.icode = 26 < ll ? line[26] : ' ';
    int resseq;
    double x = 0.0, y = 0.0, z = 0.0, occ = 0.0;
    if (!parse_int(field(line, ll, 22, 26), &resseq) ||
        !(coord_fixed(line, ll, 30, &x) || parse_double(field(line, ll, 30, 38), &x)) ||
        !(coord_fixed(line, ll, 38, &y) || parse_double(field(line, ll, 38, 46), &y)) ||
        !(coord_fixed(line, ll, 46, &z) || parse_double(field(line, ll, 46, 54), &z))) {
      r.kind = R_BAD_COORD;
      out->push_back(r);
      continue;
    }
    const Field occ_s = field(line, ll, 54, 60);
    if (!occ_s.empty() && !parse_double(occ_s, &occ)) {
      r.kind = R_BAD_OCC;
      out->push_back(r);
      continue;
    }
    r.resseq = resseq;
    r.resname = pack_name(resname.p, resname.n);
    r.het = is_het ? ((resname.n == 3 && (r.resname == pack_name("HOH", 3) || r.resname == pack_name("WAT", 3))) ? 1 : 2)
                   : 0;
    r.restype = (uint8_t)restype_index(resname);
    r.atom = (int8_t)(name.n >= 1 && name.n <= 4 ? T.find(pack_name(name.p, name.n)) : -1);
    r.xyz[0] = (float)x;
    r.xyz[1] = (float)y;
    r.xyz[2] = (float)z;
    r.occ = occ;
    out->push_back(r);
  }
}

// ---- pass 2 (sequential per file): Bio's reading order over the records of all chunks
void assemble(const char* text, size_t len, const std::vector<std::vector<Rec>>& chunks, char chain_filter,
              Parsed* out) {
  int models = 0;
  bool seen_atom_before_model = false, in_first = true, started = false;
  std::vector<Chain> chains;
  std::vector<Res> res;
  res.reserve(len / 600 + 16);  // ~8 atom records of ~81 bytes per residue
  auto line_text = [&](uint32_t at) {
    size_t next;
    const int ll = line_len_at(text, len, at, &next);
    return std::string(text + at, std::min(ll, 80));
  };
  bool stop = false;
  for (const auto& recs : chunks) {
    for (const Rec& r : recs) {
      // Bio's header ends at the first ATOM/HETATM/MODEL record and the atomic data at the first
      // CONECT or "END   " record
      if (r.kind == R_MODEL) {
        started = true;
        ++models;
        in_first = models == 1;
        continue;
      }
      if (!started && r.kind != R_ATOM && r.kind != R_HETATM && r.kind != R_BAD_COORD && r.kind != R_BAD_OCC)
        continue;
      if (r.kind == R_STOP) {
        stop = true;
        break;
      }
      if (r.kind == R_ENDMDL) {
        in_first = false;
        continue;
      }
      started = true;
      if (models == 0) seen_atom_before_model = true;
      if (!in_first && models > 0) continue;
      if (r.kind == R_BAD_COORD || r.kind == R_BAD_OCC) {
        out->status = PST_E_INVALID;
        out->error = (r.kind == R_BAD_COORD ? "malformed ATOM/HETATM record: " : "malformed occupancy: ") +
                     line_text(r.line);
        return;
      }
      const uint64_t key = (uint64_t)r.het | ((uint64_t)(uint32_t)(r.resseq + 1024) & 0xffffffu) << 2 |
                           (uint64_t)(unsigned char)r.icode << 26 |
                           (r.het == 2 ? (uint64_t)r.resname << 34 : 0ull);
      Chain* ch = nullptr;
      for (auto& c : chains)
        if (c.id == r.chain) ch = &c;
      if (!ch) {
        chains.push_back(Chain{r.chain, ~0ull, -1, {}, {}});
        ch = &chains.back();
      }
      int ri;
      if (ch->last_res >= 0 && ch->last_key == key) {  // records of a residue are contiguous
        ri = ch->last_res;
      } else {
        auto it = ch->index.find(key);
        if (it == ch->index.end()) {
          ri = (int)res.size();
          res.emplace_back();
          Res& nr = res.back();
          nr.resseq = r.resseq;
          nr.icode = r.icode;
          nr.restype = r.restype;
          nr.present = 0;
          ch->index.emplace(key, ri);
          ch->residues.push_back(ri);
        } else {
          ri = it->second;
        }
        ch->last_key = key;
        ch->last_res = ri;
      }
      const int a = r.atom;
      if (a < 0) continue;  // not an atom37 atom: never reaches the output
      Res& x = res[ri];
      const uint64_t bit = 1ull << a;
      if (!(x.present & bit) || (r.altloc != ' ' && r.occ > x.occ[a])) {
        x.present |= bit;
        x.xyz[a][0] = r.xyz[0];
        x.xyz[a][1] = r.xyz[1];
        x.xyz[a][2] = r.xyz[2];
        x.occ[a] = r.occ;
      }
    }
    if (stop) break;
  }
  const int n_models = (models || seen_atom_before_model) ? std::max(models, 1) : 0;
  if (n_models != 1) {
    out->status = PST_E_INVALID;
    out->error = "Only single model PDBs are supported. Found " + std::to_string(n_models) + " models.";
    return;
  }
  size_t n_keep = 0;
  for (const auto& ch : chains) {
    if (chain_filter && ch.id != chain_filter) continue;
    for (int ri : ch.residues) {
      const Res& r = res[ri];
      if (r.icode != ' ') {
        out->status = PST_E_INVALID;
        out->error = std::string("PDB contains an insertion code at chain ") + ch.id + " and residue index " +
                     std::to_string(r.resseq) + ". These are not supported.";
        return;
      }
      n_keep += r.present != 0;
    }
  }
  out->pos.assign(n_keep * pst::kAtomTypes * 3, 0.0f);
  out->flags.resize(n_keep * pst::kAtomTypes);
  out->aatype.resize(n_keep);
  size_t k = 0;
  for (const auto& ch : chains) {
    if (chain_filter && ch.id != chain_filter) continue;
    for (int ri : ch.residues) {
      const Res& r = res[ri];
      if (!r.present) continue;  // no atom37 atom: skipped (protein_structure_sample.py:228-230)
      float* pos = out->pos.data() + k * pst::kAtomTypes * 3;
      uint8_t* fl = out->flags.data() + k * pst::kAtomTypes;
      for (int a = 0; a < pst::kAtomTypes; ++a) fl[a] = (uint8_t)(pst::kResAtomExists[r.restype][a] << 1);
      for (uint64_t m = r.present; m; m &= m - 1) {  // the present slots (absent ones stay 0)
        const int a = __builtin_ctzll(m);
        pos[3 * a + 0] = r.xyz[a][0];
        pos[3 * a + 1] = r.xyz[a][1];
        pos[3 * a + 2] = r.xyz[a][2];
        fl[a] |= 1;
      }
      out->aatype[k] = r.restype;
      ++k;
    }
  }
  out->n = (int64_t)n_keep;
}

// Line-aligned chunk starts of a text: about `target` bytes each, cut after a '\n'
std::vector<size_t> chunk_starts(const char* text, size_t len, size_t target) {
  std::vector<size_t> st{0};
  size_t p = target;
  while (p < len) {
    const char* nl = (const char*)memchr(text + p, '\n', len - p);
    if (!nl || (size_t)(nl - text) + 1 >= len) break;
    st.push_back((size_t)(nl - text) + 1);
    p = st.back() + target;
  }
  return st;
}

bool read_file(const char* path, std::string* s, std::string* err) {
  FILE* f = fopen(path, "rb");
  if (!f) {
    *err = std::string("cannot open ") + path;
    return false;
  }
  fseek(f, 0, SEEK_END);
  long n = ftell(f);
  fseek(f, 0, SEEK_SET);
  s->resize(n > 0 ? (size_t)n : 0);
  size_t got = n > 0 ? fread(&(*s)[0], 1, (size_t)n, f) : 0;
  fclose(f);
  if ((long)got != n) {
    *err = std::string("short read: ") + path;
    return false;
  }
  return true;
}

}  // namespace

struct pst_pdb_batch {
  std::vector<Parsed> items;
};

namespace {

// fn(i) for i < n on n_threads threads of the process-wide pool, largest `size` first (the biggest
// file bounds the call)
int run_pool(int32_t n, int32_t n_threads, const std::function<size_t(int)>& size, const std::function<void(int)>& fn) {
  std::vector<int> order(n);
  std::vector<size_t> sz(n);
  for (int i = 0; i < n; ++i) {
    order[i] = i;
    sz[i] = size(i);
  }
  std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return sz[a] > sz[b]; });
  pst::HostPool::get().run(n, n_threads > 0 ? n_threads : 1, [&](int i) { fn(order[i]); });
  return PST_OK;
}

// Chunk size of pass 1: a 320 KB PDB file (the largest CASP14 one) splits into ~7 chunks
constexpr size_t kScanChunk = 48 << 10;

// Both passes over the n texts of a batch (items already marked failed are skipped) in ONE pool
// job: the tasks are the pass-1 chunks of all texts, largest text first; the worker that scans the
// LAST chunk of a text runs that text's pass 2 right away. A text's pass 2 (sequential, Bio's
// order) therefore overlaps the other texts' pass 1 instead of waiting for every chunk of the batch
// (two pool jobs before: the largest file's pass 2 ran after all of pass 1, on one thread).
void parse_texts(int32_t n, const char* const* texts, const size_t* lens, char chain_id, int32_t n_threads,
                 std::vector<Parsed>& items) {
  std::vector<std::vector<size_t>> starts(n);
  std::vector<std::vector<std::vector<Rec>>> recs(n);
  std::vector<std::pair<int, int>> tasks;
  std::vector<int> order;
  for (int32_t i = 0; i < n; ++i)
    if (items[i].status == PST_OK) order.push_back(i);
  std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return lens[a] > lens[b]; });
  std::unique_ptr<std::atomic<int>[]> left(new std::atomic<int>[std::max(1, n)]);
  for (int i : order) {
    starts[i] = chunk_starts(texts[i], lens[i], kScanChunk);
    recs[i].resize(starts[i].size());
    left[i].store((int)starts[i].size());
    for (int c = 0; c < (int)starts[i].size(); ++c) tasks.emplace_back(i, c);
  }
  auto chunk_end = [&](int i, int c) { return c + 1 < (int)starts[i].size() ? starts[i][c + 1] : lens[i]; };
  pst::HostPool::get().run((int32_t)tasks.size(), n_threads > 0 ? n_threads : 1, [&](int t) {
    const int i = tasks[t].first, c = tasks[t].second;
    scan_chunk(texts[i], lens[i], starts[i][c], chunk_end(i, c), &recs[i][c]);
    if (left[i].fetch_sub(1, std::memory_order_acq_rel) == 1) {  // this text's last chunk: pass 2
      assemble(texts[i], lens[i], recs[i], chain_id, &items[i]);
      std::vector<std::vector<Rec>>().swap(recs[i]);
    }
  });
}

}  // namespace

namespace {
// positions as float (pst_pdb_batch_copy_f32: the parser's values are Bio's float32 atom.coord,
// copied as they are) or double (pst_pdb_batch_copy: widened, exact)
template <typename T>
int batch_copy(const pst_pdb_batch* b, T* positions, uint8_t* flags, uint8_t* aatype, int64_t* offsets,
               int32_t* status) {
  if (!b) return PST_E_INVALID;
  const int32_t n = (int32_t)b->items.size();
  std::vector<int64_t> off(n + 1, 0);
  for (int32_t i = 0; i < n; ++i) off[i + 1] = off[i] + b->items[i].n;
  if (offsets) memcpy(offsets, off.data(), sizeof(int64_t) * (n + 1));
  for (int32_t i = 0; i < n; ++i)
    if (status) status[i] = b->items[i].status;
  // the copies (~481 B per residue as float32) on a few threads from a quarter megabyte on
  const int64_t bytes = off[n] * (37 + 111 * (int64_t)sizeof(T));
  const int threads = bytes > (256 << 10) ? 8 : 1;  // the pool's workers are hot after the parse
  run_pool(n, threads, [&](int i) { return (size_t)b->items[i].n; }, [&](int i) {
    const Parsed& it = b->items[i];
    const int64_t r = off[i];
    if (positions && it.n) {
      if (sizeof(T) == sizeof(float)) {
        memcpy(positions + r * 111, it.pos.data(), sizeof(float) * 111 * it.n);
      } else {
        const float* src = it.pos.data();
        T* dst = positions + r * 111;
        for (int64_t k = 0; k < 111 * (int64_t)it.n; ++k) dst[k] = (T)src[k];
      }
    }
    if (flags && it.n) memcpy(flags + r * 37, it.flags.data(), 37 * it.n);
    if (aatype && it.n) memcpy(aatype + r, it.aatype.data(), it.n);
  });
  return PST_OK;
}
}  // namespace

extern "C" {

int pst_pdb_parse_strings(const char* const* texts, const size_t* lens, int32_t n, char chain_id, int32_t n_threads,
                          pst_pdb_batch** out) {
  if (!out || n < 0 || (n > 0 && (!texts || !lens))) return PST_E_INVALID;
  auto* b = new pst_pdb_batch();
  b->items.resize(n);
  parse_texts(n, texts, lens, chain_id, n_threads, b->items);
  *out = b;
  return PST_OK;
}

int pst_pdb_parse_files(const char* const* paths, int32_t n, char chain_id, int32_t n_threads, pst_pdb_batch** out) {
  if (!out || n < 0 || (n > 0 && !paths)) return PST_E_INVALID;
  auto* b = new pst_pdb_batch();
  b->items.resize(n);
  std::vector<std::string> text(n);
  run_pool(n, n_threads, [&](int i) {
    struct stat st;
    return stat(paths[i], &st) == 0 ? (size_t)st.st_size : (size_t)0;
  }, [&](int i) {
    std::string err;
    if (!read_file(paths[i], &text[i], &err)) {
      b->items[i].status = PST_E_INVALID;
      b->items[i].error = err;
    }
  });
  std::vector<const char*> tp(n);
  std::vector<size_t> tl(n);
  for (int32_t i = 0; i < n; ++i) {
    tp[i] = text[i].data();
    tl[i] = text[i].size();
  }
  parse_texts(n, tp.data(), tl.data(), chain_id, n_threads, b->items);
  *out = b;
  return PST_OK;
}

int pst_pdb_batch_sizes(const pst_pdb_batch* b, int32_t* n, int64_t* n_residues) {
  if (!b) return PST_E_INVALID;
  int64_t r = 0;
  for (const auto& it : b->items) r += it.n;
  if (n) *n = (int32_t)b->items.size();
  if (n_residues) *n_residues = r;
  return PST_OK;
}

int pst_pdb_batch_copy(const pst_pdb_batch* b, double* positions, uint8_t* flags, uint8_t* aatype, int64_t* offsets,
                       int32_t* status) {
  return batch_copy(b, positions, flags, aatype, offsets, status);
}

int pst_pdb_batch_copy_f32(const pst_pdb_batch* b, float* positions, uint8_t* flags, uint8_t* aatype,
                           int64_t* offsets, int32_t* status) {
  return batch_copy(b, positions, flags, aatype, offsets, status);
}

const char* pst_pdb_batch_error(const pst_pdb_batch* b, int32_t i) {
  if (!b || i < 0 || (size_t)i >= b->items.size()) return "invalid index";
  return b->items[i].error.c_str();
}

void pst_pdb_batch_free(pst_pdb_batch* b) { delete b; }

int pst_write_files(int32_t n, const char* const* paths, const void* const* data, const size_t* lens,
                    int32_t n_threads) {
  if (n < 0 || (n > 0 && (!paths || !data || !lens))) return PST_E_INVALID;
  std::atomic<int> failed(-1);
  pst::HostPool::get().run(n, n_threads > 0 ? n_threads : 1, [&](int i) {
    FILE* f = fopen(paths[i], "wb");
    bool ok = f != nullptr;
    if (ok && lens[i]) ok = fwrite(data[i], 1, lens[i], f) == lens[i];
    if (f && fclose(f) != 0) ok = false;
    if (!ok) failed.store(i);
  });
  return failed.load() < 0 ? PST_OK : PST_E_INVALID;
}

}  // extern "C"
