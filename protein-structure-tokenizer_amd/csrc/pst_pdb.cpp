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

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <functional>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/pst.h"
#include "pst_residue_tables.h"

namespace {

struct AtomRec {
  char name[5];
  float xyz[3];
  double occ;
};

struct Residue {
  std::string resname;
  char icode;
  int resseq;
  std::vector<AtomRec> atoms;
};

struct ResKey;
struct ResKeyHash;

struct Parsed {
  int status = PST_OK;
  std::string error;
  std::vector<double> pos;     // [n,37,3]
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
  std::string str() const { return std::string(p, n); }
};

Field field(const char* line, int len, int a, int b) {
  if (b > len) b = len;
  while (a < b && (line[a] == ' ' || line[a] == '\t')) ++a;
  while (b > a && (line[b - 1] == ' ' || line[b - 1] == '\t')) --b;
  return Field{line + a, a < b ? b - a : 0};
}

bool parse_int(Field f, int* v) {
  if (f.empty() || f.n > 15) return false;
  char buf[16];
  memcpy(buf, f.p, f.n);
  buf[f.n] = 0;
  errno = 0;
  char* end = nullptr;
  long r = strtol(buf, &end, 10);
  if (errno || *end) return false;
  *v = (int)r;
  return true;
}

// Python float() of a field. Fast path for the fixed-point form PDB writers emit ("-12.345"):
// mantissa and 10^k are exact doubles, so one IEEE division is the correctly rounded value —
// the same double strtod returns. Anything else goes through strtod.
bool parse_double(Field f, double* v) {
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

int restype_index(const std::string& resname) {
  for (int r = 0; r < 20; ++r)
    if (resname == pst::kResName3[r]) return r;
  return 20;
}

struct ResKey {
  std::string het;
  int resseq;
  char icode;
  bool operator==(const ResKey& o) const { return resseq == o.resseq && icode == o.icode && het == o.het; }
};
struct ResKeyHash {
  size_t operator()(const ResKey& k) const {
    return std::hash<std::string>()(k.het) ^ ((size_t)k.resseq * 131u) ^ ((size_t)(unsigned char)k.icode << 20);
  }
};

struct Chain {
  char id;
  std::vector<Residue> residues;
  std::vector<ResKey> keys;
  std::unordered_map<ResKey, int, ResKeyHash> index;
};

int atom_index(const char* name) {
  for (int a = 0; a < pst::kAtomTypes; ++a)
    if (!strcmp(name, pst::kAtomNames[a])) return a;
  return -1;
}

void parse_one(const char* text, size_t len, char chain_filter, Parsed* out) {
  int models = 0;
  bool seen_atom_before_model = false, in_first = true, started = false;
  std::vector<Chain> chains;
  size_t p = 0;
  while (p < len) {
    size_t q = p;
    while (q < len && text[q] != '\n' && text[q] != '\r') ++q;
    const char* line = text + p;
    const int ll = (int)(q - p);
    p = (q + 1 < len && text[q] == '\r' && text[q + 1] == '\n') ? q + 2 : q + 1;  // \n, \r\n or \r
    // Bio names a record by its exact first 6 columns; its header ends at the first ATOM/HETATM/
    // MODEL record and the atomic data at the first CONECT or "END   " record
    auto rec = [&](const char* name6) { return ll >= 6 && !memcmp(line, name6, 6); };
    const bool is_atom = rec("ATOM  "), is_het = rec("HETATM"), is_model = rec("MODEL ");
    if (!started) {
      if (!is_atom && !is_het && !is_model) continue;
      started = true;
    }
    if (rec("CONECT") || rec("END   ")) break;
    if (is_model) {
      ++models;
      in_first = models == 1;
      continue;
    }
    if (rec("ENDMDL")) {
      in_first = false;
      continue;
    }
    if (!is_atom && !is_het) continue;
    if (models == 0) seen_atom_before_model = true;
    if (!in_first && models > 0) continue;
    const Field name = field(line, ll, 12, 16);
    const char altloc = 16 < ll ? line[16] : ' ';
    const Field resname = field(line, ll, 17, 20);
    const char chain = 21 < ll ? line[21] : ' ';
    const char icode = 26 < ll ? line[26] : ' ';
    int resseq;
    double x = 0.0, y = 0.0, z = 0.0, occ = 0.0;
    if (!parse_int(field(line, ll, 22, 26), &resseq) || !parse_double(field(line, ll, 30, 38), &x) ||
        !parse_double(field(line, ll, 38, 46), &y) || !parse_double(field(line, ll, 46, 54), &z)) {
      out->status = PST_E_INVALID;
      out->error = "malformed ATOM/HETATM record: " + std::string(line, std::min(ll, 80));
      return;
    }
    const Field occ_s = field(line, ll, 54, 60);
    if (!occ_s.empty() && !parse_double(occ_s, &occ)) {
      out->status = PST_E_INVALID;
      out->error = "malformed occupancy: " + std::string(line, std::min(ll, 80));
      return;
    }
    ResKey key{" ", resseq, icode};
    if (is_het) key.het = (resname.eq("HOH") || resname.eq("WAT")) ? std::string("W") : "H_" + resname.str();
    Chain* ch = nullptr;
    for (auto& c : chains)
      if (c.id == chain) ch = &c;
    if (!ch) {
      chains.push_back(Chain{chain, {}, {}, {}});
      ch = &chains.back();
    }
    int ri = -1;
    if (!ch->keys.empty() && ch->keys.back() == key) {  // records of a residue are contiguous
      ri = (int)ch->keys.size() - 1;
    } else {
      auto it = ch->index.find(key);
      if (it == ch->index.end()) {
        ri = (int)ch->residues.size();
        ch->index.emplace(key, ri);
        ch->keys.push_back(key);
        ch->residues.push_back(Residue{resname.str(), icode, resseq, {}});
      } else {
        ri = it->second;
      }
    }
    Residue& res = ch->residues[ri];
    AtomRec a{};
    memcpy(a.name, name.p, std::min(name.n, 4));
    a.xyz[0] = (float)x;
    a.xyz[1] = (float)y;
    a.xyz[2] = (float)z;
    a.occ = occ;
    AtomRec* prev = nullptr;
    for (auto& r : res.atoms)
      if (!strcmp(r.name, a.name)) prev = &r;
    if (!prev) {
      res.atoms.push_back(a);
    } else if (altloc != ' ' && occ > prev->occ) {
      *prev = a;
    }
  }
  const int n_models = (models || seen_atom_before_model) ? std::max(models, 1) : 0;
  if (n_models != 1) {
    out->status = PST_E_INVALID;
    out->error = "Only single model PDBs are supported. Found " + std::to_string(n_models) + " models.";
    return;
  }
  for (const auto& ch : chains) {
    if (chain_filter && ch.id != chain_filter) continue;
    for (const auto& res : ch.residues) {
      if (res.icode != ' ') {
        out->status = PST_E_INVALID;
        out->error = std::string("PDB contains an insertion code at chain ") + ch.id + " and residue index " +
                     std::to_string(res.resseq) + ". These are not supported.";
        return;
      }
      double pos[pst::kAtomTypes][3] = {};
      uint8_t mask[pst::kAtomTypes] = {};
      int n_atoms = 0;
      for (const auto& a : res.atoms) {
        const int ai = atom_index(a.name);
        if (ai < 0) continue;
        for (int d = 0; d < 3; ++d) pos[ai][d] = (double)a.xyz[d];
        if (!mask[ai]) ++n_atoms;
        mask[ai] = 1;
      }
      if (n_atoms == 0) continue;
      const int rt = restype_index(res.resname);
      out->aatype.push_back((uint8_t)rt);
      for (int ai = 0; ai < pst::kAtomTypes; ++ai) {
        for (int d = 0; d < 3; ++d) out->pos.push_back(pos[ai][d]);
        out->flags.push_back((uint8_t)(mask[ai] | (pst::kResAtomExists[rt][ai] << 1)));
      }
      ++out->n;
    }
  }
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

int run_pool(int32_t n, int32_t n_threads, const std::function<void(int)>& fn) {
  int T = std::max(1, std::min<int>(n_threads > 0 ? n_threads : 1, n));
  std::atomic<int> next(0);
  auto worker = [&]() {
    for (int i = next++; i < n; i = next++) fn(i);
  };
  std::vector<std::thread> th;
  for (int t = 1; t < T; ++t) th.emplace_back(worker);
  worker();
  for (auto& t : th) t.join();
  return PST_OK;
}

}  // namespace

extern "C" {

int pst_pdb_parse_strings(const char* const* texts, const size_t* lens, int32_t n, char chain_id, int32_t n_threads,
                          pst_pdb_batch** out) {
  if (!out || n < 0 || (n > 0 && (!texts || !lens))) return PST_E_INVALID;
  auto* b = new pst_pdb_batch();
  b->items.resize(n);
  run_pool(n, n_threads, [&](int i) { parse_one(texts[i], lens[i], chain_id, &b->items[i]); });
  *out = b;
  return PST_OK;
}

int pst_pdb_parse_files(const char* const* paths, int32_t n, char chain_id, int32_t n_threads, pst_pdb_batch** out) {
  if (!out || n < 0 || (n > 0 && !paths)) return PST_E_INVALID;
  auto* b = new pst_pdb_batch();
  b->items.resize(n);
  run_pool(n, n_threads, [&](int i) {
    std::string s, err;
    if (!read_file(paths[i], &s, &err)) {
      b->items[i].status = PST_E_INVALID;
      b->items[i].error = err;
      return;
    }
    parse_one(s.data(), s.size(), chain_id, &b->items[i]);
  });
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
  if (!b) return PST_E_INVALID;
  int64_t r = 0;
  for (size_t i = 0; i < b->items.size(); ++i) {
    const Parsed& it = b->items[i];
    if (offsets) offsets[i] = r;
    if (status) status[i] = it.status;
    if (positions && it.n) memcpy(positions + r * 111, it.pos.data(), sizeof(double) * 111 * it.n);
    if (flags && it.n) memcpy(flags + r * 37, it.flags.data(), 37 * it.n);
    if (aatype && it.n) memcpy(aatype + r, it.aatype.data(), it.n);
    r += it.n;
  }
  if (offsets) offsets[b->items.size()] = r;
  return PST_OK;
}

const char* pst_pdb_batch_error(const pst_pdb_batch* b, int32_t i) {
  if (!b || i < 0 || (size_t)i >= b->items.size()) return "invalid index";
  return b->items[i].error.c_str();
}

void pst_pdb_batch_free(pst_pdb_batch* b) { delete b; }

}  // extern "C"
