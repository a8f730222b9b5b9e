// Sanitizer harness for libpst's host code: the native PDB parser (pst_pdb_parse_strings /
// pst_pdb_parse_files), the persistent host pool (pst_pool.h) and the token-file writer
// (pst_write_files). Built only by `make -C protein-structure-tokenizer_amd/csrc asan` (ASan +
// UBSan) and `... tsan` (TSan) — never part of libpst.so.
//
// usage: pdb_harness OUT_DIR FILE.pdb...
// For every input: parse it from memory and from disk on 4 pool threads and require the two to
// agree; then parse mutated copies that exercise the malformed-input paths — every prefix
// truncation at 97 cut points (mid-line included), 64 seeded random byte corruptions, garbage in
// the numeric columns, a 4 KB line, NUL bytes, CR line ends, an empty text, an END-only text, a
// second MODEL — where any status is acceptable but the process must not fault or trip a
// sanitizer. Two host threads parse concurrently (the pool serialises them: TSan's case). All
// parsed batches are written as files through pst_write_files and read back byte for byte.
// Exit code 0 = clean; sanitizer reports abort with their own non-zero code.
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <fstream>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include "../../../include/pst.h"

namespace {

int g_fail = 0;
#define CHECK(c)                                                        \
  do {                                                                  \
    if (!(c)) {                                                         \
      fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++g_fail;                                                         \
    }                                                                   \
  } while (0)

struct Out {
  std::vector<double> pos;
  std::vector<uint8_t> flags, aatype;
  std::vector<int64_t> off;
  std::vector<int32_t> status;
};

Out copy_out(pst_pdb_batch* b) {
  int32_t n = 0;
  int64_t R = 0;
  CHECK(pst_pdb_batch_sizes(b, &n, &R) == PST_OK);
  Out o;
  o.pos.resize((size_t)R * 111 + 1);
  o.flags.resize((size_t)R * 37 + 1);
  o.aatype.resize((size_t)R + 1);
  o.off.resize((size_t)n + 1);
  o.status.resize((size_t)n + 1);
  CHECK(pst_pdb_batch_copy(b, o.pos.data(), o.flags.data(), o.aatype.data(), o.off.data(), o.status.data()) ==
        PST_OK);
  for (int32_t i = 0; i < n; ++i) CHECK(pst_pdb_batch_error(b, i) != nullptr);
  CHECK(strcmp(pst_pdb_batch_error(b, n), "invalid index") == 0);
  return o;
}

Out parse_texts(const std::vector<std::string>& texts, int threads, char chain = 0) {
  std::vector<const char*> p;
  std::vector<size_t> l;
  for (const auto& t : texts) {
    p.push_back(t.data());
    l.push_back(t.size());
  }
  pst_pdb_batch* b = nullptr;
  CHECK(pst_pdb_parse_strings(p.data(), l.data(), (int32_t)texts.size(), chain, threads, &b) == PST_OK);
  Out o = copy_out(b);
  pst_pdb_batch_free(b);
  return o;
}

std::vector<std::string> mutations(const std::string& t, uint32_t seed) {
  std::vector<std::string> v;
  for (int k = 0; k <= 96; ++k) v.push_back(t.substr(0, t.size() * k / 96));  // prefix truncations
  uint32_t s = seed * 2654435761u + 1;
  auto rnd = [&]() {
    s = s * 1664525u + 1013904223u;
    return s >> 8;
  };
  for (int k = 0; k < 64; ++k) {  // random byte corruption, 1-8 bytes each
    std::string c = t;
    const int nb = 1 + (int)(rnd() % 8);
    for (int j = 0; j < nb && !c.empty(); ++j) c[rnd() % c.size()] = (char)(rnd() & 0xff);
    v.push_back(c);
  }
  {  // letters in the coordinate / occupancy columns of every 7th ATOM line
    std::string c = t;
    size_t at = 0;
    int line = 0;
    while ((at = c.find("ATOM  ", at)) != std::string::npos) {
      if (line++ % 7 == 0 && at + 60 < c.size()) memcpy(&c[at + 30], "xx.yyyzz", 8);
      at += 6;
    }
    v.push_back(c);
  }
  v.push_back(std::string(4096, 'A') + "\n" + t);  // a long line first
  {
    std::string c = t;  // NUL bytes inside the text
    for (size_t i = 13; i < c.size(); i += 977) c[i] = '\0';
    v.push_back(c);
  }
  {
    std::string c;  // CRLF line ends
    for (char ch : t) {
      if (ch == '\n') c += '\r';
      c += ch;
    }
    v.push_back(c);
  }
  v.push_back("");
  v.push_back("END\n");
  v.push_back("MODEL        1\n" + t.substr(0, t.size() / 2) + "ENDMDL\nMODEL        2\n" + t.substr(0, t.size() / 2));
  return v;
}

std::string read_all(const char* path) {
  std::ifstream f(path, std::ios::binary);
  std::stringstream ss;
  ss << f.rdbuf();
  return ss.str();
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 3) {
    fprintf(stderr, "usage: %s OUT_DIR FILE.pdb...\n", argv[0]);
    return 2;
  }
  const std::string out_dir = argv[1];
  std::vector<std::string> paths(argv + 2, argv + argc), texts;
  for (const auto& p : paths) texts.push_back(read_all(p.c_str()));

  // memory vs disk, 1 vs 4 threads: the same batch
  Out a = parse_texts(texts, 4);
  Out a1 = parse_texts(texts, 1);
  CHECK(a.off == a1.off && a.pos == a1.pos && a.flags == a1.flags && a.aatype == a1.aatype);
  {
    std::vector<const char*> pp;
    for (const auto& p : paths) pp.push_back(p.c_str());
    pst_pdb_batch* b = nullptr;
    CHECK(pst_pdb_parse_files(pp.data(), (int32_t)pp.size(), 0, 4, &b) == PST_OK);
    Out d = copy_out(b);
    pst_pdb_batch_free(b);
    CHECK(d.off == a.off && d.pos == a.pos && d.flags == a.flags && d.status == a.status);
    const char* missing[] = {"/nonexistent/x.pdb"};
    CHECK(pst_pdb_parse_files(missing, 1, 0, 2, &b) == PST_OK);
    Out m = copy_out(b);
    CHECK(m.status[0] == PST_E_INVALID && m.off[1] == 0);
    pst_pdb_batch_free(b);
  }
  // chain filter on every input
  Out ca = parse_texts(texts, 4, 'A');
  CHECK(ca.off.size() == a.off.size());
  CHECK(pst_pdb_parse_strings(nullptr, nullptr, 1, 0, 1, nullptr) == PST_E_INVALID);

  // malformed inputs: whole mutated batches (one batch per source file) on 4 threads, while a
  // second host thread parses the clean batch concurrently
  size_t n_mut = 0, n_ok = 0;
  std::thread other([&] {
    for (int r = 0; r < 4; ++r) {
      Out o = parse_texts(texts, 3);
      CHECK(o.pos == a.pos);
    }
  });
  for (size_t i = 0; i < texts.size(); ++i) {
    std::vector<std::string> mut = mutations(texts[i], (uint32_t)i);
    Out o = parse_texts(mut, 4);
    n_mut += mut.size();
    for (size_t j = 0; j < mut.size(); ++j) n_ok += o.status[j] == PST_OK;
  }
  other.join();

  // the writer: one file per input holding its parsed positions, written on 4 pool threads
  std::vector<std::string> names;
  std::vector<const void*> data;
  std::vector<size_t> lens;
  for (size_t i = 0; i < texts.size(); ++i) {
    names.push_back(out_dir + "/w" + std::to_string(i) + ".bin");
    data.push_back(a.pos.data() + a.off[i] * 111);
    lens.push_back(sizeof(double) * 111 * (size_t)(a.off[i + 1] - a.off[i]));
  }
  std::vector<const char*> np;
  for (const auto& s : names) np.push_back(s.c_str());
  CHECK(pst_write_files((int32_t)names.size(), np.data(), data.data(), lens.data(), 4) == PST_OK);
  for (size_t i = 0; i < names.size(); ++i) {
    const std::string got = read_all(names[i].c_str());
    CHECK(got.size() == lens[i] && (lens[i] == 0 || memcmp(got.data(), data[i], lens[i]) == 0));
  }
  const char* bad[] = {"/nonexistent/dir/f.bin"};
  const void* bd[] = {data[0]};
  const size_t bl[] = {8};
  CHECK(pst_write_files(1, bad, bd, bl, 2) == PST_E_INVALID);

  printf("pdb_harness: %zu inputs, %lld residues, %zu malformed variants (%zu parsed OK), %d check failures\n",
         texts.size(), (long long)a.off.back(), n_mut, n_ok, g_fail);
  return g_fail ? 1 : 0;
}
