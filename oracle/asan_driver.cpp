// oracle/asan_driver.cpp — TEST INFRASTRUCTURE ONLY.
//
// Host code under AddressSanitizer + UBSan (SURVEY.md §5 "race detection /
// sanitizers"): the keyed oracle (kmc_oracle.cpp) and libkmc's host side
// (kmc_io.cpp: position.cpt tokenizer, KMCSTAT1 reader, writers, placement)
// linked into one executable built by `make -C oracle asan`.  Run by
// tests/test_sanitizers.py:
//
//   asan_driver <workdir> [cpt-file ...]
//
//  1. every given position.cpt (the reference-written fixtures, 150+50, the
//     dense scenario's box) is loaded, validated, written back and re-read;
//     then every truncation of it at 64 offsets and 200 single-byte
//     corruptions must load cleanly or fail with an error code;
//  2. a dense 150+50 oracle run (keyed, both neighbour modes) of 300 steps,
//     with exact-state save / load round trips, and corrupted / truncated /
//     foreign KMCSTAT1 files that must be refused;
//  3. the writers (parameter.log, test.gro, cluster.log, bond.dat line).
// Prints "asan_driver ok" and exits 0; a sanitizer report aborts non-zero.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../include/kmc.h"

extern "C" {
struct oracle_t;
oracle_t* oracle_create(const kmc_params* p, int rng_mode, uint64_t stream_t0, int nbmode);
void oracle_destroy(oracle_t* h);
int oracle_init_placement(oracle_t* h);
int oracle_set_state(oracle_t* h, const kmc_state_view* v);
int oracle_get_state(oracle_t* h, kmc_state_view* v);
int oracle_step(oracle_t* h, int64_t n, kmc_obs* obs, uint64_t* hashes);
uint64_t oracle_hash(oracle_t* h);
int oracle_get_clusters(oracle_t* h, int32_t* row_len, int32_t* members);
}

namespace {

struct Host {
  std::vector<double> ra, rb;
  std::vector<int32_t> ai, bi;
  kmc_state_view v;
  Host(int na, int nb) : ra((size_t)48 * na), rb((size_t)24 * nb), ai((size_t)5 * na), bi((size_t)8 * nb) {
    std::memset(&v, 0, sizeof v);
    v.ra = ra.data();
    v.rb = rb.data();
    v.a_int = ai.data();
    v.b_int = bi.data();
  }
};

int g_fail = 0;
#define CHECK(c)                                                        \
  do {                                                                  \
    if (!(c)) {                                                         \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++g_fail;                                                         \
    }                                                                   \
  } while (0)

std::vector<char> slurp(const std::string& path) {
  std::vector<char> b;
  FILE* f = std::fopen(path.c_str(), "rb");
  if (!f) return b;
  char buf[65536];
  size_t n;
  while ((n = std::fread(buf, 1, sizeof buf, f)) > 0) b.insert(b.end(), buf, buf + n);
  std::fclose(f);
  return b;
}

void spit(const std::string& path, const char* data, size_t n) {
  FILE* f = std::fopen(path.c_str(), "wb");
  if (!f) std::abort();
  if (n) std::fwrite(data, 1, n, f);
  std::fclose(f);
}

uint64_t lcg(uint64_t& s) {
  s = s * 6364136223846793005ull + 1442695040888963407ull;
  return s >> 33;
}

kmc_params dense_params() {
  kmc_params p;
  kmc_params_default(&p);
  p.box_x = p.box_y = 1000.0;
  p.box_z = 250.0;
  p.mono_cis_ass_rate = 0.01;
  p.cis_ass_rate = 0.09;
  p.diss_rate = 0.00002;
  p.mono_cis_diss_rate = 0.0002;
  p.cis_diss_rate = 0.00005;
  p.seed = 77;
  return p;
}

void fuzz_cpt(const kmc_params& p, const std::string& wd, const std::string& cpt) {
  Host h(p.n_a, p.n_b);
  CHECK(kmc_host_load_cpt(&p, cpt.c_str(), &h.v) == KMC_OK);
  (void)kmc_host_validate(&p, &h.v);
  const std::string out = wd + "/rt.cpt";
  CHECK(kmc_host_write_cpt(&p, &h.v, out.c_str()) == KMC_OK);
  Host h2(p.n_a, p.n_b);
  CHECK(kmc_host_load_cpt(&p, out.c_str(), &h2.v) == KMC_OK);
  CHECK(h2.v.step == h.v.step);
  const std::vector<char> bytes = slurp(cpt);
  CHECK(!bytes.empty());
  const std::string bad = wd + "/bad.cpt";
  for (int t = 0; t < 64; ++t) {  // truncations
    const size_t n = bytes.size() * t / 64;
    spit(bad, bytes.data(), n);
    Host x(p.n_a, p.n_b);
    CHECK(kmc_host_load_cpt(&p, bad.c_str(), &x.v) != KMC_OK);
  }
  uint64_t s = 12345;
  static const char junk[] = {'x', '-', '.', ' ', '\n', '9', 'e', '\0', '+', '\t'};
  for (int t = 0; t < 200; ++t) {  // single-byte corruptions: ok or an error, never a fault
    std::vector<char> b = bytes;
    b[lcg(s) % b.size()] = junk[lcg(s) % sizeof junk];
    spit(bad, b.data(), b.size());
    Host x(p.n_a, p.n_b);
    const int rc = kmc_host_load_cpt(&p, bad.c_str(), &x.v);
    if (rc == KMC_OK) (void)kmc_host_validate(&p, &x.v);
  }
  Host empty(p.n_a, p.n_b);
  CHECK(kmc_host_load_cpt(&p, (wd + "/does-not-exist.cpt").c_str(), &empty.v) == KMC_ERR_IO);
}

void oracle_run(const std::string& wd, int nbmode) {
  kmc_params p = dense_params();
  oracle_t* o = oracle_create(&p, 0, 1, nbmode);
  CHECK(o != nullptr);
  CHECK(oracle_init_placement(o) == 0);
  std::vector<kmc_obs> obs(300);
  CHECK(oracle_step(o, 150, obs.data(), nullptr) == 0);
  Host h(p.n_a, p.n_b);
  oracle_get_state(o, &h.v);
  CHECK(kmc_host_validate(&p, &h.v) == KMC_OK);
  const std::string st = wd + "/s.kmc";
  CHECK(kmc_host_save_state(&p, &h.v, st.c_str()) == KMC_OK);
  Host h2(p.n_a, p.n_b);
  CHECK(kmc_host_load_state(&p, st.c_str(), &h2.v) == KMC_OK);
  CHECK(kmc_state_hash(&p, &h2.v) == kmc_state_hash(&p, &h.v));
  oracle_t* o2 = oracle_create(&p, 0, 1, nbmode);
  oracle_set_state(o2, &h2.v);
  CHECK(oracle_step(o, 150, obs.data(), nullptr) == 0);
  CHECK(oracle_step(o2, 150, obs.data() + 150, nullptr) == 0);
  CHECK(oracle_hash(o) == oracle_hash(o2));
  // writers on the final state
  std::vector<int32_t> row(p.n_b), mem(p.n_a + p.n_b);
  oracle_get_clusters(o, row.data(), mem.data());
  oracle_get_state(o, &h.v);
  CHECK(kmc_host_write_parameter_log(&p, (wd + "/parameter.log").c_str()) == KMC_OK);
  CHECK(kmc_host_append_gro(&p, &h.v, (wd + "/test.gro").c_str()) == KMC_OK);
  CHECK(kmc_host_append_cluster_log(&p, 300, row.data(), mem.data(), (wd + "/cluster.log").c_str()) == KMC_OK);
  char line[256];
  CHECK(kmc_format_bond_line(&p, &obs[299], line, sizeof line) > 0);
  CHECK(kmc_format_bond_line(&p, &obs[299], line, 4) < 0 || std::strlen(line) < 4);
  // KMCSTAT1: truncated, corrupted and foreign files are refused
  const std::vector<char> bytes = slurp(st);
  const std::string bad = wd + "/bad.kmc";
  for (int t = 0; t < 32; ++t) {
    spit(bad, bytes.data(), bytes.size() * t / 32);
    Host x(p.n_a, p.n_b);
    CHECK(kmc_host_load_state(&p, bad.c_str(), &x.v) != KMC_OK);
  }
  uint64_t s = 99;
  for (int t = 0; t < 64; ++t) {
    std::vector<char> b = bytes;
    b[lcg(s) % b.size()] ^= (char)(1 + lcg(s) % 255);
    spit(bad, b.data(), b.size());
    Host x(p.n_a, p.n_b);
    CHECK(kmc_host_load_state(&p, bad.c_str(), &x.v) != KMC_OK);
  }
  kmc_params q = p;
  q.seed = 78;
  Host x(p.n_a, p.n_b);
  CHECK(kmc_host_load_state(&q, st.c_str(), &x.v) == KMC_ERR_ARG);
  oracle_destroy(o);
  oracle_destroy(o2);
}

void placement() {
  kmc_params p;
  kmc_params_default(&p);
  p.n_a = 3000;
  p.n_b = 1000;
  p.box_x = p.box_y = 6000.0;
  Host h(p.n_a, p.n_b);
  CHECK(kmc_host_init_random(&p, &h.v) == KMC_OK);
  CHECK(kmc_host_validate(&p, &h.v) == KMC_OK);
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 2) {
    std::fprintf(stderr, "usage: asan_driver <workdir> [cpt ...]\n");
    return 2;
  }
  const std::string wd = argv[1];
  kmc_params dp = dense_params();
  for (int i = 2; i < argc; ++i) fuzz_cpt(dp, wd, argv[i]);
  oracle_run(wd, 0);
  oracle_run(wd, 1);
  placement();
  if (g_fail) {
    std::fprintf(stderr, "asan_driver: %d checks failed\n", g_fail);
    return 1;
  }
  std::printf("asan_driver ok\n");
  return 0;
}
