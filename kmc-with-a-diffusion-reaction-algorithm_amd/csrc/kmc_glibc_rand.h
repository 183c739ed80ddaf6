// kmc_glibc_rand.h — glibc's rand() (random(3) TYPE_3 additive feedback
// generator, the state std::random_shuffle draws from in main.cpp:1285, 1345,
// 1413, 1597), restated with a call counter so a reference trajectory can be
// resumed mid-way.  Output for seed 1 equals glibc rand() without srand().
// Test infrastructure: used by oracle/ref_interpose.cpp and the oracle's
// stream mode only (the engine uses keyed Philox draws instead).
#pragma once
#include <stdint.h>

namespace kmcg {

struct GlibcRand {
  int32_t r[34];
  uint64_t calls = 0;
  int idx = 0;  // ring position
  uint32_t ring[34];
  explicit GlibcRand(uint32_t seed = 1) { reseed(seed); }
  void reseed(uint32_t seed) {
    int32_t s[344 + 34];
    s[0] = (int32_t)(seed == 0 ? 1 : seed);
    for (int i = 1; i < 31; ++i) {
      int64_t hi = s[i - 1] / 127773, lo = s[i - 1] % 127773;
      int64_t w = 16807 * lo - 2836 * hi;
      if (w < 0) w += 2147483647;
      s[i] = (int32_t)w;
    }
    for (int i = 31; i < 34; ++i) s[i] = s[i - 31];
    // ring holds the last 34 words; discard 310 outputs
    for (int i = 0; i < 34; ++i) ring[i] = (uint32_t)s[i];
    idx = 0;  // ring[(idx + k) % 34] = s[n - 34 + k] where n = next index
    n_ = 34;
    for (int i = 34; i < 344; ++i) next_word();
    calls = 0;
  }
  uint32_t next_word() {
    // s[n] = s[n-31] + s[n-3]
    uint32_t a = ring[(idx + (34 - 31)) % 34];  // s[n-31]
    uint32_t b = ring[(idx + (34 - 3)) % 34];   // s[n-3]
    uint32_t w = a + b;
    ring[idx] = w;  // overwrite s[n-34]
    idx = (idx + 1) % 34;
    ++n_;
    return w;
  }
  int next() {
    ++calls;
    return (int)(next_word() >> 1);
  }
  void skip(uint64_t n) {
    for (uint64_t i = 0; i < n; ++i) next();
  }
  uint64_t n_ = 0;
};

}  // namespace kmcg
