// kmc_state_hash.h — the per-step parity fingerprint (FNV-1a 64) of a host
// state view, in reference order: for every receptor its 16 beads
// (R_{x,y,z}[i][j][k], j,k = 1..4) then protein_status[i][2], [3],
// res_nei[i][2], [4], [3]; for every ligand and j = 1..4 its two beads then
// protein_status[.][j], res_nei[.][j]; then the five counters and the step.
// Coordinates are hashed as IEEE bit patterns, so -0.0 != +0.0: the hash only
// matches when the arithmetic is bit-identical.
#pragma once
#include <stdint.h>
#include <string.h>
#include "../../include/kmc.h"

namespace kmch {

struct Fnv {
  uint64_t h = 0xcbf29ce484222325ull;
  inline void bytes(const void* p, int n) {
    const unsigned char* c = (const unsigned char*)p;
    for (int i = 0; i < n; ++i) {
      h ^= c[i];
      h *= 0x100000001b3ull;
    }
  }
  inline void f64(double x) { bytes(&x, 8); }
  inline void i32(int32_t x) { bytes(&x, 4); }
  inline void i64(int64_t x) { bytes(&x, 8); }
};

inline uint64_t state_hash(int na, int nb, const kmc_state_view* v) {
  Fnv f;
  for (int i = 0; i < na; ++i) {
    for (int b = 0; b < 16; ++b)
      for (int c = 0; c < 3; ++c) f.f64(v->ra[(size_t)(b * 3 + c) * na + i]);
    for (int q = 0; q < 5; ++q) f.i32(v->a_int[(size_t)q * na + i]);
  }
  for (int i = 0; i < nb; ++i) {
    for (int j = 0; j < 4; ++j) {
      for (int k = 0; k < 2; ++k)
        for (int c = 0; c < 3; ++c) f.f64(v->rb[(size_t)((j * 2 + k) * 3 + c) * nb + i]);
      f.i32(v->b_int[(size_t)j * nb + i]);
      f.i32(v->b_int[(size_t)(4 + j) * nb + i]);
    }
  }
  for (int q = 0; q < 5; ++q) f.i32(v->counters[q]);
  f.i64(v->step);
  return f.h;
}

}  // namespace kmch
