// kmc_philox.h — keyed counter-based RNG (Philox4x32-10, Salmon et al. SC'11).
//
// Replaces the reference's rand2() (main.cpp:2313-2326), which re-seeds a
// std::mt19937_64 from the wall clock on every call and therefore can never be
// reproduced.  Every uniform the simulation consumes is addressed by a key
// (seed, replica) and a 128-bit counter naming the draw site:
//
//     ctr = { a, b, step, (domain << 24) | sub }
//
//   domain DIFF   a = trigger protein index (0-based), b = 0, sub = draw pair
//                 (two doubles per Philox block; free ligand uses 6 draws →
//                 pairs 0..2; receptor / dimer / complex use 3 → pairs 0..1)
//   domain RL     a = receptor, b = ligand, sub = binding site k (2..4)
//   domain MONO   a = receptor i, b = receptor j   (ordered pair, main.cpp:1952)
//   domain CIS    a = receptor i, b = receptor j   (ordered pair, main.cpp:2007)
//   domain RLD / MD / CD   a = receptor, b = 0      (dissociations)
//   domain SHUF   a = root ligand, b = shuffle call, sub = position
//   domain INIT   a = protein, b = attempt, sub = draw pair (placement)
//
// Because a draw depends only on its address, never on how many draws came
// before it, the GPU can evaluate all units and all candidate pairs
// concurrently and still reproduce the sequential CPU oracle bit for bit.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__) || defined(__HIP__)
#define KMC_HD_P __attribute__((host, device, always_inline)) inline
#else
#define KMC_HD_P static inline
#endif

namespace kmcr {

enum Domain : uint32_t {
  DOM_DIFF = 1,
  DOM_RL = 2,
  DOM_MONO = 3,
  DOM_CIS = 4,
  DOM_RLD = 5,
  DOM_MD = 6,
  DOM_CD = 7,
  DOM_SHUF = 8,
  DOM_INIT = 9,
};

struct u4 {
  uint32_t x, y, z, w;
};

KMC_HD_P void mulhilo(uint32_t a, uint32_t b, uint32_t* hi, uint32_t* lo) {
  uint64_t p = (uint64_t)a * (uint64_t)b;
  *hi = (uint32_t)(p >> 32);
  *lo = (uint32_t)p;
}

// Philox4x32 with 10 rounds.
KMC_HD_P u4 philox4x32_10(u4 c, uint32_t k0, uint32_t k1) {
  const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
  const uint32_t W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
  for (int r = 0; r < 10; ++r) {
    uint32_t hi0, lo0, hi1, lo1;
    mulhilo(M0, c.x, &hi0, &lo0);
    mulhilo(M1, c.z, &hi1, &lo1);
    u4 n;
    n.x = hi1 ^ c.y ^ k0;
    n.y = lo1;
    n.z = hi0 ^ c.w ^ k1;
    n.w = lo0;
    c = n;
    k0 += W0;
    k1 += W1;
  }
  return c;
}

struct Key {
  uint32_t k0, k1;
};

KMC_HD_P Key make_key(uint64_t seed, uint32_t replica) {
  Key k;
  k.k0 = (uint32_t)seed;
  k.k1 = (uint32_t)(seed >> 32) + replica * 0x9E3779B9u;
  return k;
}

// 53-bit uniform in [0, 1) from two 32-bit words (exact in double).
KMC_HD_P double u01(uint32_t a, uint32_t b) {
  return (double)((uint64_t)(a >> 5) * 67108864ull + (uint64_t)(b >> 6)) *
         1.1102230246251565404236316680908203125e-16;  // 2^-53
}

KMC_HD_P u4 block(Key k, uint32_t dom, uint32_t a, uint32_t b, uint32_t step, uint32_t sub) {
  u4 c;
  c.x = a;
  c.y = b;
  c.z = step;
  c.w = (dom << 24) | (sub & 0xffffffu);
  return philox4x32_10(c, k.k0, k.k1);
}

// Two uniforms from one block.
KMC_HD_P void uniform2(Key k, uint32_t dom, uint32_t a, uint32_t b, uint32_t step, uint32_t sub,
                       double* u0, double* u1) {
  u4 r = block(k, dom, a, b, step, sub);
  *u0 = u01(r.x, r.y);
  *u1 = u01(r.z, r.w);
}

KMC_HD_P double uniform(Key k, uint32_t dom, uint32_t a, uint32_t b, uint32_t step, uint32_t sub) {
  u4 r = block(k, dom, a, b, step, sub);
  return u01(r.x, r.y);
}

// Non-negative 31-bit integer, the keyed stand-in for std::rand() in the
// random_shuffle passes (main.cpp:1285, 1345, 1413, 1597).
KMC_HD_P uint32_t rand31(Key k, uint32_t dom, uint32_t a, uint32_t b, uint32_t step, uint32_t sub) {
  u4 r = block(k, dom, a, b, step, sub);
  return r.x >> 1;
}

}  // namespace kmcr
