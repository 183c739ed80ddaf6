// kmc_math.h — portable, bit-reproducible double-precision libm subset.
//
// The reference computes every geometric quantity with glibc libm
// (sin/cos in the Euler matrix, main.cpp:613-623 and its 5 copies; atan2 in
// the ligand lay-down, main.cpp:1152 and 1486; acos in gettheta,
// main.cpp:2364).  glibc's results depend on compiler flags (g++ -O2 fuses
// sin/cos pairs into sincos, which differs in the last ulp on ~0.07% of
// arguments — SURVEY.md §0.2 fact 5), and the GPU's OCML differs again.  To
// get bit-identical trajectories on the CPU oracle and on gfx950 both sides
// evaluate these functions with THIS header: the fdlibm algorithms (Cody–Waite
// argument reduction, minimax kernels), restated using only IEEE +,-,*,/,
// sqrt and exact bit manipulation.  It must be compiled with
// -ffp-contract=off on both host and device (no FMA contraction).
//
// Accuracy: < 1 ulp over the arguments the simulation produces (|x| < 2^19·π/2
// for sin/cos); checked against libm in tests/test_oracle_modes.py
// (test_portable_libm_within_one_ulp, test_portable_libm_exact_points).
#pragma once
#include <stdint.h>

#if defined(__HIPCC__) || defined(__HIP__)
#define KMC_HD __attribute__((host, device, always_inline)) inline
#else
#define KMC_HD static inline
#endif

namespace kmcm {

KMC_HD uint64_t bits(double x) { return __builtin_bit_cast(uint64_t, x); }
KMC_HD double from_bits(uint64_t u) { return __builtin_bit_cast(double, u); }
KMC_HD uint32_t hi(double x) { return (uint32_t)(bits(x) >> 32); }
KMC_HD uint32_t lo(double x) { return (uint32_t)bits(x); }
KMC_HD double with_hi_lo(uint32_t h, uint32_t l) {
  return from_bits(((uint64_t)h << 32) | (uint64_t)l);
}
KMC_HD double fabs_(double x) { return from_bits(bits(x) & 0x7fffffffffffffffull); }

// IEEE-754 correctly rounded square root (sqrtsd on x86-64; on gfx950 the
// compiler's f64 sqrt lowering is validated bit-for-bit in
// tests/test_gpu_parity.py::test_device_math_bitexact).
KMC_HD double sqrt_(double x) { return __builtin_sqrt(x); }

// round-half-away-from-zero, exact (C99 round()).  main.cpp:597 uses round()
// for the periodic wrap.
KMC_HD double round_(double x) {
  double t = __builtin_trunc(x);
  double f = x - t;  // exact: fractional part
  if (f >= 0.5) t += 1.0;
  else if (f <= -0.5) t -= 1.0;
  return t;
}

// ---------------------------------------------------------------- sin / cos
// fdlibm k_sin.c / k_cos.c kernels on [-π/4, π/4].
KMC_HD double k_sin(double x, double y, int iy) {
  const double S1 = -1.66666666666666324348e-01; /* 0xBFC55555, 0x55555549 */
  const double S2 = 8.33333333332248946124e-03;  /* 0x3F811111, 0x1110F8A6 */
  const double S3 = -1.98412698298579493134e-04; /* 0xBF2A01A0, 0x19C161D5 */
  const double S4 = 2.75573137070700676789e-06;  /* 0x3EC71DE3, 0x57B1FE7D */
  const double S5 = -2.50507602534068634195e-08; /* 0xBE5AE5E6, 0x8A2B9CEB */
  const double S6 = 1.58969099521155010221e-10;  /* 0x3DE5D93A, 0x5ACFD57C */
  uint32_t ix = hi(x) & 0x7fffffff;
  if (ix < 0x3e400000) {  // |x| < 2**-27
    if ((int)x == 0) return x;
  }
  double z = x * x;
  double v = z * x;
  double r = S2 + z * (S3 + z * (S4 + z * (S5 + z * S6)));
  if (iy == 0) return x + v * (S1 + z * r);
  return x - ((z * (0.5 * y - v * r) - y) - v * S1);
}

KMC_HD double k_cos(double x, double y) {
  const double C1 = 4.16666666666666019037e-02;  /* 0x3FA55555, 0x5555554C */
  const double C2 = -1.38888888888741095749e-03; /* 0xBF56C16C, 0x16C15177 */
  const double C3 = 2.48015872894767294178e-05;  /* 0x3EFA01A0, 0x19CB1590 */
  const double C4 = -2.75573143513906633035e-07; /* 0xBE927E4F, 0x809C52AD */
  const double C5 = 2.08757232129817482790e-09;  /* 0x3E21EE9E, 0xBDB4B1C4 */
  const double C6 = -1.13596475577881948265e-11; /* 0xBDA8FAE9, 0xBE8838D4 */
  uint32_t ix = hi(x) & 0x7fffffff;
  if (ix < 0x3e400000) {  // |x| < 2**-27
    if ((int)x == 0) return 1.0;
  }
  double z = x * x;
  double r = z * (C1 + z * (C2 + z * (C3 + z * (C4 + z * (C5 + z * C6)))));
  if (ix < 0x3FD33333) return 1.0 - (0.5 * z - (z * r - x * y));  // |x| < 0.3
  double qx;
  if (ix > 0x3fe90000) qx = 0.28125;
  else qx = with_hi_lo(ix - 0x00200000, 0);  // x/4
  double hz = 0.5 * z - qx;
  double a = 1.0 - qx;
  return a - (hz - (z * r - x * y));
}

// fdlibm e_rem_pio2.c, medium-argument path (Cody–Waite with up to three
// stages), used unconditionally for |x| > π/4.  Valid for |x| <= 2^19·π/2;
// beyond that the reduction loses accuracy but stays deterministic (the
// simulation never produces such angles: every angle is < 4π).
KMC_HD int rem_pio2(double x, double* y) {
  const double invpio2 = 6.36619772367581382433e-01; /* 0x3FE45F30, 0x6DC9C883 */
  const double pio2_1 = 1.57079632673412561417e+00;  /* 0x3FF921FB, 0x54400000 */
  const double pio2_1t = 6.07710050650619224932e-11; /* 0x3DD0B461, 0x1A626331 */
  const double pio2_2 = 6.07710050630396597660e-11;  /* 0x3DD0B461, 0x1A600000 */
  const double pio2_2t = 2.02226624879595063154e-21; /* 0x3BA3198A, 0x2E037073 */
  const double pio2_3 = 2.02226624871116645580e-21;  /* 0x3BA3198A, 0x2E000000 */
  const double pio2_3t = 8.47842766036889956997e-32; /* 0x397B839A, 0x252049C1 */
  uint32_t hx = hi(x);
  uint32_t ix = hx & 0x7fffffff;
  double t = fabs_(x);
  int n = (int)(t * invpio2 + 0.5);
  double fn = (double)n;
  double r = t - fn * pio2_1;
  double w = fn * pio2_1t;  // 1st round, good to 85 bits
  int j = (int)(ix >> 20);
  y[0] = r - w;
  int i = j - (int)((hi(y[0]) >> 20) & 0x7ff);
  if (i > 16) {  // 2nd iteration, good to 118 bits
    t = r;
    w = fn * pio2_2;
    r = t - w;
    w = fn * pio2_2t - ((t - r) - w);
    y[0] = r - w;
    i = j - (int)((hi(y[0]) >> 20) & 0x7ff);
    if (i > 49) {  // 3rd iteration, 151 bits
      t = r;
      w = fn * pio2_3;
      r = t - w;
      w = fn * pio2_3t - ((t - r) - w);
      y[0] = r - w;
    }
  }
  y[1] = (r - y[0]) - w;
  if (hx & 0x80000000u) {
    y[0] = -y[0];
    y[1] = -y[1];
    return -n;
  }
  return n;
}

KMC_HD double sin(double x) {
  uint32_t ix = hi(x) & 0x7fffffff;
  if (ix <= 0x3fe921fb) return k_sin(x, 0.0, 0);
  if (ix >= 0x7ff00000) return x - x;  // NaN
  double y[2];
  int n = rem_pio2(x, y);
  switch (n & 3) {
    case 0: return k_sin(y[0], y[1], 1);
    case 1: return k_cos(y[0], y[1]);
    case 2: return -k_sin(y[0], y[1], 1);
    default: return -k_cos(y[0], y[1]);
  }
}

KMC_HD double cos(double x) {
  uint32_t ix = hi(x) & 0x7fffffff;
  if (ix <= 0x3fe921fb) return k_cos(x, 0.0);
  if (ix >= 0x7ff00000) return x - x;
  double y[2];
  int n = rem_pio2(x, y);
  switch (n & 3) {
    case 0: return k_cos(y[0], y[1]);
    case 1: return -k_sin(y[0], y[1], 1);
    case 2: return -k_cos(y[0], y[1]);
    default: return k_sin(y[0], y[1], 1);
  }
}

// ---------------------------------------------------------------- atan/atan2
KMC_HD double atan(double x) {
  const double atanhi0 = 4.63647609000806093515e-01; /* 0x3FDDAC67, 0x0561BB4F */
  const double atanhi1 = 7.85398163397448278999e-01; /* 0x3FE921FB, 0x54442D18 */
  const double atanhi2 = 9.82793723247329054082e-01; /* 0x3FEF730B, 0xD281F69B */
  const double atanhi3 = 1.57079632679489655800e+00; /* 0x3FF921FB, 0x54442D18 */
  const double atanlo0 = 2.26987774529616870924e-17; /* 0x3C7A2B7F, 0x222F65E2 */
  const double atanlo1 = 3.06161699786838301793e-17; /* 0x3C81A626, 0x33145C07 */
  const double atanlo2 = 1.39033110312309984516e-17; /* 0x3C700788, 0x7AF0CBBD */
  const double atanlo3 = 6.12323399573676603587e-17; /* 0x3C91A626, 0x33145C07 */
  const double aT0 = 3.33333333333329318027e-01;   /* 0x3FD55555, 0x5555550D */
  const double aT1 = -1.99999999998764832476e-01;  /* 0xBFC99999, 0x9998EBC4 */
  const double aT2 = 1.42857142725034663711e-01;   /* 0x3FC24924, 0x920083FF */
  const double aT3 = -1.11111104054623557880e-01;  /* 0xBFBC71C6, 0xFE231671 */
  const double aT4 = 9.09088713343650656196e-02;   /* 0x3FB745CD, 0xC54C206E */
  const double aT5 = -7.69187620504482999495e-02;  /* 0xBFB3B0F2, 0xAF749A6D */
  const double aT6 = 6.66107313738753120669e-02;   /* 0x3FB10D66, 0xA0D03D51 */
  const double aT7 = -5.83357013379057348645e-02;  /* 0xBFADDE2D, 0x52DEFD9A */
  const double aT8 = 4.97687799461593236017e-02;   /* 0x3FA97B4B, 0x24760DEB */
  const double aT9 = -3.65315727442169155270e-02;  /* 0xBFA2B444, 0x2C6A6C2F */
  const double aT10 = 1.62858201153657823623e-02;  /* 0x3F90AD3A, 0xE322DA11 */
  uint32_t hx = hi(x);
  uint32_t ix = hx & 0x7fffffff;
  int id;
  if (ix >= 0x44100000) {  // |x| >= 2^66
    if (ix > 0x7ff00000 || (ix == 0x7ff00000 && lo(x) != 0)) return x + x;
    return (hx & 0x80000000u) ? -atanhi3 - atanlo3 : atanhi3 + atanlo3;
  }
  if (ix < 0x3fdc0000) {  // |x| < 0.4375
    if (ix < 0x3e200000) return x;  // |x| < 2^-29
    id = -1;
  } else {
    x = fabs_(x);
    if (ix < 0x3ff30000) {    // |x| < 1.1875
      if (ix < 0x3fe60000) {  // 7/16 <= |x| < 11/16
        id = 0;
        x = (2.0 * x - 1.0) / (2.0 + x);
      } else {  // 11/16 <= |x| < 19/16
        id = 1;
        x = (x - 1.0) / (x + 1.0);
      }
    } else {
      if (ix < 0x40038000) {  // |x| < 2.4375
        id = 2;
        x = (x - 1.5) / (1.0 + 1.5 * x);
      } else {  // 2.4375 <= |x| < 2^66
        id = 3;
        x = -1.0 / x;
      }
    }
  }
  double z = x * x;
  double w = z * z;
  double s1 = z * (aT0 + w * (aT2 + w * (aT4 + w * (aT6 + w * (aT8 + w * aT10)))));
  double s2 = w * (aT1 + w * (aT3 + w * (aT5 + w * (aT7 + w * aT9))));
  if (id < 0) return x - x * (s1 + s2);
  double ahi = id == 0 ? atanhi0 : id == 1 ? atanhi1 : id == 2 ? atanhi2 : atanhi3;
  double alo = id == 0 ? atanlo0 : id == 1 ? atanlo1 : id == 2 ? atanlo2 : atanlo3;
  z = ahi - ((x * (s1 + s2) - alo) - x);
  return (hx & 0x80000000u) ? -z : z;
}

// fdlibm e_atan2.c (the "+tiny" inexact-raising terms are dropped: adding
// 1e-300 to π or π/2 does not change the rounded result).
KMC_HD double atan2(double y, double x) {
  const double pi_o_4 = 7.8539816339744827900E-01; /* 0x3FE921FB, 0x54442D18 */
  const double pi_o_2 = 1.5707963267948965580E+00; /* 0x3FF921FB, 0x54442D18 */
  const double pi = 3.1415926535897931160E+00;     /* 0x400921FB, 0x54442D18 */
  const double pi_lo = 1.2246467991473531772E-16;  /* 0x3CA1A626, 0x33145C07 */
  uint32_t hx = hi(x), lx = lo(x);
  uint32_t hy = hi(y), ly = lo(y);
  uint32_t ix = hx & 0x7fffffff, iy = hy & 0x7fffffff;
  if ((ix | ((lx | (0u - lx)) >> 31)) > 0x7ff00000u ||
      (iy | ((ly | (0u - ly)) >> 31)) > 0x7ff00000u)
    return x + y;  // NaN
  if (((hx - 0x3ff00000u) | lx) == 0) return atan(y);  // x == 1.0
  int m = (int)(((hy >> 31) & 1) | ((hx >> 30) & 2));  // 2*sign(x)+sign(y)
  if ((iy | ly) == 0) {  // y == 0
    switch (m) {
      case 0:
      case 1: return y;
      case 2: return pi;
      default: return -pi;
    }
  }
  if ((ix | lx) == 0) return (hy & 0x80000000u) ? -pi_o_2 : pi_o_2;  // x == 0
  if (ix == 0x7ff00000) {
    if (iy == 0x7ff00000) {
      switch (m) {
        case 0: return pi_o_4;
        case 1: return -pi_o_4;
        case 2: return 3.0 * pi_o_4;
        default: return -3.0 * pi_o_4;
      }
    } else {
      switch (m) {
        case 0: return 0.0;
        case 1: return -0.0;
        case 2: return pi;
        default: return -pi;
      }
    }
  }
  if (iy == 0x7ff00000) return (hy & 0x80000000u) ? -pi_o_2 : pi_o_2;
  int k = ((int)iy - (int)ix) >> 20;
  double z;
  if (k > 60) z = pi_o_2 + 0.5 * pi_lo;
  else if ((hx & 0x80000000u) && k < -60) z = 0.0;
  else z = atan(fabs_(y / x));
  switch (m) {
    case 0: return z;
    case 1: return -z;  // flips the sign bit only, as __HI(z) ^= 0x80000000
    case 2: return pi - (z - pi_lo);
    default: return (z - pi_lo) - pi;
  }
}

// ---------------------------------------------------------------- acos
KMC_HD double acos(double x) {
  const double pi = 3.14159265358979311600e+00;       /* 0x400921FB, 0x54442D18 */
  const double pio2_hi = 1.57079632679489655800e+00;  /* 0x3FF921FB, 0x54442D18 */
  const double pio2_lo = 6.12323399573676603587e-17;  /* 0x3C91A626, 0x33145C07 */
  const double pS0 = 1.66666666666666657415e-01;      /* 0x3FC55555, 0x55555555 */
  const double pS1 = -3.25565818622400915405e-01;     /* 0xBFD4D612, 0x03EB6F7D */
  const double pS2 = 2.01212532134862925881e-01;      /* 0x3FC9C155, 0x0E884455 */
  const double pS3 = -4.00555345006794114027e-02;     /* 0xBFA48228, 0xB5688F3B */
  const double pS4 = 7.91534994289814532176e-04;      /* 0x3F49EFE0, 0x7501B288 */
  const double pS5 = 3.47933107596021167570e-05;      /* 0x3F023DE1, 0x0DFDF709 */
  const double qS1 = -2.40339491173441421878e+00;     /* 0xC0033A27, 0x1C8A2D4B */
  const double qS2 = 2.02094576023350569471e+00;      /* 0x40002AE5, 0x9C598AC8 */
  const double qS3 = -6.88283971605453293030e-01;     /* 0xBFE6066C, 0x1B8D0159 */
  const double qS4 = 7.70381505559019352791e-02;      /* 0x3FB3B8C5, 0xB12E9282 */
  uint32_t hx = hi(x);
  uint32_t ix = hx & 0x7fffffff;
  if (ix >= 0x3ff00000) {  // |x| >= 1
    if (((ix - 0x3ff00000) | lo(x)) == 0) {
      if (!(hx & 0x80000000u)) return 0.0;
      return pi + 2.0 * pio2_lo;
    }
    return (x - x) / (x - x);  // NaN
  }
  if (ix < 0x3fe00000) {  // |x| < 0.5
    if (ix <= 0x3c600000) return pio2_hi + pio2_lo;
    double z = x * x;
    double p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
    double q = 1.0 + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
    double r = p / q;
    return pio2_hi - (x - (pio2_lo - x * r));
  } else if (hx & 0x80000000u) {  // x < -0.5
    double z = (1.0 + x) * 0.5;
    double p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
    double q = 1.0 + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
    double s = sqrt_(z);
    double r = p / q;
    double w = r * s - pio2_lo;
    return pi - 2.0 * (s + w);
  } else {  // x > 0.5
    double z = (1.0 - x) * 0.5;
    double s = sqrt_(z);
    double df = with_hi_lo(hi(s), 0);
    double c = (z - df * df) / (s + df);
    double p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
    double q = 1.0 + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
    double r = p / q;
    double w = r * s + c;
    return 2.0 * (df + w);
  }
}

}  // namespace kmcm
