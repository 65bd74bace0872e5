// ORACLE — test infrastructure only (see orb_oracle.cpp header).
//
// The oracle's own transcription of the pinned double-precision math (DESIGN.md
// P10/P11): the reference links glibc's libm, whose results are not pinned
// across versions, so oracle and kernels both implement Sun's fdlibm 5.3
// algorithms (e_exp.c, e_log.c, e_log10.c, e_rem_pio2.c medium range, k_sin.c,
// k_cos.c, s_sin.c, s_cos.c, s_atan.c, e_atan2.c), written here from the
// published fdlibm sources' algorithm and constants, independently of the
// product's csrc/lsd_math.h, so that a slip on either side fails GPU parity.
// P11: pow(x, n) for integral n >= 0 by binary exponentiation; sinh by the odd
// Taylor series below |x| = 0.125 (the reference only evaluates sinh(1/x),
// x > 15), e^x formula above.
//
// Probe (tests/test_math_divergence.py): with pmath::probe_on() every call
// also evaluates glibc and counts, per function, the calls and the results
// that differ - the divergence of a glibc-built reference on the arguments the
// path actually hits.
#ifndef ORACLE_PINNED_MATH_H
#define ORACLE_PINNED_MATH_H

#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstring>

namespace pmath {

enum Fn { kExp, kLog, kLog10, kSin, kCos, kAtan2, kCosF, kSinF, kNumFn };

struct Probe {
  std::atomic<int> on{0};
  std::atomic<long long> calls[kNumFn];
  std::atomic<long long> differ[kNumFn];
  std::atomic<long long> max_ulp[kNumFn];
};
inline Probe& probe() {
  static Probe p;
  return p;
}

inline uint32_t hiw(double x) {
  uint64_t u;
  std::memcpy(&u, &x, 8);
  return (uint32_t)(u >> 32);
}
inline uint32_t low(double x) {
  uint64_t u;
  std::memcpy(&u, &x, 8);
  return (uint32_t)u;
}
inline double make(uint32_t hi, uint32_t lo) {
  const uint64_t u = ((uint64_t)hi << 32) | lo;
  double x;
  std::memcpy(&x, &u, 8);
  return x;
}
inline double set_hi(double x, uint32_t hi) { return make(hi, low(x)); }

inline long long ulp_dist(double a, double b) {
  int64_t ia, ib;
  std::memcpy(&ia, &a, 8);
  std::memcpy(&ib, &b, 8);
  if (ia < 0) ia = INT64_MIN - ia;
  if (ib < 0) ib = INT64_MIN - ib;
  const long long d = (long long)(ia > ib ? ia - ib : ib - ia);
  return d;
}
inline void record(Fn f, double pinned, double libm) {
  Probe& p = probe();
  p.calls[f]++;
  if (std::memcmp(&pinned, &libm, 8) != 0) {
    p.differ[f]++;
    const long long d = ulp_dist(pinned, libm);
    long long m = p.max_ulp[f].load();
    while (d > m && !p.max_ulp[f].compare_exchange_weak(m, d)) {
    }
  }
}
inline void recordf(Fn f, float pinned, float libm) {
  Probe& p = probe();
  p.calls[f]++;
  if (std::memcmp(&pinned, &libm, 4) != 0) {
    p.differ[f]++;
    int32_t a, b;
    std::memcpy(&a, &pinned, 4);
    std::memcpy(&b, &libm, 4);
    const long long d = a > b ? (long long)a - b : (long long)b - a;
    long long m = p.max_ulp[f].load();
    while (d > m && !p.max_ulp[f].compare_exchange_weak(m, d)) {
    }
  }
}

// ---------------------------------------------------------------- e_exp.c
inline double exp_raw(double x) {
  const double halF[2] = {0.5, -0.5};
  const double o_threshold = 7.09782712893383973096e+02;
  const double u_threshold = -7.45133219101941108420e+02;
  const double ln2HI[2] = {6.93147180369123816490e-01, -6.93147180369123816490e-01};
  const double ln2LO[2] = {1.90821492927058770002e-10, -1.90821492927058770002e-10};
  const double invln2 = 1.44269504088896338700e+00;
  const double P1 = 1.66666666666666019037e-01, P2 = -2.77777777770155933842e-03,
               P3 = 6.61375632143793436117e-05, P4 = -1.65339022054652515390e-06,
               P5 = 4.13813679705723846039e-08;
  const double twom1000 = 9.33263618503218878990e-302;
  uint32_t hx = hiw(x);
  const int xsb = (int)((hx >> 31) & 1);
  hx &= 0x7fffffffu;
  double hi = 0.0, lo = 0.0;
  int k = 0;
  if (hx >= 0x40862E42u) {
    if (hx >= 0x7ff00000u) {
      if (((hx & 0xfffffu) | low(x)) != 0) return x + x;
      return xsb == 0 ? x : 0.0;
    }
    if (x > o_threshold) return HUGE_VAL;
    if (x < u_threshold) return 0.0;
  }
  if (hx > 0x3fd62e42u) {          // |x| > 0.5 ln2
    if (hx < 0x3FF0A2B2u) {        // and |x| < 1.5 ln2
      hi = x - ln2HI[xsb];
      lo = ln2LO[xsb];
      k = 1 - xsb - xsb;
    } else {
      k = (int)(invln2 * x + halF[xsb]);
      const double t = k;
      hi = x - t * ln2HI[0];
      lo = t * ln2LO[0];
    }
    x = hi - lo;
  } else if (hx < 0x3e300000u) {   // |x| < 2^-28
    return 1.0 + x;
  } else {
    k = 0;
  }
  const double t = x * x;
  const double c = x - t * (P1 + t * (P2 + t * (P3 + t * (P4 + t * P5))));
  if (k == 0) return 1.0 - ((x * c) / (c - 2.0) - x);
  double y = 1.0 - ((lo - (x * c) / (2.0 - c)) - hi);
  if (k >= -1021) return set_hi(y, hiw(y) + ((uint32_t)k << 20));
  y = set_hi(y, hiw(y) + ((uint32_t)(k + 1000) << 20));
  return y * twom1000;
}

// ---------------------------------------------------------------- e_log.c
inline double log_raw(double x) {
  const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10,
               two54 = 1.80143985094819840000e+16;
  const double Lg1 = 6.666666666666735130e-01, Lg2 = 3.999999999940941908e-01,
               Lg3 = 2.857142874366239149e-01, Lg4 = 2.222219843214978396e-01,
               Lg5 = 1.818357216161805012e-01, Lg6 = 1.531383769920937332e-01,
               Lg7 = 1.479819860511658591e-01;
  int32_t hx = (int32_t)hiw(x);
  const uint32_t lx = low(x);
  int k = 0;
  if (hx < 0x00100000) {
    if (((hx & 0x7fffffff) | (int32_t)lx) == 0) return -HUGE_VAL;
    if (hx < 0) return NAN;
    k -= 54;
    x *= two54;
    hx = (int32_t)hiw(x);
  }
  if (hx >= 0x7ff00000) return x + x;
  k += (hx >> 20) - 1023;
  hx &= 0x000fffff;
  int32_t i = (hx + 0x95f64) & 0x100000;
  x = set_hi(x, (uint32_t)(hx | (i ^ 0x3ff00000)));   // x or x/2 in [sqrt(2)/2, sqrt(2))
  k += (i >> 20);
  const double f = x - 1.0;
  double dk;
  if ((0x000fffff & (2 + hx)) < 3) {                  // |f| < 2^-20
    if (f == 0.0) {
      if (k == 0) return 0.0;
      dk = (double)k;
      return dk * ln2_hi + dk * ln2_lo;
    }
    const double R = f * f * (0.5 - 0.33333333333333333 * f);
    if (k == 0) return f - R;
    dk = (double)k;
    return dk * ln2_hi - ((R - dk * ln2_lo) - f);
  }
  const double s = f / (2.0 + f);
  dk = (double)k;
  const double z = s * s;
  i = hx - 0x6147a;
  const double w = z * z;
  const int32_t j = 0x6b851 - hx;
  const double t1 = w * (Lg2 + w * (Lg4 + w * Lg6));
  const double t2 = z * (Lg1 + w * (Lg3 + w * (Lg5 + w * Lg7)));
  i |= j;
  const double R = t2 + t1;
  if (i > 0) {
    const double hfsq = 0.5 * f * f;
    if (k == 0) return f - (hfsq - s * (hfsq + R));
    return dk * ln2_hi - ((hfsq - (s * (hfsq + R) + dk * ln2_lo)) - f);
  }
  if (k == 0) return f - s * (f - R);
  return dk * ln2_hi - ((s * (f - R) - dk * ln2_lo) - f);
}

// -------------------------------------------------------------- e_log10.c
inline double log10_raw(double x) {
  const double two54 = 1.80143985094819840000e+16, ivln10 = 4.34294481903251816668e-01,
               log10_2hi = 3.01029995663611771306e-01, log10_2lo = 3.69423907715893078616e-13;
  int32_t hx = (int32_t)hiw(x);
  const uint32_t lx = low(x);
  int k = 0;
  if (hx < 0x00100000) {
    if (((hx & 0x7fffffff) | (int32_t)lx) == 0) return -HUGE_VAL;
    if (hx < 0) return NAN;
    k -= 54;
    x *= two54;
    hx = (int32_t)hiw(x);
  }
  if (hx >= 0x7ff00000) return x + x;
  k += (hx >> 20) - 1023;
  const int i = (int)(((uint32_t)k & 0x80000000u) >> 31);
  hx = (hx & 0x000fffff) | ((0x3ff - i) << 20);
  const double y = (double)(k + i);
  x = set_hi(x, (uint32_t)hx);
  const double z = y * log10_2lo + ivln10 * log_raw(x);
  return z + y * log10_2hi;
}

// --------------------------------------------------- k_sin.c / k_cos.c
inline double kernel_sin(double x, double y, int iy) {
  const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
               S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
               S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
  const uint32_t ix = hiw(x) & 0x7fffffffu;
  if (ix < 0x3e400000u && (int)x == 0) return x;   // |x| < 2^-27
  const double z = x * x;
  const double v = z * x;
  const double r = S2 + z * (S3 + z * (S4 + z * (S5 + z * S6)));
  if (iy == 0) return x + v * (S1 + z * r);
  return x - ((z * (0.5 * y - v * r) - y) - v * S1);
}

inline double kernel_cos(double x, double y) {
  const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
               C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
               C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
  const uint32_t ix = hiw(x) & 0x7fffffffu;
  if (ix < 0x3e400000u && (int)x == 0) return 1.0;
  const double z = x * x;
  const double r = z * (C1 + z * (C2 + z * (C3 + z * (C4 + z * (C5 + z * C6)))));
  if (ix < 0x3FD33333u) return 1.0 - (0.5 * z - (z * r - x * y));
  const double qx = ix > 0x3fe90000u ? 0.28125 : make(ix - 0x00200000u, 0);
  const double hz = 0.5 * z - qx;
  const double a = 1.0 - qx;
  return a - (hz - (z * r - x * y));
}

// ----------------------------------------- e_rem_pio2.c, |x| < 2^19 pi/2
inline int rem_pio2(double x, double* y) {
  static const uint32_t npio2_hw[32] = {
      0x3FF921FB, 0x400921FB, 0x4012D97C, 0x401921FB, 0x401F6A7A, 0x4022D97C, 0x4025FDBB,
      0x402921FB, 0x402C463A, 0x402F6A7A, 0x4031475C, 0x4032D97C, 0x40346B9C, 0x4035FDBB,
      0x40378FDB, 0x403921FB, 0x403AB41B, 0x403C463A, 0x403DD85A, 0x403F6A7A, 0x40407E4C,
      0x4041475C, 0x4042106C, 0x4042D97C, 0x4043A28C, 0x40446B9C, 0x404534AC, 0x4045FDBB,
      0x4046C6CB, 0x40478FDB, 0x404858EB, 0x404921FB};
  const double invpio2 = 6.36619772367581382433e-01, pio2_1 = 1.57079632673412561417e+00,
               pio2_1t = 6.07710050650619224932e-11, pio2_2 = 6.07710050630396597660e-11,
               pio2_2t = 2.02226624879595063154e-21, pio2_3 = 2.02226624871116645580e-21,
               pio2_3t = 8.47842766036889956997e-32;
  const int32_t hx = (int32_t)hiw(x);
  const uint32_t ix = (uint32_t)hx & 0x7fffffffu;
  if (ix <= 0x3fe921fbu) {
    y[0] = x;
    y[1] = 0;
    return 0;
  }
  if (ix < 0x4002d97cu) {   // |x| < 3pi/4: n = +-1
    if (hx > 0) {
      double z = x - pio2_1;
      if (ix != 0x3ff921fbu) {
        y[0] = z - pio2_1t;
        y[1] = (z - y[0]) - pio2_1t;
      } else {
        z -= pio2_2;
        y[0] = z - pio2_2t;
        y[1] = (z - y[0]) - pio2_2t;
      }
      return 1;
    }
    double z = x + pio2_1;
    if (ix != 0x3ff921fbu) {
      y[0] = z + pio2_1t;
      y[1] = (z - y[0]) + pio2_1t;
    } else {
      z += pio2_2;
      y[0] = z + pio2_2t;
      y[1] = (z - y[0]) + pio2_2t;
    }
    return -1;
  }
  // medium size (the path never reaches 2^19 pi/2; larger arguments would
  // need __kernel_rem_pio2's Payne-Hanek reduction)
  const double t = std::fabs(x);
  const int n = (int)(t * invpio2 + 0.5);
  const double fn = (double)n;
  double r = t - fn * pio2_1;
  double w = fn * pio2_1t;
  if (n < 32 && ix != npio2_hw[n - 1]) {
    y[0] = r - w;
  } else {
    const int j = (int)(ix >> 20);
    y[0] = r - w;
    int i = j - (int)((hiw(y[0]) >> 20) & 0x7ff);
    if (i > 16) {
      double tt = r;
      w = fn * pio2_2;
      r = tt - w;
      w = fn * pio2_2t - ((tt - r) - w);
      y[0] = r - w;
      i = j - (int)((hiw(y[0]) >> 20) & 0x7ff);
      if (i > 49) {
        tt = r;
        w = fn * pio2_3;
        r = tt - w;
        w = fn * pio2_3t - ((tt - r) - w);
        y[0] = r - w;
      }
    }
  }
  y[1] = (r - y[0]) - w;
  if (hx < 0) {
    y[0] = -y[0];
    y[1] = -y[1];
    return -n;
  }
  return n;
}

// ---------------------------------------------------- s_sin.c / s_cos.c
inline double sin_raw(double x) {
  const uint32_t ix = hiw(x) & 0x7fffffffu;
  if (ix <= 0x3fe921fbu) return kernel_sin(x, 0.0, 0);
  if (ix >= 0x7ff00000u) return x - x;
  double y[2];
  const int n = rem_pio2(x, y);
  switch (n & 3) {
    case 0: return kernel_sin(y[0], y[1], 1);
    case 1: return kernel_cos(y[0], y[1]);
    case 2: return -kernel_sin(y[0], y[1], 1);
    default: return -kernel_cos(y[0], y[1]);
  }
}

inline double cos_raw(double x) {
  const uint32_t ix = hiw(x) & 0x7fffffffu;
  if (ix <= 0x3fe921fbu) return kernel_cos(x, 0.0);
  if (ix >= 0x7ff00000u) return x - x;
  double y[2];
  const int n = rem_pio2(x, y);
  switch (n & 3) {
    case 0: return kernel_cos(y[0], y[1]);
    case 1: return -kernel_sin(y[0], y[1], 1);
    case 2: return -kernel_cos(y[0], y[1]);
    default: return kernel_sin(y[0], y[1], 1);
  }
}

// -------------------------------------------------------------- s_atan.c
inline double atan_raw(double x) {
  static const double atanhi[4] = {4.63647609000806093515e-01, 7.85398163397448278999e-01,
                                   9.82793723247329054082e-01, 1.57079632679489655800e+00};
  static const double atanlo[4] = {2.26987774529616870924e-17, 3.06161699786838301793e-17,
                                   1.39033110312309984516e-17, 6.12323399573676603587e-17};
  static const double aT[11] = {
      3.33333333333329318027e-01,  -1.99999999998764832476e-01, 1.42857142725034663711e-01,
      -1.11111104054623557880e-01, 9.09088713343650656196e-02,  -7.69187620504482999495e-02,
      6.66107313738753120669e-02,  -5.83357013379057348645e-02, 4.97687799461593236017e-02,
      -3.65315727442169155270e-02, 1.62858201153657823623e-02};
  const int32_t hx = (int32_t)hiw(x);
  const uint32_t ix = (uint32_t)hx & 0x7fffffffu;
  int id;
  if (ix >= 0x44100000u) {   // |x| >= 2^66
    if (ix > 0x7ff00000u || (ix == 0x7ff00000u && low(x) != 0)) return x + x;
    return hx > 0 ? atanhi[3] + atanlo[3] : -atanhi[3] - atanlo[3];
  }
  if (ix < 0x3fdc0000u) {    // |x| < 0.4375
    if (ix < 0x3e200000u) return x;   // |x| < 2^-29
    id = -1;
  } else {
    x = std::fabs(x);
    if (ix < 0x3ff30000u) {          // |x| < 1.1875
      if (ix < 0x3fe60000u) {        // 7/16 <= |x| < 11/16
        id = 0;
        x = (2.0 * x - 1.0) / (2.0 + x);
      } else {                       // 11/16 <= |x| < 19/16
        id = 1;
        x = (x - 1.0) / (x + 1.0);
      }
    } else if (ix < 0x40038000u) {   // |x| < 2.4375
      id = 2;
      x = (x - 1.5) / (1.0 + 1.5 * x);
    } else {                         // 2.4375 <= |x| < 2^66
      id = 3;
      x = -1.0 / x;
    }
  }
  const double z = x * x;
  const double w = z * z;
  const double s1 = z * (aT[0] + w * (aT[2] + w * (aT[4] + w * (aT[6] + w * (aT[8] + w * aT[10])))));
  const double s2 = w * (aT[1] + w * (aT[3] + w * (aT[5] + w * (aT[7] + w * aT[9]))));
  if (id < 0) return x - x * (s1 + s2);
  const double r = atanhi[id] - ((x * (s1 + s2) - atanlo[id]) - x);
  return hx < 0 ? -r : r;
}

// ------------------------------------------------------------- e_atan2.c
inline double atan2_raw(double y, double x) {
  const double tiny = 1.0e-300, pi_o_4 = 7.8539816339744827900E-01,
               pi_o_2 = 1.5707963267948965580E+00, pi = 3.1415926535897931160E+00,
               pi_lo = 1.2246467991473531772E-16;
  const int32_t hx = (int32_t)hiw(x), hy = (int32_t)hiw(y);
  const uint32_t ix = (uint32_t)hx & 0x7fffffffu, iy = (uint32_t)hy & 0x7fffffffu;
  const uint32_t lx = low(x), ly = low(y);
  if ((ix | ((lx | (0u - lx)) >> 31)) > 0x7ff00000u || (iy | ((ly | (0u - ly)) >> 31)) > 0x7ff00000u)
    return x + y;
  if ((((uint32_t)hx - 0x3ff00000u) | lx) == 0) return atan_raw(y);   // x = 1.0
  const int m = ((hy >> 31) & 1) | ((hx >> 30) & 2);
  if ((iy | ly) == 0) {
    switch (m) {
      case 0:
      case 1: return y;
      case 2: return pi + tiny;
      default: return -pi - tiny;
    }
  }
  if ((ix | lx) == 0) return hy < 0 ? -pi_o_2 - tiny : pi_o_2 + tiny;
  if (ix == 0x7ff00000u) {
    if (iy == 0x7ff00000u) {
      switch (m) {
        case 0: return pi_o_4 + tiny;
        case 1: return -pi_o_4 - tiny;
        case 2: return 3.0 * pi_o_4 + tiny;
        default: return -3.0 * pi_o_4 - tiny;
      }
    }
    switch (m) {
      case 0: return 0.0;
      case 1: return -0.0;
      case 2: return pi + tiny;
      default: return -pi - tiny;
    }
  }
  if (iy == 0x7ff00000u) return hy < 0 ? -pi_o_2 - tiny : pi_o_2 + tiny;
  const int k = ((int)iy - (int)ix) >> 20;
  double z;
  if (k > 60) z = pi_o_2 + 0.5 * pi_lo;
  else if (hx < 0 && k < -60) z = 0.0;
  else z = atan_raw(std::fabs(y / x));
  switch (m) {
    case 0: return z;
    case 1: return -z;
    case 2: return pi - (z - pi_lo);
    default: return (z - pi_lo) - pi;
  }
}

// ------------------------------------------------------------------ P11
inline double powi(double x, double n_as_double) {
  // x^n, n a non-negative integer: bits of n from the least significant,
  // the running square updated only while bits remain
  unsigned long long n = (unsigned long long)n_as_double;
  double acc = 1.0, sq = x;
  for (; n != 0; n >>= 1) {
    if (n & 1ull) acc = acc * sq;
    if (n > 1ull) sq = sq * sq;
  }
  return acc;
}

inline double sinh_(double x) {
  const double a = std::fabs(x);
  if (a < 0.125) {
    // x + x^3/3! + x^5/5! + ... + x^11/11!, Horner in z = x^2 with the
    // factors 1/6, 1/20, 1/42, 1/72, 1/110 between consecutive terms
    const double z = x * x;
    double h = 1.0 + z / 110.0;
    h = 1.0 + z / 72.0 * h;
    h = 1.0 + z / 42.0 * h;
    h = 1.0 + z / 20.0 * h;
    return x + x * (z / 6.0 * h);
  }
  const double e = exp_raw(a);
  const double s = 0.5 * (e - 1.0 / e);
  return x < 0 ? -s : s;
}

// ------------------------------------------------ probed entry points
inline double exp_(double x) {
  const double r = exp_raw(x);
  if (probe().on.load(std::memory_order_relaxed)) record(kExp, r, std::exp(x));
  return r;
}
inline double log_(double x) {
  const double r = log_raw(x);
  if (probe().on.load(std::memory_order_relaxed)) record(kLog, r, std::log(x));
  return r;
}
inline double log10_(double x) {
  const double r = log10_raw(x);
  if (probe().on.load(std::memory_order_relaxed)) record(kLog10, r, std::log10(x));
  return r;
}
inline double sin_(double x) {
  const double r = sin_raw(x);
  if (probe().on.load(std::memory_order_relaxed)) record(kSin, r, std::sin(x));
  return r;
}
inline double cos_(double x) {
  const double r = cos_raw(x);
  if (probe().on.load(std::memory_order_relaxed)) record(kCos, r, std::cos(x));
  return r;
}
inline double atan2_(double y, double x) {
  const double r = atan2_raw(y, x);
  if (probe().on.load(std::memory_order_relaxed)) record(kAtan2, r, std::atan2(y, x));
  return r;
}
// P2: float cos / sin of the descriptor steering angle, correctly rounded
// (glibc's double cos / sin are correctly rounded on these arguments; the
// probe counts how often glibc's cosf / sinf give another float)
inline float cosf_cr(float a) {
  const float r = (float)std::cos((double)a);
  if (probe().on.load(std::memory_order_relaxed)) recordf(kCosF, r, cosf(a));
  return r;
}
inline float sinf_cr(float a) {
  const float r = (float)std::sin((double)a);
  if (probe().on.load(std::memory_order_relaxed)) recordf(kSinF, r, sinf(a));
  return r;
}

}  // namespace pmath

#endif
