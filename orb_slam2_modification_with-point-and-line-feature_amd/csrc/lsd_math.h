// Deterministic double-precision elementary functions for the line path
// (LSD NFA / rectangle geometry, LBD weights, KeyLine angles).
//
// The reference calls glibc's libm (exp, log, log10, pow, sinh, sin, cos,
// atan2). Those are not bit-reproducible on the GPU, so the line path pins
// them (pinned semantics P10-P12) to the fdlibm algorithms below,
// written with plain IEEE-754 +,-,*,/ and bit manipulation only, compiled with
// -ffp-contract=off. The oracle has its own transcription (oracle/
// pinned_math.h); tests/test_math_divergence.py compares the two bit for bit
// and both against glibc (<= 1 ulp).
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define LSDM_HD __host__ __device__ __forceinline__
#else
#define LSDM_HD static inline
#endif

namespace lsdm {

LSDM_HD uint64_t bits(double x) {
  union { double d; uint64_t u; } v;
  v.d = x;
  return v.u;
}
LSDM_HD double from_bits(uint64_t u) {
  union { double d; uint64_t u; } v;
  v.u = u;
  return v.d;
}
LSDM_HD int32_t hi_word(double x) { return (int32_t)(bits(x) >> 32); }
LSDM_HD uint32_t lo_word(double x) { return (uint32_t)bits(x); }
LSDM_HD double with_hi(double x, int32_t hi) {
  return from_bits(((uint64_t)(uint32_t)hi << 32) | (uint64_t)lo_word(x));
}
LSDM_HD double fabs_(double x) { return from_bits(bits(x) & 0x7FFFFFFFFFFFFFFFull); }

// ---- exp (fdlibm e_exp.c) ----
LSDM_HD double exp_(double x) {
  const double ln2HI = 6.93147180369123816490e-01, ln2LO = 1.90821492927058770002e-10,
               invln2 = 1.44269504088896338700e+00, P1 = 1.66666666666666019037e-01,
               P2 = -2.77777777770155933842e-03, P3 = 6.61375632143793436117e-05,
               P4 = -1.65339022054652515390e-06, P5 = 4.13813679705723846039e-08,
               o_threshold = 7.09782712893383973096e+02,
               u_threshold = -7.45133219101941108420e+02,
               twom1000 = 9.33263618503218878990e-302;
  uint32_t hx = (uint32_t)hi_word(x);
  const int xsb = (hx >> 31) & 1;
  hx &= 0x7fffffff;
  if (hx >= 0x40862E42u) {
    if (hx >= 0x7ff00000u) {
      if (((hx & 0xfffff) | lo_word(x)) != 0) return x + x;
      return xsb == 0 ? x : 0.0;
    }
    if (x > o_threshold) return from_bits(0x7FF0000000000000ull);
    if (x < u_threshold) return 0.0;
  }
  double hi = 0, lo = 0, c, t, y;
  int k = 0;
  if (hx > 0x3fd62e42u) {
    if (hx < 0x3FF0A2B2u) {
      hi = xsb ? x + ln2HI : x - ln2HI;
      lo = xsb ? -ln2LO : ln2LO;
      k = 1 - xsb - xsb;
    } else {
      k = (int)(invln2 * x + (xsb ? -0.5 : 0.5));
      t = k;
      hi = x - t * ln2HI;
      lo = t * ln2LO;
    }
    x = hi - lo;
  } else if (hx < 0x3e300000u) {
    return 1.0 + x;
  } else {
    k = 0;
  }
  t = x * x;
  c = x - t * (P1 + t * (P2 + t * (P3 + t * (P4 + t * P5))));
  if (k == 0) return 1.0 - ((x * c) / (c - 2.0) - x);
  y = 1.0 - ((lo - (x * c) / (2.0 - c)) - hi);
  // exponent adjust without shifting a negative int (UB before C++20)
  if (k >= -1021) return with_hi(y, (int32_t)((uint32_t)hi_word(y) + ((uint32_t)k << 20)));
  return with_hi(y, (int32_t)((uint32_t)hi_word(y) + ((uint32_t)(k + 1000) << 20))) * twom1000;
}

// ---- log (fdlibm e_log.c), x > 0 finite ----
LSDM_HD double log_(double x) {
  const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10,
               two54 = 1.80143985094819840000e+16, Lg1 = 6.666666666666735130e-01,
               Lg2 = 3.999999999940941908e-01, Lg3 = 2.857142874366239149e-01,
               Lg4 = 2.222219843214978396e-01, Lg5 = 1.818357216161805012e-01,
               Lg6 = 1.531383769920937332e-01, Lg7 = 1.479819860511658591e-01;
  int32_t hx = hi_word(x);
  const uint32_t lx = lo_word(x);
  int k = 0;
  if (hx < 0x00100000) {
    if (((hx & 0x7fffffff) | lx) == 0) return -from_bits(0x7FF0000000000000ull);
    if (hx < 0) return from_bits(0x7FF8000000000000ull);
    k -= 54;
    x *= two54;
    hx = hi_word(x);
  }
  if (hx >= 0x7ff00000) return x + x;
  k += (hx >> 20) - 1023;
  hx &= 0x000fffff;
  int i = (hx + 0x95f64) & 0x100000;
  x = with_hi(x, hx | (i ^ 0x3ff00000));
  k += (i >> 20);
  const double f = x - 1.0;
  double dk, R;
  if ((0x000fffff & (2 + hx)) < 3) {
    if (f == 0.0) {
      if (k == 0) return 0.0;
      dk = (double)k;
      return dk * ln2_hi + dk * ln2_lo;
    }
    R = f * f * (0.5 - 0.33333333333333333 * f);
    if (k == 0) return f - R;
    dk = (double)k;
    return dk * ln2_hi - ((R - dk * ln2_lo) - f);
  }
  const double s = f / (2.0 + f);
  dk = (double)k;
  const double z = s * s;
  i = hx - 0x6147a;
  const double w = z * z;
  const int j = 0x6b851 - hx;
  const double t1 = w * (Lg2 + w * (Lg4 + w * Lg6));
  const double t2 = z * (Lg1 + w * (Lg3 + w * (Lg5 + w * Lg7)));
  i |= j;
  R = t2 + t1;
  if (i > 0) {
    const double hfsq = 0.5 * f * f;
    if (k == 0) return f - (hfsq - s * (hfsq + R));
    return dk * ln2_hi - ((hfsq - (s * (hfsq + R) + dk * ln2_lo)) - f);
  }
  if (k == 0) return f - s * (f - R);
  return dk * ln2_hi - ((s * (f - R) - dk * ln2_lo) - f);
}

// ---- log10 (fdlibm e_log10.c), x > 0 finite ----
LSDM_HD double log10_(double x) {
  const double two54 = 1.80143985094819840000e+16, ivln10 = 4.34294481903251816668e-01,
               log10_2hi = 3.01029995663611771306e-01, log10_2lo = 3.69423907715893078616e-13;
  int32_t hx = hi_word(x);
  int k = 0;
  if (hx < 0x00100000) {
    if (((hx & 0x7fffffff) | lo_word(x)) == 0) return -from_bits(0x7FF0000000000000ull);
    if (hx < 0) return from_bits(0x7FF8000000000000ull);
    k -= 54;
    x *= two54;
    hx = hi_word(x);
  }
  if (hx >= 0x7ff00000) return x + x;
  k += (hx >> 20) - 1023;
  const int i = (int)(((uint32_t)k & 0x80000000u) >> 31);
  hx = (hx & 0x000fffff) | ((0x3ff - i) << 20);
  const double y = (double)(k + i);
  x = with_hi(x, hx);
  const double z = y * log10_2lo + ivln10 * log_(x);
  return z + y * log10_2hi;
}

// ---- pow for a non-negative integral exponent (pinned P11): binary
// exponentiation from the least significant bit; pow(x, 0) = 1 ----
LSDM_HD double powi_(double x, double yd) {
  long long n = (long long)yd;
  double r = 1.0, b = x;
  while (n > 0) {
    if (n & 1) r *= b;
    n >>= 1;
    if (n) b *= b;
  }
  return r;
}

// ---- sinh (pinned P11): odd Taylor series for |x| < 0.125 (the reference
// evaluates sinh(1/x) with x > 15 only), exp formula otherwise ----
LSDM_HD double sinh_(double x) {
  const double ax = fabs_(x);
  if (ax < 0.125) {
    const double z = x * x;
    // x (1 + z/6 (1 + z/20 (1 + z/42 (1 + z/72 (1 + z/110)))))
    return x + x * (z / 6.0 * (1.0 + z / 20.0 * (1.0 + z / 42.0 * (1.0 + z / 72.0 * (1.0 + z / 110.0)))));
  }
  const double e = exp_(ax);
  const double r = 0.5 * (e - 1.0 / e);
  return x < 0 ? -r : r;
}

// ---- sin / cos (fdlibm k_sin.c, k_cos.c, e_rem_pio2.c, s_sin.c, s_cos.c) ----
// iy = 0: y is zero (the |x| <= pi/4 entry of sin); iy = 1: x + y is the
// reduced argument (two formulas: they round differently)
LSDM_HD double ksin_(double x, double y, int iy) {
  const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
               S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
               S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
  if ((hi_word(x) & 0x7fffffff) < 0x3e400000 && (int)x == 0) return x;   // |x| < 2^-27
  const double z = x * x;
  const double v = z * x;
  const double r = S2 + z * (S3 + z * (S4 + z * (S5 + z * S6)));
  if (iy == 0) return x + v * (S1 + z * r);
  return x - ((z * (0.5 * y - v * r) - y) - v * S1);
}

LSDM_HD double kcos_(double x, double y) {
  const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
               C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
               C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
  const int32_t ix = hi_word(x) & 0x7fffffff;
  if (ix < 0x3e400000 && (int)x == 0) return 1.0;
  const double z = x * x;
  const double r = z * (C1 + z * (C2 + z * (C3 + z * (C4 + z * (C5 + z * C6)))));
  if (ix < 0x3FD33333) return 1.0 - (0.5 * z - (z * r - x * y));
  double qx;
  if (ix > 0x3fe90000) qx = 0.28125;
  else qx = from_bits((uint64_t)(uint32_t)(ix - 0x00200000) << 32);
  const double hz = 0.5 * z - qx;
  const double a = 1.0 - qx;
  return a - (hz - (z * r - x * y));
}

// high word of n * pi/2, n = 1..32 (e_rem_pio2.c's npio2_hw): equal high
// words flag a cancellation that needs the second reduction round
LSDM_HD int32_t npio2_hw_(int n) {
  switch (n) {
    case 1: return 0x3FF921FB; case 2: return 0x400921FB; case 3: return 0x4012D97C;
    case 4: return 0x401921FB; case 5: return 0x401F6A7A; case 6: return 0x4022D97C;
    case 7: return 0x4025FDBB; case 8: return 0x402921FB; case 9: return 0x402C463A;
    case 10: return 0x402F6A7A; case 11: return 0x4031475C; case 12: return 0x4032D97C;
    case 13: return 0x40346B9C; case 14: return 0x4035FDBB; case 15: return 0x40378FDB;
    case 16: return 0x403921FB; case 17: return 0x403AB41B; case 18: return 0x403C463A;
    case 19: return 0x403DD85A; case 20: return 0x403F6A7A; case 21: return 0x40407E4C;
    case 22: return 0x4041475C; case 23: return 0x4042106C; case 24: return 0x4042D97C;
    case 25: return 0x4043A28C; case 26: return 0x40446B9C; case 27: return 0x404534AC;
    case 28: return 0x4045FDBB; case 29: return 0x4046C6CB; case 30: return 0x40478FDB;
    case 31: return 0x404858EB; default: return 0x404921FB;
  }
}

// |x| < 2^19 * pi/2 (the line path's angles are within a few pi). Returns the
// quadrant; *y0 + *y1 = x - n*pi/2.
LSDM_HD int rem_pio2_(double x, double* y0, double* y1) {
  const double invpio2 = 6.36619772367581382433e-01, pio2_1 = 1.57079632673412561417e+00,
               pio2_1t = 6.07710050650619224932e-11, pio2_2 = 6.07710050630396597660e-11,
               pio2_2t = 2.02226624879595063154e-21, pio2_3 = 2.02226624871116645580e-21,
               pio2_3t = 8.47842766036889956997e-32;
  const int32_t hx = hi_word(x), ix = hx & 0x7fffffff;
  if (ix <= 0x3fe921fb) {   // |x| <= pi/4
    *y0 = x;
    *y1 = 0.0;
    return 0;
  }
  if (ix < 0x4002d97c) {    // |x| < 3pi/4: n = +-1, a 33+53-bit pi/2 suffices
    const double sg = hx > 0 ? 1.0 : -1.0;
    double z = x - sg * pio2_1;
    if (ix != 0x3ff921fb) {
      *y0 = z - sg * pio2_1t;
      *y1 = (z - *y0) - sg * pio2_1t;
    } else {                // near pi/2: 33+33+53 bits
      z -= sg * pio2_2;
      *y0 = z - sg * pio2_2t;
      *y1 = (z - *y0) - sg * pio2_2t;
    }
    return hx > 0 ? 1 : -1;
  }
  const double t = fabs_(x);
  const int n = (int)(t * invpio2 + 0.5);
  const double fn = (double)n;
  double r = t - fn * pio2_1;
  double w = fn * pio2_1t;   // first round: 85 bits
  double y = r - w;
  if (!(n < 32 && ix != npio2_hw_(n))) {
    const int j = ix >> 20;
    int i = j - ((hi_word(y) >> 20) & 0x7ff);
    if (i > 16) {            // second round: 118 bits
      double tt = r;
      w = fn * pio2_2;
      r = tt - w;
      w = fn * pio2_2t - ((tt - r) - w);
      y = r - w;
      i = j - ((hi_word(y) >> 20) & 0x7ff);
      if (i > 49) {          // third round: 151 bits
        tt = r;
        w = fn * pio2_3;
        r = tt - w;
        w = fn * pio2_3t - ((tt - r) - w);
        y = r - w;
      }
    }
  }
  const double yt = (r - y) - w;
  if (x < 0) {
    *y0 = -y;
    *y1 = -yt;
    return -n;
  }
  *y0 = y;
  *y1 = yt;
  return n;
}

LSDM_HD double sin_(double x) {
  if ((hi_word(x) & 0x7fffffff) <= 0x3fe921fb) return ksin_(x, 0.0, 0);
  double a, b;
  const int n = rem_pio2_(x, &a, &b);
  switch (n & 3) {
    case 0: return ksin_(a, b, 1);
    case 1: return kcos_(a, b);
    case 2: return -ksin_(a, b, 1);
    default: return -kcos_(a, b);
  }
}

// sin_(x) and cos_(x) together (the same results as the two calls)
LSDM_HD void sincos_(double x, double* s, double* c) {
  if ((hi_word(x) & 0x7fffffff) <= 0x3fe921fb) {
    *s = ksin_(x, 0.0, 0);
    *c = kcos_(x, 0.0);
    return;
  }
  double a, b;
  const int n = rem_pio2_(x, &a, &b);
  const double ks = ksin_(a, b, 1), kc = kcos_(a, b);
  switch (n & 3) {
    case 0: *s = ks; *c = kc; break;
    case 1: *s = kc; *c = -ks; break;
    case 2: *s = -ks; *c = -kc; break;
    default: *s = -kc; *c = ks; break;
  }
}

LSDM_HD double cos_(double x) {
  if ((hi_word(x) & 0x7fffffff) <= 0x3fe921fb) return kcos_(x, 0.0);
  double a, b;
  const int n = rem_pio2_(x, &a, &b);
  switch (n & 3) {
    case 0: return kcos_(a, b);
    case 1: return -ksin_(a, b, 1);
    case 2: return -kcos_(a, b);
    default: return ksin_(a, b, 1);
  }
}

// ---- atan / atan2 (fdlibm s_atan.c, e_atan2.c) ----
LSDM_HD double atan_(double x) {
  const double atanhi[4] = {4.63647609000806093515e-01, 7.85398163397448278999e-01,
                            9.82793723247329054082e-01, 1.57079632679489655800e+00};
  const double atanlo[4] = {2.26987774529616870924e-17, 3.06161699786838301793e-17,
                            1.39033110312309984516e-17, 6.12323399573676603587e-17};
  const double aT0 = 3.33333333333329318027e-01, aT1 = -1.99999999998764832476e-01,
               aT2 = 1.42857142725034663711e-01, aT3 = -1.11111104054623557880e-01,
               aT4 = 9.09088713343650656196e-02, aT5 = -7.69187620504482999495e-02,
               aT6 = 6.66107313738753120669e-02, aT7 = -5.83357013379057348645e-02,
               aT8 = 4.97687799461593236017e-02, aT9 = -3.65315727442169155270e-02,
               aT10 = 1.62858201153657823623e-02;
  const int32_t hx = hi_word(x);
  const int32_t ix = hx & 0x7fffffff;
  int id;
  if (ix >= 0x44100000) {  // |x| >= 2^66
    if (ix > 0x7ff00000 || (ix == 0x7ff00000 && lo_word(x) != 0)) return x + x;
    return hx > 0 ? atanhi[3] + atanlo[3] : -atanhi[3] - atanlo[3];
  }
  if (ix < 0x3fdc0000) {  // |x| < 0.4375
    if (ix < 0x3e200000) return x;
    id = -1;
  } else {
    x = fabs_(x);
    if (ix < 0x3ff30000) {
      if (ix < 0x3fe60000) {
        id = 0;
        x = (2.0 * x - 1.0) / (2.0 + x);
      } else {
        id = 1;
        x = (x - 1.0) / (x + 1.0);
      }
    } else {
      if (ix < 0x40038000) {
        id = 2;
        x = (x - 1.5) / (1.0 + 1.5 * x);
      } else {
        id = 3;
        x = -1.0 / x;
      }
    }
  }
  const double z = x * x;
  const double w = z * z;
  const double s1 = z * (aT0 + w * (aT2 + w * (aT4 + w * (aT6 + w * (aT8 + w * aT10)))));
  const double s2 = w * (aT1 + w * (aT3 + w * (aT5 + w * (aT7 + w * aT9))));
  if (id < 0) return x - x * (s1 + s2);
  const double zz = atanhi[id] - ((x * (s1 + s2) - atanlo[id]) - x);
  return hx < 0 ? -zz : zz;
}

LSDM_HD double atan2_(double y, double x) {
  const double pi_o_4 = 7.8539816339744827900E-01, pi_o_2 = 1.5707963267948965580E+00,
               pi = 3.1415926535897931160E+00, pi_lo = 1.2246467991473531772E-16;
  const int32_t hx = hi_word(x), hy = hi_word(y);
  const uint32_t lx = lo_word(x), ly = lo_word(y);
  const int32_t ix = hx & 0x7fffffff, iy = hy & 0x7fffffff;
  if ((ix | ((lx | (0u - lx)) >> 31)) > 0x7ff00000 || (iy | ((ly | (0u - ly)) >> 31)) > 0x7ff00000)
    return x + y;  // NaN
  if ((((uint32_t)hx - 0x3ff00000u) | lx) == 0) return atan_(y);  // x == 1 (no signed wrap)
  const int m = ((hy >> 31) & 1) | ((hx >> 30) & 2);
  if ((iy | ly) == 0) {  // y == 0
    switch (m) {
      case 0:
      case 1: return y;
      case 2: return pi;
      default: return -pi;
    }
  }
  if ((ix | lx) == 0) return hy < 0 ? -pi_o_2 : pi_o_2;  // x == 0
  if (ix == 0x7ff00000) {
    if (iy == 0x7ff00000) {
      switch (m) {
        case 0: return pi_o_4;
        case 1: return -pi_o_4;
        case 2: return 3.0 * pi_o_4;
        default: return -3.0 * pi_o_4;
      }
    }
    switch (m) {
      case 0: return 0.0;
      case 1: return -0.0;
      case 2: return pi;
      default: return -pi;
    }
  }
  if (iy == 0x7ff00000) return hy < 0 ? -pi_o_2 : pi_o_2;
  const int k = (iy - ix) >> 20;
  double z;
  if (k > 60) z = pi_o_2 + 0.5 * pi_lo;
  else if (hx < 0 && k < -60) z = 0.0;
  else z = atan_(fabs_(y / x));
  switch (m) {
    case 0: return z;
    case 1: return -z;
    case 2: return pi - (z - pi_lo);
    default: return (z - pi_lo) - pi;
  }
}

}  // namespace lsdm
