// Deterministic scalar math used by the ORB kernels. Every routine is written
// with plain IEEE-754 +,-,*,/ (the library is compiled with -ffp-contract=off
// and correctly rounded f32 division), so the device result equals the result
// of the same expression evaluated on the host: this is what makes keypoint
// angles and descriptor bits bit-exact against the CPU oracle.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define ORBPL_HD __host__ __device__ __forceinline__
#else
#define ORBPL_HD static inline
#include <math.h>
#endif

namespace orbpl {

// cvRound(float): round half to even (OpenCV uses cvtss2si, default MXCSR).
ORBPL_HD int cv_round(float v) {
#if defined(__HIP_DEVICE_COMPILE__)
  return (int)__builtin_rintf(v);
#else
  return (int)rintf(v);
#endif
}

ORBPL_HD float f_abs(float v) { return v < 0.f ? -v : v; }

// cv::fastAtan2 (OpenCV 3.4 core, scalar path), degrees in [0, 360).
// Polynomial constants are OpenCV's published atan2 minimax coefficients
// scaled by (float)(180/pi).
ORBPL_HD float fast_atan2_deg(float y, float x) {
  const float k180pi = (float)(180.0 / 3.14159265358979323846);
  const float p1 = 0.9997878412794807f * k180pi;
  const float p3 = -0.3258083974640975f * k180pi;
  const float p5 = 0.1555786518463281f * k180pi;
  const float p7 = -0.04432655554792128f * k180pi;
  const float eps = (float)2.220446049250313080847e-16;  // (float)DBL_EPSILON
  float ax = f_abs(x), ay = f_abs(y);
  float a, c, c2;
  if (ax >= ay) {
    c = ay / (ax + eps);
    c2 = c * c;
    a = (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
  } else {
    c = ax / (ay + eps);
    c2 = c * c;
    a = 90.f - (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
  }
  if (x < 0) a = 180.f - a;
  if (y < 0) a = 360.f - a;
  return a;
}

// Correctly rounded float cos/sin of a float argument in [0, 8) (pinned P2).
// Double-precision Cody-Waite reduction by pi/2 followed by the classic
// fdlibm minimax kernels (error < 1 double ulp), then one rounding to float.
// Verified against (float)cos((double)x) for every float angle the
// descriptor stage can produce (tests/test_math_exhaustive.py).
ORBPL_HD double k_sin(double x) {
  const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
               S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
               S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
  double z = x * x;
  double v = z * x;
  double r = S2 + z * (S3 + z * (S4 + z * (S5 + z * S6)));
  return x + v * (S1 + z * r);
}

ORBPL_HD double k_cos(double x) {
  const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
               C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
               C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
  double z = x * x;
  double r = z * (C1 + z * (C2 + z * (C3 + z * (C4 + z * (C5 + z * C6)))));
  double ax = x < 0 ? -x : x;
  if (ax < 0.3) return 1.0 - (0.5 * z - (z * r));
  double qx;
  if (ax > 0.78125) {
    qx = 0.28125;
  } else {
    // qx = x/4 with the low 32 bits of the mantissa cleared (fdlibm)
    union { double d; uint64_t u; } q;
    q.d = ax * 0.25;
    q.u &= 0xFFFFFFFF00000000ull;
    qx = q.d;
  }
  double hz = 0.5 * z - qx;
  double a = 1.0 - qx;
  return a - (hz - (z * r));
}

ORBPL_HD void cr_cos_sin(float xf, float* c, float* s) {
  const double x = (double)xf;
  const double two_over_pi = 6.36619772367581382433e-01;
  const double pio2_1 = 1.57079632673412561417e+00;   // first 33 bits of pi/2
  const double pio2_1t = 6.07710050650619224932e-11;  // pi/2 - pio2_1
#if defined(__HIP_DEVICE_COMPILE__)
  double k = __builtin_rint(x * two_over_pi);
#else
  double k = rint(x * two_over_pi);
#endif
  double r = (x - k * pio2_1) - k * pio2_1t;
  int q = ((int)k) & 3;
  double sr = k_sin(r), cr = k_cos(r);
  double cc, ss;
  switch (q) {
    case 0: cc = cr; ss = sr; break;
    case 1: cc = -sr; ss = cr; break;
    case 2: cc = -cr; ss = -sr; break;
    default: cc = sr; ss = -cr; break;
  }
  *c = (float)cc;
  *s = (float)ss;
}

}  // namespace orbpl
