// ============================================================================
// ORACLE — TEST INFRASTRUCTURE ONLY. NOT PART OF THE PRODUCT PATH.
//
// CPU restatement of the reference's line-feature extraction
//   /root/reference/src/LineExtractor.cpp:12-74  LineExtractor::ExtractLineSegment
//     LSDDetector::detect(img, keylines, scale=1, octaves=1)   (opencv_contrib 3.4)
//     keep the 80 longest (std::sort by response, :26-33)
//     BinaryDescriptor::compute(img, keylines, desc)           (opencv_contrib 3.4)
//     homogeneous line coefficients (Eigen cross + normalize, :62-72)
// and of the third-party algorithms it calls, which are absent from
// /root/reference (EXTERNAL, restated from their published algorithms):
//   LSD  — OpenCV 3.4 LineSegmentDetectorImpl (von Gioi et al., IPOL 2012, as
//          adapted by OpenCV: 8-bit image, fastAtan2 angles, float region angle
//          sums, std::sort pseudo-ordering, rect_nfa raster walk), refine mode
//          LSD_REFINE_ADV, scale 0.8, sigma_scale 0.6, quant 2, ang_th 22.5,
//          log_eps 0, density_th 0.7, n_bins 1024.
//   LBD  — opencv_contrib BinaryDescriptor::computeLBD (Zhang & Koch 2013):
//          Gaussian 5x5 sigma 1, Sobel 3x3 16S, 9 bands of width 7, local and
//          global Gaussian weights, clamp 0.4, 32 band-pair comparisons.
//   cv::LineIterator (8-connectivity) / clipLine, GaussianBlur 8U fixed point,
//   resize INTER_LINEAR_EXACT 8U.
//
// PARITY STATUS: "parity unpinned" against the real reference (OpenCV 3.4 and
// opencv_contrib are not in this image and the reference ships no line
// fixtures). Pinned semantic choices (DESIGN.md §Pinned semantics):
//   P2  float cos/sin = correctly rounded, computed as (float)cos((double)x).
//   P9  LSD resize = INTER_LINEAR_EXACT 8U (bit-exact resize, 8-bit coefficients).
//   P10 double sin/cos/exp/log/log10/atan2 = the fdlibm algorithms, the
//       oracle's own transcription in pinned_math.h (the product has its own
//       in csrc/lsd_math.h; the oracle includes nothing from csrc/).
//   P11 pow(x, integer) = binary exponentiation; sinh = odd Taylor series.
//   P12 atan2f (KeyLine::angle) = (float)atan2((double)y, (double)x) (P10).
//   P13 rect_nfa walks the rectangle with double-valued edge steps and the
//       tail corner's y (OpenCV 3.4 after its rect_nfa fix).
// std::sort calls are the reference's own (libstdc++ introsort), so ties
// follow libstdc++'s order exactly as in the reference build.
// ============================================================================
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "pinned_math.h"
#include "oracle_api.h"

namespace lsdo {

static const double kPi = 3.14159265358979323846;  // CV_PI
static const double DEG_TO_RADS = kPi / 180;
static const double NOTDEF = -1024.0;
static const uint8_t NOTUSED = 0, USED = 1;

static inline int reflect101(int i, int n) {
  if (n == 1) return 0;
  while (i < 0 || i >= n) i = i < 0 ? -i : 2 * n - 2 - i;
  return i;
}

static inline float cosf_cr(float x) { return pmath::cosf_cr(x); }
static inline float sinf_cr(float x) { return pmath::sinf_cr(x); }

// ---------------------------------------------------------------------------
// GaussianBlur, 8U fixed-point path (OpenCV >= 3.4.2 smooth.cpp): kernel in
// 8.8 fixed point from getGaussianKernelBitExact, separable, REFLECT_101.
// ---------------------------------------------------------------------------
void fixed_gauss_kernel(int n, double sigma, int* k) {
  const double scale2X = -0.125 / (sigma * sigma);
  const int n2 = (n - 1) / 2;
  std::vector<double> values(n2 + 1);
  double sum = 0;
  for (int i = 0, x = 1 - n; i < n2; i++, x += 2) {
    values[i] = pmath::exp_((double)(x * x) * scale2X);
    sum += values[i];
  }
  sum *= 2;
  sum += 1.0;
  const double mul1 = 1.0 / sum;
  int sum2 = 0;
  for (int i = 0; i < n2; i++) {
    const double v = values[i] * mul1 * 256.0;
    const int t = (int)std::lrint(v);
    k[i] = t;
    k[n - 1 - i] = t;
    sum2 += t;
  }
  k[n2] = 256 - 2 * sum2;
}

static void gauss_fixed(const uint8_t* src, int W, int H, const int* k, int n, uint8_t* dst) {
  const int r = n / 2;
  std::vector<int> tmp((size_t)W * H);
  for (int y = 0; y < H; y++)
    for (int x = 0; x < W; x++) {
      int acc = 0;
      for (int j = 0; j < n; j++) acc += k[j] * src[(size_t)y * W + reflect101(x + j - r, W)];
      tmp[(size_t)y * W + x] = acc;
    }
  for (int y = 0; y < H; y++)
    for (int x = 0; x < W; x++) {
      int acc = 0;
      for (int j = 0; j < n; j++) acc += k[j] * tmp[(size_t)reflect101(y + j - r, H) * W + x];
      dst[(size_t)y * W + x] = (uint8_t)std::min(255, (acc + (1 << 15)) >> 16);
    }
}

// ---------------------------------------------------------------------------
// resize INTER_LINEAR_EXACT, 8U (OpenCV resize_bitExact / interpolationLinear):
// 8.8 fixed-point coefficients, horizontal then vertical, round at the end.
// ---------------------------------------------------------------------------
struct LinCoeffs {
  std::vector<int> ofs, c1;  // c0 = 256 - c1
  int mn = 0, mx = 0;
};

static LinCoeffs lin_coeffs(double inv_scale, int ssize, int dsize) {
  LinCoeffs L;
  L.ofs.assign(dsize, 0);
  L.c1.assign(dsize, 0);
  const double scale = 1.0 / inv_scale;
  int minofst = 0, maxofst = dsize;
  for (int d = 0; d < dsize; d++) {
    const double fval = scale * ((double)d + 0.5) - 0.5;
    const int ival = (int)std::floor(fval);
    if (ival >= 0 && ssize > 1) {
      if (ival < ssize - 1) {
        L.ofs[d] = ival;
        L.c1[d] = (int)std::lrint((fval - (double)ival) * 256.0);
      } else {
        L.ofs[d] = ssize - 1;
        maxofst = std::min(maxofst, d);
      }
    } else {
      minofst = std::max(minofst, d + 1);
    }
  }
  L.mn = minofst;
  L.mx = maxofst;
  return L;
}

void resize_exact(const uint8_t* src, int sw, int sh, double fx, uint8_t* dst, int dw, int dh) {
  const LinCoeffs X = lin_coeffs(fx, sw, dw), Y = lin_coeffs(fx, sh, dh);
  auto hrow = [&](int sy, std::vector<int>& out) {
    const uint8_t* S = src + (size_t)sy * sw;
    out.resize(dw);
    for (int dx = 0; dx < dw; dx++) {
      if (dx < X.mn) out[dx] = S[0] << 8;
      else if (dx >= X.mx) out[dx] = S[X.ofs[dw - 1]] << 8;
      else out[dx] = (256 - X.c1[dx]) * S[X.ofs[dx]] + X.c1[dx] * S[X.ofs[dx] + 1];
    }
  };
  std::vector<int> r0, r1;
  for (int dy = 0; dy < dh; dy++) {
    uint8_t* D = dst + (size_t)dy * dw;
    if (dy < Y.mn || dy >= Y.mx) {
      hrow(dy < Y.mn ? 0 : sh - 1, r0);
      for (int dx = 0; dx < dw; dx++) D[dx] = (uint8_t)std::min(255, (r0[dx] + 0x80) >> 8);
      continue;
    }
    hrow(Y.ofs[dy], r0);
    hrow(Y.ofs[dy] + 1, r1);
    const int b1 = Y.c1[dy], b0 = 256 - b1;
    for (int dx = 0; dx < dw; dx++)
      D[dx] = (uint8_t)std::min(255, (r0[dx] * b0 + r1[dx] * b1 + 0x8000) >> 16);
  }
}

// ---------------------------------------------------------------------------
// LSD (OpenCV 3.4 lsd.cpp LineSegmentDetectorImpl), LSD_REFINE_ADV
// ---------------------------------------------------------------------------
struct RegionPoint {
  int x, y;
  uint8_t* used;
  double angle, modgrad;
};

struct Rect {
  double x1, y1, x2, y2, width, x, y, theta, dx, dy, prec, p;
};

struct NormPoint {
  int x, y;
  int norm;
};

struct Edge {
  int x, y;
  bool taken;
};

static inline bool double_equal(double a, double b) {
  if (a == b) return true;
  const double abs_diff = std::fabs(a - b);
  const double aa = std::fabs(a), bb = std::fabs(b);
  double abs_max = aa > bb ? aa : bb;
  if (abs_max < DBL_MIN) abs_max = DBL_MIN;
  return (abs_diff / abs_max) <= (100.0 * DBL_EPSILON);
}

static inline double angle_diff_signed(double a, double b) {
  double diff = a - b;
  while (diff <= -kPi) diff += 2 * kPi;
  while (diff > kPi) diff -= 2 * kPi;
  return diff;
}
static inline double angle_diff(double a, double b) { return std::fabs(angle_diff_signed(a, b)); }

static inline double dist(double x1, double y1, double x2, double y2) {
  return std::sqrt((x2 - x1) * (x2 - x1) + (y2 - y1) * (y2 - y1));
}
static inline double distSq(double x1, double y1, double x2, double y2) {
  return (x2 - x1) * (x2 - x1) + (y2 - y1) * (y2 - y1);
}

static inline double log_gamma_windschitl(double x) {
  return 0.918938533204673 + (x - 0.5) * pmath::log_(x) - x +
         0.5 * x * pmath::log_(x * pmath::sinh_(1 / x) + 1 / (810.0 * pmath::powi(x, 6.0)));
}
static inline double log_gamma_lanczos(double x) {
  static const double q[7] = {75122.6331530, 80916.6278952, 36308.2951477, 8687.24529705,
                              1168.92649479, 83.8676043424, 2.50662827511};
  double a = (x + 0.5) * pmath::log_(x + 5.5) - (x + 5.5);
  double b = 0;
  for (int n = 0; n < 7; ++n) {
    a -= pmath::log_(x + double(n));
    b += q[n] * pmath::powi(x, double(n));
  }
  return a + pmath::log_(b);
}
static inline double log_gamma(double x) {
  return x > 15.0 ? log_gamma_windschitl(x) : log_gamma_lanczos(x);
}

// Element accesses of the sequential algorithm, by stage (test / measurement
// infrastructure: the algorithmic-traffic floor of the LSD kernels, see
// oracle_lsd_traffic). Counted, not timed; the detection result is unchanged.
struct LsdTraffic {
  long long sort_cmp = 0, sort_moves = 0;    // pseudo-order std::sort: compares, element writes
  long long seeds = 0;                       // ordered entries the seed loop visits
  long long grow_nb = 0, grow_add = 0;       // region_grow: in-image neighbour reads, adds
  long long grow_expand = 0;                 // region list reads (points expanded)
  long long grows = 0;                       // region_grow calls (first + refine's second)
  long long fit_reads = 0, fit_writes = 0;   // region list element reads / writes of the fit
  long long nfa_evals = 0, nfa_px = 0;       // rect_nfa calls, rectangle pixels visited
  // distinct addresses (touched-address bitmaps over the scaled image): the
  // unique-bytes floor of each stage, every element fetched or stored once
  long long sort_n = 0;                      // pseudo-ordered entries (keys read + written)
  long long max_reg = 0;                     // longest region list (list scratch slots)
  long long rects = 0;                       // rectangles validated (rect_improve calls)
  std::vector<uint8_t> px;                   // bit 0 seed-loop pixel read, 1 USED written,
                                             // 2 q (weight) read, 3 NFA angle read
  void mark(int W, int x, int y, uint8_t bit) { px[(size_t)y * W + x] |= bit; }
};

struct LSD {
  LsdTraffic* tr = nullptr;   // non-NULL: count element accesses
  // parameters (LSD_REFINE_ADV defaults)
  const double SCALE = 0.8, SIGMA_SCALE = 0.6, QUANT = 2.0, ANG_TH = 22.5, LOG_EPS = 0,
               DENSITY_TH = 0.7;
  const int N_BINS = 1024;

  int img_width = 0, img_height = 0;
  double LOG_NT = 0;
  std::vector<uint8_t> scaled;       // 8-bit scaled image
  std::vector<double> angles, modgrad;
  std::vector<uint8_t> used;
  std::vector<NormPoint> ordered;

  double ang(int x, int y) const { return angles[(size_t)y * img_width + x]; }

  bool isAligned(int x, int y, double theta, double prec) const {
    if (x < 0 || y < 0 || x >= img_width || y >= img_height) return false;
    const double a = ang(x, y);
    if (a == NOTDEF) return false;
    double n_theta = theta - a;
    if (n_theta < 0) n_theta = -n_theta;
    if (n_theta > (3 * kPi) / 2) {
      n_theta -= (2 * kPi);
      if (n_theta < 0) n_theta = -n_theta;
    }
    return n_theta <= prec;
  }

  void ll_angle(double threshold) {
    const int W = img_width, H = img_height;
    angles.assign((size_t)W * H, 0.0);
    modgrad.assign((size_t)W * H, 0.0);
    for (int x = 0; x < W; x++) angles[(size_t)(H - 1) * W + x] = NOTDEF;
    for (int y = 0; y < H; y++) angles[(size_t)y * W + W - 1] = NOTDEF;
    double max_grad = -1;
    for (int y = 0; y < H - 1; ++y) {
      const uint8_t* r0 = &scaled[(size_t)y * W];
      const uint8_t* r1 = &scaled[(size_t)(y + 1) * W];
      for (int x = 0; x < W - 1; ++x) {
        const int DA = r1[x + 1] - r0[x];
        const int BC = r0[x + 1] - r1[x];
        const int gx = DA + BC, gy = DA - BC;
        const double norm = std::sqrt((gx * gx + gy * gy) / 4.0);
        modgrad[(size_t)y * W + x] = norm;
        if (norm <= threshold) {
          angles[(size_t)y * W + x] = NOTDEF;
        } else {
          angles[(size_t)y * W + x] = oracle_fast_atan2(float(gx), float(-gy)) * DEG_TO_RADS;
          if (norm > max_grad) max_grad = norm;
        }
      }
    }
    const double bin_coef = (max_grad > 0) ? double(N_BINS - 1) / max_grad : 0;
    ordered.clear();
    ordered.reserve((size_t)(W - 1) * (H - 1));
    for (int y = 0; y < H - 1; ++y)
      for (int x = 0; x < W - 1; ++x) {
        NormPoint p;
        p.x = x;
        p.y = y;
        p.norm = int(modgrad[(size_t)y * W + x] * bin_coef);
        ordered.push_back(p);
      }
    if (!tr) {
      std::sort(ordered.begin(), ordered.end(),
                [](const NormPoint& a, const NormPoint& b) { return a.norm > b.norm; });
    } else {
      // the same std::sort over a counting element type: same comparisons,
      // same permutation; compares and element writes counted
      struct CP {
        NormPoint v;
        long long* mv;
        CP(NormPoint a, long long* m) : v(a), mv(m) {}
        CP(const CP& o) : v(o.v), mv(o.mv) { ++*mv; }
        CP& operator=(const CP& o) {
          v = o.v;
          mv = o.mv;
          ++*mv;
          return *this;
        }
      };
      std::vector<CP> c;
      c.reserve(ordered.size());
      for (const NormPoint& q : ordered) c.emplace_back(q, &tr->sort_moves);
      tr->sort_moves = 0;
      tr->sort_n = (long long)ordered.size();
      long long* nc = &tr->sort_cmp;
      std::sort(c.begin(), c.end(), [nc](const CP& a, const CP& b) {
        ++*nc;
        return a.v.norm > b.v.norm;
      });
      for (size_t i = 0; i < c.size(); i++) ordered[i] = c[i].v;
    }
  }

  void region_grow(int sx, int sy, std::vector<RegionPoint>& reg, double& reg_angle,
                   double prec) {
    const int W = img_width, H = img_height;
    reg.clear();
    RegionPoint seed;
    seed.x = sx;
    seed.y = sy;
    seed.used = &used[(size_t)sy * W + sx];
    reg_angle = ang(sx, sy);
    seed.angle = reg_angle;
    seed.modgrad = modgrad[(size_t)sy * W + sx];
    reg.push_back(seed);
    float sumdx = float(pmath::cos_(reg_angle));
    float sumdy = float(pmath::sin_(reg_angle));
    *seed.used = USED;
    if (tr) {
      tr->grows++;
      tr->grow_add++;
      tr->mark(W, sx, sy, 1 | 2);
    }
    for (size_t i = 0; i < reg.size(); i++) {
      const RegionPoint rpoint = reg[i];
      const int xx_min = std::max(rpoint.x - 1, 0), xx_max = std::min(rpoint.x + 1, W - 1);
      const int yy_min = std::max(rpoint.y - 1, 0), yy_max = std::min(rpoint.y + 1, H - 1);
      if (tr) {
        tr->grow_expand++;
        tr->grow_nb += (long long)(xx_max - xx_min + 1) * (yy_max - yy_min + 1) - 1;
        for (int yy = yy_min; yy <= yy_max; ++yy)
          for (int xx = xx_min; xx <= xx_max; ++xx) tr->mark(W, xx, yy, 1);
      }
      for (int yy = yy_min; yy <= yy_max; ++yy)
        for (int xx = xx_min; xx <= xx_max; ++xx) {
          uint8_t& is_used = used[(size_t)yy * W + xx];
          if (is_used != USED && isAligned(xx, yy, reg_angle, prec)) {
            const double angle = ang(xx, yy);
            is_used = USED;
            RegionPoint rp;
            rp.x = xx;
            rp.y = yy;
            rp.used = &is_used;
            rp.modgrad = modgrad[(size_t)yy * W + xx];
            rp.angle = angle;
            reg.push_back(rp);
            sumdx += cosf_cr(float(angle));
            sumdy += sinf_cr(float(angle));
            reg_angle = oracle_fast_atan2(sumdy, sumdx) * DEG_TO_RADS;
            if (tr) {
              tr->grow_add++;
              tr->mark(W, xx, yy, 2);
            }
          }
        }
    }
  }

  double get_theta(const std::vector<RegionPoint>& reg, double x, double y, double reg_angle,
                   double prec) const {
    double Ixx = 0.0, Iyy = 0.0, Ixy = 0.0;
    for (size_t i = 0; i < reg.size(); ++i) {
      const double regx = reg[i].x, regy = reg[i].y;
      const double weight = reg[i].modgrad;
      const double dx = regx - x, dy = regy - y;
      Ixx += dy * dy * weight;
      Iyy += dx * dx * weight;
      Ixy -= dx * dy * weight;
    }
    const double lambda = 0.5 * (Ixx + Iyy - std::sqrt((Ixx - Iyy) * (Ixx - Iyy) + 4.0 * Ixy * Ixy));
    double theta = (std::fabs(Ixx) > std::fabs(Iyy))
                       ? double(oracle_fast_atan2(float(lambda - Ixx), float(Ixy)))
                       : double(oracle_fast_atan2(float(Ixy), float(lambda - Iyy)));
    theta *= DEG_TO_RADS;
    if (angle_diff(theta, reg_angle) > prec) theta += kPi;
    return theta;
  }

  void region2rect(const std::vector<RegionPoint>& reg, double reg_angle, double prec, double p,
                   Rect& rec) const {
    if (tr) {
      tr->fit_reads += 3 * (long long)reg.size();   // centroid, inertia, extents passes
      tr->max_reg = std::max(tr->max_reg, (long long)reg.size());
      for (const RegionPoint& r : reg) tr->mark(img_width, r.x, r.y, 4);
    }
    double x = 0, y = 0, sum = 0;
    for (size_t i = 0; i < reg.size(); ++i) {
      const double weight = reg[i].modgrad;
      x += double(reg[i].x) * weight;
      y += double(reg[i].y) * weight;
      sum += weight;
    }
    x /= sum;
    y /= sum;
    const double theta = get_theta(reg, x, y, reg_angle, prec);
    const double dx = pmath::cos_(theta), dy = pmath::sin_(theta);
    double l_min = 0, l_max = 0, w_min = 0, w_max = 0;
    for (size_t i = 0; i < reg.size(); ++i) {
      const double regdx = double(reg[i].x) - x, regdy = double(reg[i].y) - y;
      const double l = regdx * dx + regdy * dy;
      const double w = -regdx * dy + regdy * dx;
      if (l > l_max) l_max = l;
      else if (l < l_min) l_min = l;
      if (w > w_max) w_max = w;
      else if (w < w_min) w_min = w;
    }
    rec.x1 = x + l_min * dx;
    rec.y1 = y + l_min * dy;
    rec.x2 = x + l_max * dx;
    rec.y2 = y + l_max * dy;
    rec.width = w_max - w_min;
    rec.x = x;
    rec.y = y;
    rec.theta = theta;
    rec.dx = dx;
    rec.dy = dy;
    rec.prec = prec;
    rec.p = p;
    if (rec.width < 1.0) rec.width = 1.0;
  }

  bool reduce_region_radius(std::vector<RegionPoint>& reg, double reg_angle, double prec,
                            double p, Rect& rec, double density) {
    const double xc = double(reg[0].x), yc = double(reg[0].y);
    const double radSq1 = distSq(xc, yc, rec.x1, rec.y1);
    const double radSq2 = distSq(xc, yc, rec.x2, rec.y2);
    double radSq = radSq1 > radSq2 ? radSq1 : radSq2;
    while (density < DENSITY_TH) {
      radSq *= 0.75 * 0.75;
      for (size_t i = 0; i < reg.size(); ++i) {
        if (tr) tr->fit_reads++;
        if (distSq(xc, yc, double(reg[i].x), double(reg[i].y)) > radSq) {
          if (tr) {
            tr->fit_writes += 2;   // the USED flag, the swapped-in element
            tr->mark(img_width, reg[i].x, reg[i].y, 2);
          }
          *(reg[i].used) = NOTUSED;
          std::swap(reg[i], reg[reg.size() - 1]);
          reg.pop_back();
          --i;
        }
      }
      if (reg.size() < 2) return false;
      region2rect(reg, reg_angle, prec, p, rec);
      density = double(reg.size()) / (dist(rec.x1, rec.y1, rec.x2, rec.y2) * rec.width);
    }
    return true;
  }

  bool refine(std::vector<RegionPoint>& reg, double reg_angle, double prec, double p, Rect& rec) {
    double density = double(reg.size()) / (dist(rec.x1, rec.y1, rec.x2, rec.y2) * rec.width);
    if (density >= DENSITY_TH) return true;
    const double xc = double(reg[0].x), yc = double(reg[0].y);
    const double ang_c = reg[0].angle;
    double sum = 0, s_sum = 0;
    int n = 0;
    if (tr) {
      tr->fit_reads += (long long)reg.size();
      tr->fit_writes += (long long)reg.size();   // USED flags released before the regrow
      for (const RegionPoint& r : reg) tr->mark(img_width, r.x, r.y, 2);
    }
    for (size_t i = 0; i < reg.size(); ++i) {
      *(reg[i].used) = NOTUSED;
      if (dist(xc, yc, reg[i].x, reg[i].y) < rec.width) {
        const double angle = reg[i].angle;
        const double ang_d = angle_diff_signed(angle, ang_c);
        sum += ang_d;
        s_sum += ang_d * ang_d;
        ++n;
      }
    }
    const double mean_angle = sum / double(n);
    const double tau =
        2.0 * std::sqrt((s_sum - 2.0 * mean_angle * sum) / double(n) + mean_angle * mean_angle);
    region_grow(reg[0].x, reg[0].y, reg, reg_angle, tau);
    if (reg.size() < 2) return false;
    region2rect(reg, reg_angle, prec, p, rec);
    density = double(reg.size()) / (dist(rec.x1, rec.y1, rec.x2, rec.y2) * rec.width);
    if (density < DENSITY_TH) return reduce_region_radius(reg, reg_angle, prec, p, rec, density);
    return true;
  }

  double nfa(int n, int k, double p) const {
    if (n == 0 || k == 0) return -LOG_NT;
    if (n == k) return -LOG_NT - double(n) * pmath::log10_(p);
    const double p_term = p / (1 - p);
    const double log1term = log_gamma(double(n) + 1) - log_gamma(double(k) + 1) -
                            log_gamma(double(n - k) + 1) + double(k) * pmath::log_(p) +
                            double(n - k) * pmath::log_(1.0 - p);
    double term = pmath::exp_(log1term);
    if (double_equal(term, 0)) {
      if (k > n * p) return -log1term / 2.30258509299404568402 - LOG_NT;
      return -LOG_NT;
    }
    double bin_tail = term;
    const double tolerance = 0.1;
    for (int i = k + 1; i <= n; ++i) {
      const double bin_term = double(n - i + 1) / double(i);
      const double mult_term = bin_term * p_term;
      term *= mult_term;
      bin_tail += term;
      if (bin_term < 1) {
        const double err =
            term * ((1 - pmath::powi(mult_term, double(n - i + 1))) / (1 - mult_term) - 1);
        if (err < tolerance * std::fabs(-pmath::log10_(bin_tail) - LOG_NT) * bin_tail) break;
      }
    }
    return -pmath::log10_(bin_tail) - LOG_NT;
  }

  double rect_nfa(const Rect& rec) const {
    int total_pts = 0, alg_pts = 0;
    const double half_width = rec.width / 2.0;
    const double dyhw = rec.dy * half_width;
    const double dxhw = rec.dx * half_width;
    Edge ordered_x[4];
    ordered_x[0] = {int(rec.x1 - dyhw), int(rec.y1 + dxhw), false};
    ordered_x[1] = {int(rec.x2 - dyhw), int(rec.y2 + dxhw), false};
    ordered_x[2] = {int(rec.x2 + dyhw), int(rec.y2 - dxhw), false};
    ordered_x[3] = {int(rec.x1 + dyhw), int(rec.y1 - dxhw), false};
    std::sort(ordered_x, ordered_x + 4, [](const Edge& a, const Edge& b) {
      return (a.x < b.x) || (a.x == b.x && a.y < b.y);
    });
    Edge* min_y = &ordered_x[0];
    Edge* max_y = &ordered_x[0];
    for (int i = 1; i < 4; ++i) {
      if (min_y->y > ordered_x[i].y) min_y = &ordered_x[i];
      if (max_y->y < ordered_x[i].y) max_y = &ordered_x[i];
    }
    min_y->taken = true;
    Edge* leftmost = nullptr;
    for (int i = 0; i < 4; ++i)
      if (!ordered_x[i].taken) {
        if (!leftmost) leftmost = &ordered_x[i];
        else if (leftmost->x > ordered_x[i].x) leftmost = &ordered_x[i];
      }
    leftmost->taken = true;
    Edge* rightmost = nullptr;
    for (int i = 0; i < 4; ++i)
      if (!ordered_x[i].taken) {
        if (!rightmost) rightmost = &ordered_x[i];
        else if (rightmost->x < ordered_x[i].x) rightmost = &ordered_x[i];
      }
    rightmost->taken = true;
    Edge* tailp = nullptr;
    for (int i = 0; i < 4; ++i)
      if (!ordered_x[i].taken) {
        if (!tailp) tailp = &ordered_x[i];
        else if (tailp->x > ordered_x[i].x) tailp = &ordered_x[i];
      }
    tailp->taken = true;
    // pinned P13: double-valued steps and the tail corner's y (OpenCV 3.4
    // after its rect_nfa fix). The pre-fix text divides integer corner
    // coordinates and uses the tail's x for its y; that walk loses most
    // oblique segments (a 30-degree square keeps 1 of 4 sides), see DESIGN.md.
    const double flstep =
        (min_y->y != leftmost->y) ? (min_y->x - leftmost->x) / double(min_y->y - leftmost->y) : 0;
    const double slstep =
        (leftmost->y != tailp->y) ? (leftmost->x - tailp->x) / double(leftmost->y - tailp->y) : 0;
    const double frstep =
        (min_y->y != rightmost->y) ? (min_y->x - rightmost->x) / double(min_y->y - rightmost->y) : 0;
    const double srstep =
        (rightmost->y != tailp->y) ? (rightmost->x - tailp->x) / double(rightmost->y - tailp->y) : 0;
    double lstep = flstep, rstep = frstep;
    double left_x = min_y->x, right_x = min_y->x;
    const int min_iter = min_y->y, max_iter = max_y->y;
    for (int y = min_iter; y <= max_iter; ++y) {
      if (y < 0 || y >= img_height) continue;
      for (int x = int(left_x); x <= int(right_x); ++x) {
        if (x < 0 || x >= img_width) continue;
        ++total_pts;
        if (tr) tr->mark(img_width, x, y, 8);
        if (isAligned(x, y, rec.theta, rec.prec)) ++alg_pts;
      }
      if (y >= leftmost->y) lstep = slstep;
      if (y >= rightmost->y) rstep = srstep;
      left_x += lstep;
      right_x += rstep;
    }
    if (tr) {
      tr->nfa_evals++;
      tr->nfa_px += total_pts;
    }
    return nfa(total_pts, alg_pts, rec.p);
  }

  double rect_improve(Rect& rec) const {
    const double delta = 0.5, delta_2 = delta / 2.0;
    double log_nfa = rect_nfa(rec);
    if (log_nfa > LOG_EPS) return log_nfa;
    Rect r = rec;
    for (int n = 0; n < 5; ++n) {
      r.p /= 2;
      r.prec = r.p * kPi;
      const double log_nfa_new = rect_nfa(r);
      if (log_nfa_new > log_nfa) {
        log_nfa = log_nfa_new;
        rec = r;
      }
    }
    if (log_nfa > LOG_EPS) return log_nfa;
    r = rec;
    for (int n = 0; n < 5; ++n) {
      if ((r.width - delta) >= 0.5) {
        r.width -= delta;
        const double log_nfa_new = rect_nfa(r);
        if (log_nfa_new > log_nfa) {
          rec = r;
          log_nfa = log_nfa_new;
        }
      }
    }
    if (log_nfa > LOG_EPS) return log_nfa;
    r = rec;
    for (int n = 0; n < 5; ++n) {
      if ((r.width - delta) >= 0.5) {
        r.x1 += -r.dy * delta_2;
        r.y1 += r.dx * delta_2;
        r.x2 += -r.dy * delta_2;
        r.y2 += r.dx * delta_2;
        r.width -= delta;
        const double log_nfa_new = rect_nfa(r);
        if (log_nfa_new > log_nfa) {
          rec = r;
          log_nfa = log_nfa_new;
        }
      }
    }
    if (log_nfa > LOG_EPS) return log_nfa;
    r = rec;
    for (int n = 0; n < 5; ++n) {
      if ((r.width - delta) >= 0.5) {
        r.x1 -= -r.dy * delta_2;
        r.y1 -= r.dx * delta_2;
        r.x2 -= -r.dy * delta_2;
        r.y2 -= r.dx * delta_2;
        r.width -= delta;
        const double log_nfa_new = rect_nfa(r);
        if (log_nfa_new > log_nfa) {
          rec = r;
          log_nfa = log_nfa_new;
        }
      }
    }
    if (log_nfa > LOG_EPS) return log_nfa;
    r = rec;
    for (int n = 0; n < 5; ++n) {
      if ((r.width - delta) >= 0.5) {
        r.p /= 2;
        r.prec = r.p * kPi;
        const double log_nfa_new = rect_nfa(r);
        if (log_nfa_new > log_nfa) {
          rec = r;
          log_nfa = log_nfa_new;
        }
      }
    }
    return log_nfa;
  }

  // LineSegmentDetectorImpl::detect + flsd on an 8-bit image.
  void detect(const uint8_t* img, int W, int H, std::vector<float>& lines) {
    lines.clear();
    const double prec = kPi * ANG_TH / 180;
    const double p = ANG_TH / 180;
    const double rho = QUANT / pmath::sin_(prec);
    // Gaussian sub-sampling
    const double sigma = (SCALE < 1) ? (SIGMA_SCALE / SCALE) : SIGMA_SCALE;
    const double sprec = 3;
    const unsigned h = (unsigned)std::ceil(sigma * std::sqrt(2 * sprec * pmath::log_(10.0)));
    const int ksize = 1 + 2 * (int)h;
    std::vector<int> k(ksize);
    fixed_gauss_kernel(ksize, sigma, k.data());
    std::vector<uint8_t> g((size_t)W * H);
    gauss_fixed(img, W, H, k.data(), ksize, g.data());
    img_width = (int)std::lrint(W * SCALE);
    img_height = (int)std::lrint(H * SCALE);
    scaled.assign((size_t)img_width * img_height, 0);
    resize_exact(g.data(), W, H, SCALE, scaled.data(), img_width, img_height);
    ll_angle(rho);
    LOG_NT = 5 * (pmath::log10_(double(img_width)) + pmath::log10_(double(img_height))) / 2 +
             pmath::log10_(11.0);
    const size_t min_reg_size = size_t(-LOG_NT / pmath::log10_(p));
    used.assign((size_t)img_width * img_height, NOTUSED);
    if (tr) tr->px.assign((size_t)img_width * img_height, 0);
    std::vector<RegionPoint> reg;
    for (size_t i = 0; i < ordered.size(); ++i) {
      const int px = ordered[i].x, py = ordered[i].y;
      if (tr) {
        tr->seeds++;
        tr->mark(img_width, px, py, 1);
      }
      if (used[(size_t)py * img_width + px] != NOTUSED || ang(px, py) == NOTDEF) continue;
      double reg_angle;
      region_grow(px, py, reg, reg_angle, prec);
      if (reg.size() < min_reg_size) continue;
      Rect rec;
      region2rect(reg, reg_angle, prec, p, rec);
      if (!refine(reg, reg_angle, prec, p, rec)) continue;
      if (tr) tr->rects++;
      const double log_nfa = rect_improve(rec);
      if (log_nfa <= LOG_EPS) continue;
      rec.x1 += 0.5;
      rec.y1 += 0.5;
      rec.x2 += 0.5;
      rec.y2 += 0.5;
      rec.x1 /= SCALE;
      rec.y1 /= SCALE;
      rec.x2 /= SCALE;
      rec.y2 /= SCALE;
      lines.push_back(float(rec.x1));
      lines.push_back(float(rec.y1));
      lines.push_back(float(rec.x2));
      lines.push_back(float(rec.y2));
    }
  }
};

// ---------------------------------------------------------------------------
// cv::LineIterator(img, Point(pt1), Point(pt2), 8).count with clipLine.
// ---------------------------------------------------------------------------
static int cv_round_f(float v) { return (int)std::nearbyint(v); }

static bool clip_line(int W, int H, long long& x1, long long& y1, long long& x2, long long& y2) {
  const long long right = W - 1, bottom = H - 1;
  if (W <= 0 || H <= 0) return false;
  int c1 = (x1 < 0) + (x1 > right) * 2 + (y1 < 0) * 4 + (y1 > bottom) * 8;
  int c2 = (x2 < 0) + (x2 > right) * 2 + (y2 < 0) * 4 + (y2 > bottom) * 8;
  if ((c1 & c2) == 0 && (c1 | c2) != 0) {
    long long a;
    if (c1 & 12) {
      a = c1 < 8 ? 0 : bottom;
      x1 += (long long)((double)(a - y1) * (x2 - x1) / (y2 - y1));
      y1 = a;
      c1 = (x1 < 0) + (x1 > right) * 2;
    }
    if (c2 & 12) {
      a = c2 < 8 ? 0 : bottom;
      x2 += (long long)((double)(a - y2) * (x2 - x1) / (y2 - y1));
      y2 = a;
      c2 = (x2 < 0) + (x2 > right) * 2;
    }
    if ((c1 & c2) == 0 && (c1 | c2) != 0) {
      if (c1) {
        a = c1 == 1 ? 0 : right;
        y1 += (long long)((double)(a - x1) * (y2 - y1) / (x2 - x1));
        x1 = a;
        c1 = 0;
      }
      if (c2) {
        a = c2 == 1 ? 0 : right;
        y2 += (long long)((double)(a - x2) * (y2 - y1) / (x2 - x1));
        x2 = a;
        c2 = 0;
      }
    }
  }
  return (c1 | c2) == 0;
}

int line_iterator_count(int W, int H, float fx1, float fy1, float fx2, float fy2) {
  long long x1 = cv_round_f(fx1), y1 = cv_round_f(fy1), x2 = cv_round_f(fx2), y2 = cv_round_f(fy2);
  if ((unsigned long long)x1 >= (unsigned long long)W || (unsigned long long)x2 >= (unsigned long long)W ||
      (unsigned long long)y1 >= (unsigned long long)H || (unsigned long long)y2 >= (unsigned long long)H) {
    if (!clip_line(W, H, x1, y1, x2, y2)) return 0;
  }
  long long dx = x2 - x1, dy = y2 - y1;
  if (dx < 0) dx = -dx;
  if (dy < 0) dy = -dy;
  return (int)(std::max(dx, dy) + 1);
}

// ---------------------------------------------------------------------------
// LBD (opencv_contrib BinaryDescriptor): weights, Sobel images, descriptor.
// ---------------------------------------------------------------------------
static const int kBandW = 7, kBands = 9;
static const int kComb[32][2] = {{0, 1}, {0, 2}, {0, 3}, {0, 4}, {0, 5}, {0, 6}, {1, 2}, {1, 3},
                                 {1, 4}, {1, 5}, {1, 6}, {2, 3}, {2, 4}, {2, 5}, {2, 6}, {2, 7},
                                 {2, 8}, {3, 4}, {3, 5}, {3, 6}, {3, 7}, {3, 8}, {4, 5}, {4, 6},
                                 {4, 7}, {4, 8}, {5, 6}, {5, 7}, {5, 8}, {6, 7}, {6, 8}, {7, 8}};

void lbd_weights(float* gL /*21*/, float* gG /*63*/) {
  double u = (kBandW * 3 - 1) / 2;
  double sigma = (kBandW * 2 + 1) / 2;
  double invsigma2 = -1 / (2 * sigma * sigma);
  for (int i = 0; i < kBandW * 3; i++) {
    const double dis = i - u;
    gL[i] = (float)pmath::exp_(dis * dis * invsigma2);
  }
  u = (kBands * kBandW - 1) / 2;
  sigma = u;
  invsigma2 = -1 / (2 * sigma * sigma);
  for (int i = 0; i < kBands * kBandW; i++) {
    const double dis = i - u;
    gG[i] = (float)pmath::exp_(dis * dis * invsigma2);
  }
}

void sobel_images(const uint8_t* img, int W, int H, int16_t* dx, int16_t* dy) {
  int k5[5];
  fixed_gauss_kernel(5, 1.0, k5);
  std::vector<uint8_t> g((size_t)W * H);
  gauss_fixed(img, W, H, k5, 5, g.data());
  auto G = [&](int x, int y) { return (int)g[(size_t)reflect101(y, H) * W + reflect101(x, W)]; };
  for (int y = 0; y < H; y++)
    for (int x = 0; x < W; x++) {
      const int gx = (G(x + 1, y - 1) - G(x - 1, y - 1)) + 2 * (G(x + 1, y) - G(x - 1, y)) +
                     (G(x + 1, y + 1) - G(x - 1, y + 1));
      const int gy = (G(x - 1, y + 1) - G(x - 1, y - 1)) + 2 * (G(x, y + 1) - G(x, y - 1)) +
                     (G(x + 1, y + 1) - G(x + 1, y - 1));
      dx[(size_t)y * W + x] = (int16_t)gx;
      dy[(size_t)y * W + x] = (int16_t)gy;
    }
}

void lbd_descriptor(const orbpl_keyline& kl, const int16_t* pdx, const int16_t* pdy, int W, int H,
                    const float* gL, const float* gG, uint8_t* out32) {
  const short heightOfLSP = kBandW * kBands;
  const short halfHeight = (heightOfLSP - 1) / 2;
  const short imageWidth = (short)(W - 1), imageHeight = (short)(H - 1);
  float pL[kBands] = {}, nL[kBands] = {}, pL2[kBands] = {}, nL2[kBands] = {};
  float pO[kBands] = {}, nO[kBands] = {}, pO2[kBands] = {}, nO2[kBands] = {};
  const short lengthOfLSP = (short)kl.numOfPixels;
  const short halfWidth = (lengthOfLSP - 1) / 2;
  const float midX = (float)(0.5 * (kl.sPointInOctaveX + kl.ePointInOctaveX));
  const float midY = (float)(0.5 * (kl.sPointInOctaveY + kl.ePointInOctaveY));
  float dL[2], dO[2];
  dL[0] = cosf_cr(kl.angle);
  dL[1] = sinf_cr(kl.angle);
  dO[0] = -dL[1];
  dO[1] = dL[0];
  float sCorX0 = -dL[0] * halfWidth + dL[1] * halfHeight + midX;
  float sCorY0 = -dL[1] * halfWidth - dL[0] * halfHeight + midY;
  for (short hID = 0; hID < heightOfLSP; hID++) {
    float sCorX = sCorX0, sCorY = sCorY0;
    float pLr = 0, nLr = 0, pOr = 0, nOr = 0;
    for (short wID = 0; wID < lengthOfLSP; wID++) {
      short t = (short)std::round(sCorX);
      const short xCor = (t < 0) ? 0 : (t > imageWidth) ? imageWidth : t;
      t = (short)std::round(sCorY);
      const short yCor = (t < 0) ? 0 : (t > imageHeight) ? imageHeight : t;
      const short dx = pdx[yCor * W + xCor], dy = pdy[yCor * W + xCor];
      const float gDL = dx * dL[0] + dy * dL[1];
      const float gDO = dx * dO[0] + dy * dO[1];
      if (gDL > 0) pLr += gDL;
      else nLr -= gDL;
      if (gDO > 0) pOr += gDO;
      else nOr -= gDO;
      sCorX += dL[0];
      sCorY += dL[1];
    }
    sCorX0 -= dL[1];
    sCorY0 += dL[0];
    float c = gG[hID];
    pLr = c * pLr;
    nLr = c * nLr;
    const float pL2r = pLr * pLr, nL2r = nLr * nLr;
    pOr = c * pOr;
    nOr = c * nOr;
    const float pO2r = pOr * pOr, nO2r = nOr * nOr;
    short b = hID / kBandW;
    c = gL[hID % kBandW + kBandW];
    pL[b] += c * pLr; nL[b] += c * nLr;
    pL2[b] += c * c * pL2r; nL2[b] += c * c * nL2r;
    pO[b] += c * pOr; nO[b] += c * nOr;
    pO2[b] += c * c * pO2r; nO2[b] += c * c * nO2r;
    b--;
    if (b >= 0) {
      c = gL[hID % kBandW + 2 * kBandW];
      pL[b] += c * pLr; nL[b] += c * nLr;
      pL2[b] += c * c * pL2r; nL2[b] += c * c * nL2r;
      pO[b] += c * pOr; nO[b] += c * nOr;
      pO2[b] += c * c * pO2r; nO2[b] += c * c * nO2r;
    }
    b = b + 2;
    if (b < kBands) {
      c = gL[hID % kBandW];
      pL[b] += c * pLr; nL[b] += c * nLr;
      pL2[b] += c * c * pL2r; nL2[b] += c * c * nL2r;
      pO[b] += c * pOr; nO[b] += c * nOr;
      pO2[b] += c * c * pO2r; nO2[b] += c * c * nO2r;
    }
  }
  float d[kBands * 8];
  const float invN2 = (float)(1.0 / (kBandW * 2.0)), invN3 = (float)(1.0 / (kBandW * 3.0));
  for (int b = 0; b < kBands; b++) {
    const float invN = (b == 0 || b == kBands - 1) ? invN2 : invN3;
    float t = pL[b] * invN;
    d[b * 8 + 0] = t;
    d[b * 8 + 4] = std::sqrt(pL2[b] * invN - t * t);
    t = nL[b] * invN;
    d[b * 8 + 1] = t;
    d[b * 8 + 5] = std::sqrt(nL2[b] * invN - t * t);
    t = pO[b] * invN;
    d[b * 8 + 2] = t;
    d[b * 8 + 6] = std::sqrt(pO2[b] * invN - t * t);
    t = nO[b] * invN;
    d[b * 8 + 3] = t;
    d[b * 8 + 7] = std::sqrt(nO2[b] * invN - t * t);
  }
  float tempM = 0, tempS = 0;
  for (int b = 0; b < kBands; b++) {
    const float* v = d + 8 * b;
    tempM += v[0] * v[0];
    tempM += v[1] * v[1];
    tempM += v[2] * v[2];
    tempM += v[3] * v[3];
    tempS += v[4] * v[4];
    tempS += v[5] * v[5];
    tempS += v[6] * v[6];
    tempS += v[7] * v[7];
  }
  tempM = 1 / std::sqrt(tempM);
  tempS = 1 / std::sqrt(tempS);
  for (int b = 0; b < kBands; b++) {
    float* v = d + 8 * b;
    for (int q = 0; q < 4; q++) v[q] = v[q] * tempM;
    for (int q = 4; q < 8; q++) v[q] = v[q] * tempS;
  }
  for (int i = 0; i < kBands * 8; i++)
    if ((double)d[i] > 0.4) d[i] = (float)0.4;
  float tempSum = 0;
  for (int i = 0; i < kBands * 8; i++) tempSum += d[i] * d[i];
  tempSum = 1 / std::sqrt(tempSum);
  for (int i = 0; i < kBands * 8; i++) d[i] = d[i] * tempSum;
  for (int c = 0; c < 32; c++) {
    const float* f1 = d + 8 * kComb[c][0];
    const float* f2 = d + 8 * kComb[c][1];
    uint8_t r = 0;
    for (int i = 0; i < 8; i++)
      if (f1[i] > f2[i]) r = (uint8_t)(r + (1u << i));
    out32[c] = r;
  }
}

}  // namespace lsdo

using namespace lsdo;

extern "C" {

int oracle_lsd_detect(const uint8_t* img, int W, int H, float* lines, int cap, int* n_out) {
  LSD lsd;
  std::vector<float> L;
  lsd.detect(img, W, H, L);
  const int n = (int)(L.size() / 4);
  *n_out = n;
  if (n > cap) return -2;
  std::memcpy(lines, L.data(), L.size() * sizeof(float));
  return 0;
}

// The element accesses of one detection (LsdTraffic, in declaration order:
// sort_cmp, sort_moves, seeds, grow_nb, grow_add, grow_expand, grows,
// fit_reads, fit_writes, nfa_evals, nfa_px), then the distinct-address counts
// (sort_n, max_reg, rects, and the distinct scaled-image pixels the seed loop
// reads, whose USED state it writes, whose weight q it reads, and whose angle
// the NFA walks read); bench.py turns them into the LSD kernels' access
// volume and unique-bytes floor. Returns the number of segments.
int oracle_lsd_traffic(const uint8_t* img, int W, int H, long long* out18) {
  LSD lsd;
  LsdTraffic t;
  lsd.tr = &t;
  std::vector<float> L;
  lsd.detect(img, W, H, L);
  long long u[4] = {0, 0, 0, 0};
  for (uint8_t b : t.px)
    for (int k = 0; k < 4; k++) u[k] += (b >> k) & 1;
  const long long v[18] = {t.sort_cmp, t.sort_moves, t.seeds, t.grow_nb, t.grow_add, t.grow_expand,
                           t.grows, t.fit_reads, t.fit_writes, t.nfa_evals, t.nfa_px,
                           t.sort_n, t.max_reg, t.rects, u[0], u[1], u[2], u[3]};
  std::memcpy(out18, v, sizeof(v));
  return (int)(L.size() / 4);
}

// Intermediate LSD stages for stage-wise parity: the 8-bit scaled image
// (sw*sh), the per-pixel angle (NOTDEF = -1024) and the seed order (x | y<<16).
int oracle_lsd_stages(const uint8_t* img, int W, int H, uint8_t* scaled, double* angles,
                      uint32_t* order, int* sw, int* sh, int* n_order) {
  LSD lsd;
  const double prec = kPi * lsd.ANG_TH / 180;
  const double rho = lsd.QUANT / pmath::sin_(prec);
  const double sigma = lsd.SIGMA_SCALE / lsd.SCALE;
  const unsigned h = (unsigned)std::ceil(sigma * std::sqrt(2 * 3.0 * pmath::log_(10.0)));
  const int ksize = 1 + 2 * (int)h;
  std::vector<int> k(ksize);
  fixed_gauss_kernel(ksize, sigma, k.data());
  std::vector<uint8_t> g((size_t)W * H);
  gauss_fixed(img, W, H, k.data(), ksize, g.data());
  lsd.img_width = (int)std::lrint(W * lsd.SCALE);
  lsd.img_height = (int)std::lrint(H * lsd.SCALE);
  lsd.scaled.assign((size_t)lsd.img_width * lsd.img_height, 0);
  resize_exact(g.data(), W, H, lsd.SCALE, lsd.scaled.data(), lsd.img_width, lsd.img_height);
  lsd.ll_angle(rho);
  *sw = lsd.img_width;
  *sh = lsd.img_height;
  if (scaled) std::memcpy(scaled, lsd.scaled.data(), lsd.scaled.size());
  if (angles) std::memcpy(angles, lsd.angles.data(), lsd.angles.size() * sizeof(double));
  if (order)
    for (size_t i = 0; i < lsd.ordered.size(); i++)
      order[i] = (uint32_t)lsd.ordered[i].x | ((uint32_t)lsd.ordered[i].y << 16);
  *n_order = (int)lsd.ordered.size();
  return 0;
}

// LineExtractor::ExtractLineSegment(img, key_lines, desc, coef, scale=1, octaves=1)
int oracle_line_extract(const uint8_t* img, int W, int H, orbpl_keyline* kl_out, uint8_t* desc,
                        double* coef, int cap, int* n_out, int* n_detected) {
  LSD lsd;
  std::vector<float> L;
  lsd.detect(img, W, H, L);
  const int nl = (int)(L.size() / 4);
  if (n_detected) *n_detected = nl;
  std::vector<orbpl_keyline> kls(nl);
  for (int k = 0; k < nl; k++) {
    const float* e = &L[4 * k];
    orbpl_keyline& kl = kls[k];
    kl.startPointX = e[0] * 1.0f;
    kl.startPointY = e[1] * 1.0f;
    kl.endPointX = e[2] * 1.0f;
    kl.endPointY = e[3] * 1.0f;
    kl.sPointInOctaveX = e[0];
    kl.sPointInOctaveY = e[1];
    kl.ePointInOctaveX = e[2];
    kl.ePointInOctaveY = e[3];
    const double ddx = (double)(e[0] - e[2]), ddy = (double)(e[1] - e[3]);
    kl.lineLength = (float)std::sqrt(ddx * ddx + ddy * ddy);
    kl.numOfPixels = line_iterator_count(W, H, e[0], e[1], e[2], e[3]);
    kl.angle = (float)pmath::atan2_((double)(kl.endPointY - kl.startPointY),
                                   (double)(kl.endPointX - kl.startPointX));
    kl.class_id = k;
    kl.octave = 0;
    kl.size = (kl.endPointX - kl.startPointX) * (kl.endPointY - kl.startPointY);
    kl.response = kl.lineLength / (float)std::max(W, H);
    kl.pt_x = (kl.endPointX + kl.startPointX) / 2;
    kl.pt_y = (kl.endPointY + kl.startPointY) / 2;
  }
  const int kMaxLines = 80;  // LineExtractor.cpp:24
  if ((int)kls.size() > kMaxLines) {
    std::sort(kls.begin(), kls.end(),
              [](const orbpl_keyline& a, const orbpl_keyline& b) { return a.response > b.response; });
    kls.resize(kMaxLines);
  }
  const int n = (int)kls.size();
  *n_out = n;
  if (n > cap) return -2;
  if (n == 0) return 0;
  std::vector<int16_t> dx((size_t)W * H), dy((size_t)W * H);
  sobel_images(img, W, H, dx.data(), dy.data());
  float gL[21], gG[63];
  lbd_weights(gL, gG);
  for (int i = 0; i < n; i++) {
    kl_out[i] = kls[i];
    lbd_descriptor(kls[i], dx.data(), dy.data(), W, H, gL, gG, desc + 32 * i);
    // Eigen: s.cross(e).normalized()
    const double s0 = kls[i].startPointX, s1 = kls[i].startPointY, s2 = 1.0;
    const double e0 = kls[i].endPointX, e1 = kls[i].endPointY, e2 = 1.0;
    double c0 = s1 * e2 - s2 * e1, c1 = s2 * e0 - s0 * e2, c2 = s0 * e1 - s1 * e0;
    const double nrm = std::sqrt(c0 * c0 + c1 * c1 + c2 * c2);
    if (nrm > 0) {
      c0 /= nrm;
      c1 /= nrm;
      c2 /= nrm;
    }
    coef[3 * i] = c0;
    coef[3 * i + 1] = c1;
    coef[3 * i + 2] = c2;
  }
  return 0;
}

// pinned math, exported for the accuracy tests
double oracle_lsdm(int fn, double x, double y) {
  switch (fn) {
    case 0: return pmath::exp_(x);
    case 1: return pmath::log_(x);
    case 2: return pmath::log10_(x);
    case 3: return pmath::sin_(x);
    case 4: return pmath::cos_(x);
    case 5: return pmath::atan2_(y, x);
    case 6: return pmath::sinh_(x);
    case 7: return pmath::powi(x, y);
    default: return 0;
  }
}

// divergence probe (pinned_math.h): on != 0 starts counting (and resets the
// counters), on == 0 stops; oracle_math_probe_read fills per function (exp,
// log, log10, sin, cos, atan2, cosf, sinf) calls, results differing from
// glibc, and the largest difference in ulps.
int oracle_math_probe(int on) {
  pmath::Probe& p = pmath::probe();
  if (on)
    for (int i = 0; i < pmath::kNumFn; i++) p.calls[i] = p.differ[i] = p.max_ulp[i] = 0;
  p.on = on ? 1 : 0;
  return 0;
}

int oracle_math_probe_read(long long* calls, long long* differ, long long* max_ulp) {
  pmath::Probe& p = pmath::probe();
  for (int i = 0; i < pmath::kNumFn; i++) {
    calls[i] = p.calls[i];
    differ[i] = p.differ[i];
    max_ulp[i] = p.max_ulp[i];
  }
  return pmath::kNumFn;
}

int oracle_line_iterator_count(int W, int H, float x1, float y1, float x2, float y2) {
  return line_iterator_count(W, H, x1, y1, x2, y2);
}

}  // extern "C"

extern "C" {
// std::sort (libstdc++ introsort) of (key, index) records by key descending,
// the comparator of LSD's ordered_points; returns the index permutation.
int oracle_introsort_perm(const int* keys, int n, int* perm) {
  std::vector<lsdo::NormPoint> v(n);
  for (int i = 0; i < n; i++) v[i] = {i, 0, keys[i]};
  std::sort(v.begin(), v.end(),
            [](const lsdo::NormPoint& a, const lsdo::NormPoint& b) { return a.norm > b.norm; });
  for (int i = 0; i < n; i++) perm[i] = v[i].x;
  return 0;
}
}  // extern "C"
