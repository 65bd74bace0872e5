// LSD greedy seed loop on gfx950 (OpenCV 3.4 LineSegmentDetectorImpl::flsd
// after ll_angle; restated in oracle/lsd_oracle.cpp LSD::detect).
//
// The seed loop is inherently sequential (each region marks pixels USED for
// every later seed), so one wave runs one frame and all 64 lanes execute the
// same serial control flow on the same (uniform) values; a batch of frames
// fills the GPU with independent waves. Lanes work in parallel where the
// reference's result does not depend on order:
//   * seed screening: 64 pseudo-ordered pixels are tested per step, the next
//     seed is the lowest lane whose pixel is defined and still NOTUSED,
//     re-evaluated after every region (refinement can release pixels);
//   * rect_nfa: the rectangle's pixels are counted by all lanes (integer
//     counts), the walk's row ranges are computed serially first.
// Per-frame state in LDS: the USED map as bits and the region list (first
// kRegLds points; longer regions continue in global scratch).
#include <hip/hip_runtime.h>

#include "lsd_kernels.h"
#include "lsd_math.h"
#include "orbpl_math.h"

namespace orbpl {

namespace {

constexpr double kPi = 3.14159265358979323846;
constexpr double kDegToRad = kPi / 180;
constexpr int kRegLds = 4096;

struct Rect {
  double x1, y1, x2, y2, width, x, y, theta, dx, dy, prec, p;
};

struct Frame {
  int sw, sh;
  const float* deg;
  const int* q;
  uint32_t* used;     // LDS bits
  uint32_t* reg_l;    // LDS region list
  uint32_t* reg_g;    // global continuation
  int4* rows;         // LDS rect_nfa rows
  int row_cap;
  double log_nt;
  int lane;
};

__device__ __forceinline__ bool used_get(const Frame& F, int x, int y) {
  const int i = y * F.sw + x;
  return (F.used[i >> 5] >> (i & 31)) & 1u;
}
__device__ __forceinline__ void used_set(Frame& F, int x, int y, bool v) {
  const int i = y * F.sw + x;
  // every lane performs the same update (wave-uniform serial execution)
  if (F.lane == 0) {
    if (v) atomicOr(&F.used[i >> 5], 1u << (i & 31));
    else atomicAnd(&F.used[i >> 5], ~(1u << (i & 31)));
  }
  __builtin_amdgcn_wave_barrier();
}
__device__ __forceinline__ uint32_t reg_get(const Frame& F, int i) {
  return i < kRegLds ? F.reg_l[i] : F.reg_g[i - kRegLds];
}
__device__ __forceinline__ void reg_set(Frame& F, int i, uint32_t v) {
  if (i < kRegLds) F.reg_l[i] = v;
  else F.reg_g[i - kRegLds] = v;
  __builtin_amdgcn_wave_barrier();
}
__device__ __forceinline__ double deg2ang(float d) { return (double)d * kDegToRad; }
__device__ __forceinline__ double modgrad(const Frame& F, int x, int y) {
  return sqrt(F.q[y * F.sw + x] / 4.0);
}

__device__ __forceinline__ bool aligned_deg(float d, double theta, double prec) {
  if (d < 0.f) return false;  // NOTDEF
  double n_theta = theta - deg2ang(d);
  if (n_theta < 0) n_theta = -n_theta;
  if (n_theta > (3 * kPi) / 2) {
    n_theta -= (2 * kPi);
    if (n_theta < 0) n_theta = -n_theta;
  }
  return n_theta <= prec;
}

__device__ __forceinline__ double angle_diff_signed(double a, double b) {
  double diff = a - b;
  while (diff <= -kPi) diff += 2 * kPi;
  while (diff > kPi) diff -= 2 * kPi;
  return diff;
}

__device__ __forceinline__ double dist(double x1, double y1, double x2, double y2) {
  return sqrt((x2 - x1) * (x2 - x1) + (y2 - y1) * (y2 - y1));
}
__device__ __forceinline__ double distSq(double x1, double y1, double x2, double y2) {
  return (x2 - x1) * (x2 - x1) + (y2 - y1) * (y2 - y1);
}

__device__ bool double_equal(double a, double b) {
  if (a == b) return true;
  const double abs_diff = fabs(a - b);
  const double aa = fabs(a), bb = fabs(b);
  double abs_max = aa > bb ? aa : bb;
  if (abs_max < 2.2250738585072014e-308) abs_max = 2.2250738585072014e-308;
  return (abs_diff / abs_max) <= (100.0 * 2.220446049250313080847e-16);
}

__device__ double log_gamma(double x) {
  if (x > 15.0)
    return 0.918938533204673 + (x - 0.5) * lsdm::log_(x) - x +
           0.5 * x * lsdm::log_(x * lsdm::sinh_(1 / x) + 1 / (810.0 * lsdm::powi_(x, 6.0)));
  const double q[7] = {75122.6331530, 80916.6278952, 36308.2951477, 8687.24529705,
                       1168.92649479, 83.8676043424, 2.50662827511};
  double a = (x + 0.5) * lsdm::log_(x + 5.5) - (x + 5.5);
  double b = 0;
  for (int n = 0; n < 7; ++n) {
    a -= lsdm::log_(x + double(n));
    b += q[n] * lsdm::powi_(x, double(n));
  }
  return a + lsdm::log_(b);
}

__device__ double nfa(int n, int k, double p, double log_nt) {
  if (n == 0 || k == 0) return -log_nt;
  if (n == k) return -log_nt - double(n) * lsdm::log10_(p);
  const double p_term = p / (1 - p);
  const double log1term = log_gamma(double(n) + 1) - log_gamma(double(k) + 1) -
                          log_gamma(double(n - k) + 1) + double(k) * lsdm::log_(p) +
                          double(n - k) * lsdm::log_(1.0 - p);
  double term = lsdm::exp_(log1term);
  if (double_equal(term, 0)) {
    if (k > n * p) return -log1term / 2.30258509299404568402 - log_nt;
    return -log_nt;
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
          term * ((1 - lsdm::powi_(mult_term, double(n - i + 1))) / (1 - mult_term) - 1);
      if (err < tolerance * fabs(-lsdm::log10_(bin_tail) - log_nt) * bin_tail) break;
    }
  }
  return -lsdm::log10_(bin_tail) - log_nt;
}

// region_grow (lsd.cpp): returns the region size; the region list holds the
// points in insertion order.
__device__ int region_grow(Frame& F, int sx, int sy, double& reg_angle, double prec) {
  const int sw = F.sw, sh = F.sh;
  int n = 0;
  reg_set(F, n++, (uint32_t)sx | ((uint32_t)sy << 16));
  reg_angle = deg2ang(F.deg[sy * sw + sx]);
  float sumdx = (float)lsdm::cos_(reg_angle);
  float sumdy = (float)lsdm::sin_(reg_angle);
  used_set(F, sx, sy, true);
  for (int i = 0; i < n; i++) {
    const uint32_t pt = reg_get(F, i);
    const int x = (int)(pt & 0xFFFF), y = (int)(pt >> 16);
    // the nine degree values are static: load them together
    float dv[9];
#pragma unroll
    for (int k = 0; k < 9; k++) {
      const int xx = x + (k % 3) - 1, yy = y + (k / 3) - 1;
      dv[k] = (xx >= 0 && xx < sw && yy >= 0 && yy < sh) ? F.deg[yy * sw + xx] : kLsdNotdef;
    }
#pragma unroll
    for (int k = 0; k < 9; k++) {
      const int xx = x + (k % 3) - 1, yy = y + (k / 3) - 1;
      if (xx < 0 || xx >= sw || yy < 0 || yy >= sh) continue;
      if (!used_get(F, xx, yy) && aligned_deg(dv[k], reg_angle, prec)) {
        used_set(F, xx, yy, true);
        reg_set(F, n++, (uint32_t)xx | ((uint32_t)yy << 16));
        float c, s;
        cr_cos_sin((float)deg2ang(dv[k]), &c, &s);
        sumdx += c;
        sumdy += s;
        reg_angle = (double)fast_atan2_deg(sumdy, sumdx) * kDegToRad;
      }
    }
  }
  return n;
}

__device__ void region2rect(Frame& F, int n, double reg_angle, double prec, double p, Rect& rec) {
  double x = 0, y = 0, sum = 0;
  for (int i = 0; i < n; ++i) {
    const uint32_t pt = reg_get(F, i);
    const int px = (int)(pt & 0xFFFF), py = (int)(pt >> 16);
    const double weight = modgrad(F, px, py);
    x += double(px) * weight;
    y += double(py) * weight;
    sum += weight;
  }
  x /= sum;
  y /= sum;
  // get_theta
  double Ixx = 0.0, Iyy = 0.0, Ixy = 0.0;
  for (int i = 0; i < n; ++i) {
    const uint32_t pt = reg_get(F, i);
    const int px = (int)(pt & 0xFFFF), py = (int)(pt >> 16);
    const double weight = modgrad(F, px, py);
    const double dx = double(px) - x, dy = double(py) - y;
    Ixx += dy * dy * weight;
    Iyy += dx * dx * weight;
    Ixy -= dx * dy * weight;
  }
  const double lambda = 0.5 * (Ixx + Iyy - sqrt((Ixx - Iyy) * (Ixx - Iyy) + 4.0 * Ixy * Ixy));
  double theta = (fabs(Ixx) > fabs(Iyy)) ? double(fast_atan2_deg(float(lambda - Ixx), float(Ixy)))
                                         : double(fast_atan2_deg(float(Ixy), float(lambda - Iyy)));
  theta *= kDegToRad;
  if (fabs(angle_diff_signed(theta, reg_angle)) > prec) theta += kPi;
  const double dx = lsdm::cos_(theta), dy = lsdm::sin_(theta);
  double l_min = 0, l_max = 0, w_min = 0, w_max = 0;
  for (int i = 0; i < n; ++i) {
    const uint32_t pt = reg_get(F, i);
    const double regdx = double((int)(pt & 0xFFFF)) - x, regdy = double((int)(pt >> 16)) - y;
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

__device__ bool reduce_region_radius(Frame& F, int& n, double reg_angle, double prec, double p,
                                     Rect& rec, double density, double density_th) {
  const uint32_t p0 = reg_get(F, 0);
  const double xc = double((int)(p0 & 0xFFFF)), yc = double((int)(p0 >> 16));
  const double radSq1 = distSq(xc, yc, rec.x1, rec.y1);
  const double radSq2 = distSq(xc, yc, rec.x2, rec.y2);
  double radSq = radSq1 > radSq2 ? radSq1 : radSq2;
  while (density < density_th) {
    radSq *= 0.75 * 0.75;
    for (int i = 0; i < n; ++i) {
      const uint32_t pt = reg_get(F, i);
      const int px = (int)(pt & 0xFFFF), py = (int)(pt >> 16);
      if (distSq(xc, yc, double(px), double(py)) > radSq) {
        used_set(F, px, py, false);
        const uint32_t last = reg_get(F, n - 1);
        reg_set(F, i, last);
        reg_set(F, n - 1, pt);
        n--;
        --i;
      }
    }
    if (n < 2) return false;
    region2rect(F, n, reg_angle, prec, p, rec);
    density = double(n) / (dist(rec.x1, rec.y1, rec.x2, rec.y2) * rec.width);
  }
  return true;
}

__device__ bool refine(Frame& F, int& n, double reg_angle, double prec, double p, Rect& rec,
                       double density_th) {
  double density = double(n) / (dist(rec.x1, rec.y1, rec.x2, rec.y2) * rec.width);
  if (density >= density_th) return true;
  const uint32_t p0 = reg_get(F, 0);
  const int x0 = (int)(p0 & 0xFFFF), y0 = (int)(p0 >> 16);
  const double xc = double(x0), yc = double(y0);
  const double ang_c = deg2ang(F.deg[y0 * F.sw + x0]);
  double sum = 0, s_sum = 0;
  int cnt = 0;
  for (int i = 0; i < n; ++i) {
    const uint32_t pt = reg_get(F, i);
    const int px = (int)(pt & 0xFFFF), py = (int)(pt >> 16);
    used_set(F, px, py, false);
    if (dist(xc, yc, px, py) < rec.width) {
      const double ang_d = angle_diff_signed(deg2ang(F.deg[py * F.sw + px]), ang_c);
      sum += ang_d;
      s_sum += ang_d * ang_d;
      ++cnt;
    }
  }
  const double mean_angle = sum / double(cnt);
  const double tau =
      2.0 * sqrt((s_sum - 2.0 * mean_angle * sum) / double(cnt) + mean_angle * mean_angle);
  n = region_grow(F, x0, y0, reg_angle, tau);
  if (n < 2) return false;
  region2rect(F, n, reg_angle, prec, p, rec);
  density = double(n) / (dist(rec.x1, rec.y1, rec.x2, rec.y2) * rec.width);
  if (density < density_th) return reduce_region_radius(F, n, reg_angle, prec, p, rec, density, density_th);
  return true;
}

struct Edge {
  int x, y;
  bool taken;
};

__device__ double rect_nfa(Frame& F, const Rect& rec) {
  const double half_width = rec.width / 2.0;
  const double dyhw = rec.dy * half_width;
  const double dxhw = rec.dx * half_width;
  Edge e[4];
  e[0] = {int(rec.x1 - dyhw), int(rec.y1 + dxhw), false};
  e[1] = {int(rec.x2 - dyhw), int(rec.y2 + dxhw), false};
  e[2] = {int(rec.x2 + dyhw), int(rec.y2 - dxhw), false};
  e[3] = {int(rec.x1 + dyhw), int(rec.y1 - dxhw), false};
  // std::sort of 4 elements = insertion sort (AsmallerB_XorYisSmaller)
  for (int i = 1; i < 4; i++) {
    const Edge v = e[i];
    int j = i;
    while (j > 0 && ((v.x < e[j - 1].x) || (v.x == e[j - 1].x && v.y < e[j - 1].y))) {
      e[j] = e[j - 1];
      j--;
    }
    e[j] = v;
  }
  int imin = 0, imax = 0;
  for (int i = 1; i < 4; ++i) {
    if (e[imin].y > e[i].y) imin = i;
    if (e[imax].y < e[i].y) imax = i;
  }
  e[imin].taken = true;
  int il = -1;
  for (int i = 0; i < 4; ++i)
    if (!e[i].taken) {
      if (il < 0) il = i;
      else if (e[il].x > e[i].x) il = i;
    }
  e[il].taken = true;
  int ir = -1;
  for (int i = 0; i < 4; ++i)
    if (!e[i].taken) {
      if (ir < 0) ir = i;
      else if (e[ir].x < e[i].x) ir = i;
    }
  e[ir].taken = true;
  int it = -1;
  for (int i = 0; i < 4; ++i)
    if (!e[i].taken) {
      if (it < 0) it = i;
      else if (e[it].x > e[i].x) it = i;
    }
  e[it].taken = true;
  const Edge mn = e[imin], mx = e[imax], lf = e[il], rt = e[ir], tl = e[it];
  // double-valued steps, tail corner's y (pinned P13, oracle rect_nfa)
  const double flstep = (mn.y != lf.y) ? (mn.x - lf.x) / double(mn.y - lf.y) : 0;
  const double slstep = (lf.y != tl.y) ? (lf.x - tl.x) / double(lf.y - tl.y) : 0;
  const double frstep = (mn.y != rt.y) ? (mn.x - rt.x) / double(mn.y - rt.y) : 0;
  const double srstep = (rt.y != tl.y) ? (rt.x - tl.x) / double(rt.y - tl.y) : 0;
  double lstep = flstep, rstep = frstep;
  double left_x = mn.x, right_x = mn.x;
  // serial walk: row ranges into LDS (prefix offsets in .w)
  int nrows = 0, total = 0;
  for (int y = mn.y; y <= mx.y; ++y) {
    // rows outside the image skip the step updates too (the reference's
    // `continue` precedes them)
    if (y < 0 || y >= F.sh) continue;
    const int xa = max((int)left_x, 0), xb = min((int)right_x, F.sw - 1);
    if (xb >= xa && nrows < F.row_cap) {
      if (F.lane == 0) F.rows[nrows] = make_int4(y, xa, xb, total);
      total += xb - xa + 1;
      nrows++;
    }
    if (y >= lf.y) lstep = slstep;
    if (y >= rt.y) rstep = srstep;
    left_x += lstep;
    right_x += rstep;
  }
  __builtin_amdgcn_wave_barrier();
  // parallel count of aligned pixels
  int alg = 0, r = 0;
  for (int k = F.lane; k < total; k += 64) {
    while (r + 1 < nrows && F.rows[r + 1].w <= k) r++;
    const int4 rw = F.rows[r];
    const int x = rw.y + (k - rw.w);
    alg += aligned_deg(F.deg[rw.x * F.sw + x], rec.theta, rec.prec) ? 1 : 0;
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) alg += __shfl_xor(alg, o, 64);
  __builtin_amdgcn_wave_barrier();
  return nfa(total, alg, rec.p, F.log_nt);
}

__device__ double rect_improve(Frame& F, Rect& rec) {
  const double delta = 0.5, delta_2 = delta / 2.0;
  double log_nfa = rect_nfa(F, rec);
  if (log_nfa > 0) return log_nfa;
  Rect r = rec;
  for (int n = 0; n < 5; ++n) {
    r.p /= 2;
    r.prec = r.p * kPi;
    const double v = rect_nfa(F, r);
    if (v > log_nfa) {
      log_nfa = v;
      rec = r;
    }
  }
  if (log_nfa > 0) return log_nfa;
  r = rec;
  for (int n = 0; n < 5; ++n) {
    if ((r.width - delta) >= 0.5) {
      r.width -= delta;
      const double v = rect_nfa(F, r);
      if (v > log_nfa) {
        rec = r;
        log_nfa = v;
      }
    }
  }
  if (log_nfa > 0) return log_nfa;
  r = rec;
  for (int n = 0; n < 5; ++n) {
    if ((r.width - delta) >= 0.5) {
      r.x1 += -r.dy * delta_2;
      r.y1 += r.dx * delta_2;
      r.x2 += -r.dy * delta_2;
      r.y2 += r.dx * delta_2;
      r.width -= delta;
      const double v = rect_nfa(F, r);
      if (v > log_nfa) {
        rec = r;
        log_nfa = v;
      }
    }
  }
  if (log_nfa > 0) return log_nfa;
  r = rec;
  for (int n = 0; n < 5; ++n) {
    if ((r.width - delta) >= 0.5) {
      r.x1 -= -r.dy * delta_2;
      r.y1 -= r.dx * delta_2;
      r.x2 -= -r.dy * delta_2;
      r.y2 -= r.dx * delta_2;
      r.width -= delta;
      const double v = rect_nfa(F, r);
      if (v > log_nfa) {
        rec = r;
        log_nfa = v;
      }
    }
  }
  if (log_nfa > 0) return log_nfa;
  r = rec;
  for (int n = 0; n < 5; ++n) {
    if ((r.width - delta) >= 0.5) {
      r.p /= 2;
      r.prec = r.p * kPi;
      const double v = rect_nfa(F, r);
      if (v > log_nfa) {
        rec = r;
        log_nfa = v;
      }
    }
  }
  return log_nfa;
}

}  // namespace

__global__ void __launch_bounds__(64) k_lsd_grow(LsdGeom g, LsdScratch sc) {
  extern __shared__ uint32_t grow_smem[];
  const int f = blockIdx.x, lane = threadIdx.x;
  const int sw = g.sw, sh = g.sh;
  const int used_words = (sw * sh + 31) / 32;
  Frame F;
  F.sw = sw;
  F.sh = sh;
  F.deg = sc.deg + (long long)f * sw * sh;
  F.q = sc.q + (long long)f * sw * sh;
  F.used = grow_smem;
  F.reg_l = grow_smem + used_words;
  F.reg_g = sc.reg + (long long)f * sw * sh;
  F.rows = reinterpret_cast<int4*>(grow_smem + ((used_words + kRegLds + 3) & ~3));
  F.row_cap = sh + 2;
  F.log_nt = g.log_nt;
  F.lane = lane;
  for (int i = lane; i < used_words; i += 64) F.used[i] = 0;
  __builtin_amdgcn_wave_barrier();
  const uint32_t* A = sc.A + (long long)f * g.n;
  float* out = sc.lines + (long long)f * kLsdMaxLines * 4;
  const int w1 = sw - 1;
  const double prec = g.prec, p = g.p;
  int nl = 0;
  for (int base = 0; base < g.n; base += 64) {
    const int i = base + lane;
    int px = 0, py = 0;
    bool def = false;
    if (i < g.n) {
      const int idx = (int)(A[i] & 0x3FFFFFu);
      py = idx / w1;
      px = idx - py * w1;
      def = F.deg[py * sw + px] >= 0.f;
    }
    unsigned long long mask = __ballot(def && !used_get(F, px, py));
    while (mask) {
      const int l = __ffsll((long long)mask) - 1;
      const int sx = __shfl(px, l, 64), sy = __shfl(py, l, 64);
      double reg_angle;
      int n = region_grow(F, sx, sy, reg_angle, prec);
      if (n >= g.min_reg_size) {
        Rect rec;
        region2rect(F, n, reg_angle, prec, p, rec);
        if (refine(F, n, reg_angle, prec, p, rec, 0.7)) {
          const double log_nfa = rect_improve(F, rec);
          if (log_nfa > 0) {
            if (nl < kLsdMaxLines) {
              if (lane == 0) {
                out[nl * 4 + 0] = float((rec.x1 + 0.5) / 0.8);
                out[nl * 4 + 1] = float((rec.y1 + 0.5) / 0.8);
                out[nl * 4 + 2] = float((rec.x2 + 0.5) / 0.8);
                out[nl * 4 + 3] = float((rec.y2 + 0.5) / 0.8);
              }
            } else if (lane == 0) {
              atomicOr(sc.err + f, 8);
            }
            nl++;
          }
        }
      }
      mask = __ballot(def && lane > l && !used_get(F, px, py));
    }
  }
  if (lane == 0) sc.nlines[f] = min(nl, kLsdMaxLines);
}

size_t lsd_grow_smem(const LsdGeom& g) {
  const int used_words = (g.sw * g.sh + 31) / 32;
  return 4 * (size_t)(((used_words + kRegLds + 3) & ~3) + 4 * (g.sh + 2));
}

void launch_lsd_grow(const LsdGeom& g, const LsdScratch& sc, int batch, hipStream_t s) {
  const size_t smem = lsd_grow_smem(g);
  if (smem > 65536)
    (void)hipFuncSetAttribute((const void*)k_lsd_grow, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)smem);
  hipLaunchKernelGGL(k_lsd_grow, dim3(batch), dim3(64), smem, s, g, sc);
}

}  // namespace orbpl
