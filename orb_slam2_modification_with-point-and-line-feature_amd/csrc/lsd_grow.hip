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

#include <cstdlib>

#include "lsd_kernels.h"
#include "lsd_math.h"
#include "orbpl_math.h"

namespace orbpl {

// Scope of the seed loop's stamp loads / stores. One wave owns a frame's
// stamps, and the CU's vector L1 is coherent for its own waves' stores and
// atomics (the memory model's workgroup scope needs no L1 invalidation outside
// tgsplit mode), so workgroup-scope loads may hit L1 where agent-scope ones
// (sc1) went to L2 for every neighbourhood: 153.8 -> 140.7 ms per 3072 frames,
// bit-exact (test_gpu_lsd). A/B builds override.
#ifndef ORBPL_LSD_SCOPE
#define ORBPL_LSD_SCOPE __HIP_MEMORY_SCOPE_WORKGROUP
#endif

namespace {

constexpr double kPi = 3.14159265358979323846;
constexpr double kDegToRad = kPi / 180;
constexpr int kRegLds = 512;

struct Rect {
  double x1, y1, x2, y2, width, x, y, theta, dx, dy, prec, p;
};

struct Frame {
  int sw, sh;
  const float* deg;   // lsd_deg_index tiles
  int dtw;
  const int* q;
  uint32_t* used;     // LDS bits (k_lsd_grow)
  uint64_t* usd;      // k_lsd_spec: USED lives in the claim stamps (high words, 0 = USED)
  const uint64_t* cs; // k_lsd_spec: the angle-term plane (cos | sin << 32, lsd_sd_frame_words)
  int tw;             // tiles per row of usd
  uint32_t* reg_l;    // LDS region points (x | y << 16)
  int* regq_l;        // LDS q (gx^2 + gy^2) of each region point
  float* regd_l;      // LDS degrees of each region point
  uint32_t* reg_g;    // global continuation: (pt, q, deg) triples
  float* ring;        // LDS 64 x 9 prefetched 3x3 degree neighbourhoods
  int4* rows;         // LDS rect_nfa rows
  Rect* rect0;        // LDS: the current rectangle (rec)
  Rect* rect1;        // LDS: rect_improve's trial rectangle (r)
  int row_cap;
  double log_nt;
  int lane;
  long long pf_cyc, pf_cnt, seed_cyc;
};

// USED state. k_lsd_grow keeps a bitmap in LDS. k_lsd_spec keeps it in the
// per-pixel claim stamp (global, read at L2 like the claims): 0 = USED
// (below every claim tag), anything else = not USED. Freeing LDS of the
// 24 KB bitmap lets twice as many frames share a CU.
__device__ __forceinline__ uint32_t* sd_hi(uint64_t* sd, int idx) {
  return reinterpret_cast<uint32_t*>(sd + idx) + 1;
}
__device__ __forceinline__ bool used_get(const Frame& F, int x, int y) {
  if (F.usd)
    return __hip_atomic_load(sd_hi(F.usd, lsd_sd_index(x, y, F.tw)), __ATOMIC_RELAXED,
                             ORBPL_LSD_SCOPE) == 0u;
  const int i = y * F.sw + x;
  return (F.used[i >> 5] >> (i & 31)) & 1u;
}
__device__ __forceinline__ void used_set(Frame& F, int x, int y, bool v) {
  const int i = y * F.sw + x;
  // the lanes run the same serial program; one of them updates the word
  // (single writer: a plain read-modify-write)
  if (F.usd) {
    if (F.lane == 0)
      __hip_atomic_store(sd_hi(F.usd, lsd_sd_index(x, y, F.tw)), v ? 0u : 0xFFFFFFFFu,
                         __ATOMIC_RELAXED, ORBPL_LSD_SCOPE);
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  } else if (F.lane == 0) {
    const uint32_t w = F.used[i >> 5], b = 1u << (i & 31);
    F.used[i >> 5] = v ? (w | b) : (w & ~b);
  }
  __builtin_amdgcn_wave_barrier();
}
__device__ __forceinline__ uint32_t reg_get(const Frame& F, int i) {
  return i < kRegLds ? F.reg_l[i] : F.reg_g[3 * (i - kRegLds)];
}
__device__ __forceinline__ int regq_get(const Frame& F, int i) {
  return i < kRegLds ? F.regq_l[i] : (int)F.reg_g[3 * (i - kRegLds) + 1];
}
__device__ __forceinline__ float regd_get(const Frame& F, int i) {
  return i < kRegLds ? F.regd_l[i] : __uint_as_float(F.reg_g[3 * (i - kRegLds) + 2]);
}
// point + degree (q is filled in bulk by fill_q when the region is fitted)
__device__ __forceinline__ void reg_put(Frame& F, int i, uint32_t pt, float d) {
  if (F.lane == 0) {
    if (i < kRegLds) {
      F.reg_l[i] = pt;
      F.regd_l[i] = d;
    } else {
      F.reg_g[3 * (i - kRegLds)] = pt;
      F.reg_g[3 * (i - kRegLds) + 2] = __float_as_uint(d);
    }
  }
  __builtin_amdgcn_wave_barrier();
}
__device__ __forceinline__ void reg_swap(Frame& F, int i, int j) {
  const uint32_t pi = reg_get(F, i), pj = reg_get(F, j);
  const int qi = regq_get(F, i), qj = regq_get(F, j);
  const float di = regd_get(F, i), dj = regd_get(F, j);
  __builtin_amdgcn_wave_barrier();
  if (F.lane == 0) {
    if (i < kRegLds) { F.reg_l[i] = pj; F.regq_l[i] = qj; F.regd_l[i] = dj; }
    else { F.reg_g[3 * (i - kRegLds)] = pj; F.reg_g[3 * (i - kRegLds) + 1] = (uint32_t)qj; F.reg_g[3 * (i - kRegLds) + 2] = __float_as_uint(dj); }
    if (j < kRegLds) { F.reg_l[j] = pi; F.regq_l[j] = qi; F.regd_l[j] = di; }
    else { F.reg_g[3 * (j - kRegLds)] = pi; F.reg_g[3 * (j - kRegLds) + 1] = (uint32_t)qi; F.reg_g[3 * (j - kRegLds) + 2] = __float_as_uint(di); }
  }
  __threadfence_block();
  __builtin_amdgcn_wave_barrier();
}
// q of region points [0, n): all lanes load in parallel
__device__ __forceinline__ void fill_q(Frame& F, int n) {
  for (int j = F.lane; j < n; j += 64) {
    const uint32_t pt = reg_get(F, j);
    const int v = F.q[(int)(pt >> 16) * F.sw + (int)(pt & 0xFFFF)];
    if (j < kRegLds) F.regq_l[j] = v;
    else F.reg_g[3 * (j - kRegLds) + 1] = (uint32_t)v;
  }
  __threadfence_block();
  __builtin_amdgcn_wave_barrier();
}
__device__ __forceinline__ double deg2ang(float d) { return (double)d * kDegToRad; }
__device__ __forceinline__ double modgrad_q(int q) { return sqrt(q / 4.0); }

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
#pragma unroll
  for (int n = 0; n < 7; ++n) {
    a -= lsdm::log_(x + double(n));
    b += q[n] * lsdm::powi_(x, double(n));
  }
  return a + lsdm::log_(b);
}

__device__ __forceinline__ double shfl_d(double v, int src) {
  const long long b = __double_as_longlong(v);
  const int lo = __shfl((int)(b & 0xFFFFFFFF), src, 64), hi = __shfl((int)(b >> 32), src, 64);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

// nfa (lsd.cpp). Wave-parallel, same values as the serial reference: the
// three log_gamma terms are evaluated on lanes 0-2, and the tail loop's
// term / bin_tail recurrence is replayed serially while the (expensive)
// stopping test of 64 consecutive iterations is evaluated one per lane.
__device__ double nfa(int n, int k, double p, double log_nt, int lane) {
  if (n == 0 || k == 0) return -log_nt;
  if (n == k) return -log_nt - double(n) * lsdm::log10_(p);
  const double p_term = p / (1 - p);
  const double garg = lane == 0 ? double(n) + 1 : (lane == 1 ? double(k) + 1 : double(n - k) + 1);
  const double lg = log_gamma(garg);
  const double lg0 = shfl_d(lg, 0), lg1 = shfl_d(lg, 1), lg2 = shfl_d(lg, 2);
  const double log1term = lg0 - lg1 - lg2 + double(k) * lsdm::log_(p) +
                          double(n - k) * lsdm::log_(1.0 - p);
  double term = lsdm::exp_(log1term);
  if (double_equal(term, 0)) {
    if (k > n * p) return -log1term / 2.30258509299404568402 - log_nt;
    return -log_nt;
  }
  double bin_tail = term;
  const double tolerance = 0.1;
  for (int i0 = k + 1; i0 <= n; i0 += 64) {
    // serial recurrence; lane l keeps iteration i0 + l
    double my_term = 0, my_tail = 0, my_bin = 2, my_mult = 0;
    const int cnt = min(64, n - i0 + 1);
    for (int l = 0; l < cnt; l++) {
      const int i = i0 + l;
      const double bin_term = double(n - i + 1) / double(i);
      const double mult_term = bin_term * p_term;
      term *= mult_term;
      bin_tail += term;
      if (lane == l) {
        my_term = term;
        my_tail = bin_tail;
        my_bin = bin_term;
        my_mult = mult_term;
      }
    }
    bool stop = false;
    double my_res = 0;
    if (lane < cnt && my_bin < 1) {
      const int i = i0 + lane;
      const double err =
          my_term * ((1 - lsdm::powi_(my_mult, double(n - i + 1))) / (1 - my_mult) - 1);
      const double lt = lsdm::log10_(my_tail);
      stop = err < tolerance * fabs(-lt - log_nt) * my_tail;
      my_res = -lt - log_nt;
    }
    const unsigned long long m = __ballot(stop);
    if (m) return shfl_d(my_res, __ffsll((long long)m) - 1);
  }
  return -lsdm::log10_(bin_tail) - log_nt;
}

// Prefetch the 3x3 degree neighbourhoods of region points [i0, i1) (at most
// 64) into the ring, one point per lane.
__device__ __forceinline__ void prefetch_ring(Frame& F, int i0, int i1) {
  const int j = i0 + F.lane;
  if (j < i1) {
    const uint32_t pt = reg_get(F, j);
    const int x = (int)(pt & 0xFFFF), y = (int)(pt >> 16);
    float v[9];
#pragma unroll
    for (int k = 0; k < 9; k++) {
      const int xx = x + (k % 3) - 1, yy = y + (k / 3) - 1;
      v[k] = (xx >= 0 && xx < F.sw && yy >= 0 && yy < F.sh) ? F.deg[lsd_deg_index(xx, yy, F.dtw)] : kLsdNotdef;
    }
    float* r = F.ring + (j & 63) * 9;
#pragma unroll
    for (int k = 0; k < 9; k++) r[k] = v[k];
  }
  __threadfence_block();
  __builtin_amdgcn_wave_barrier();
}

// region_grow (lsd.cpp): returns the region size; the region list holds the
// points in insertion order. Degree neighbourhoods of pending points are
// fetched 64 at a time (they are static), the USED tests stay in order.
__device__ __forceinline__ int region_grow(Frame& F, int sx, int sy, double& reg_angle, double prec) {
  const int sw = F.sw, sh = F.sh;
  int n = 1;
  const uint32_t p0 = (uint32_t)sx | ((uint32_t)sy << 16);
  if (F.lane == 0) F.reg_l[0] = p0;
  __builtin_amdgcn_wave_barrier();
  const long long tq0 = clock64();
  prefetch_ring(F, 0, 1);
  F.pf_cyc += clock64() - tq0;
  F.pf_cnt++;
  int pf_end = 1;
  const float d0 = F.ring[4];
  reg_put(F, 0, p0, d0);
  reg_angle = deg2ang(d0);
  double s0, c0;
  lsdm::sincos_(reg_angle, &s0, &c0);
  float sumdx = (float)c0;
  float sumdy = (float)s0;
  used_set(F, sx, sy, true);
  for (int i = 0; i < n; i++) {
    if (i == pf_end) {
      pf_end = min(n, i + 64);
      const long long tq = clock64();
      prefetch_ring(F, i, pf_end);
      F.pf_cyc += clock64() - tq;
      F.pf_cnt++;
    }
    const uint32_t pt = reg_get(F, i);
    const int x = (int)(pt & 0xFFFF), y = (int)(pt >> 16);
    const float* dv = F.ring + (i & 63) * 9;
    // USED bits of the 3x3 block, read once: marking a pixel below changes
    // only that pixel's own bit, which is not visited again in this block
    unsigned ub = 0;
#pragma unroll
    for (int k = 0; k < 9; k++) {
      const int xx = x + (k % 3) - 1, yy = y + (k / 3) - 1;
      if (xx >= 0 && xx < sw && yy >= 0 && yy < sh && used_get(F, xx, yy)) ub |= 1u << k;
    }
#pragma unroll
    for (int k = 0; k < 9; k++) {
      const int xx = x + (k % 3) - 1, yy = y + (k / 3) - 1;
      if (xx < 0 || xx >= sw || yy < 0 || yy >= sh) continue;
      const float d = dv[k];
      if (!((ub >> k) & 1u) && aligned_deg(d, reg_angle, prec)) {
        used_set(F, xx, yy, true);
        reg_put(F, n++, (uint32_t)xx | ((uint32_t)yy << 16), d);
        float c, sn;
        cr_cos_sin((float)deg2ang(d), &c, &sn);
        sumdx += c;
        sumdy += sn;
        reg_angle = (double)fast_atan2_deg(sumdy, sumdx) * kDegToRad;
      }
    }
  }
  return n;
}

__device__ __forceinline__ void region2rect(Frame& F, int n, double reg_angle, double prec, double p, Rect& rec) {
  double x = 0, y = 0, sum = 0;
#pragma unroll 4
  for (int i = 0; i < n; ++i) {
    const uint32_t pt = reg_get(F, i);
    const int px = (int)(pt & 0xFFFF), py = (int)(pt >> 16);
    const double weight = modgrad_q(regq_get(F, i));
    x += double(px) * weight;
    y += double(py) * weight;
    sum += weight;
  }
  x /= sum;
  y /= sum;
  // get_theta
  double Ixx = 0.0, Iyy = 0.0, Ixy = 0.0;
#pragma unroll 4
  for (int i = 0; i < n; ++i) {
    const uint32_t pt = reg_get(F, i);
    const int px = (int)(pt & 0xFFFF), py = (int)(pt >> 16);
    const double weight = modgrad_q(regq_get(F, i));
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

__device__ __forceinline__ bool reduce_region_radius(Frame& F, int& n, double reg_angle, double prec, double p,
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
        reg_swap(F, i, n - 1);
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

__device__ __forceinline__ bool refine(Frame& F, int& n, double reg_angle, double prec, double p, Rect& rec,
                       double density_th) {
  double density = double(n) / (dist(rec.x1, rec.y1, rec.x2, rec.y2) * rec.width);
  if (density >= density_th) return true;
  const uint32_t p0 = reg_get(F, 0);
  const int x0 = (int)(p0 & 0xFFFF), y0 = (int)(p0 >> 16);
  const double xc = double(x0), yc = double(y0);
  const double ang_c = deg2ang(regd_get(F, 0));
  double sum = 0, s_sum = 0;
  int cnt = 0;
  for (int i = 0; i < n; ++i) {
    const uint32_t pt = reg_get(F, i);
    const int px = (int)(pt & 0xFFFF), py = (int)(pt >> 16);
    used_set(F, px, py, false);
    if (dist(xc, yc, px, py) < rec.width) {
      const double ang_d = angle_diff_signed(deg2ang(regd_get(F, i)), ang_c);
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
  fill_q(F, n);
  region2rect(F, n, reg_angle, prec, p, rec);
  density = double(n) / (dist(rec.x1, rec.y1, rec.x2, rec.y2) * rec.width);
  if (density < density_th) return reduce_region_radius(F, n, reg_angle, prec, p, rec, density, density_th);
  return true;
}

__device__ __forceinline__ double rect_nfa(Frame& F, const Rect& rec_lds) {
  const Rect rec = rec_lds;
  const double half_width = rec.width / 2.0;
  const double dyhw = rec.dy * half_width;
  const double dxhw = rec.dx * half_width;
  // corners, sorted by (x, y) (std::sort of 4 = insertion sort; corners
  // with equal (x, y) are indistinguishable, so a sorting network is exact)
  int ex0 = int(rec.x1 - dyhw), ey0 = int(rec.y1 + dxhw);
  int ex1 = int(rec.x2 - dyhw), ey1 = int(rec.y2 + dxhw);
  int ex2 = int(rec.x2 + dyhw), ey2 = int(rec.y2 - dxhw);
  int ex3 = int(rec.x1 + dyhw), ey3 = int(rec.y1 - dxhw);
  auto cswap = [](int& ax, int& ay, int& bx, int& by) {
    if ((bx < ax) || (bx == ax && by < ay)) {
      const int tx = ax, ty = ay;
      ax = bx; ay = by; bx = tx; by = ty;
    }
  };
  cswap(ex0, ey0, ex1, ey1);
  cswap(ex2, ey2, ex3, ey3);
  cswap(ex0, ey0, ex2, ey2);
  cswap(ex1, ey1, ex3, ey3);
  cswap(ex1, ey1, ex2, ey2);
  auto X = [&](int i) { return i == 0 ? ex0 : (i == 1 ? ex1 : (i == 2 ? ex2 : ex3)); };
  auto Y = [&](int i) { return i == 0 ? ey0 : (i == 1 ? ey1 : (i == 2 ? ey2 : ey3)); };
  int imin = 0, imax = 0;
#pragma unroll
  for (int i = 1; i < 4; ++i) {
    if (Y(imin) > Y(i)) imin = i;
    if (Y(imax) < Y(i)) imax = i;
  }
  unsigned taken = 1u << imin;
  int il = -1;
#pragma unroll
  for (int i = 0; i < 4; ++i)
    if (!((taken >> i) & 1u)) {
      if (il < 0) il = i;
      else if (X(il) > X(i)) il = i;
    }
  taken |= 1u << il;
  int ir = -1;
#pragma unroll
  for (int i = 0; i < 4; ++i)
    if (!((taken >> i) & 1u)) {
      if (ir < 0) ir = i;
      else if (X(ir) < X(i)) ir = i;
    }
  taken |= 1u << ir;
  int it = -1;
#pragma unroll
  for (int i = 0; i < 4; ++i)
    if (!((taken >> i) & 1u)) {
      if (it < 0) it = i;
      else if (X(it) > X(i)) it = i;
    }
  const int mnx = X(imin), mny = Y(imin), mxy = Y(imax);
  const int lfx = X(il), lfy = Y(il), rtx = X(ir), rty = Y(ir), tlx = X(it), tly = Y(it);
  // double-valued steps, tail corner's y (pinned P13, oracle rect_nfa)
  const double flstep = (mny != lfy) ? (mnx - lfx) / double(mny - lfy) : 0;
  const double slstep = (lfy != tly) ? (lfx - tlx) / double(lfy - tly) : 0;
  const double frstep = (mny != rty) ? (mnx - rtx) / double(mny - rty) : 0;
  const double srstep = (rty != tly) ? (rtx - tlx) / double(rty - tly) : 0;
  double lstep = flstep, rstep = frstep;
  double left_x = mnx, right_x = mnx;
  // serial walk: row ranges into LDS (prefix offsets in .w)
  int nrows = 0, total = 0;
  for (int y = mny; y <= mxy; ++y) {
    // rows outside the image skip the step updates too (the reference's
    // `continue` precedes them)
    if (y < 0 || y >= F.sh) continue;
    const int xa = max((int)left_x, 0), xb = min((int)right_x, F.sw - 1);
    if (xb >= xa && nrows < F.row_cap) {
      if (F.lane == 0) F.rows[nrows] = make_int4(y, xa, xb, total);
      total += xb - xa + 1;
      nrows++;
    }
    if (y >= lfy) lstep = slstep;
    if (y >= rty) rstep = srstep;
    left_x += lstep;
    right_x += rstep;
  }
  __builtin_amdgcn_wave_barrier();
  // parallel count of aligned pixels, 8 loads in flight per lane
  int alg = 0, r = 0;
  for (int k0 = F.lane; k0 < total; k0 += 64 * 8) {
    float dv[8];
#pragma unroll
    for (int u = 0; u < 8; u++) {
      const int k = k0 + 64 * u;
      dv[u] = kLsdNotdef;
      if (k < total) {
        while (r + 1 < nrows && F.rows[r + 1].w <= k) r++;
        const int4 rw = F.rows[r];
        dv[u] = F.deg[lsd_deg_index(rw.y + (k - rw.w), rw.x, F.dtw)];
      }
    }
#pragma unroll
    for (int u = 0; u < 8; u++) alg += aligned_deg(dv[u], rec.theta, rec.prec) ? 1 : 0;
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) alg += __shfl_xor(alg, o, 64);
  __builtin_amdgcn_wave_barrier();
  return nfa(total, alg, rec.p, F.log_nt, F.lane);
}

// rect_improve (lsd.cpp): the five refinement phases in order, each trying
// five variations of a copy of the best rectangle. Both rectangles live in
// LDS so that the (non-inlined) rect_nfa calls keep few registers live.
__device__ __forceinline__ double rect_improve(Frame& F, Rect& rec) {
  const double delta = 0.5, delta_2 = delta / 2.0;
  Rect& r = *F.rect1;
  double log_nfa = rect_nfa(F, rec);
  if (log_nfa > 0) return log_nfa;
  for (int phase = 0; phase < 5; phase++) {
    r = rec;
    __builtin_amdgcn_wave_barrier();
    for (int n = 0; n < 5; ++n) {
      bool eval = true;
      if (phase == 0) {
        r.p /= 2;
        r.prec = r.p * kPi;
      } else if ((r.width - delta) >= 0.5) {
        if (phase == 1) {
          r.width -= delta;
        } else if (phase == 2) {
          r.x1 += -r.dy * delta_2;
          r.y1 += r.dx * delta_2;
          r.x2 += -r.dy * delta_2;
          r.y2 += r.dx * delta_2;
          r.width -= delta;
        } else if (phase == 3) {
          r.x1 -= -r.dy * delta_2;
          r.y1 -= r.dx * delta_2;
          r.x2 -= -r.dy * delta_2;
          r.y2 -= r.dx * delta_2;
          r.width -= delta;
        } else {
          r.p /= 2;
          r.prec = r.p * kPi;
        }
      } else {
        eval = false;
      }
      __builtin_amdgcn_wave_barrier();
      if (eval) {
        const double v = rect_nfa(F, r);
        if (v > log_nfa) {
          log_nfa = v;
          rec = r;
          __builtin_amdgcn_wave_barrier();
        }
      }
    }
    if (log_nfa > 0) return log_nfa;
  }
  return log_nfa;
}


// ---------------------------------------------------------------------------
// Speculative lane-parallel seed loop (k_lsd_spec).
//
// Each round takes the next (up to) 64 seeds of the pseudo-ordered list that
// are defined and NOTUSED, and every lane runs the whole serial per-seed
// program (region_grow, region2rect, refine) for its own seed against the
// committed USED map, claiming the pixels it adds in a per-pixel stamp word
// with atomicMin(round | seed rank | grow generation). A region's result
// equals the sequential one unless an earlier seed of the same round
// claimed a pixel the region wanted to add (the region's outcome depends on
// the USED state of exactly the aligned pixels it adds); such regions see a
// smaller stamp (during growth or when their claims are re-read after the
// round) and are not committed. Regions are committed in seed order up to
// the first real conflict; a conflicting seed that an earlier committed
// region has covered is skipped exactly as the sequential loop skips USED
// seeds; the next round resumes at the first uncommitted seed (whose rank 0
// guarantees progress). The committed regions' final pixel sets are OR-ed
// into the USED bits, rectangles of refined regions go to the candidate
// list in seed order. A region longer than a lane's buffer is processed by
// the wave-cooperative serial code once it is the first uncommitted seed.
// ---------------------------------------------------------------------------
// One wave owns a frame's speculative state, so ordering its own global
// stores and loads needs only a workgroup-scope fence (s_waitcnt; the CU's
// L1 is coherent for its waves) - an agent-scope __threadfence would write
// back the whole L2 on gfx950.
__device__ __forceinline__ void wg_fence() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup"); }

enum { kSpecConflict = -1, kSpecOverflow = -2, kSpecSmall = 0, kSpecFail = 1, kSpecCand = 2 };

__device__ __forceinline__ uint32_t ld_stamp(uint64_t* sd, int idx) {
  return __hip_atomic_load(sd_hi(sd, idx), __ATOMIC_RELAXED, ORBPL_LSD_SCOPE);
}
__device__ __forceinline__ uint64_t ld_sd(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, ORBPL_LSD_SCOPE);
}
__device__ __forceinline__ int pt_x(const uint4& e) { return (int)(e.x & 0xFFFF); }
__device__ __forceinline__ int pt_y(const uint4& e) { return (int)(e.x >> 16); }

// region_grow for one lane over the packed pixel words (degrees + claim
// stamp, one 8-byte load per neighbour). buf entries: (x | y << 16, degrees,
// modgrad as a double split lo / hi), the weight stored by lane_rect's first
// pass. Claims are fire-and-forget 64-bit atomicMin on (stamp << 32 | deg
// bits) - the low word is constant per pixel, so the minimum is the stamps'.
// The own-pixel test re-reads the stamp from L2 (same-address order within
// the wave). The angle terms cos / sin of an added pixel (the reference's
// region_grow arithmetic, P2) come precomputed from the angle-term plane,
// loaded with the neighbourhood, so the serial chain per added pixel is the
// two adds and the atan2. Returns the
// length, kSpecConflict or kSpecOverflow.
__device__ __forceinline__ double entry_w(const uint4& e) {
  return __hiloint2double((int)e.w, (int)e.z);
}
__device__ __forceinline__ float entry_deg(const uint4& e) { return __uint_as_float(e.y); }

// A lane's region list: lbuf[frame][lane][i] (a lane's batch of 8 entries is
// one cache line; lane-interleaved lists measured slower, 231 vs 222 ms per
// 3072 frames).
struct LaneBuf {
  uint4* p;
  __device__ __forceinline__ uint4& operator[](int i) const { return p[i]; }
  __device__ __forceinline__ LaneBuf operator+(int o) const { return LaneBuf{p + o}; }
  __device__ __forceinline__ uint32_t pt(int i) const { return p[i].x; }
  __device__ __forceinline__ void set_pt(int i, uint32_t v) const { p[i].x = v; }
  __device__ __forceinline__ double w(int i) const {
    const uint2 v = *reinterpret_cast<const uint2*>(&p[i].z);
    return __hiloint2double((int)v.y, (int)v.x);
  }
  __device__ __forceinline__ void set_w(int i, double v) const {
    *reinterpret_cast<uint2*>(&p[i].z) =
        make_uint2((uint32_t)__double2loint(v), (uint32_t)__double2hiint(v));
  }
};

// cv::fastAtan2 with one division: both branches of fast_atan2_deg divide the
// smaller of |x|, |y| by the larger + eps and evaluate the same polynomial, so
// selecting the operands first gives the same float operations in the same
// order (bit-identical) without executing both branches when lanes diverge.
__device__ __forceinline__ float fast_atan2_deg_1div(float y, float x) {
  const float k180pi = (float)(180.0 / 3.14159265358979323846);
  const float p1 = 0.9997878412794807f * k180pi;
  const float p3 = -0.3258083974640975f * k180pi;
  const float p5 = 0.1555786518463281f * k180pi;
  const float p7 = -0.04432655554792128f * k180pi;
  const float eps = (float)2.220446049250313080847e-16;
  const float ax = f_abs(x), ay = f_abs(y);
  const bool ge = ax >= ay;
  const float c = (ge ? ay : ax) / ((ge ? ax : ay) + eps);
  const float c2 = c * c;
  const float pc = (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
  float a = ge ? pc : 90.f - pc;
  a = x < 0 ? 180.f - a : a;
  a = y < 0 ? 360.f - a : a;
  return a;
}

// region_grow for one lane (same result as the step below). Per step the 8
// neighbour addresses come from 3 row and 3 column terms of the tile index;
// the neighbour's flags (in image, not USED, not already in this region,
// defined) are computed for all 8 before the in-order walk, so the walk per
// position is the aligned test (sub, abs, compare, a conditional 2 pi fold)
// and the add body under one branch. The centre (the point being expanded)
// is skipped: its stamp is this grow's own claim unless an earlier seed of
// the round claimed it, and then the claim re-check after the round flags the
// lane anyway (a conflict ends the lane's speculation whichever step finds
// it).
__device__ __forceinline__ int lane_grow(const Frame& F, uint64_t* sd, LaneBuf buf, int cap, int sx,
                                         int sy, double& reg_angle, double prec, uint32_t myval) {
  const uint32_t mytag = myval >> 1;
  const int sw = F.sw, sh = F.sh, tw = F.tw;
  const int si = lsd_sd_index(sx, sy, tw);
  if (cap < 1) return kSpecOverflow;
  const uint64_t v0 = ld_sd(sd + si);
  if (((uint32_t)(v0 >> 32) >> 1) < mytag) return kSpecConflict;
  atomicMin(reinterpret_cast<unsigned long long*>(sd + si),
            ((unsigned long long)myval << 32) | (uint32_t)v0);
  uint4 cur = make_uint4((uint32_t)sx | ((uint32_t)sy << 16), (uint32_t)v0, 0u, 0u);
  buf[0] = cur;
  reg_angle = deg2ang(entry_deg(cur));
  double s0, c0;
  lsdm::sincos_(reg_angle, &s0, &c0);
  float sumdx = (float)c0;
  float sumdy = (float)s0;
  const double k3pi2 = (3 * kPi) / 2, k2pi = 2 * kPi;
  int n = 1;
  for (int i = 0; i < n; i++) {
    const int x = pt_x(cur), y = pt_y(cur);
    const int n_start = n;
    const uint4 pref = buf[min(i + 1, n_start - 1)];
    // tile index = row term + column term (disjoint bit fields), x2 for the
    // paired 16-byte entries
    // byte offsets from the frame's (wave-uniform) pixel-word base as 32-bit
    // unsigned values: the loads and claims take the scalar-base + 32-bit
    // vector-offset form (no 64-bit address arithmetic per neighbour)
    uint32_t rterm[3], cterm[3];
    bool rin[3], cin[3];
#pragma unroll
    for (int d = 0; d < 3; d++) {
      const int yy = y + d - 1, xx = x + d - 1;
      rin[d] = yy >= 0 && yy < sh;
      cin[d] = xx >= 0 && xx < sw;
      const int cy = min(max(yy, 0), sh - 1), cx = min(max(xx, 0), sw - 1);
      rterm[d] = ((((uint32_t)(cy >> 2) * (uint32_t)tw) << 5) | ((uint32_t)(cy & 3) << 3)) << 3;
      cterm[d] = (((uint32_t)(cx >> 2) << 5) | ((uint32_t)(cx & 3) << 1)) << 3;
    }
    uint4 w[9];
#pragma unroll
    for (int k = 0; k < 9; k++) {
      if (k == 4) continue;
      w[k] = *reinterpret_cast<const uint4*>(reinterpret_cast<const char*>(sd) +
                                             (rterm[k / 3] + cterm[k % 3]));
    }
    unsigned ok = 0;
#pragma unroll
    for (int k = 0; k < 9; k++) {
      if (k == 4) continue;
      // bitwise, not short-circuit: no branch per neighbour
      const unsigned f = (unsigned)(rin[k / 3] & cin[k % 3]) & (unsigned)(w[k].y != 0u) &
                         (unsigned)(w[k].y != myval) & (unsigned)(__uint_as_float(w[k].x) >= 0.f);
      ok |= f << k;
    }
    uint4 first_add = cur;
#pragma unroll
    for (int k = 0; k < 9; k++) {
      if (k == 4) continue;
      // aligned_deg(d, reg_angle, prec) for a defined d
      double nt = fabs(reg_angle - deg2ang(__uint_as_float(w[k].x)));
      nt = nt > k3pi2 ? fabs(nt - k2pi) : nt;
      if (((ok >> k) & 1u) && nt <= prec) {
        if ((w[k].y >> 1) < mytag) return kSpecConflict;   // an earlier seed's pixel
        atomicMin(reinterpret_cast<unsigned long long*>(reinterpret_cast<char*>(sd) +
                                                        (rterm[k / 3] + cterm[k % 3])),
                  ((unsigned long long)myval << 32) | w[k].x);
        if (n >= cap) return kSpecOverflow;
        const int xx = x + (k % 3) - 1, yy = y + (k / 3) - 1;
        const uint4 e = make_uint4((uint32_t)xx | ((uint32_t)yy << 16), w[k].x, 0u, 0u);
        if (n == n_start) first_add = e;
        buf[n++] = e;
        sumdx += __uint_as_float(w[k].z);   // add_angle(d) terms
        sumdy += __uint_as_float(w[k].w);
        reg_angle = (double)fast_atan2_deg_1div(sumdy, sumdx) * kDegToRad;
      }
    }
    cur = (i + 1 < n_start) ? pref : first_add;
  }
  return n;
}

// One pass of reduce_region_radius's removal scan (lsd.cpp reduce_region_radius:
// "swap with the last point, pop, re-test i") over a lane list, without its
// chain of dependent loads. The scan's result is fixed by the points alone:
// the kept ("near") points end in [0, nn), nn = their count; a near point in
// [0, nn) keeps its slot and the k-th far point there (in index order) is
// replaced by the k-th near point of [nn, n) counted from the end. So one
// batched counting pass, then a merge of a forward stream over [0, nn) and a
// backward stream over [nn, n), several loads in flight per refill. Each slot
// is read by one stream before any store reaches it (stores go to slots the
// storing stream has consumed), so the windows never hold stale points. The
// far points stay in [nn, n) (their order is immaterial: the claim re-check
// reads the touched prefix as a set), and only their point words: the scan
// tests only point words, a near point moved forward carries all four.
// distSq of two pixel positions is an integer below 2^21, exact in double
// whichever way it is summed: the integer form gives the same comparison.
__device__ __forceinline__ bool lane_far(uint32_t pt, int xc, int yc, double radSq) {
  const int dx = (int)(pt & 0xFFFF) - xc, dy = (int)(pt >> 16) - yc;
  return (double)(dx * dx + dy * dy) > radSq;
}
// Profiling build (-DORBPL_FIT_PROF): wall time of the fit's phases per
// round, as seen by the lanes in them, reduced to the wave maximum per round
// and printed for frame 0 (0 first rect, 1 refine statistics, 2 second grow,
// 3 second rect, 4 reduce_region_radius loop).
struct FitProf {
#ifdef ORBPL_FIT_PROF
  long long d[5] = {0, 0, 0, 0, 0};
  long long last = 0;
  __device__ __forceinline__ void start() { last = clock64(); }
  __device__ __forceinline__ void lap(int k) {
    const long long c = clock64();
    d[k] += c - last;
    last = c;
  }
#else
  __device__ __forceinline__ void start() {}
  __device__ __forceinline__ void lap(int) {}
#endif
};

// ---------------------------------------------------------------------------
// NFA validation with one lane per rectangle (k_lsd_validate): most
// candidates are small (tens of pixels) and go through all rect_improve
// phases, so the serial parts (corner walk, log_gamma, binomial tail)
// dominate; a lane runs them for its own rectangle exactly as the reference
// orders them, 64 rectangles per wave.
// ---------------------------------------------------------------------------
// log(p) and log(1 - p) of the last p a lane's NFA saw (rect_improve changes
// p only in its first and last phase)
struct NfaLogs {
  double p = -1, lp = 0, l1p = 0;
  __device__ __forceinline__ void set(double q) {
    if (q != p) {
      p = q;
      lp = lsdm::log_(q);
      l1p = lsdm::log_(1.0 - q);
    }
  }
};

// nfa for one lane. The three log_gamma terms take integer arguments n + 1,
// k + 1, n - k + 1: they come from a table the same log_gamma filled
// (k_lgamma_table; Lanczos below 15, 8 logs and 7 powers, Windschitl above)
// when n is inside it.
__device__ __forceinline__ double nfa_lane(int n, int k, double p, double log_nt,
                                           const double* __restrict__ lgam, int lgam_n,
                                           NfaLogs& L) {
  if (n == 0 || k == 0) return -log_nt;
  if (n == k) return -log_nt - double(n) * lsdm::log10_(p);
  const double p_term = p / (1 - p);
  L.set(p);
  const double lgn = n < lgam_n ? lgam[n] : log_gamma(double(n) + 1);
  const double lgk = n < lgam_n ? lgam[k] : log_gamma(double(k) + 1);
  const double lgnk = n < lgam_n ? lgam[n - k] : log_gamma(double(n - k) + 1);
  const double log1term = lgn - lgk - lgnk + double(k) * L.lp + double(n - k) * L.l1p;
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

// rect_nfa for one lane: the reference's row walk, pixels counted in
// batches of 8 loads generated across rows.
__device__ __forceinline__ double rect_nfa_lane(const float* __restrict__ deg, int sw, int sh,
                                                const Rect& rec, double log_nt,
                                                const double* __restrict__ lgam, int lgam_n,
                                                NfaLogs& L) {
  const double half_width = rec.width / 2.0;
  const double dyhw = rec.dy * half_width;
  const double dxhw = rec.dx * half_width;
  int ex0 = int(rec.x1 - dyhw), ey0 = int(rec.y1 + dxhw);
  int ex1 = int(rec.x2 - dyhw), ey1 = int(rec.y2 + dxhw);
  int ex2 = int(rec.x2 + dyhw), ey2 = int(rec.y2 - dxhw);
  int ex3 = int(rec.x1 + dyhw), ey3 = int(rec.y1 - dxhw);
  auto cswap = [](int& ax, int& ay, int& bx, int& by) {
    if ((bx < ax) || (bx == ax && by < ay)) {
      const int tx = ax, ty = ay;
      ax = bx; ay = by; bx = tx; by = ty;
    }
  };
  cswap(ex0, ey0, ex1, ey1);
  cswap(ex2, ey2, ex3, ey3);
  cswap(ex0, ey0, ex2, ey2);
  cswap(ex1, ey1, ex3, ey3);
  cswap(ex1, ey1, ex2, ey2);
  auto X = [&](int i) { return i == 0 ? ex0 : (i == 1 ? ex1 : (i == 2 ? ex2 : ex3)); };
  auto Y = [&](int i) { return i == 0 ? ey0 : (i == 1 ? ey1 : (i == 2 ? ey2 : ey3)); };
  int imin = 0, imax = 0;
#pragma unroll
  for (int i = 1; i < 4; ++i) {
    if (Y(imin) > Y(i)) imin = i;
    if (Y(imax) < Y(i)) imax = i;
  }
  unsigned taken = 1u << imin;
  int il = -1;
#pragma unroll
  for (int i = 0; i < 4; ++i)
    if (!((taken >> i) & 1u)) {
      if (il < 0) il = i;
      else if (X(il) > X(i)) il = i;
    }
  taken |= 1u << il;
  int ir = -1;
#pragma unroll
  for (int i = 0; i < 4; ++i)
    if (!((taken >> i) & 1u)) {
      if (ir < 0) ir = i;
      else if (X(ir) < X(i)) ir = i;
    }
  taken |= 1u << ir;
  int it = -1;
#pragma unroll
  for (int i = 0; i < 4; ++i)
    if (!((taken >> i) & 1u)) {
      if (it < 0) it = i;
      else if (X(it) > X(i)) it = i;
    }
  const int mnx = X(imin), mny = Y(imin), mxy = Y(imax);
  const int lfx = X(il), lfy = Y(il), rtx = X(ir), rty = Y(ir), tlx = X(it), tly = Y(it);
  const double flstep = (mny != lfy) ? (mnx - lfx) / double(mny - lfy) : 0;
  const double slstep = (lfy != tly) ? (lfx - tlx) / double(lfy - tly) : 0;
  const double frstep = (mny != rty) ? (mnx - rtx) / double(mny - rty) : 0;
  const double srstep = (rty != tly) ? (rtx - tlx) / double(rty - tly) : 0;
  double lstep = flstep, rstep = frstep;
  double left_x = mnx, right_x = mnx;
  // walk state: row y, next pixel x, last pixel xe (rows outside the image
  // are skipped without step updates, as the reference's `continue`)
  int y = mny, x = 1, xe = 0;
  while (y <= mxy && (y < 0 || y >= sh)) y++;
  if (y <= mxy) {
    x = max((int)left_x, 0);
    xe = min((int)right_x, sw - 1);
  }
  int total = 0, alg = 0;
  const int dtw = lsd_deg_tw(sw);
  const double theta = rec.theta, prec = rec.prec;
  while (y <= mxy) {
    int idx[8];
    unsigned valid = 0;
#pragma unroll
    for (int u = 0; u < 8; u++) {
      while (y <= mxy && x > xe) {
        if (y >= lfy) lstep = slstep;
        if (y >= rty) rstep = srstep;
        left_x += lstep;
        right_x += rstep;
        y++;
        while (y <= mxy && (y < 0 || y >= sh)) y++;
        if (y <= mxy) {
          x = max((int)left_x, 0);
          xe = min((int)right_x, sw - 1);
        }
      }
      idx[u] = 0;
      if (y <= mxy) {
        idx[u] = lsd_deg_index(x, y, dtw);
        valid |= 1u << u;
        x++;
      }
    }
    float dv[8];
#pragma unroll
    for (int u = 0; u < 8; u++) dv[u] = deg[idx[u]];
#pragma unroll
    for (int u = 0; u < 8; u++) {
      if ((valid >> u) & 1u) {
        total++;
        alg += aligned_deg(dv[u], theta, prec) ? 1 : 0;
      }
    }
  }
  return nfa_lane(total, alg, rec.p, log_nt, lgam, lgam_n, L);
}

__device__ __forceinline__ double rect_improve_lane(const float* __restrict__ deg, int sw, int sh,
                                                    Rect& rec, double log_nt,
                                                    const double* __restrict__ lgam, int lgam_n) {
  const double delta = 0.5, delta_2 = delta / 2.0;
  NfaLogs L;
  double log_nfa = rect_nfa_lane(deg, sw, sh, rec, log_nt, lgam, lgam_n, L);
  if (log_nfa > 0) return log_nfa;
  for (int phase = 0; phase < 5; phase++) {
    Rect r = rec;
    for (int n = 0; n < 5; ++n) {
      bool eval = true;
      if (phase == 0) {
        r.p /= 2;
        r.prec = r.p * kPi;
      } else if ((r.width - delta) >= 0.5) {
        if (phase == 1) {
          r.width -= delta;
        } else if (phase == 2) {
          r.x1 += -r.dy * delta_2;
          r.y1 += r.dx * delta_2;
          r.x2 += -r.dy * delta_2;
          r.y2 += r.dx * delta_2;
          r.width -= delta;
        } else if (phase == 3) {
          r.x1 -= -r.dy * delta_2;
          r.y1 -= r.dx * delta_2;
          r.x2 -= -r.dy * delta_2;
          r.y2 -= r.dx * delta_2;
          r.width -= delta;
        } else {
          r.p /= 2;
          r.prec = r.p * kPi;
        }
      } else {
        eval = false;
      }
      if (eval) {
        const double v = rect_nfa_lane(deg, sw, sh, r, log_nt, lgam, lgam_n, L);
        if (v > log_nfa) {
          log_nfa = v;
          rec = r;
        }
      }
    }
    if (log_nfa > 0) return log_nfa;
  }
  return log_nfa;
}

// rect_improve with the best rectangle's changing fields (x1, y1, x2, y2,
// width, prec, p) in a per-lane LDS slot instead of registers: the trial
// rectangle is re-read from it at each phase start and written on an
// improvement, so the 8-wave register budget holds the walk without scratch
// spills (whose write-backs were most of the kernel's HBM writes).
__device__ __forceinline__ double rect_improve_lds(const float* __restrict__ deg, int sw, int sh,
                                                   Rect& rec, double* __restrict__ slot,
                                                   double log_nt, const double* __restrict__ lgam,
                                                   int lgam_n) {
  const double delta = 0.5, delta_2 = delta / 2.0;
  NfaLogs L;
  double log_nfa = rect_nfa_lane(deg, sw, sh, rec, log_nt, lgam, lgam_n, L);
  if (log_nfa > 0) return log_nfa;
  slot[0] = rec.x1; slot[1] = rec.y1; slot[2] = rec.x2; slot[3] = rec.y2;
  slot[4] = rec.width; slot[5] = rec.prec; slot[6] = rec.p;
  Rect r = rec;
  for (int phase = 0; phase < 5; phase++) {
    r.x1 = slot[0]; r.y1 = slot[1]; r.x2 = slot[2]; r.y2 = slot[3];
    r.width = slot[4]; r.prec = slot[5]; r.p = slot[6];
    for (int n = 0; n < 5; ++n) {
      bool eval = true;
      if (phase == 0) {
        r.p /= 2;
        r.prec = r.p * kPi;
      } else if ((r.width - delta) >= 0.5) {
        if (phase == 1) {
          r.width -= delta;
        } else if (phase == 2) {
          r.x1 += -r.dy * delta_2;
          r.y1 += r.dx * delta_2;
          r.x2 += -r.dy * delta_2;
          r.y2 += r.dx * delta_2;
          r.width -= delta;
        } else if (phase == 3) {
          r.x1 -= -r.dy * delta_2;
          r.y1 -= r.dx * delta_2;
          r.x2 -= -r.dy * delta_2;
          r.y2 -= r.dx * delta_2;
          r.width -= delta;
        } else {
          r.p /= 2;
          r.prec = r.p * kPi;
        }
      } else {
        eval = false;
      }
      if (eval) {
        const double v = rect_nfa_lane(deg, sw, sh, r, log_nt, lgam, lgam_n, L);
        if (v > log_nfa) {
          log_nfa = v;
          slot[0] = r.x1; slot[1] = r.y1; slot[2] = r.x2; slot[3] = r.y2;
          slot[4] = r.width; slot[5] = r.prec; slot[6] = r.p;
        }
      }
    }
    if (log_nfa > 0) break;
  }
  rec.x1 = slot[0]; rec.y1 = slot[1]; rec.x2 = slot[2]; rec.y2 = slot[3];
  rec.width = slot[4]; rec.prec = slot[5]; rec.p = slot[6];
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
  F.deg = sc.deg + (long long)f * lsd_deg_words(sw, sh);
  F.dtw = lsd_deg_tw(sw);
  F.q = sc.q + (long long)f * sw * sh;
  F.used = grow_smem;
  F.usd = nullptr;
  F.tw = 0;
  F.reg_l = grow_smem + used_words;
  F.regq_l = reinterpret_cast<int*>(F.reg_l + kRegLds);
  F.regd_l = reinterpret_cast<float*>(F.regq_l + kRegLds);
  F.ring = F.regd_l + kRegLds;
  F.reg_g = sc.reg + (long long)f * 3 * sw * sh;
  F.rows = reinterpret_cast<int4*>(grow_smem + ((used_words + 3 * kRegLds + 64 * 9 + 3) & ~3));
  F.rect0 = reinterpret_cast<Rect*>(F.rows);
  F.rect1 = F.rect0 + 1;
  F.row_cap = 0;
  F.log_nt = g.log_nt;
  F.lane = lane;
  F.pf_cyc = 0;
  F.pf_cnt = 0;
  for (int i = lane; i < used_words; i += 64) F.used[i] = 0;
  __builtin_amdgcn_wave_barrier();
  const uint32_t* A = sc.A + (long long)f * g.n;
  const int nlist = sc.sort_nge[f];   // later list entries are NOTDEF
  const int w1 = sw - 1;
  const double prec = g.prec, p = g.p;
  int nl = 0;
  long long pc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const long long tstart = clock64();
  for (int base = 0; base < nlist; base += 64) {
    const int i = base + lane;
    int px = 0, py = 0;
    bool def = false;
    if (i < nlist) {
      const int idx = (int)(A[i] & 0x3FFFFFu);
      py = idx / w1;
      px = idx - py * w1;
      def = F.deg[lsd_deg_index(px, py, F.dtw)] >= 0.f;
    }
    unsigned long long mask = __ballot(def && !used_get(F, px, py));
    while (mask) {
      const int l = __ffsll((long long)mask) - 1;
      const int sx = __shfl(px, l, 64), sy = __shfl(py, l, 64);
      double reg_angle;
      long long t0 = clock64();
      int n = region_grow(F, sx, sy, reg_angle, prec);
      long long t1 = clock64();
      pc[0] += t1 - t0;
      pc[4] += n;
      pc[5] += 1;
      if (n >= g.min_reg_size) {
        Rect& rec = *F.rect0;
        fill_q(F, n);
        region2rect(F, n, reg_angle, prec, p, rec);
        const bool ok = refine(F, n, reg_angle, prec, p, rec, 0.7);
        pc[1] += clock64() - t1;
        if (ok) {
          // NFA validation (rect_improve) does not touch the USED map: it
          // runs later for all rectangles at once (k_lsd_validate)
          if (nl < kLsdMaxCand) {
            const double* rv = reinterpret_cast<const double*>(F.rect0);
            if (lane < 12) sc.cand[((long long)f * kLsdMaxCand + nl) * 12 + lane] = rv[lane];
          } else if (lane == 0) {
            atomicOr(sc.err + f, 8);
          }
          nl++;
        }
      }
      mask = __ballot(def && lane > l && !used_get(F, px, py));
    }
  }
  if (lane == 0) sc.ncand[f] = min(nl, kLsdMaxCand);
  if (sc.prof && lane == 0) {
    pc[3] = clock64() - tstart;
    pc[7] = nl;
    pc[6] = F.pf_cyc;
    pc[5] = F.pf_cnt;
    for (int k = 0; k < 8; k++) sc.prof[f * 8 + k] = pc[k];
  }
}


// Speculative seed loop (see lane_grow): W waves per frame, 64 W seeds per
// round. W = 1 for large batches (every frame co-resident, one wave each);
// mid-size batches take 4 waves per frame (lsd_spec_waves):
// a round of 128 / 256 seeds needs 2.4x fewer rounds (388 -> 159 per frame),
// but each round waits for the slowest of more lanes and wastes more
// speculative regions (24.8k -> 40.5k per frame), so a lone frame gains
// nothing; with the GPU partly empty the extra waves fill it (batch 256:
// -5 %, 1024: -10 % per batch).
#ifndef ORBPL_SPEC_SMALL_BATCH
#define ORBPL_SPEC_SMALL_BATCH 96
#endif
constexpr int kSpecSmallBatch = ORBPL_SPEC_SMALL_BATCH;
// ORBPL_SPEC_MINW: waves per SIMD the one-wave-per-frame variant's register
// budget must allow. Round 2 chose 4 (128 VGPRs) although the batches that
// use it hold 3 frames per SIMD, so that the concurrent ORB extraction /
// tracking waves fit beside the seed loop (LSD alone 222.9 -> 235 ms per 3072
// frames, lines workload 10.5k -> 11.4k frames/s then). With the round-4 seed
// loop the 128-VGPR build spills 77 registers; 3 (168 VGPRs) measured (two
// rounds each, tools/ab_lines_lib.sh, tools/ab_kitti_lib.sh): LSD at 3072
// frames 167.0 -> 156.6 ms, the lines leg's seed stage 86-90 -> 74 ms, the
// lines leg equal (15.7-16.0k vs 15.9k), the stereo leg 5.4-5.8k -> 5.85-5.89k
#ifndef ORBPL_SPEC_MINW
#define ORBPL_SPEC_MINW 3
#endif
// Carried seeds (one wave per frame): a round ends at its first seed whose
// region met an earlier seed's claim; the later seeds of the window whose
// claim re-check passed keep their regions and fits for the next round
// instead of growing them again. Their results are the reference's unless a
// seed before them in the list (the stopping seed, regrown, or another
// regrown one) now claims one of their pixels: at the next round's start
// their touched pixels are re-stamped with that round's claim tag (ranks in
// list order, so the regrown seeds before them win and the new seeds after
// them lose), and the next re-check decides again. Lanes take the carried
// seeds first, in list order, then new seeds from the scan; a lane's list
// buffer travels with its seed (bufid). After a cooperative fallback nothing
// is carried (the fallback uses buffer 0 as scratch).
// ---------------------------------------------------------------------------
// Wave-wide fits. After a round's grows, the fits of the regions that reach
// min_reg_size (~4 per round) keep the per-lane control flow, but every pass
// over a region's list - region2rect's centroid, inertia and extent passes,
// refine's angle statistics, reduce_region_radius' count and merge - has
// independent per-point work and ordered double sums: the wave computes 64
// points' terms at once, then the sums are added in list order from LDS, so
// each rounds exactly as the sequential loop's (the extents and the counts
// are order-free). refine's second region grow stays one lane per region.
// Measured on three boxes against per-lane fits (round 4, bit-exact): LSD
// batch 1 44.0-47.4 vs 44.4-51.5 ms, batch 16 51.8-53.1 vs 54.6-55.5 ms,
// batch 1536 115.3 vs 118.8 ms. One region at a time across the whole wave
// measured no faster (the per-region fixed costs outweigh the parallel
// points). The A/B records are under profiles/r04/.
// ---------------------------------------------------------------------------

// fitters whose terms share LDS at once
constexpr int kCoopG = 4;
struct CoopScratch {
  union {
    struct {   // one row per fitter of a group, padded so that the lanes'
               // rows start in different banks
      double ga[kCoopG][65], gb[kCoopG][65], gc[kCoopG][65];
    };
    struct {
      uint16_t farpos[kLaneCap / 2], nearpos[kLaneCap / 2];
    };
  };
};

// the wave's LDS operations so far are complete; no memory access moves across
__device__ __forceinline__ void coop_lds_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ int coop_rl(int v, int l) { return __builtin_amdgcn_readlane(v, l); }
__device__ __forceinline__ double coop_rl(double v, int l) {
  return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), l),
                          __builtin_amdgcn_readlane(__double2loint(v), l));
}
__device__ __forceinline__ uint4* coop_rl(uint4* v, int l) {
  const uintptr_t u = reinterpret_cast<uintptr_t>(v);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)u, l);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), l);
  return reinterpret_cast<uint4*>(((uintptr_t)hi << 32) | lo);
}

// The fits stay one lane per region (the round's fitting lanes together),
// but every pass's per-point work is
// spread over the whole wave: for a group of up to kCoopG fitting lanes and
// a window of 64 points, the wave evaluates each lane's 64 terms in turn
// (term(f, i, ...) with f the owning lane) into that lane's LDS row, then
// every lane of the group adds its own row in point order. The sums round as
// the sequential loop's; the serial part per point is three LDS reads and
// three adds instead of the point's whole load / weight / product chain.
// The three sums of a slot run on three lanes.
template <bool kSubC, class Load, class Term>
__device__ __forceinline__ void group_sums(CoopScratch& S, int lane, bool act, int n, double& A,
                                           double& B, double& C, Load load, Term term) {
  unsigned long long am = __ballot(act);
  while (am) {
    // the group: the first kCoopG lanes of am, slot s = the s-th of them
    int fs[kCoopG], nfs[kCoopG];
    unsigned long long gm = 0;
#pragma unroll
    for (int s = 0; s < kCoopG; s++) {
      fs[s] = am ? __ffsll((long long)am) - 1 : -1;
      nfs[s] = fs[s] >= 0 ? coop_rl(n, fs[s]) : 0;
      if (am) {
        gm |= am & (~am + 1ull);
        am &= am - 1;
      }
    }
    const bool ing = (gm >> lane) & 1ull;
    const int myslot = __popcll(gm & ((1ull << lane) - 1ull));
    // chain lanes: lane c * kCoopG + s adds sum c (A, B, C) of slot s, so a
    // point's three ordered adds run on three lanes at once; C's terms are
    // stored negated where the sum subtracts (x - y == x + (-y) exactly)
    const int cs = lane % kCoopG, cc = lane / kCoopG;
    int myf = -1, mynf = 0;
#pragma unroll
    for (int s2 = 0; s2 < kCoopG; s2++) {
      myf = cs == s2 ? fs[s2] : myf;
      mynf = cs == s2 ? nfs[s2] : mynf;
    }
    const bool chain = cc < 3 && myf >= 0;
    const double a0 = shfl_d(A, max(myf, 0)), b0 = shfl_d(B, max(myf, 0)),
                 c0 = shfl_d(C, max(myf, 0));
    double acc = cc == 0 ? a0 : (cc == 1 ? b0 : c0);
    const double* prow = cc == 0 ? S.ga[cs] : (cc == 1 ? S.gb[cs] : S.gc[cs]);
    int nmax = ing ? n : 0;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) nmax = max(nmax, __shfl_xor(nmax, o, 64));
    for (int k0 = 0; k0 < nmax; k0 += 64) {
      const int i = k0 + lane;
      // every slot's loads issue before any term is formed
      uint4 v[kCoopG];
#pragma unroll
      for (int s = 0; s < kCoopG; s++)
        v[s] = (i < nfs[s]) ? load(fs[s], i) : make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
      for (int s = 0; s < kCoopG; s++) {
        if (i < nfs[s]) {
          double ta, tb, tc;
          term(fs[s], i, v[s], ta, tb, tc);
          S.ga[s][lane] = ta;
          S.gb[s][lane] = tb;
          S.gc[s][lane] = kSubC ? -tc : tc;
        }
      }
      coop_lds_sync();
      if (chain) {
        const int cnt = min(64, mynf - k0);
        int k = 0;
        for (; k + 4 <= cnt; k += 4) {
          double xv[4];
#pragma unroll
          for (int u = 0; u < 4; u++) xv[u] = prow[k + u];
#pragma unroll
          for (int u = 0; u < 4; u++) acc += xv[u];
        }
        for (; k < cnt; k++) acc += prow[k];
      }
      coop_lds_sync();
    }
    // the chain lanes' sums back to their fitters
    const double ra = shfl_d(acc, myslot), rb = shfl_d(acc, kCoopG + myslot),
                 rc = shfl_d(acc, 2 * kCoopG + myslot);
    if (ing) {
      A = ra;
      B = rb;
      C = rc;
    }
  }
}

// region2rect's first pass for every act lane over its list bp[0, n) (with q:
// the weights computed and stored into the entries first)
__device__ __forceinline__ void group_centroid(CoopScratch& S, int lane, bool act, uint4* bp,
                                               int n, const int* __restrict__ q, int sw,
                                               double& x, double& y, double& sum) {
  x = 0;
  y = 0;
  sum = 0;
  if (q) {
    group_sums<false>(
        S, lane, act, n, x, y, sum,
        [&](int f, int i) {
          const uint32_t pt = LaneBuf{coop_rl(bp, f)}.pt(i);
          return make_uint4(pt, (uint32_t)q[(int)(pt >> 16) * sw + (int)(pt & 0xFFFF)], 0u, 0u);
        },
        [&](int f, int i, const uint4& e, double& ta, double& tb, double& tc) {
          const double w = modgrad_q((int)e.y);
          LaneBuf{coop_rl(bp, f)}.set_w(i, w);
          ta = double(e.x & 0xFFFF) * w;
          tb = double(e.x >> 16) * w;
          tc = w;
        });
  } else {
    group_sums<false>(
        S, lane, act, n, x, y, sum, [&](int f, int i) { return LaneBuf{coop_rl(bp, f)}[i]; },
        [&](int f, int i, const uint4& e, double& ta, double& tb, double& tc) {
          const double w = entry_w(e);
          ta = double(e.x & 0xFFFF) * w;
          tb = double(e.x >> 16) * w;
          tc = w;
        });
  }
}

// lane_rect_tail for every act lane: inertia sums (group_sums), theta per
// lane, the extents fitter by fitter over the whole wave
__device__ __forceinline__ void group_rect_tail(CoopScratch& S, int lane, bool act, uint4* bp,
                                                int n, double x, double y, double sum,
                                                double reg_angle, double prec, double p,
                                                Rect& rec) {
  if (act) {
    x /= sum;
    y /= sum;
  }
  double Ixx = 0.0, Iyy = 0.0, Ixy = 0.0;
  group_sums<true>(
      S, lane, act, n, Ixx, Iyy, Ixy, [&](int f, int i) { return LaneBuf{coop_rl(bp, f)}[i]; },
      [&](int f, int i, const uint4& e, double& ta, double& tb, double& tc) {
        const double xf = coop_rl(x, f), yf = coop_rl(y, f);
        const double weight = entry_w(e);
        const double dx = double(pt_x(e)) - xf, dy = double(pt_y(e)) - yf;
        ta = dy * dy * weight;
        tb = dx * dx * weight;
        tc = dx * dy * weight;
      });
  double theta = 0, dx = 0, dy = 0;
  if (act) {
    const double lambda = 0.5 * (Ixx + Iyy - sqrt((Ixx - Iyy) * (Ixx - Iyy) + 4.0 * Ixy * Ixy));
    theta = (fabs(Ixx) > fabs(Iyy)) ? double(fast_atan2_deg(float(lambda - Ixx), float(Ixy)))
                                    : double(fast_atan2_deg(float(Ixy), float(lambda - Iyy)));
    theta *= kDegToRad;
    if (fabs(angle_diff_signed(theta, reg_angle)) > prec) theta += kPi;
    dx = lsdm::cos_(theta);
    dy = lsdm::sin_(theta);
  }
  // the extents: order-free max / min, one lane per region (lane_rect_tail)
  double l_min = 0, l_max = 0, w_min = 0, w_max = 0;
  if (act) {
    const LaneBuf bf{bp};
    constexpr int kB3 = 16;
    for (int i0 = 0; i0 < n; i0 += kB3) {
      uint32_t pt[kB3];
#pragma unroll
      for (int u = 0; u < kB3; u++) pt[u] = bf.pt(min(i0 + u, n - 1));
#pragma unroll
      for (int u = 0; u < kB3; u++) {
        const double regdx = double(pt[u] & 0xFFFF) - x, regdy = double(pt[u] >> 16) - y;
        const double l = regdx * dx + regdy * dy;
        const double w = -regdx * dy + regdy * dx;
        l_max = l > l_max ? l : l_max;
        l_min = l < l_min ? l : l_min;
        w_max = w > w_max ? w : w_max;
        w_min = w < w_min ? w : w_min;
      }
    }
  }
  if (act) {
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
}

// refine's angle statistics for every act lane over bp[0, n) -> tau (the
// count as a third sum: whole numbers, exact in double)
__device__ __forceinline__ double group_tau(CoopScratch& S, int lane, bool act, uint4* bp, int n,
                                           const Rect& rec) {
  double sum = 0, s_sum = 0, cnt = 0;
  const double width = rec.width;
  group_sums<false>(
      S, lane, act, n, sum, s_sum, cnt, [&](int f, int i) { return LaneBuf{coop_rl(bp, f)}[i]; },
      [&](int f, int i, const uint4& e, double& ta, double& tb, double& tc) {
        const LaneBuf bf{coop_rl(bp, f)};
        const double wf = coop_rl(width, f);
        const uint4 e0 = bf[0];
        const double xc = double(pt_x(e0)), yc = double(pt_y(e0));
        const double ang_c = deg2ang(entry_deg(e0));
        ta = 0;
        tb = 0;
        tc = 0;
        // a point outside adds +0.0: the sums start at +0 and never become
        // -0, so x + 0.0 == x (skipping it)
        if (dist(xc, yc, pt_x(e), pt_y(e)) < wf) {
          const double ang_d = angle_diff_signed(deg2ang(entry_deg(e)), ang_c);
          ta = ang_d;
          tb = ang_d * ang_d;
          tc = 1.0;
        }
      });
  if (!act) return 0.0;
  const int c = (int)cnt;
  const double mean_angle = sum / double(c);
  return 2.0 * sqrt((s_sum - 2.0 * mean_angle * sum) / double(c) + mean_angle * mean_angle);
}

// lane_reduce_pass's merge for fitter f (count nn < n already known): the
// k-th far point of [0, nn) in index order takes the k-th near point of
// [nn, n) counted from the end; that slot keeps the far point's word
__device__ __forceinline__ void group_merge(CoopScratch& S, int lane, LaneBuf g1, int n, int nn,
                                            int xc, int yc, double radSq) {
  const unsigned long long lt = (1ull << lane) - 1ull;
  int m = 0;
  for (int i0 = 0; i0 < nn; i0 += 64) {
    const int i = i0 + lane;
    const bool fr = i < nn && lane_far(g1.pt(i), xc, yc, radSq);
    const unsigned long long mk = __ballot(fr);
    if (fr) S.farpos[m + __popcll(mk & lt)] = (uint16_t)i;
    m += __popcll(mk);
  }
  int m2 = 0;
  for (int j0 = 0; j0 < n - nn; j0 += 64) {
    const int j = n - 1 - (j0 + lane);
    const bool nr = j >= nn && !lane_far(g1.pt(j), xc, yc, radSq);
    const unsigned long long mk = __ballot(nr);
    if (nr) S.nearpos[m2 + __popcll(mk & lt)] = (uint16_t)j;
    m2 += __popcll(mk);
  }
  coop_lds_sync();
  for (int k0 = 0; k0 < m; k0 += 64) {
    const int k = k0 + lane;
    if (k < m) {
      const int i = S.farpos[k], j = S.nearpos[k];
      const uint32_t farw = g1.pt(i);
      const uint4 b = g1[j];
      g1[i] = b;
      g1.set_pt(j, farw);
    }
  }
  coop_lds_sync();
}

// The round's fits: region2rect + refine + reduce_region_radius with the
// per-lane control flow and the wave-wide passes above
__device__ __forceinline__ void group_fit(CoopScratch& S, int lane, bool fitter, int n,
                                          double reg_angle, uint4* fbuf, int bufid,
                                          const Frame& F, uint64_t* sd, double prec, double p,
                                          uint32_t myval1, int& status, Rect& rec, int& off,
                                          int& len, int& touched, FitProf& fp) {
  uint4* bp = fbuf + (long long)bufid * kLaneCap;
  double cx, cy, cs;
  fp.start();
  group_centroid(S, lane, fitter, bp, n, F.q, F.sw, cx, cy, cs);
  wg_fence();
  __builtin_amdgcn_wave_barrier();
  group_rect_tail(S, lane, fitter, bp, n, cx, cy, cs, reg_angle, prec, p, rec);
  fp.lap(0);
  bool refine = false;
  if (fitter) {
    const double density = double(n) / (dist(rec.x1, rec.y1, rec.x2, rec.y2) * rec.width);
    off = 0;
    len = n;
    touched = n;
    status = kSpecCand;
    refine = density < 0.7;
  }
  const double tau = group_tau(S, lane, refine, bp, n, rec);
  fp.lap(1);
  // refine's second grow, one lane per region
  const LaneBuf buf{bp};
  int n1 = 0, x0 = 0, y0 = 0;
  double ra2 = reg_angle;
  if (refine) {
    const uint4 e0 = buf[0];
    x0 = pt_x(e0);
    y0 = pt_y(e0);
  }
  if (refine) {
    n1 = lane_grow(F, sd, buf + n, kLaneCap - n, x0, y0, ra2, tau, myval1);
  }
  if (refine) {
    if (n1 < 0) {
      status = n1;
      refine = false;
    } else {
      off = n;
      len = n1;
      touched = n + n1;
      if (n1 < 2) {
        status = kSpecFail;
        refine = false;
      }
    }
  }
  __builtin_amdgcn_wave_barrier();
  fp.lap(2);
  uint4* gp = bp + n;   // the second region's list
  group_centroid(S, lane, refine, gp, n1, F.q, F.sw, cx, cy, cs);
  wg_fence();
  __builtin_amdgcn_wave_barrier();
  group_rect_tail(S, lane, refine, gp, n1, cx, cy, cs, ra2, prec, p, rec);
  fp.lap(3);
  bool red = false;
  double radSq = 0;
  if (refine) {
    const double density = double(n1) / (dist(rec.x1, rec.y1, rec.x2, rec.y2) * rec.width);
    if (density < 0.7) {
      red = true;
      const double xc = double(x0), yc = double(y0);
      const double radSq1 = distSq(xc, yc, rec.x1, rec.y1);
      const double radSq2 = distSq(xc, yc, rec.x2, rec.y2);
      radSq = radSq1 > radSq2 ? radSq1 : radSq2;
    }
  }
  // reduce_region_radius, one iteration of every reducing lane per pass
  while (__ballot(red)) {
    if (red) radSq *= 0.75 * 0.75;
    int nn = n1;
    for (unsigned long long m = __ballot(red); m; m &= m - 1) {
      const int f = __ffsll((long long)m) - 1;
      const int nf = coop_rl(n1, f), xf = coop_rl(x0, f), yf = coop_rl(y0, f);
      const double rf = coop_rl(radSq, f);
      const LaneBuf g1{coop_rl(gp, f)};
      int c = 0;
      for (int i0 = 0; i0 < nf; i0 += 64) {
        const int i = i0 + lane;
        c += __popcll(__ballot(i < nf && !lane_far(g1.pt(i), xf, yf, rf)));
      }
      if (c < nf) group_merge(S, lane, g1, nf, c, xf, yf, rf);
      if (lane == f) nn = c;
    }
    wg_fence();
    __builtin_amdgcn_wave_barrier();
    const bool merged = red && nn < n1;
    group_centroid(S, lane, merged, gp, nn, nullptr, 0, cx, cy, cs);
    bool tail = false;
    if (red) {
      const int n_prev = n1;
      n1 = nn;
      len = n1;
      if (n1 < 2) {
        status = kSpecFail;
        red = false;
      } else if (n1 != n_prev) {
        tail = true;
      }
    }
    group_rect_tail(S, lane, tail, gp, n1, cx, cy, cs, ra2, prec, p, rec);
    if (tail) {
      const double density = double(n1) / (dist(rec.x1, rec.y1, rec.x2, rec.y2) * rec.width);
      if (density >= 0.7) red = false;
    }
  }
  fp.lap(4);
}


#ifndef ORBPL_SPEC_WIN
#define ORBPL_SPEC_WIN 64
#endif
// the block's first index >= j whose bit is set in the per-wave masks, or n
template <int W>
__device__ __forceinline__ int next_set(const unsigned long long* m, int j, int n) {
#pragma unroll
  for (int w = 0; w < W; w++) {
    if (j >= 64 * (w + 1)) continue;
    const int b = j - 64 * w;
    const unsigned long long r = b <= 0 ? m[w] : (m[w] & ~((1ull << b) - 1ull));
    if (r) return min(n, 64 * w + __ffsll((long long)r) - 1);
  }
  return n;
}
template <int W>
__device__ __forceinline__ void block_sync() {
  if (W == 1) {
    __builtin_amdgcn_wave_barrier();
  } else {
    __syncthreads();
  }
}

template <int W, int MINW = (W == 1 ? ORBPL_SPEC_MINW : 1)>
__global__ void __launch_bounds__(64 * W, MINW) k_lsd_spec(LsdGeom g, LsdScratch sc) {
  constexpr int SL = 64 * W;
  // seeds per round (one-wave variant: ORBPL_SPEC_WIN, an A/B build override)
  constexpr int WIN = W == 1 ? ORBPL_SPEC_WIN : SL;
  constexpr bool KEEP = W == 1;
  extern __shared__ uint32_t grow_smem[];
  __shared__ uint32_t s_pt[SL];
  __shared__ int s_pos[SL];
  __shared__ int s_src[KEEP ? SL : 1];
  __shared__ int s_cnt[2][W];
  __shared__ unsigned long long s_cm[W], s_km[W];
  __shared__ int s_misc[2];   // next_pos, status of the stop seed / nl after a fallback
  __shared__ CoopScratch s_coop[W];
  const int f = blockIdx.x, t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int sw = g.sw, sh = g.sh;
  Frame F;
  F.sw = sw;
  F.sh = sh;
  F.deg = sc.deg + (long long)f * lsd_deg_words(sw, sh);
  F.dtw = lsd_deg_tw(sw);
  F.q = sc.q + (long long)f * sw * sh;
  F.used = nullptr;
  // the cooperative fallback's region list head and prefetch ring live in
  // the (then idle) lane buffers, so LDS holds only the USED bits
  uint4* fbuf = sc.lbuf + (long long)f * SL * kLaneCap;
  uint32_t* coop = reinterpret_cast<uint32_t*>(fbuf);
  F.reg_l = coop;
  F.regq_l = reinterpret_cast<int*>(F.reg_l + kRegLds);
  F.regd_l = reinterpret_cast<float*>(F.regq_l + kRegLds);
  F.ring = F.regd_l + kRegLds;
  F.reg_g = sc.reg + (long long)f * 3 * sw * sh;
  F.rows = reinterpret_cast<int4*>(grow_smem);
  F.rect0 = reinterpret_cast<Rect*>(F.rows);
  F.rect1 = F.rect0 + 1;
  F.row_cap = 0;
  F.log_nt = g.log_nt;
  F.lane = lane;
  F.pf_cyc = 0;
  F.pf_cnt = 0;
  uint64_t* sd = sc.sd + (long long)f * lsd_sd_frame_words(sw, sh);   // stamps unclaimed at launch
  F.usd = sd;
  F.cs = sd + lsd_cs_offset(sw, sh);
  F.tw = lsd_sd_tw(sw);
  int bufid = t;       // this lane's list buffer (KEEP: travels with a carried seed)
  bool keep = false;   // KEEP: the lane's seed, region and fit carried from the last round
  int ncarry = 0;      // KEEP: lanes [0, ncarry) hold carried seeds
  int status = kSpecConflict, off = 0, len = 0, touched = 0;
  Rect rec;
  const uint32_t* A = sc.A + (long long)f * g.n;
  const int nlist = sc.sort_nge[f];   // later list entries are NOTDEF
  double* cand_out = sc.cand + (long long)f * kLsdMaxCand * 12;
  const int w1 = sw - 1;
  const double prec = g.prec, p = g.p;
  const unsigned long long lt_mask = (1ull << lane) - 1ull;
  int nl = 0, pos = 0, it = 0;
  uint32_t round = 0;
#ifdef ORBPL_FIT_PROF
  long long fpr[5] = {0, 0, 0, 0, 0}, fpt[5] = {0, 0, 0, 0, 0};
#endif
  long long n_spec = 0, n_rounds = 0, cyc_spec = 0, cyc_fit = 0, cyc_val = 0, max_steps = 0,
            n_coop = 0;
  const long long t_all = clock64();
  while (pos < nlist || ncarry > 0) {
    const LaneBuf buf{fbuf + (long long)bufid * kLaneCap};
    // ---- the next SL defined, NOTUSED seeds in list order (after the
    // carried ones) ----
    int ncand = ncarry, scan = pos, next_pos = nlist;
    while (ncand < WIN && scan < nlist) {
      const int i = scan + t;
      bool c = false;
      int px = 0, py = 0;
      if (i < nlist) {
        const int idx = (int)(A[i] & 0x3FFFFFu);
        py = idx / w1;
        px = idx - py * w1;
        // one packed load: defined (degrees) and NOTUSED (stamp)
        const uint64_t v = ld_sd(sd + lsd_sd_index(px, py, F.tw));
        c = __uint_as_float((uint32_t)v) >= 0.f && (uint32_t)(v >> 32) != 0u;
      }
      const unsigned long long m = __ballot(c);
      int before = __popcll(m & lt_mask), cnt = __popcll(m);
      if (W > 1) {
        const int par = it++ & 1;   // double-buffered: no barrier before the next write
        if (lane == 0) s_cnt[par][wv] = cnt;
        __syncthreads();
        int off = 0, tot = 0;
#pragma unroll
        for (int w = 0; w < W; w++) {
          const int v = s_cnt[par][w];
          off += w < wv ? v : 0;
          tot += v;
        }
        before += off;
        cnt = tot;
      }
      if (c && ncand + before < WIN) {
        s_pt[ncand + before] = (uint32_t)px | ((uint32_t)py << 16);
        s_pos[ncand + before] = i;
      }
      if (ncand + cnt >= WIN) {
        if (W == 1) {
          const unsigned long long mm = __ballot(c && before == WIN - ncand - 1);
          next_pos = scan + __ffsll((long long)mm);
        } else {
          if (c && before == WIN - ncand - 1) s_misc[0] = i + 1;
          __syncthreads();
          next_pos = s_misc[0];
        }
        ncand = WIN;
      } else {
        ncand += cnt;
        scan += SL;
      }
    }
    if (ncand == 0) break;
    __threadfence_block();
    block_sync<W>();
    n_rounds++;
    n_spec += ncand - (KEEP ? __popcll(__ballot(keep)) : 0);
    // ---- speculative per-lane processing ----
    const long long t0 = clock64();
    // claim tags: a later round's are smaller (stale claims of uncommitted
    // seeds lose to them), an earlier seed's of the same round smaller
    const uint32_t tag = ((0x3FFFFFu - round) << 9) | (uint32_t)t;
    const uint32_t myval0 = (tag << 1) | 1u, myval1 = tag << 1;
    if (!keep) {
      status = kSpecConflict;
      off = 0;
      len = 0;
      touched = 0;
    } else {
      // a carried seed's touched pixels take this round's tag (a USED pixel
      // keeps its 0 and fails the re-check)
      for (int j0 = 0; j0 < touched; j0 += 8) {
        uint32_t ev[8];
#pragma unroll
        for (int u = 0; u < 8; u++) ev[u] = buf[min(j0 + u, touched - 1)].x;
#pragma unroll
        for (int u = 0; u < 8; u++)
          atomicMin(sd_hi(sd, lsd_sd_index((int)(ev[u] & 0xFFFF), (int)(ev[u] >> 16), F.tw)),
                    myval0);
      }
      wg_fence();
    }
    __builtin_amdgcn_wave_barrier();
    double reg_angle = 0;
    int n = 0;
    if (t < ncand && !keep) {
      const uint32_t pt = s_pt[t];
      n = lane_grow(F, sd, buf, kLaneCap, (int)(pt & 0xFFFF), (int)(pt >> 16), reg_angle, prec,
                    myval0);
    }
    __builtin_amdgcn_wave_barrier();
    const long long t1 = clock64();
    {
      int mx = n;
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) mx = max(mx, __shfl_xor(mx, o, 64));
      max_steps += mx;
    }
    {
      // the round's fits: per-lane control flow, wave-wide passes (group_fit)
      const bool mine = t < ncand && !keep;
      if (mine && n < 0) {
        status = n;
      } else if (mine && n < g.min_reg_size) {
        status = kSpecSmall;
        len = n;
        touched = n;
      }
      FitProf fp;
      group_fit(s_coop[wv], lane, mine && n >= g.min_reg_size, n, reg_angle, fbuf, bufid, F, sd,
                prec, p, myval1, status, rec, off, len, touched, fp);
#ifdef ORBPL_FIT_PROF
      for (int k = 0; k < 5; k++) fpr[k] = fp.d[k];
#endif
    }
#ifdef ORBPL_FIT_PROF
#pragma unroll
    for (int k = 0; k < 5; k++) {
      long long v = fpr[k];
      for (int o = 32; o >= 1; o >>= 1) v = max(v, __shfl_xor(v, o, 64));
      fpt[k] += v;
      fpr[k] = 0;
    }
#endif
    wg_fence();
    block_sync<W>();
    const long long t2 = clock64();
    cyc_spec += t1 - t0;
    cyc_fit += t2 - t1;
    // ---- re-read the claims: an earlier seed's smaller stamp = conflict ----
    bool conflict = t < ncand && status < 0;
    if (t < ncand && status >= 0) {
      for (int j0 = 0; j0 < touched && !conflict; j0 += 8) {
        uint32_t ev[8], sv[8];
#pragma unroll
        for (int u = 0; u < 8; u++) ev[u] = buf[min(j0 + u, touched - 1)].x;
#pragma unroll
        for (int u = 0; u < 8; u++)
          sv[u] = ld_stamp(sd, lsd_sd_index((int)(ev[u] & 0xFFFF), (int)(ev[u] >> 16), F.tw));
#pragma unroll
        for (int u = 0; u < 8; u++) conflict |= (sv[u] >> 1) != tag;
      }
    }
    // ---- commit in seed order: seeds [lo, hi) ----
    unsigned long long cmw[W];
    {
      const unsigned long long cm1 = __ballot(conflict);
      if (W == 1) {
        cmw[0] = cm1;
      } else {
        if (lane == 0) s_cm[wv] = cm1;
        __syncthreads();
#pragma unroll
        for (int w = 0; w < W; w++) cmw[w] = s_cm[w];
      }
    }
    int first = next_set<W>(cmw, 0, ncand);
    int lo = 0, hi = first;
    int stop = ncand;
    while (true) {
      const bool mine = t >= lo && t < hi;
      if (mine && len > 0) {
        for (int j0 = off; j0 < off + len; j0 += 8) {
          uint32_t ev[8];
#pragma unroll
          for (int u = 0; u < 8; u++) ev[u] = buf[min(j0 + u, off + len - 1)].x;
#pragma unroll
          for (int u = 0; u < 8; u++) {
            const int id = lsd_sd_index((int)(ev[u] & 0xFFFF), (int)(ev[u] >> 16), F.tw);
            __hip_atomic_store(sd_hi(sd, id), 0u, __ATOMIC_RELAXED, ORBPL_LSD_SCOPE);
          }
        }
      }
      const bool is_cand = mine && status == kSpecCand;
      const unsigned long long cm = __ballot(is_cand);
      int kbefore = __popcll(cm & lt_mask), ktot = __popcll(cm);
      if (W > 1) {
        if (lane == 0) s_km[wv] = cm;
        __syncthreads();
        ktot = 0;
#pragma unroll
        for (int w = 0; w < W; w++) {
          const int v = __popcll(s_km[w]);
          kbefore += w < wv ? v : 0;
          ktot += v;
        }
      }
      if (is_cand) {
        const int k = nl + kbefore;
        if (k < kLsdMaxCand) {
          double* o = cand_out + (long long)k * 12;
          o[0] = rec.x1; o[1] = rec.y1; o[2] = rec.x2; o[3] = rec.y2;
          o[4] = rec.width; o[5] = rec.x; o[6] = rec.y; o[7] = rec.theta;
          o[8] = rec.dx; o[9] = rec.dy; o[10] = rec.prec; o[11] = rec.p;
        }
      }
      nl += ktot;
      __threadfence_block();
      block_sync<W>();
      if (first >= ncand) break;
      const uint32_t spt = s_pt[first];
      if (used_get(F, (int)(spt & 0xFFFF), (int)(spt >> 16))) {
        // covered by a committed region: the sequential loop skips it
        const int nxt = next_set<W>(cmw, first + 1, ncand);
        lo = first + 1;
        hi = nxt;
        first = nxt;
        if (W > 1) __syncthreads();   // every wave has read the USED bit before new stores
        continue;
      }
      stop = first;
      break;
    }
    cyc_val += clock64() - t2;
    bool carry = false;   // KEEP: this round's seeds from `stop` on go to the next one
    if (stop < ncand) {
      pos = s_pos[stop];
      int st_stop;
      if (W == 1) {
        st_stop = __shfl(status, stop, 64);
      } else {
        if (t == stop) s_misc[1] = status;
        __syncthreads();
        st_stop = s_misc[1];
      }
      if (st_stop == kSpecOverflow) {
        // a region longer than a lane buffer: the wave-cooperative program
        // (wave 0; the lane lists it uses as scratch are idle)
        if (wv == 0) {
          const uint32_t spt = s_pt[stop];
          double reg_angle;
          int n = region_grow(F, (int)(spt & 0xFFFF), (int)(spt >> 16), reg_angle, prec);
          if (n >= g.min_reg_size) {
            Rect& rc = *F.rect0;
            fill_q(F, n);
            region2rect(F, n, reg_angle, prec, p, rc);
            if (refine(F, n, reg_angle, prec, p, rc, 0.7)) {
              if (nl < kLsdMaxCand) {
                const double* rv = reinterpret_cast<const double*>(F.rect0);
                if (lane < 12) cand_out[(long long)nl * 12 + lane] = rv[lane];
              }
              nl++;
            }
          }
          if (W > 1 && lane == 0) s_misc[1] = nl;
        }
        if (W > 1) {
          __threadfence_block();
          __syncthreads();
          nl = s_misc[1];
        }
        n_coop++;
        pos++;
      } else if (KEEP) {
        carry = true;
        pos = next_pos;
      }
    } else {
      pos = next_pos;
    }
    if constexpr (KEEP) {
      // carry the seeds from `stop` on (the stopping seed and every later
      // one, kept when its re-check passed; a conflicting one whose seed
      // pixel a committed region now covers is dropped, as the sequential
      // loop skips it) to lanes [0, ncarry) in list order; the other lanes'
      // buffers go to the lanes the scan fills
      bool car = carry && t >= stop && t < ncand;
      const bool kp = car && t > stop && !conflict;
      const uint32_t my_pt = s_pt[t];
      const int my_pos = s_pos[t];
      if (car && !kp && used_get(F, (int)(my_pt & 0xFFFF), (int)(my_pt >> 16))) car = false;
      const unsigned long long cm = __ballot(car);
      const int ncar = __popcll(cm);
      s_src[car ? __popcll(cm & lt_mask) : ncar + __popcll(~cm & lt_mask)] = t;
      __threadfence_block();
      __builtin_amdgcn_wave_barrier();
      const int src = s_src[t];
      keep = __shfl((int)kp, src, 64) != 0 && t < ncar;
      bufid = __shfl(bufid, src, 64);
      status = __shfl(status, src, 64);
      off = __shfl(off, src, 64);
      len = __shfl(len, src, 64);
      touched = __shfl(touched, src, 64);
      rec.x1 = shfl_d(rec.x1, src); rec.y1 = shfl_d(rec.y1, src);
      rec.x2 = shfl_d(rec.x2, src); rec.y2 = shfl_d(rec.y2, src);
      rec.width = shfl_d(rec.width, src); rec.x = shfl_d(rec.x, src);
      rec.y = shfl_d(rec.y, src); rec.theta = shfl_d(rec.theta, src);
      rec.dx = shfl_d(rec.dx, src); rec.dy = shfl_d(rec.dy, src);
      rec.prec = shfl_d(rec.prec, src); rec.p = shfl_d(rec.p, src);
      const uint32_t npt = (uint32_t)__shfl((int)my_pt, src, 64);
      const int npos = __shfl(my_pos, src, 64);
      if (t < ncar) {
        s_pt[t] = npt;
        s_pos[t] = npos;
      }
      ncarry = ncar;
      __threadfence_block();
      __builtin_amdgcn_wave_barrier();
    }
    round++;
    if (W > 1) __syncthreads();   // s_pt / s_pos / s_misc reads done before the next round
  }
  if (t == 0) {
    sc.ncand[f] = min(nl, kLsdMaxCand);
    if (nl > kLsdMaxCand) atomicOr(sc.err + f, 8);
  }
#ifdef ORBPL_FIT_PROF
  if (f == 0 && t == 0)
    printf("fitprof rect1 %lld stats %lld grow2 %lld rect2 %lld reduce %lld (grow %lld fit %lld val %lld)\n",
           fpt[0], fpt[1], fpt[2], fpt[3], fpt[4], cyc_spec, cyc_fit, cyc_val);
#endif
  if (sc.prof && t == 0) {
    long long* pr = sc.prof + f * 8;
    pr[0] = cyc_spec;
    pr[1] = n_rounds;
    pr[2] = n_spec;
    pr[3] = clock64() - t_all;
    pr[4] = cyc_fit;
    pr[5] = cyc_val;
    pr[6] = max_steps | (n_coop << 40);
    pr[7] = nl;
  }
}

// NFA validation of every refined rectangle (rect_improve), one lane per
// rectangle; the accepted segments are compacted in seed order by
// k_lsd_compact.
// workgroups per frame: 8 for small batches (one frame's rectangles spread
// wide), 2 from 1024 frames on (each lane then takes ~3 rectangles from the
// counter: 27.4 -> 24.2 ms per 3072 frames)
#ifndef ORBPL_VAL_BLOCKS_LARGE
#define ORBPL_VAL_BLOCKS_LARGE 2
#endif
constexpr int kValBlocksSmall = 8, kValBlocksLarge = ORBPL_VAL_BLOCKS_LARGE;

#ifndef ORBPL_VAL_MINW
// 6 waves/SIMD (80 VGPRs, the best rectangle in LDS): the same time as 8 (64
// VGPRs) and a third less HBM traffic - 8 spilled doubles to scratch inside
// the phase loop (A/B at 1536 frames, tools/gpu_r04_h.sh: 9.42 vs 9.44 ms,
// 12.3 vs 16.8 MB per frame of FETCH x2 + WRITE; round 3, before the LDS
// slot and the tiled degree plane: 8: 33.1 ms per 3072 frames, 6: 34.5,
// unbounded (111 VGPRs, 4 waves): 39.8)
#define ORBPL_VAL_MINW 6
#endif
// Lanes take rectangles from a workgroup-wide counter (block b owns the
// rectangles c = b (mod gridDim.x)): a lane whose rectangle was cheap takes
// the next one instead of idling until the wave's costliest walk ends (the
// improvement loop runs rect_nfa up to ~25 times on rejected rectangles).
// gridDim.x = workgroups per frame.
// The workgroups of one frame run on one XCD (workgroups are dealt
// round-robin over the 8 XCDs by linear id; the remap gives each XCD a
// contiguous range of frames), so the frame's degree-plane lines one block
// fetched into that XCD's L2 serve its other blocks' walks too.
__global__ void __launch_bounds__(256, ORBPL_VAL_MINW) k_lsd_validate(LsdGeom g, LsdScratch sc) {
  __shared__ int s_next;
  __shared__ double s_rec[256][7];
  const int nx = gridDim.x, nwg = nx * gridDim.y;
  const int orig = blockIdx.x + nx * blockIdx.y;
  const int xcd = orig & 7, qq = nwg >> 3, rr = nwg & 7;
  const int wg = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (orig >> 3);
  const int f = wg / nx, bxv = wg - f * nx;
  const int nc = sc.ncand[f];
  const float* deg = sc.deg + (long long)f * lsd_deg_words(g.sw, g.sh);
  if (threadIdx.x == 0) s_next = 256;
  __syncthreads();
  for (int k = threadIdx.x;; k = atomicAdd(&s_next, 1)) {
    const int c = bxv + k * (int)gridDim.x;
    if (c >= nc) break;
    const long long o = (long long)f * kLsdMaxCand + c;
    const double* rv = sc.cand + o * 12;
    Rect rec;
    rec.x1 = rv[0]; rec.y1 = rv[1]; rec.x2 = rv[2]; rec.y2 = rv[3];
    rec.width = rv[4]; rec.x = rv[5]; rec.y = rv[6]; rec.theta = rv[7];
    rec.dx = rv[8]; rec.dy = rv[9]; rec.prec = rv[10]; rec.p = rv[11];
    const double log_nfa =
        rect_improve_lds(deg, g.sw, g.sh, rec, s_rec[threadIdx.x], g.log_nt, sc.lgam, sc.lgam_n);
    const bool ok = log_nfa > 0;
    sc.cand_ok[o] = ok;
    if (ok) {
      sc.cand_line[o * 4 + 0] = float((rec.x1 + 0.5) / 0.8);
      sc.cand_line[o * 4 + 1] = float((rec.y1 + 0.5) / 0.8);
      sc.cand_line[o * 4 + 2] = float((rec.x2 + 0.5) / 0.8);
      sc.cand_line[o * 4 + 3] = float((rec.y2 + 0.5) / 0.8);
    }
  }
}

__global__ void __launch_bounds__(64) k_lsd_compact(LsdScratch sc) {
  const int f = blockIdx.x, lane = threadIdx.x;
  const int nc = sc.ncand[f];
  float* out = sc.lines + (long long)f * kLsdMaxLines * 4;
  int nl = 0;
  for (int b = 0; b < nc; b += 64) {
    const int c = b + lane;
    const long long o = (long long)f * kLsdMaxCand + c;
    const bool ok = c < nc && sc.cand_ok[o];
    const unsigned long long m = __ballot(ok);
    const int pos = nl + __popcll(m & ((1ull << lane) - 1ull));
    if (ok && pos < kLsdMaxLines) {
      const float4 v = *reinterpret_cast<const float4*>(sc.cand_line + o * 4);
      *reinterpret_cast<float4*>(out + pos * 4) = v;
    }
    nl += __popcll(m);
  }
  if (lane == 0) {
    sc.nlines[f] = min(nl, kLsdMaxLines);
    if (nl > kLsdMaxLines) atomicOr(sc.err + f, 8);
  }
}

__global__ void __launch_bounds__(256) k_lgamma_table(double* t, int n) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) t[i] = log_gamma(double(i) + 1);
}

void launch_lgamma_table(double* t, int n, hipStream_t s) {
  hipLaunchKernelGGL(k_lgamma_table, dim3((n + 255) / 256), dim3(256), 0, s, t, n);
}

void launch_lsd_validate(const LsdGeom& g, const LsdScratch& sc, int batch, hipStream_t s) {
  const int nblk = batch >= 1024 ? kValBlocksLarge : kValBlocksSmall;
  hipLaunchKernelGGL(k_lsd_validate, dim3(nblk, batch), dim3(256), 0, s, g, sc);
  hipLaunchKernelGGL(k_lsd_compact, dim3(batch), dim3(64), 0, s, sc);
}

size_t lsd_grow_smem(const LsdGeom& g) {
  const int used_words = (g.sw * g.sh + 31) / 32;
  return 4 * (size_t)(((used_words + 3 * kRegLds + 64 * 9 + 3) & ~3)) + 2 * sizeof(Rect);
}

void launch_lsd_grow(const LsdGeom& g, const LsdScratch& sc, int batch, hipStream_t s,
                     bool serial) {
  const size_t smem = serial ? lsd_grow_smem(g) : 2 * sizeof(Rect);
  if (serial) {
    if (smem > 65536)
      (void)hipFuncSetAttribute((const void*)k_lsd_grow, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)smem);
    hipLaunchKernelGGL(k_lsd_grow, dim3(batch), dim3(64), smem, s, g, sc);
    return;
  }
  switch (lsd_spec_waves(batch)) {
    case 4: hipLaunchKernelGGL(k_lsd_spec<4>, dim3(batch), dim3(256), smem, s, g, sc); break;
    case 2: hipLaunchKernelGGL(k_lsd_spec<2>, dim3(batch), dim3(128), smem, s, g, sc); break;
    default:
      // few frames leave the GPU mostly idle: the register budget of one wave
      // per SIMD (no spills on the seed chain) instead of the co-residence bound
      static const char* sb_env = getenv("ORBPL_SPEC_SMALL");
      static const int small_batch = sb_env ? atoi(sb_env) : kSpecSmallBatch;
      if (batch <= small_batch)
        hipLaunchKernelGGL((k_lsd_spec<1, 1>), dim3(batch), dim3(64), smem, s, g, sc);
      else
        hipLaunchKernelGGL(k_lsd_spec<1>, dim3(batch), dim3(64), smem, s, g, sc);
      break;
  }
}

}  // namespace orbpl
