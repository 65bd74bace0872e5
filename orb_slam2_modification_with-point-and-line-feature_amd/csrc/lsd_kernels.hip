// LSD line segment detection on gfx950 — LineExtractor::ExtractLineSegment's
// LSDDetector::detect (/root/reference/src/LineExtractor.cpp:20-21; the
// algorithm is OpenCV 3.4's LineSegmentDetectorImpl, restated in
// oracle/lsd_oracle.cpp). One launch per stage covers the whole batch:
//
//   k_lsd_blur    GaussianBlur 7x7 sigma 0.75, 8U fixed point, REFLECT_101
//   k_lsd_resize  resize x0.8, INTER_LINEAR_EXACT (8.8 fixed point)
//   k_lsd_grad    ll_angle: 2x2 gradient, norm, fastAtan2 degrees, max norm
//   k_lsd_sort    the reference's std::sort of pixels by gradient bin,
//                 replayed exactly: libstdc++ introsort with every partition
//                 level executed in parallel (one 1024-thread block / frame)
//   k_lsd_grow    the greedy seed loop (region growing, rectangle fit,
//                 refinement, NFA): one wave per frame, wave-uniform serial
//                 control flow, parallel seed screening and NFA pixel counts
#include <algorithm>
#include <hip/hip_runtime.h>

#include "lsd_kernels.h"
#include "lsd_math.h"
#include "orbpl_math.h"

namespace orbpl {
// region_grow's accumulation terms of a pixel (lsd.cpp region_grow: sumdx +=
// cos(angle), sumdy += sin(angle), float angle; P2 pins correctly rounded
// float cos / sin): (cos | sin << 32), the same expression k_lsd_spec's
// add_angle evaluated per added pixel. NOTDEF pixels are never added.
__device__ __forceinline__ uint64_t lsd_angle_terms(float d) {
  if (d < 0.f) return 0;
  float c, s;
  cr_cos_sin((float)((double)d * (3.14159265358979323846 / 180)), &c, &s);
  return ((uint64_t)__float_as_uint(s) << 32) | (uint64_t)__float_as_uint(c);
}
}  // namespace orbpl

namespace orbpl {

__device__ __forceinline__ int refl101(int i, int n) {
  if (n == 1) return 0;
  while (i < 0 || i >= n) i = i < 0 ? -i : 2 * n - 2 - i;
  return i;
}

// ---------------------------------------------------------------------------
// GaussianBlur (fixed point): 64x32 output tile per 256-thread block; input
// (64+6)x(32+6) staged in LDS, horizontal pass into LDS, vertical to HBM.
// ---------------------------------------------------------------------------
constexpr int kBlTW = 64, kBlTH = 32, kBlR = 3;

__global__ void __launch_bounds__(256) k_lsd_blur(LsdGeom g, const uint8_t* __restrict__ img,
                                                  int stride, long long frame_pitch,
                                                  uint8_t* __restrict__ out) {
  __shared__ uint8_t s_in[kBlTH + 2 * kBlR][kBlTW + 2 * kBlR];
  __shared__ int s_h[kBlTH + 2 * kBlR][kBlTW];
  const int f = blockIdx.z, t = threadIdx.x;
  const int x0 = blockIdx.x * kBlTW, y0 = blockIdx.y * kBlTH;
  const int W = g.W, H = g.H;
  const uint8_t* src = img + (long long)f * frame_pitch;
  for (int i = t; i < (kBlTH + 2 * kBlR) * (kBlTW + 2 * kBlR); i += 256) {
    const int r = i / (kBlTW + 2 * kBlR), c = i - r * (kBlTW + 2 * kBlR);
    const int sy = refl101(y0 + r - kBlR, H), sx = refl101(x0 + c - kBlR, W);
    s_in[r][c] = src[(long long)sy * stride + sx];
  }
  __syncthreads();
  const int n = g.ksize, rr = n / 2;
  for (int i = t; i < (kBlTH + 2 * kBlR) * kBlTW; i += 256) {
    const int r = i / kBlTW, c = i - r * kBlTW;
    int acc = 0;
    for (int j = 0; j < n; j++) acc += g.gk[j] * s_in[r][c + kBlR + j - rr];
    s_h[r][c] = acc;
  }
  __syncthreads();
  uint8_t* dst = out + (long long)f * W * H;
  for (int i = t; i < kBlTH * kBlTW; i += 256) {
    const int r = i / kBlTW, c = i - r * kBlTW;
    const int x = x0 + c, y = y0 + r;
    if (x >= W || y >= H) continue;
    int acc = 0;
    // tile row r holds source row refl101(y0 + r - kBlR)
    for (int j = 0; j < n; j++) acc += g.gk[j] * s_h[r + kBlR + j - rr][c];
    dst[(long long)y * W + x] = (uint8_t)min(255, (acc + (1 << 15)) >> 16);
  }
}

// ---------------------------------------------------------------------------
// resize x0.8 INTER_LINEAR_EXACT. tabs = xofs[sw], xc1[sw], yofs[sh], yc1[sh].
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_lsd_resize(LsdGeom g, const int* __restrict__ tabs,
                                                    const uint8_t* __restrict__ blur,
                                                    uint8_t* __restrict__ scaled) {
  const int f = blockIdx.y;
  const int i = blockIdx.x * 256 + threadIdx.x;
  const int sw = g.sw, sh = g.sh;
  if (i >= sw * sh) return;
  const int dy = i / sw, dx = i - dy * sw;
  const int* xofs = tabs;
  const int* xc1 = tabs + sw;
  const int* yofs = tabs + 2 * sw;
  const int* yc1 = tabs + 2 * sw + sh;
  const uint8_t* S = blur + (long long)f * g.W * g.H;
  auto hval = [&](int sy) -> int {
    const uint8_t* row = S + (long long)sy * g.W;
    if (dx < g.rx0) return row[0] << 8;
    if (dx >= g.rx1) return row[xofs[sw - 1]] << 8;
    const int c1 = xc1[dx], o = xofs[dx];
    return (256 - c1) * row[o] + c1 * row[o + 1];
  };
  int v;
  if (dy < g.ry0 || dy >= g.ry1) {
    v = (hval(dy < g.ry0 ? 0 : g.H - 1) + 0x80) >> 8;
  } else {
    const int b1 = yc1[dy], b0 = 256 - b1, oy = yofs[dy];
    v = (hval(oy) * b0 + hval(oy + 1) * b1 + 0x8000) >> 16;
  }
  scaled[(long long)f * sw * sh + i] = (uint8_t)min(255, v);
}

// ---------------------------------------------------------------------------
// ll_angle: per pixel gx, gy, q = gx^2 + gy^2, degrees (or NOTDEF), max q.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_lsd_grad(LsdGeom g, const uint8_t* __restrict__ scaled,
                                                  float* __restrict__ deg, int* __restrict__ q,
                                                  uint64_t* __restrict__ sd,
                                                  unsigned* __restrict__ maxq) {
  const int f = blockIdx.y;
  const int i = blockIdx.x * 256 + threadIdx.x;
  const int sw = g.sw, sh = g.sh;
  unsigned mq = 0;
  if (i < sw * sh) {
    const int y = i / sw, x = i - y * sw;
    const long long o = (long long)f * sw * sh + i;
    float d = kLsdNotdef;
    int qq = 0;
    if (x < sw - 1 && y < sh - 1) {
      const uint8_t* r0 = scaled + (long long)f * sw * sh + (long long)y * sw;
      const uint8_t* r1 = r0 + sw;
      const int DA = r1[x + 1] - r0[x];
      const int BC = r0[x + 1] - r1[x];
      const int gx = DA + BC, gy = DA - BC;
      qq = gx * gx + gy * gy;
      const double norm = sqrt(qq / 4.0);
      if (norm > g.rho) {
        d = fast_atan2_deg((float)gx, (float)-gy);
        mq = (unsigned)qq;
      }
    }
    deg[(long long)f * lsd_deg_words(sw, sh) + lsd_deg_index(x, y, lsd_deg_tw(sw))] = d;
    q[o] = qq;
    // the speculative seed loop's pixel word: degrees + unclaimed stamp
    uint64_t* fsd = sd + (long long)f * lsd_sd_frame_words(sw, sh);
    const int si = lsd_sd_index(x, y, lsd_sd_tw(sw));
    fsd[si] = (0xFFFFFFFFull << 32) | (uint64_t)__float_as_uint(d);
    fsd[lsd_cs_offset(sw, sh) + si] = lsd_angle_terms(d);
  }
  // block max, one atomic per block
  __shared__ unsigned s_m[4];
  unsigned m = mq;
  for (int o = 32; o >= 1; o >>= 1) m = max(m, (unsigned)__shfl_xor((int)m, o, 64));
  if ((threadIdx.x & 63) == 0) s_m[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned bm = max(max(s_m[0], s_m[1]), max(s_m[2], s_m[3]));
    if (bm) atomicMax(maxq + f, bm);
  }
}

// element e of a wave-uniform array by a 32-bit byte offset (the scalar-base
// + vector-offset addressing form; e * sizeof(T) < 2^32 for every array here)
template <class T>
__device__ __forceinline__ T& ix(T* base, int e) {
  return *reinterpret_cast<T*>(reinterpret_cast<char*>(base) + (uint32_t)e * (uint32_t)sizeof(T));
}

// a * b for operands that fit 16 bits (full-rate v_mul_u32_u24, not the
// quarter-rate v_mul_lo_u32)
__device__ __forceinline__ uint32_t umul16(uint32_t a, uint32_t b) {
  return (uint32_t)(uint16_t)a * (uint32_t)(uint16_t)b;
}

// ---------------------------------------------------------------------------
// k_lsd_prep: k_lsd_blur + k_lsd_resize + k_lsd_grad fused per tile of the
// scaled image (the same integer arithmetic, in the same order): the block's
// source span (rows / columns the resize taps of its kPrTW+1 x kPrTH+1 scaled
// pixels read) is loaded once with the blur halo, blurred in LDS (horizontal
// sums as u16: 255 x 256 fits), resized in LDS, and the gradient of the core
// kPrTW x kPrTH pixels written with the scaled image. The blurred image never
// goes to HBM. The host checks the spans fit (lsdx_create) and the kernel
// size is 7, else the three-kernel path runs.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_lsd_prep(LsdGeom g, const int* __restrict__ tabs,
                                                  const uint8_t* __restrict__ img, int stride,
                                                  long long frame_pitch,
                                                  uint8_t* __restrict__ scaled,
                                                  float* __restrict__ deg, int* __restrict__ q,
                                                  uint64_t* __restrict__ sd,
                                                  unsigned* __restrict__ maxq) {
  __shared__ uint8_t s_in[kPrSR + 2 * kPrR][kPrSC + 2 * kPrR];
  __shared__ uint16_t s_h[kPrSR + 2 * kPrR][kPrSC];
  __shared__ uint8_t s_b[kPrSR][kPrSC];
  __shared__ uint8_t s_s[kPrTH + 1][kPrTW + 4];
  __shared__ int s_xo[kPrTW + 1], s_xc[kPrTW + 1], s_yo[kPrTH + 1], s_yc[kPrTH + 1];
  __shared__ int s_span[4];   // source column min / max, row min / max
  __shared__ unsigned s_m[4];
  const int f = blockIdx.z, t = threadIdx.x;
  const int x0 = blockIdx.x * kPrTW, y0 = blockIdx.y * kPrTH;
  const int W = g.W, H = g.H, sw = g.sw, sh = g.sh;
  const int nx = min(kPrTW + 1, sw - x0), ny = min(kPrTH + 1, sh - y0);
  const int* xofs = tabs;
  const int* xc1 = tabs + sw;
  const int* yofs = tabs + 2 * sw;
  const int* yc1 = tabs + 2 * sw + sh;
  const int xlast = xofs[sw - 1];
  if (t < 4) s_span[t] = (t & 1) ? -1 : 0x7fffffff;
  __syncthreads();
  if (t < nx) {
    const int dx = x0 + t;
    int lo, hi;
    if (dx < g.rx0) lo = hi = 0;
    else if (dx >= g.rx1) lo = hi = xlast;
    else {
      lo = xofs[dx];
      hi = lo + 1;
    }
    s_xo[t] = xofs[dx];
    s_xc[t] = xc1[dx];
    atomicMin(&s_span[0], lo);
    atomicMax(&s_span[1], hi);
  }
  if (t >= 128 && t - 128 < ny) {
    const int i = t - 128, dy = y0 + i;
    int lo, hi;
    if (dy < g.ry0) lo = hi = 0;
    else if (dy >= g.ry1) lo = hi = H - 1;
    else {
      lo = yofs[dy];
      hi = lo + 1;
    }
    s_yo[i] = yofs[dy];
    s_yc[i] = yc1[dy];
    atomicMin(&s_span[2], lo);
    atomicMax(&s_span[3], hi);
  }
  __syncthreads();
  const int sx0 = s_span[0], sy0 = s_span[2];
  const int ncol = s_span[1] - sx0 + 1, nrow = s_span[3] - sy0 + 1;
  // the source span with the blur halo (REFLECT_101 as k_lsd_blur). The
  // passes below map a thread to column t % 128 and rows t / 128 + 2k (every
  // span is at most kPrSC + 2 kPrR < 128 wide): no division per element, and
  // 32-bit offsets from the frame's (uniform) base
  static_assert(kPrSC + 2 * kPrR <= 128 && kPrTW + 1 <= 128, "prep column mapping");
  const uint8_t* src = img + (long long)f * frame_pitch;
  const int icols = ncol + 2 * kPrR, irows = nrow + 2 * kPrR;
  const int tc = t & 127, tr = t >> 7;
  if (tc < icols) {
    const uint32_t sc = (uint32_t)refl101(sx0 + tc - kPrR, W);
    for (int r = tr; r < irows; r += 2)
      s_in[r][tc] = src[umul16((uint32_t)refl101(sy0 + r - kPrR, H), (uint32_t)stride) + sc];
  }
  __syncthreads();
  if (tc < ncol)
    for (int r = tr; r < irows; r += 2) {
      uint32_t acc = 0;
#pragma unroll
      for (int j = 0; j < 2 * kPrR + 1; j++) acc += umul16((uint32_t)g.gk[j], s_in[r][tc + j]);
      s_h[r][tc] = (uint16_t)acc;
    }
  __syncthreads();
  if (tc < ncol)
    for (int r = tr; r < nrow; r += 2) {
      int acc = 0;
#pragma unroll
      for (int j = 0; j < 2 * kPrR + 1; j++) acc += (int)umul16((uint32_t)g.gk[j], s_h[r + j][tc]);
      s_b[r][tc] = (uint8_t)min(255, (acc + (1 << 15)) >> 16);
    }
  __syncthreads();
  // resize (k_lsd_resize's arithmetic) of the scaled tile incl. the +1 halo
  for (int r = tr; tc < nx && r < ny; r += 2) {
    const int c = tc;
    const int dx = x0 + c, dy = y0 + r;
    auto hval = [&](int sy) -> int {
      const uint8_t* row = s_b[sy - sy0];
      if (dx < g.rx0) return row[0 - sx0] << 8;
      if (dx >= g.rx1) return row[xlast - sx0] << 8;
      const int c1 = s_xc[c], o = s_xo[c] - sx0;
      // coefficients <= 256, pixels <= 255: 16-bit operands
      return (int)(umul16((uint32_t)(256 - c1), row[o]) + umul16((uint32_t)c1, row[o + 1]));
    };
    int v;
    if (dy < g.ry0 || dy >= g.ry1) {
      v = (hval(dy < g.ry0 ? 0 : H - 1) + 0x80) >> 8;
    } else {
      const int b1 = s_yc[r], b0 = 256 - b1, oy = s_yo[r];
      v = (int)((umul16((uint32_t)hval(oy), (uint32_t)b0) + umul16((uint32_t)hval(oy + 1), (uint32_t)b1) +
                 0x8000u) >> 16);
    }
    s_s[r][c] = (uint8_t)min(255, v);
  }
  __syncthreads();
  // the scaled image and ll_angle (k_lsd_grad's arithmetic) of the core tile
  unsigned mq = 0;
  const int tw = lsd_sd_tw(sw);
  const int dtw = lsd_deg_tw(sw);
  // the frame's planes (uniform bases) and 32-bit element offsets
  uint8_t* fscaled = scaled + (long long)f * sw * sh;
  int* fq = q + (long long)f * sw * sh;
  float* fdeg = deg + (long long)f * lsd_deg_words(sw, sh);
  uint64_t* fsd = sd + (long long)f * lsd_sd_frame_words(sw, sh);
  const int csw = (int)lsd_cs_offset(sw, sh);
  for (int i = t; i < kPrTH * kPrTW; i += 256) {
    const int r = i / kPrTW, c = i - r * kPrTW;
    const int x = x0 + c, y = y0 + r;
    if (x >= sw || y >= sh) continue;
    const int o = (int)umul16((uint32_t)y, (uint32_t)sw) + x;
    ix(fscaled, o) = s_s[r][c];
    float d = kLsdNotdef;
    int qq = 0;
    if (x < sw - 1 && y < sh - 1) {
      const int DA = s_s[r + 1][c + 1] - s_s[r][c];
      const int BC = s_s[r][c + 1] - s_s[r + 1][c];
      const int gx = DA + BC, gy = DA - BC;
      qq = gx * gx + gy * gy;
      const double norm = sqrt(qq / 4.0);
      if (norm > g.rho) {
        d = fast_atan2_deg((float)gx, (float)-gy);
        mq = max(mq, (unsigned)qq);
      }
    }
    ix(fdeg, lsd_deg_index(x, y, dtw)) = d;
    ix(fq, o) = qq;
    const int si = lsd_sd_index(x, y, tw);
    ix(fsd, si) = (0xFFFFFFFFull << 32) | (uint64_t)__float_as_uint(d);
    ix(fsd, csw + si) = lsd_angle_terms(d);
  }
  unsigned m = mq;
  for (int o = 32; o >= 1; o >>= 1) m = max(m, (unsigned)__shfl_xor((int)m, o, 64));
  if ((t & 63) == 0) s_m[t >> 6] = m;
  __syncthreads();
  if (t == 0) {
    const unsigned bm = max(max(s_m[0], s_m[1]), max(s_m[2], s_m[3]));
    if (bm) atomicMax(maxq + f, bm);
  }
}

// ---------------------------------------------------------------------------
// libstdc++ std::sort replay (introsort, comparator key(a) > key(b)).
//
// Elements are key << 22 | raster index. The recursion of __introsort_loop
// is executed level by level: every active segment (> 16 elements, depth
// left) is partitioned in the same pass. __unguarded_partition on the
// original array is reproduced in closed form: with L_k the k-th position
// (from first+1 upwards) whose key <= pivot and R_k the k-th position (from
// last-1 downwards) whose key >= pivot, the sequential loop swaps pairs
// (L_k, R_k) while L_k < R_k and returns cut = min(L_K, R_{K-1}) for the
// first failing K. Segments whose depth budget is exhausted are heap-sorted
// (std::__partial_sort); the final insertion sort never moves an element
// across a leaf segment, so it is a stable sort of each leaf.
// ---------------------------------------------------------------------------
struct SortPtrs {
  uint32_t* A;
  int *Lpos, *Rpos;
  int4 *seg0, *seg1, *heap;
  int* si;   // 8 arrays of seg_cap
  int* ci;   // 4 arrays of chunk_cap
  int2* leaves;
  uint32_t* leaves_p;   // LDS variant: first | last << 16 (positions < 65536); null = leaves
  int seg_cap, chunk_cap, leaf_cap;
  int* err;
  int4* local;     // segments of <= local_max elements deferred to k_lsd_sort_local
  int* nlocal;
  int local_max;   // 0: partition everything here
  int kt;          // segments whose key bound is < kt hold only NOTDEF pixels
  // the level's stopper ballots by chunk (CH / 64 L then CH / 64 R words per
  // chunk), kept from the count sweep for the scatter sweep so that it does
  // not read the keys again; null or a level above mask_cap chunks: re-read
  unsigned long long* masks;
  int mask_cap;
};

__device__ __forceinline__ int skey(uint32_t e) { return (int)(e >> 22); }

#ifndef ORBPL_SORT_THREADS
#define ORBPL_SORT_THREADS 512
#endif
constexpr int kSortThreads = ORBPL_SORT_THREADS;   // k_lsd_sort's workgroup (A/B build override)
// k_lsd_sort's partition chunk (elements; a multiple of 64, at least
// kLsdSortChunk so that the chunk scratch sized for kLsdSortChunk suffices):
// every lane keeps CH / 64 loads in flight per chunk
#ifndef ORBPL_SORT_CHUNK_G
#define ORBPL_SORT_CHUNK_G 1024
#endif
constexpr int kSortChunkG = ORBPL_SORT_CHUNK_G;
static_assert(kSortChunkG % 64 == 0 && kSortChunkG >= kLsdSortChunk, "sort chunk");
#ifndef ORBPL_SORT_MAP_G
#define ORBPL_SORT_MAP_G 4096
#endif
// segments of one level whose table k_lsd_sort keeps in LDS (more: global)
constexpr int kSortTab = 1024;
// k_lsd_sort's chunk -> segment map capacity (chunks of one level)
constexpr int kSortMapG = ORBPL_SORT_MAP_G;
// batches up to this many frames sort with 1024-thread workgroups
#ifndef ORBPL_SORT_WIDE_BATCH
#define ORBPL_SORT_WIDE_BATCH 256
#endif
constexpr int kSortWideBatch = ORBPL_SORT_WIDE_BATCH;

// Exclusive scan of a[0..len) (global) in place by the whole block; returns
// the total in every thread.
template <int NT>
__device__ __forceinline__ int block_scan_global(int* a, int len, int* s_w) {
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int per = (len + NT - 1) / NT;
  const int b = min(len, t * per), e = min(len, b + per);
  int sum = 0;
  for (int i = b; i < e; i++) sum += a[i];
  int incl = sum;
  for (int o = 1; o < 64; o <<= 1) {
    const int u = __shfl_up(incl, o, 64);
    if (lane >= o) incl += u;
  }
  if (lane == 63) s_w[wave] = incl;
  __syncthreads();
  int off = 0, tot = 0;
  for (int w = 0; w < (NT / 64); w++) {
    const int v = s_w[w];
    if (w < wave) off += v;
    tot += v;
  }
  int run = off + incl - sum;
  for (int i = b; i < e; i++) {
    const int v = a[i];
    a[i] = run;
    run += v;
  }
  __syncthreads();
  return tot;
}

__device__ void move_median_to_first(uint32_t* A, int result, int a, int b, int c) {
  const int ka = skey(A[a]), kb = skey(A[b]), kc = skey(A[c]);
  int m;
  if (ka > kb) {
    if (kb > kc) m = b;
    else if (ka > kc) m = c;
    else m = a;
  } else if (ka > kc) {
    m = a;
  } else if (kb > kc) {
    m = c;
  } else {
    m = b;
  }
  const uint32_t tmp = A[result];
  A[result] = A[m];
  A[m] = tmp;
}

// libstdc++ __adjust_heap / __push_heap with comp = key greater.
__device__ void adjust_heap(uint32_t* A, int hole, int len, uint32_t value) {
  const int top = hole;
  int second = hole;
  while (second < (len - 1) / 2) {
    second = 2 * (second + 1);
    if (skey(A[second]) > skey(A[second - 1])) second--;
    A[hole] = A[second];
    hole = second;
  }
  if ((len & 1) == 0 && second == (len - 2) / 2) {
    second = 2 * (second + 1);
    A[hole] = A[second - 1];
    hole = second - 1;
  }
  int parent = (hole - 1) / 2;
  while (hole > top && skey(A[parent]) > skey(value)) {
    A[hole] = A[parent];
    hole = parent;
    parent = (hole - 1) / 2;
  }
  A[hole] = value;
}

// std::__partial_sort(first, last, last): make_heap + sort_heap.
__device__ void heap_sort_seg(uint32_t* A, int len) {
  if (len < 2) return;
  for (int parent = (len - 2) / 2;; parent--) {
    adjust_heap(A, parent, len, A[parent]);
    if (parent == 0) break;
  }
  for (int last = len; last > 1;) {
    --last;
    const uint32_t v = A[last];
    A[last] = A[0];
    adjust_heap(A, 0, last, v);
  }
}

// Sorts A[first, last) whose introsort depth budget is depth0 (the top
// level: 2 * floor(log2(n))). NT threads, CH elements per partition chunk
// (the decomposition only: any CH gives the same permutation). TAB: a level's
// segment table (first, last, pivot key, first chunk) is copied to LDS so that
// a chunk finds its segment by a binary search in LDS instead of a chain of
// dependent global loads (the global-memory kernel; up to kSortTab segments).
// MAPCAP > 0: a chunk -> segment map (one LDS read per chunk instead of the
// binary search) for levels of at most MAPCAP chunks.
template <int NT, int CH = kLsdSortChunk, bool TAB = false, int MAPCAP = 0>
//
// Segments carry an upper bound of their keys in .w: the right part of a
// partition (keys <= pivot) gets min(bound, pivot key). A segment whose bound
// is below P.kt holds only NOTDEF pixels (ll_angle: key < int(rho *
// bin_coef) implies norm < rho), which the seed loop never takes, so its
// internal order is irrelevant and it is not sorted further; every other
// segment is replayed exactly.
__device__ __forceinline__ void sort_core(const SortPtrs& P, int first0, int last0, int depth0,
                                          int ub0) {
  __shared__ int s_w[(NT / 64)];
  __shared__ int s_nseg, s_next, s_nheap, s_nleaf;
  __shared__ int4 s_tab[TAB ? kSortTab : 1];
  __shared__ uint16_t s_map[MAPCAP > 0 ? MAPCAP : 1];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  uint32_t* A = P.A;
  int* piv = P.si;
  int* choff = P.si + P.seg_cap;
  int* nch = P.si + 2 * P.seg_cap;
  int* sK = P.si + 3 * P.seg_cap;
  int* scut = P.si + 4 * P.seg_cap;
  int* Lc = P.ci;
  int* Rc = P.ci + P.chunk_cap;
  int* Lpre = P.ci + 2 * P.chunk_cap;
  int* Rsuf = P.ci + 3 * P.chunk_cap;
  if (t == 0) {
    s_nheap = 0;
    s_nleaf = 0;
    s_nseg = 0;
    const int n = last0 - first0;
    if (ub0 < P.kt) {
      // nothing to order
    } else if (n > 16) {
      P.seg0[0] = make_int4(first0, last0, depth0, ub0);
      s_nseg = 1;
    } else if (n > 1) {
      if (P.leaves_p) P.leaves_p[0] = (uint32_t)first0 | ((uint32_t)last0 << 16);
      else P.leaves[0] = make_int2(first0, last0);
      s_nleaf = 1;
    }
  }
  __syncthreads();
  int4* cur = P.seg0;
  int4* nxt = P.seg1;
  const unsigned long long below = (1ull << lane) - 1ull;
  while (true) {
    const int nseg = s_nseg;
    if (nseg == 0) break;
    if (t == 0) s_next = 0;
    // R1: median of three into first, pivot key, chunk counts
    for (int s = t; s < nseg; s += NT) {
      const int4 sg = cur[s];
      const int first = sg.x, last = sg.y;
      const int mid = first + (last - first) / 2;
      move_median_to_first(A, first, first + 1, mid, last - 1);
      piv[s] = skey(A[first]);
      nch[s] = (last - first + CH - 1) / CH;
      choff[s] = nch[s];
    }
    __syncthreads();
    const int nchunks = block_scan_global<NT>(choff, nseg, s_w);
    if (nchunks > P.chunk_cap) {
      if (t == 0) *P.err |= 1;
      return;
    }
    const bool tab = TAB && nseg <= kSortTab;
    const bool use_masks =
        P.masks != nullptr && (long long)nchunks * (2 * CH / 64) <= (long long)P.mask_cap * 32 &&
        2 * CH / 64 <= 64;
    const bool map = MAPCAP > 0 && nchunks <= MAPCAP && nseg <= 65536;
    if (tab || map) {
      for (int s = t; s < nseg; s += NT) {
        const int4 sg = cur[s];
        const int c0 = choff[s];
        if (tab) s_tab[s] = make_int4(sg.x, sg.y, piv[s], c0);
        if (map) {
          const int c1 = c0 + (sg.y - sg.x + CH - 1) / CH;
          for (int c = c0; c < c1; c++) s_map[c] = (uint16_t)s;
        }
      }
      __syncthreads();
    }
    // the segment of chunk ch: (first, last, pivot key, first chunk) and its index
    auto seg_of = [&](int ch, int& s) -> int4 {
      int lo = 0, hi = nseg;  // last segment with choff <= ch
      if (map) {
        lo = s_map[ch];
        s = lo;
        if (tab) return s_tab[lo];
        const int4 sg = cur[lo];
        return make_int4(sg.x, sg.y, piv[lo], choff[lo]);
      }
      if (tab) {
        while (hi - lo > 1) {
          const int m = (lo + hi) >> 1;
          if (s_tab[m].w <= ch) lo = m;
          else hi = m;
        }
        s = lo;
        return s_tab[lo];
      }
      while (hi - lo > 1) {
        const int m = (lo + hi) >> 1;
        if (choff[m] <= ch) lo = m;
        else hi = m;
      }
      s = lo;
      const int4 sg = cur[lo];
      return make_int4(sg.x, sg.y, piv[lo], choff[lo]);
    };
    // R3: per chunk L / R stopper counts
    for (int ch = wave; ch < nchunks; ch += (NT / 64)) {
      int s;
      const int4 sq = seg_of(ch, s);
      const int first = sq.x, last = sq.y, p = sq.z;
      const int b = first + (ch - sq.w) * CH;
      const int e = min(b + CH, last);
      int cl = 0, cr = 0;
      unsigned long long myL = 0ull, myR = 0ull;   // lane j: chunk word j's ballots
#pragma unroll
      for (int j = 0; j < CH / 64; j++) {
        const int i = b + j * 64 + lane;
        bool fl = false, fr = false;
        if (i < e) {
          const int k = skey(ix(A, i));
          fl = i > first && k <= p;
          fr = k >= p;
        }
        const unsigned long long bL = __ballot(fl), bR = __ballot(fr);
        cl += __popcll(bL);
        cr += __popcll(bR);
        if (lane == j) {
          myL = bL;
          myR = bR;
        }
      }
      if (use_masks && lane < CH / 64) {
        P.masks[(size_t)ch * (2 * CH / 64) + lane] = myL;
        P.masks[(size_t)ch * (2 * CH / 64) + CH / 64 + lane] = myR;
      }
      if (lane == 0) {
        Lc[ch] = cl;
        Rc[ch] = cr;
        Lpre[ch] = cl;
        Rsuf[ch] = cr;
      }
    }
    __syncthreads();
    block_scan_global<NT>(Lpre, nchunks, s_w);
    const int totR = block_scan_global<NT>(Rsuf, nchunks, s_w);
    for (int c = t; c < nchunks; c += NT) Rsuf[c] = totR - Rsuf[c] - Rc[c];
    __syncthreads();
    // R5: scatter stopper positions by rank
    for (int ch = wave; ch < nchunks; ch += (NT / 64)) {
      int s;
      const int4 sq = seg_of(ch, s);
      const int first = sq.x, last = sq.y, p = sq.z;
      const int c0 = sq.w, c1 = c0 + (last - first + CH - 1) / CH - 1;
      const int b = first + (ch - c0) * CH;
      const int e = min(b + CH, last);
      int runL = Lpre[ch] - Lpre[c0];
      int sufR = Rsuf[ch] - Rsuf[c1];
      // only ranks 0 .. (last - first) / 2 are ever read: K <= n / 2 (the K
      // swap pairs are 2K distinct positions), R6 reads L_K and R_{K-1}
      const int lim = (last - first) >> 1;
      auto scatter_r = [&](unsigned long long m, int j) {
        const int i = b + j * 64 + lane;
        if ((m >> lane) & 1ull) {
          const int k = sufR + __popcll(m & ~(below | (1ull << lane)));
          if (k <= lim) ix(P.Rpos, first + k) = i;
        }
        sufR += __popcll(m);
      };
      auto scatter_l = [&](unsigned long long m, int j) {
        const int i = b + j * 64 + lane;
        const int k = runL + __popcll(m & below);
        if (((m >> lane) & 1ull) && k <= lim) ix(P.Lpos, first + k) = i;
        runL += __popcll(m);
      };
      if (use_masks) {
        // the count sweep's ballots (vector loads: the words are rewritten
        // every level), one word per lane, each broadcast by v_readlane where
        // it is used
        const unsigned long long v =
            lane < 2 * CH / 64 ? P.masks[(size_t)ch * (2 * CH / 64) + lane] : 0ull;
        const int vlo = (int)(uint32_t)v, vhi = (int)(uint32_t)(v >> 32);
        auto word = [&](int w) {
          return (unsigned long long)(uint32_t)__builtin_amdgcn_readlane(vlo, w) |
                 ((unsigned long long)(uint32_t)__builtin_amdgcn_readlane(vhi, w) << 32);
        };
#pragma unroll
        for (int j = CH / 64 - 1; j >= 0; j--) scatter_r(word(CH / 64 + j), j);
#pragma unroll
        for (int j = 0; j < CH / 64; j++) scatter_l(word(j), j);
      } else {
        unsigned long long mL[CH / 64], mR[CH / 64];
#pragma unroll
        for (int j = 0; j < CH / 64; j++) {
          const int i = b + j * 64 + lane;
          bool fl = false, fr = false;
          if (i < e) {
            const int k = skey(ix(A, i));
            fl = i > first && k <= p;
            fr = k >= p;
          }
          mL[j] = __ballot(fl);
          mR[j] = __ballot(fr);
        }
#pragma unroll
        for (int j = CH / 64 - 1; j >= 0; j--) scatter_r(mR[j], j);
#pragma unroll
        for (int j = 0; j < CH / 64; j++) scatter_l(mL[j], j);
      }
    }
    __syncthreads();
    // R6: swap count K and cut per segment
    for (int s = t; s < nseg; s += NT) {
      const int4 sg = cur[s];
      const int first = sg.x, last = sg.y;
      const int c0 = choff[s], c1 = c0 + nch[s] - 1;
      const int nL = Lpre[c1] + Lc[c1] - Lpre[c0];
      const int nR = Rsuf[c0] + Rc[c0] - Rsuf[c1];
      // the first k with L_k >= R_k lies at or below (last - first) / 2 when
      // min(nL, nR) exceeds it (ranks beyond it were not written)
      const int mn = min(nL, nR);
      int lo = 0, hi = min(mn, ((last - first) >> 1) + 1);
      while (lo < hi) {
        const int m = (lo + hi) >> 1;
        if (ix(P.Lpos, first + m) < ix(P.Rpos, first + m)) lo = m + 1;
        else hi = m;
      }
      const int K = lo < min(mn, ((last - first) >> 1) + 1) ? lo : mn;
      int cut = last;
      if (K < nL) cut = min(cut, P.Lpos[first + K]);
      if (K > 0) cut = min(cut, P.Rpos[first + K - 1]);
      sK[s] = K;
      scut[s] = cut;
    }
    __syncthreads();
    // R7: swaps (disjoint pairs)
    for (int ch = wave; ch < nchunks; ch += (NT / 64)) {
      int s;
      const int4 sq = seg_of(ch, s);
      const int first = sq.x;
      const int kb = Lpre[ch] - Lpre[sq.w];
      const int ke = min(kb + Lc[ch], sK[s]);
      // kSwapU x 64 pairs per round: positions, then elements, then stores
      // (one round trip each instead of two per 64 pairs)
      constexpr int kSwapU = 4;
      for (int k0 = kb; k0 < ke; k0 += kSwapU * 64) {
        int pi[kSwapU], pj[kSwapU];
        uint32_t va[kSwapU], vb[kSwapU];
#pragma unroll
        for (int u = 0; u < kSwapU; u++) {
          const int k = min(k0 + u * 64 + lane, ke - 1);
          pi[u] = ix(P.Lpos, first + k);
          pj[u] = ix(P.Rpos, first + k);
        }
#pragma unroll
        for (int u = 0; u < kSwapU; u++) {
          va[u] = ix(A, pi[u]);
          vb[u] = ix(A, pj[u]);
        }
#pragma unroll
        for (int u = 0; u < kSwapU; u++)
          if (k0 + u * 64 + lane < ke) {
            ix(A, pi[u]) = vb[u];
            ix(A, pj[u]) = va[u];
          }
      }
    }
    __syncthreads();
    // R8: children
    for (int s = t; s < nseg; s += NT) {
      const int4 sg = cur[s];
      const int cut = scut[s], d = sg.z - 1;
      const int bs[2] = {cut, sg.x}, es[2] = {sg.y, cut};
      const int ubs[2] = {min(sg.w, piv[s]), sg.w};   // [cut, last): keys <= pivot
      for (int c = 0; c < 2; c++) {
        const int b = bs[c], e = es[c], size = e - b, ub = ubs[c];
        if (ub < P.kt) {
          // only NOTDEF pixels: order irrelevant
        } else if (size > 16) {
          if (d > 0 && size <= P.local_max) {
            const int idx = atomicAdd(P.nlocal, 1);
            if (idx < P.seg_cap) P.local[idx] = make_int4(b, e, d, ub);
            else atomicOr(P.err, 2);
          } else if (d > 0) {
            const int idx = atomicAdd(&s_next, 1);
            if (idx < P.seg_cap) nxt[idx] = make_int4(b, e, d, ub);
            else atomicOr(P.err, 2);
          } else {
            const int idx = atomicAdd(&s_nheap, 1);
            if (idx < P.seg_cap) P.heap[idx] = make_int4(b, e, 0, 0);
            else atomicOr(P.err, 2);
          }
        } else if (size > 1) {
          const int idx = atomicAdd(&s_nleaf, 1);
          if (idx < P.leaf_cap) {
            if (P.leaves_p) P.leaves_p[idx] = (uint32_t)b | ((uint32_t)e << 16);
            else P.leaves[idx] = make_int2(b, e);
          }
          else atomicOr(P.err, 4);
        }
      }
    }
    __syncthreads();
    if (t == 0) s_nseg = min(s_next, P.seg_cap);
    int4* tmp = cur;
    cur = nxt;
    nxt = tmp;
    __syncthreads();
  }
  const int nheap = min(s_nheap, P.seg_cap), nleaf = min(s_nleaf, P.leaf_cap);
  for (int h = t; h < nheap; h += NT) {
    const int4 sg = P.heap[h];
    heap_sort_seg(A + sg.x, sg.y - sg.x);
  }
  for (int l = t; l < nleaf; l += NT) {
    const int2 lf = P.leaves_p ? make_int2((int)(P.leaves_p[l] & 0xFFFFu), (int)(P.leaves_p[l] >> 16))
                               : P.leaves[l];
    for (int i = lf.x + 1; i < lf.y; i++) {
      const uint32_t v = A[i];
      int j = i;
      while (j > lf.x && skey(v) > skey(A[j - 1])) {
        A[j] = A[j - 1];
        j--;
      }
      A[j] = v;
    }
  }
  __syncthreads();
}

__device__ SortPtrs sort_ptrs(const LsdGeom& g, const LsdScratch& sc, int f) {
  SortPtrs P;
  const long long n = g.n;
  P.A = sc.A + f * n;
  P.Lpos = sc.Lpos + f * n;
  P.Rpos = sc.Rpos + f * n;
  P.seg0 = sc.seg0 + (long long)f * g.seg_cap;
  P.seg1 = sc.seg1 + (long long)f * g.seg_cap;
  P.heap = sc.heap + (long long)f * g.seg_cap;
  P.si = sc.seg_i + (long long)f * 8 * g.seg_cap;
  P.ci = sc.chunk_i + (long long)f * 4 * g.chunk_cap;
  P.leaves = sc.leaves + (long long)f * g.leaf_cap;
  P.leaves_p = nullptr;
  P.seg_cap = g.seg_cap;
  P.chunk_cap = g.chunk_cap;
  P.leaf_cap = g.leaf_cap;
  P.err = sc.err + f;
  P.local = sc.sort_local + (long long)f * g.seg_cap;
  P.nlocal = sc.sort_nlocal + f;
  P.local_max = kSortLocalMax;
  P.kt = -(1 << 30);
  P.masks = sc.sort_masks + (long long)f * g.mask_cap * 32;
  P.mask_cap = g.mask_cap;   // in 1024-element chunks (32 words each)
  return P;
}

// The top levels of the introsort run in k_lsd_sort over global memory;
// segments of at most kSortLocalMax elements are finished here, each loaded
// into LDS and sorted by one 256-thread block (same partition replay).
constexpr int kLocalThreads = 256;
constexpr int kLSeg = kSortLocalMax / 17 + 2;
constexpr int kLChunk = kSortLocalMax / kLsdSortChunk + kLSeg + 2;
constexpr int kLLeaf = kSortLocalMax / 2 + 2;
// the local sort's chunk -> segment map (ORBPL_SORT_MAP=0: binary search; the
// map's 264 B fit the 4-blocks-per-CU LDS budget)
#ifndef ORBPL_SORT_MAP
#define ORBPL_SORT_MAP 1
#endif
constexpr int kLocalMap = ORBPL_SORT_MAP ? kLChunk : 0;
constexpr int kSortLocalBlocks = 4;

__global__ void __launch_bounds__(kLocalThreads, 4) k_lsd_sort_local(LsdGeom g, LsdScratch sc) {
  __shared__ uint32_t sA[kSortLocalMax];
  __shared__ int sL[kSortLocalMax], sR[kSortLocalMax];
  __shared__ int4 sseg0[kLSeg], sseg1[kLSeg], sheap[kLSeg];
  __shared__ int ssi[8 * kLSeg];
  __shared__ int sci[4 * kLChunk];
  __shared__ uint32_t sleaves[kLLeaf];   // packed: 40.6 KB of LDS in all, 4 blocks per CU
  const int f = blockIdx.y, t = threadIdx.x;
  uint32_t* A = sc.A + (long long)f * g.n;
  const int nloc = min(sc.sort_nlocal[f], g.seg_cap);
  const int4* loc = sc.sort_local + (long long)f * g.seg_cap;
  SortPtrs L;
  L.A = sA;
  L.Lpos = sL;
  L.Rpos = sR;
  L.seg0 = sseg0;
  L.seg1 = sseg1;
  L.heap = sheap;
  L.si = ssi;
  L.ci = sci;
  L.leaves = nullptr;
  L.leaves_p = sleaves;
  L.seg_cap = kLSeg;
  L.chunk_cap = kLChunk;
  L.leaf_cap = kLLeaf;
  L.err = sc.err + f;
  L.local = nullptr;
  L.nlocal = nullptr;
  L.local_max = 0;
  L.masks = nullptr;
  L.mask_cap = 0;
  L.kt = sc.sort_kt[f];
  for (int k = blockIdx.x; k < nloc; k += gridDim.x) {
    const int4 sg = loc[k];
    const int m = sg.y - sg.x;
    // the segment's loads all in flight at once (m <= kSortLocalMax)
    constexpr int kLU = kSortLocalMax / kLocalThreads;
    uint32_t lv[kLU];
#pragma unroll
    for (int u = 0; u < kLU; u++) lv[u] = A[sg.x + min(t + u * kLocalThreads, m - 1)];
#pragma unroll
    for (int u = 0; u < kLU; u++)
      if (t + u * kLocalThreads < m) sA[t + u * kLocalThreads] = lv[u];
    __syncthreads();
    sort_core<kLocalThreads, kLsdSortChunk, false, kLocalMap>(L, 0, m, sg.z, sg.w);
    for (int i = t; i < m; i += kLocalThreads) A[sg.x + i] = sA[i];
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// k_lsd_sort_wave: the deferred segments (<= kSortLocalMax elements) finished
// by ONE wave each, in its own LDS, with no block barriers. The same replay
// of libstdc++'s introsort as sort_core (median of three into first, the
// closed-form Hoare partition, depth budget -> heap sort, <= 16 -> insertion
// sort of the leaf), organised for a single wave:
//   * a segment of more than 64 elements is scanned in 64-element chunks (all
//     keys loaded at once): one ballot per chunk gives the L stoppers' ranks
//     (bottom-up, the running count in a scalar register), a second pass in
//     reverse chunk order the R stoppers' (top-down); ranks 0 .. n/2 go to two
//     position tables in LDS (K <= n/2), K is the first rank whose L_k >= R_k
//     (64 ranks per ballot), and the K swaps are table-driven; the pending
//     segments are a depth-first stack in LDS (at most one more per level);
//   * a segment of at most 64 elements is sorted entirely in registers, one
//     element per lane (ws_small_sort): every active sub-segment is
//     partitioned in the same pass, and the leaves are ranked stably.
// The level-synchronous sort_core paid ~10 block barriers per level per
// segment for its 256 threads. Exactness: the same permutation
// (tests/test_gpu_lsd.py test_introsort_replica_matches_std_sort, every LSD
// parity test).
// ---------------------------------------------------------------------------
constexpr int kWsStack = 64;    // pending segments (depth-first: <= depth budget + 1)
struct WaveSortLds {
  uint32_t a[kSortLocalMax];
  // L / R stopper position by rank, ranks 0 .. n / 2 (K <= n / 2: the K swap
  // pairs are 2K distinct positions)
  uint16_t lp[kSortLocalMax / 2 + 2], rp[kSortLocalMax / 2 + 2];
  int4 stack[kWsStack];
  uint8_t tl[64], tr[64];   // in-register sort: stopper lane by (segment start + rank)
};

// __unguarded_partition_pivot on S.a[f, l) (l - f > 64): returns the cut;
// *pkey = the pivot key. Every lane returns the same values.
__device__ int ws_partition(WaveSortLds& S, int f, int l, int* pkey, int lane) {
  uint32_t* A = S.a;
  const int n = l - f;
  {
    // std::__move_median_to_first(first, first + 1, mid, last - 1)
    const int a = f + 1, b = f + n / 2, c = l - 1;
    const int ka = skey(A[a]), kb = skey(A[b]), kc = skey(A[c]);
    int m;
    if (ka > kb) {
      if (kb > kc) m = b;
      else if (ka > kc) m = c;
      else m = a;
    } else if (ka > kc) {
      m = a;
    } else if (kb > kc) {
      m = c;
    } else {
      m = b;
    }
    const uint32_t vf = A[f], vm = A[m];
    __syncthreads();
    if (lane == 0) {
      A[f] = vm;
      A[m] = vf;
    }
    *pkey = skey(vm);
    __syncthreads();
  }
  const int p = *pkey;
  const unsigned long long bl = (1ull << lane) - 1ull;
  const unsigned long long ab = ~bl & ~(1ull << lane);   // bits above the lane
  // 64-element chunks, four chunks' key loads in flight per group: L
  // stoppers ranked bottom-up in chunk order, R stoppers top-down in reverse
  // chunk order (a second read of the keys), the running counts in scalar
  // registers; ranks 0 .. lim (positions relative to f) go to the tables
  const int nc = (n + 63) >> 6;
  const int lim = n >> 1;
  int nL = 0, nR = 0;
  for (int c0 = 0; c0 < nc; c0 += 4) {
    int kk[4];
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const int j = f + 64 * (c0 + u) + lane;
      kk[u] = (j < l) ? skey(A[j]) : -1;   // keys are >= 0
    }
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const int c = c0 + u;
      if (c < nc) {
        const int j = f + 64 * c + lane;
        const bool isl = kk[u] >= 0 && j > f && kk[u] <= p;
        const unsigned long long lm = __ballot(isl);
        const int kl = nL + __popcll(lm & bl);
        if (isl && kl <= lim) S.lp[kl] = (uint16_t)(64 * c + lane);
        nL += __popcll(lm);
      }
    }
  }
  for (int c1 = nc - 1; c1 >= 0; c1 -= 4) {
    int kk[4];
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const int j = f + 64 * (c1 - u) + lane;
      kk[u] = (c1 - u >= 0 && j < l) ? skey(A[j]) : -1;
    }
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const int c = c1 - u;
      if (c >= 0) {
        const bool isr = kk[u] >= p;
        const unsigned long long rm = __ballot(isr);
        const int kr = nR + __popcll(rm & ab);
        if (isr && kr <= lim) S.rp[kr] = (uint16_t)(64 * c + lane);
        nR += __popcll(rm);
      }
    }
  }
  const int mn = min(nL, nR);
  __syncthreads();
  // K: the first k with L_k >= R_k (k < mn; it exists below lim + 1 when
  // mn > lim), else mn
  const int kend = min(mn, lim + 1);
  int K = mn;
  for (int k0 = 0; k0 < kend; k0 += 128) {
    const int ka = k0 + lane, kb2 = k0 + 64 + lane;
    const bool fa = ka < kend && S.lp[ka] >= S.rp[ka];
    const bool fb = kb2 < kend && S.lp[kb2] >= S.rp[kb2];
    const unsigned long long Fa = __ballot(fa), Fb = __ballot(fb);
    if (Fa | Fb) {
      K = Fa ? k0 + __builtin_ctzll(Fa) : k0 + 64 + __builtin_ctzll(Fb);
      break;
    }
  }
  int cut = n;
  if (K < nL) cut = min(cut, (int)S.lp[K]);
  if (K > 0) cut = min(cut, (int)S.rp[K - 1]);
  for (int k0 = 0; k0 < K; k0 += 4 * 64) {   // 4 x 64 pairs per round, loads first
    int pi[4], pj[4];
    uint32_t vi[4], vj[4];
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const int k = min(k0 + u * 64 + lane, K - 1);
      pi[u] = f + S.lp[k];
      pj[u] = f + S.rp[k];
    }
#pragma unroll
    for (int u = 0; u < 4; u++) {
      vi[u] = A[pi[u]];
      vj[u] = A[pj[u]];
    }
#pragma unroll
    for (int u = 0; u < 4; u++)
      if (k0 + u * 64 + lane < K) {
        A[pi[u]] = vj[u];
        A[pj[u]] = vi[u];
      }
  }
  __syncthreads();
  return f + cut;
}

// S.a[b, b + n) (n <= 64) sorted entirely in registers, one element per
// lane: every lane carries the bounds [sa, sb) of its current segment, so one
// pass partitions every active segment at once (median of three by three
// lane reads, the pivot swap and the Hoare swaps as lane permutations, the
// stopper ranks by popcounts of the segment-masked ballots, the k-th stopper's
// lane from a rank table in LDS). Leaves (2 .. 16 elements) are then ranked stably in registers
// (the final insertion sort's order); a depth-exhausted segment is heap-sorted
// in LDS by lane 0 afterwards (libstdc++'s partial_sort).
__device__ void ws_small_sort(WaveSortLds& S, int b, int n, int d, int ub, int kt, int lane) {
  const bool in = lane < n;
  uint32_t x = in ? S.a[b + lane] : 0u;
  int sa = 0, sb = n, sd = d, su = ub;
  auto part_of = [&]() { return in && su >= kt && sb - sa > 16 && sd > 0; };
  bool part = part_of();
  while (__ballot(part)) {
    const int nn = sb - sa;
    const int p1 = min(sa + 1, 63), p2 = min(sa + nn / 2, 63), p3 = max(min(sb - 1, 63), 0);
    const int k0 = skey(x);
    const int ka = __shfl(k0, p1, 64), kb = __shfl(k0, p2, 64), kc = __shfl(k0, p3, 64);
    int m, km;
    if (ka > kb) {
      if (kb > kc) { m = p2; km = kb; }
      else if (ka > kc) { m = p3; km = kc; }
      else { m = p1; km = ka; }
    } else if (ka > kc) {
      m = p1; km = ka;
    } else if (kb > kc) {
      m = p3; km = kc;
    } else {
      m = p2; km = kb;
    }
    int src = lane;
    if (part) src = lane == sa ? m : (lane == m ? sa : lane);
    x = (uint32_t)__shfl((int)x, src, 64);
    const int k = skey(x);
    const unsigned long long segm =
        part ? (((nn >= 64 ? ~0ull : ((1ull << nn) - 1ull))) << sa) : 0ull;
    const unsigned long long Ls = __ballot(part && lane > sa && k <= km) & segm;
    const unsigned long long Rs = __ballot(part && k >= km) & segm;
    const unsigned long long bl = (1ull << lane) - 1ull;
    const int nL = __popcll(Ls), nR = __popcll(Rs), mn = min(nL, nR);
    const bool isL = (Ls >> lane) & 1ull, isR = (Rs >> lane) & 1ull;
    const int rkl = __popcll(Ls & bl), rkr = __popcll(Rs & ~bl & ~(1ull << lane));
    // stopper lane by rank: S.tl / S.tr[sa + rank] (segments are disjoint lane ranges)
    if (isL) S.tl[sa + rkl] = (uint8_t)lane;
    if (isR) S.tr[sa + rkr] = (uint8_t)lane;
    __syncthreads();
    const bool hasp = isL && rkl < mn;
    const int partner = hasp ? (int)S.tr[sa + rkl] : 64;   // R_rkl
    const int partL = (isR && rkr < nL) ? (int)S.tl[sa + rkr] : lane;   // L_rkr
    const unsigned long long F = __ballot(hasp && lane >= partner) & segm;
    const int K = F ? __popcll(Ls & ((1ull << __builtin_ctzll(F)) - 1ull)) : mn;
    int cut = sb;
    if (part) {
      if (K < nL) cut = min(cut, (int)S.tl[sa + K]);
      if (K > 0) cut = min(cut, (int)S.tr[sa + K - 1]);
    }
    src = lane;
    if (isL && rkl < K) src = partner;
    if (isR && rkr < K) src = partL;
    __syncthreads();
    x = (uint32_t)__shfl((int)x, src, 64);
    if (part) {
      if (lane >= cut) {
        sa = cut;
        su = min(su, km);   // [cut, last): keys <= pivot
      } else {
        sb = cut;
      }
      sd--;
      part = part_of();
    }
  }
  // leaves: stable rank by key (descending) within [sa, sb)
  const int len = sb - sa;
  const bool leaf = in && su >= kt && len > 1 && len <= 16;
  int dst = lane;
  if (__ballot(leaf)) {
    const int k = skey(x);
    int rank = 0;
    // as many steps as the longest leaf (<= 16), two lane reads per step
    for (int t = 0; __ballot(leaf && t < len); t += 2) {
      const int o0 = min(sa + t, 63), o1 = min(sa + t + 1, 63);
      const int k0 = __shfl(k, o0, 64), k1 = __shfl(k, o1, 64);
      if (leaf && t < len && o0 != lane) rank += (k0 > k) || (k0 == k && o0 < lane);
      if (leaf && t + 1 < len && o1 != lane) rank += (k1 > k) || (k1 == k && o1 < lane);
    }
    if (leaf) dst = sa + rank;
  }
  __syncthreads();
  if (in) S.a[b + dst] = x;
  // depth-exhausted segments (> 16 elements, budget 0): heap sort in LDS
  const unsigned long long H = __ballot(in && su >= kt && len > 16 && sd <= 0 && lane == sa);
  __syncthreads();
  for (unsigned long long h = H; h; h &= h - 1ull) {
    const int a0 = __builtin_ctzll(h);
    const int e0 = __builtin_amdgcn_readlane(sb, a0);
    if (lane == 0) heap_sort_seg(S.a + b + a0, e0 - a0);
  }
  __syncthreads();
}

// Sorts S.a[0, m) as __introsort_loop with depth budget d0 and key bound ub0
// (segments whose bound is below kt hold only NOTDEF pixels: left as they are).
__device__ void ws_sort_segment(WaveSortLds& S, int m, int d0, int ub0, int kt, int lane,
                                int* err) {
  int sp = 0;
  auto add = [&](int b, int e, int d, int ub) {   // uniform
    const int sz = e - b;
    if (ub < kt || sz < 2) return;
    if (sz <= 64) {
      ws_small_sort(S, b, sz, d, ub, kt, lane);
    } else if (d > 0) {
      if (sp < kWsStack) {
        if (lane == 0) S.stack[sp] = make_int4(b, e, d, ub);
        sp++;
      } else if (lane == 0) {
        atomicOr(err, 8);
      }
    } else {
      __syncthreads();
      if (lane == 0) heap_sort_seg(S.a + b, sz);
      __syncthreads();
    }
  };
  add(0, m, d0, ub0);
  while (sp > 0) {
    __syncthreads();
    const int4 e = S.stack[--sp];
    int p;
    const int cut = ws_partition(S, e.x, e.y, &p, lane);
    add(cut, e.y, e.z - 1, min(e.w, p));   // [cut, last): keys <= pivot
    add(e.x, cut, e.z - 1, e.w);
  }
}

__global__ void __launch_bounds__(64) k_lsd_sort_wave(LsdGeom g, LsdScratch sc) {
  __shared__ WaveSortLds S;
  const int f = blockIdx.y, lane = threadIdx.x;
  uint32_t* A = sc.A + (long long)f * g.n;
  const int nloc = min(sc.sort_nlocal[f], g.seg_cap);
  const int4* loc = sc.sort_local + (long long)f * g.seg_cap;
  const int kt = sc.sort_kt[f];
  for (int k = blockIdx.x; k < nloc; k += gridDim.x) {
    const int4 sg = loc[k];
    const int m = sg.y - sg.x;
    for (int i0 = 0; i0 < m; i0 += 8 * 64) {
      uint32_t lv[8];
#pragma unroll
      for (int u = 0; u < 8; u++) lv[u] = A[sg.x + min(i0 + lane + u * 64, m - 1)];
#pragma unroll
      for (int u = 0; u < 8; u++)
        if (i0 + lane + u * 64 < m) S.a[i0 + lane + u * 64] = lv[u];
    }
    __syncthreads();
    ws_sort_segment(S, m, sg.z, sg.w, kt, lane, sc.err + f);
    __syncthreads();
    for (int i = lane; i < m; i += 64) A[sg.x + i] = S.a[i];
    __syncthreads();
  }
}

// waves per SIMD k_lsd_sort's register budget must allow (A/B build override):
// 8 = 64 VGPRs, 4 workgroups of 512 per CU (unbounded, the 1024-element chunks
// take 94). Measured with the LDS segment table (tools/gpu_r04_s.sh, kernel
// time per launch, bit-exact): batch 1 2.39 ms (previous sort) -> 1.68 (1024,
// unbounded) / 1.73 (1024, 8 waves) / 1.80 (512, 8 waves) / 2.06 (256, table
// only); 1536 frames 18.1 -> 15.1 / 12.0 / 12.3 / 17.8 ms; LSD at 3072 frames
// 187.4 -> 172.7 ms (512, 8 waves), lines leg 14.3-14.6k -> 15.2-15.8k frames/s
#ifndef ORBPL_SORT_MINW
#define ORBPL_SORT_MINW 8
#endif
template <int NT>
__global__ void __launch_bounds__(NT, NT >= 1024 ? 4 : ORBPL_SORT_MINW) k_lsd_sort(LsdGeom g, LsdScratch sc) {
  const int f = blockIdx.x;
  SortPtrs P = sort_ptrs(g, sc, f);
  // bins: int(norm * bin_coef), bin_coef = 1023 / max_grad (ll_angle)
  const unsigned mq = sc.maxq[f];
  const double max_grad = mq ? sqrt(mq / 4.0) : -1.0;
  const double bin_coef = max_grad > 0 ? 1023.0 / max_grad : 0.0;
  // key < kt => norm < rho => NOTDEF (both from the same double norm; no
  // defined pixel at all: everything is NOTDEF)
  const int kt = mq ? (int)(g.rho * bin_coef) : 1 << 30;
  P.kt = kt;
  const int sw = g.sw, w1 = g.sw - 1;
  const int* q = sc.q + (long long)f * sw * g.sh;
  __shared__ int s_nge;
  if (threadIdx.x == 0) s_nge = 0;
  __syncthreads();
  int nge = 0;
  // the keys, kU gradient loads of a thread in flight at once
  constexpr int kU = 4;
  for (int i0 = threadIdx.x; i0 < g.n; i0 += NT * kU) {
    int qv[kU];
#pragma unroll
    for (int u = 0; u < kU; u++) {
      const int i = min(i0 + u * NT, g.n - 1);
      const int y = i / w1, x = i - y * w1;
      qv[u] = q[y * sw + x];
    }
#pragma unroll
    for (int u = 0; u < kU; u++) {
      const int i = i0 + u * NT;
      if (i < g.n) {
        const int key = (int)(sqrt(qv[u] / 4.0) * bin_coef);
        P.A[i] = ((uint32_t)key << 22) | (uint32_t)i;
        nge += key >= kt;
      }
    }
  }
  for (int o = 32; o >= 1; o >>= 1) nge += __shfl_xor(nge, o, 64);
  if ((threadIdx.x & 63) == 0 && nge) atomicAdd(&s_nge, nge);
  if (threadIdx.x == 0) *P.nlocal = 0;
  __syncthreads();
  if (threadIdx.x == 0) {
    sc.sort_kt[f] = kt;
    sc.sort_nge[f] = s_nge;
  }
  sort_core<NT, kSortChunkG, true, kSortMapG>(P, 0, g.n, g.n > 16 ? 2 * (31 - __clz(g.n)) : 0,
                                              1023);
}

// test hook: sort caller-provided keys (frame slot 0) with the configuration
// a one-frame batch uses (NT = 1024 threads, LDS segment table and chunk map)
template <int NT>
__global__ void __launch_bounds__(NT) k_lsd_sort_keys(LsdGeom g, LsdScratch sc,
                                                      const int* __restrict__ keys) {
  const SortPtrs P = sort_ptrs(g, sc, 0);
  for (int i = threadIdx.x; i < g.n; i += NT)
    P.A[i] = ((uint32_t)keys[i] << 22) | (uint32_t)i;
  if (threadIdx.x == 0) {
    *P.nlocal = 0;
    sc.sort_kt[0] = P.kt;   // no NOTDEF semantics: sort everything
    sc.sort_nge[0] = g.n;
  }
  __syncthreads();
  sort_core<NT, kSortChunkG, true, kSortMapG>(P, 0, g.n, g.n > 16 ? 2 * (31 - __clz(g.n)) : 0,
                                              1 << 30);
}

void launch_lsd_blur(const LsdGeom& g, const uint8_t* img, int stride, long long frame_pitch,
                     uint8_t* out, int batch, hipStream_t s) {
  dim3 grid((g.W + kBlTW - 1) / kBlTW, (g.H + kBlTH - 1) / kBlTH, batch);
  hipLaunchKernelGGL(k_lsd_blur, grid, dim3(256), 0, s, g, img, stride, frame_pitch, out);
}

void launch_lsd_resize(const LsdGeom& g, const int* tabs, const uint8_t* blur, uint8_t* scaled,
                       int batch, hipStream_t s) {
  hipLaunchKernelGGL(k_lsd_resize, dim3((g.sw * g.sh + 255) / 256, batch), dim3(256), 0, s, g,
                     tabs, blur, scaled);
}

void launch_lsd_prep(const LsdGeom& g, const int* tabs, const uint8_t* img, int stride,
                     long long frame_pitch, uint8_t* scaled, float* deg, int* q, uint64_t* sd,
                     unsigned* maxq, int batch, hipStream_t s) {
  dim3 grid((g.sw + kPrTW - 1) / kPrTW, (g.sh + kPrTH - 1) / kPrTH, batch);
  hipLaunchKernelGGL(k_lsd_prep, grid, dim3(256), 0, s, g, tabs, img, stride, frame_pitch, scaled,
                     deg, q, sd, maxq);
}

void launch_lsd_grad(const LsdGeom& g, const uint8_t* scaled, float* deg, int* q, uint64_t* sd,
                     unsigned* maxq, int batch, hipStream_t s) {
  hipLaunchKernelGGL(k_lsd_grad, dim3((g.sw * g.sh + 255) / 256, batch), dim3(256), 0, s, g,
                     scaled, deg, q, sd, maxq);
}

// workgroups per frame of k_lsd_sort_local: the LDS segments are independent,
// so a small batch spreads a frame's ~50-100 segments over more CUs (batch 1:
// 128 blocks instead of 4, the stage 2.0 ms -> one segment's sort); from 256
// frames on the batch alone fills the GPU
__host__ int lsd_sort_local_blocks(int batch) {
  return std::max(kSortLocalBlocks, std::min(128, 1024 / std::max(batch, 1)));
}
// one-wave workgroups per frame of k_lsd_sort_wave (a frame has ~50-100
// deferred segments): 16 from 512 frames on, up to 128 for small batches
__host__ int lsd_sort_wave_blocks(int batch) {
  return std::max(16, std::min(128, 8192 / std::max(batch, 1)));
}

// the deferred segments: one wave per segment (k_lsd_sort_wave), or the
// 256-thread level-synchronous replay (ORBPL_SORT_WAVE=0, k_lsd_sort_local)
static void launch_lsd_sort_local(const LsdGeom& g, const LsdScratch& sc, int batch,
                                  hipStream_t s) {
  static const char* we = getenv("ORBPL_SORT_WAVE");
  static const bool wave = !(we && we[0] == '0');
  if (wave)
    hipLaunchKernelGGL(k_lsd_sort_wave, dim3(lsd_sort_wave_blocks(batch), batch), dim3(64), 0, s, g,
                       sc);
  else
    hipLaunchKernelGGL(k_lsd_sort_local, dim3(lsd_sort_local_blocks(batch), batch),
                       dim3(kLocalThreads), 0, s, g, sc);
}

void launch_lsd_sort(const LsdGeom& g, const LsdScratch& sc, int batch, hipStream_t s) {
  // a batch that leaves CUs idle: 1024-thread workgroups (twice the chunks in
  // flight per frame); ORBPL_SORT_WIDE_BATCH overrides the batch bound
  static const char* wb_env = getenv("ORBPL_SORT_WIDE_BATCH");
  static const int wide_batch = wb_env ? atoi(wb_env) : kSortWideBatch;
  if (kSortThreads < 1024 && batch <= wide_batch)
    hipLaunchKernelGGL(k_lsd_sort<1024>, dim3(batch), dim3(1024), 0, s, g, sc);
  else
    hipLaunchKernelGGL(k_lsd_sort<kSortThreads>, dim3(batch), dim3(kSortThreads), 0, s, g, sc);
  launch_lsd_sort_local(g, sc, batch, s);
}

void launch_lsd_sort_keys(int n, const int* keys, const LsdScratch& sc, hipStream_t s) {
  LsdGeom g{};
  g.n = n;
  g.seg_cap = n / 17 + 2;
  g.chunk_cap = n / kLsdSortChunk + g.seg_cap + 2;
  g.leaf_cap = n / 2 + 2;
  g.mask_cap = 2 * (n / 1024) + 8;
  if (kSortThreads < 1024 && 1 <= kSortWideBatch)
    hipLaunchKernelGGL(k_lsd_sort_keys<1024>, dim3(1), dim3(1024), 0, s, g, sc, keys);
  else
    hipLaunchKernelGGL(k_lsd_sort_keys<kSortThreads>, dim3(1), dim3(kSortThreads), 0, s, g, sc,
                       keys);
  launch_lsd_sort_local(g, sc, 1, s);
}

}  // namespace orbpl
