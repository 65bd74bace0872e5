// ORB extraction kernels for gfx950 (CDNA4): the MI355X-native replacement of
// ORB_SLAM2::ORBextractor::operator() (src/ORBextractor.cc:1043-1105).
//
// Pipeline per batch of frames (all kernels take the frame index from
// blockIdx.y/z, so one launch covers the whole batch):
//   k_pyramid                  : ComputePyramid (ORBextractor.cc:1107-1132) +
//                                GaussianBlur 7x7 s=2 per level (:1084-1086)
//   k_fast_cells               : per-cell FAST(20) -> FAST(7) fallback (:789-827)
//   k_octree                   : DistributeOctTree (:539-763) + border/octave (:837-847)
//   k_orient_desc              : IC_Angle (:77-104) + computeOrbDescriptor (:108-147)
//                                + level concatenation and pt *= scale (:1075-1104)
// Bit-exactness against the CPU oracle relies on integer arithmetic for every
// image stage and on orbpl_math.h for the two float stages.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <stdint.h>

#include <cstdlib>

#include "orb_geom.h"
#include "orbpl_math.h"
#include "orb_kernels.h"
#include "orbpl_runtime.h"

namespace orbpl {

#include "orb_pattern.inc"
__constant__ int c_pattern[1024];
// the same 256 point pairs as floats (x1, y1, x2, y2): the ints are small,
// so the conversion is exact and the steered coordinates bit-identical
__constant__ float4 c_pattern_f[256];

__device__ __forceinline__ int reflect101_dev(int p, int len) {
  // BORDER_REFLECT_101 for |p| < 2*len (always true for the 19 px border on
  // levels >= 20 px; smaller levels are rejected at create time).
  if (p < 0) p = -p;
  if (p >= len) p = 2 * len - 2 - p;
  return p;
}

// ---------------------------------------------------------------------------
// FAST-9/16 per cell window with per-window 3x3 NMS (cv::FAST semantics on a
// ROI, features2d/fast.cpp FAST_t<16> + cornerScore<16>), threshold
// iniThFAST then minThFAST if the window produced nothing.
//
// For every pixel the kernel computes m = max(A, -B), A/B = max/min over the
// 16 circular 9-arcs of min/max(v - ring). Then, for any threshold t,
//   is_corner_t  <=>  m >= t + 1,   cornerScore_t = m - 1,
// which is exactly what FAST_t emits (see DESIGN.md for the derivation).
// One wave per window, 4 windows per 256-thread block. Candidates are
// written in the reference's row-major emission order into the window's slot.
// ---------------------------------------------------------------------------
// LDS layout of one window (one wave): P[r][q] = pix(a0+q) | pix(a0+q+1) << 16
// for window row r, where a0 = x0 & ~3 (dword-aligned start of the row), so
// one ds_read_b32 gives a ring pixel for two horizontally adjacent centres and
// the 9-arc min/max runs on packed i16 pairs (v_pk_min_i16 / v_pk_max_i16).
// M[r][q] = m(q) | m(q+1) << 16 in the same coordinates, m clamped to [0,255]
// and zero outside the detection region.
//
// 3x3 NMS at threshold t (FAST_t nonmax_suppression on cornerScore = m - 1):
// keep p  <=>  m >= max(t+1, 2)  and  m > max(m of the 8 neighbours).
// (A neighbour n with m_n >= m >= t+1 is itself a corner, so comparing raw m
// values is the same as the reference's comparison of neighbour scores, where
// non-corners score 0.)
// m plane of a FAST window: one u16 per window pixel, rows of fast_pstride
// u16 (a multiple of 8: whole uint4s), then 4 candidate mask words per row
__host__ __device__ constexpr int fast_pstride(int win_w) { return (win_w + 7) & ~7; }
__host__ __device__ constexpr int fast_wave_words(int win_w, int win_h) {
  return win_h * (fast_pstride(win_w) / 2) + 4 * win_h;
}

typedef short fshort2 __attribute__((ext_vector_type(2)));
typedef unsigned short fushort2 __attribute__((ext_vector_type(2)));

// Integer and address helpers for the per-lane index arithmetic.
// a * b for operands that fit 16 bits: the zero / sign extensions let the
// compiler pick the full-rate v_mul_u32_u24 / v_mul_i32_i24 instead of the
// quarter-rate v_mul_lo_u32
__device__ __forceinline__ uint32_t umul24(uint32_t a, uint32_t b) {
  return (uint32_t)(uint16_t)a * (uint32_t)(uint16_t)b;
}
// i / D for i < 2^16 / D (D = 9, 10: exact below 32768 / 16384)
template <uint32_t D>
__device__ __forceinline__ uint32_t div_c16(uint32_t i) {
  return umul24(i, (65536u + D - 1) / D) >> 16;
}
__device__ __forceinline__ int imul24(int a, int b) {
  return (int)(int16_t)a * (int)(int16_t)b;
}
// dword `dw` of a wave-uniform base: the scalar-base + 32-bit vector-offset
// load form, no 64-bit address arithmetic per lane
__device__ __forceinline__ uint32_t ld_dw(const uint32_t* base, uint32_t dw) {
  return *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(base) + (dw << 2));
}
// dwords dw, dw + 1, dw + 2 of a wave-uniform base: one 32-bit offset and
// immediate offsets, so the three loads merge into one dwordx3
__device__ __forceinline__ void ld_dw3(const uint32_t* base, uint32_t dw, uint32_t* a, uint32_t* b,
                                       uint32_t* c) {
  const char* p = reinterpret_cast<const char*>(base) + (dw << 2);
  *a = *reinterpret_cast<const uint32_t*>(p);
  *b = *reinterpret_cast<const uint32_t*>(p + 4);
  *c = *reinterpret_cast<const uint32_t*>(p + 8);
}
// byte `off` of a wave-uniform base as a dword / for a dword store (same form)
__device__ __forceinline__ uint32_t ld_b4(const uint8_t* base, uint32_t off) {
  return *reinterpret_cast<const uint32_t*>(base + off);
}
__device__ __forceinline__ void st_b4(uint8_t* base, uint32_t off, uint32_t v) {
  *reinterpret_cast<uint32_t*>(base + off) = v;
}

__device__ __forceinline__ fshort2 as_s2(uint32_t v) { return __builtin_bit_cast(fshort2, v); }
__device__ __forceinline__ fushort2 as_u2(uint32_t v) { return __builtin_bit_cast(fushort2, v); }
__device__ __forceinline__ fshort2 pmin(fshort2 a, fshort2 b) { return __builtin_elementwise_min(a, b); }
__device__ __forceinline__ fshort2 pmax(fshort2 a, fshort2 b) { return __builtin_elementwise_max(a, b); }
__device__ __forceinline__ fushort2 pmaxu(fushort2 a, fushort2 b) { return __builtin_elementwise_max(a, b); }
__device__ __forceinline__ fushort2 pminu(fushort2 a, fushort2 b) { return __builtin_elementwise_min(a, b); }

// m = max(A, -B) for the centre pair (x, x+1) from a register window: R[k] =
// bytes x-3 .. x+4 of row (centre row + k - 3) as two dwords (.x = bytes
// 0-3, .y = bytes 4-7). A ring pixel at (dx, dy) pairs with its right
// neighbour in one v_perm_b32: (pix(x+dx) | pix(x+1+dx) << 16).
__device__ __forceinline__ uint32_t ring_pair(const uint2* R, int dy, int dx) {
  const uint32_t j = (uint32_t)(3 + dx);
  return __builtin_amdgcn_perm(R[3 + dy].y, R[3 + dy].x, j | (0x0cu << 8) | ((j + 1) << 16) | (0x0cu << 24));
}

// Arc extrema of one side for the 8 windows of 8 ring pixels that start at
// an odd index: W[j] = op(p[2j+1 .. 2j+8]) (indices mod 16). With the halves
// p[0..7], p[8..15], the window from odd j < 8 is suffix(first half, j) +
// prefix(second half, j - 1) and the one from j + 8 the mirror; only odd
// suffixes and even prefixes are needed, and they share the pair ops
// (1,2), (3,4), (5,6) of each half: 9 ops per half + 8 combines.
template <bool kMax>
__device__ __forceinline__ void fast_windows(const fushort2* p, fushort2* W) {
  auto op = [](fushort2 a, fushort2 b) { return kMax ? pmaxu(a, b) : pminu(a, b); };
  fushort2 s[2][4], pr[2][4];   // s[h][i] = suffix from 2i+1, pr[h][i] = prefix to 2i
#pragma unroll
  for (int h = 0; h < 2; h++) {
    const fushort2* d = p + 8 * h;
    const fushort2 q12 = op(d[1], d[2]), q34 = op(d[3], d[4]), q56 = op(d[5], d[6]);
    s[h][3] = d[7];
    s[h][2] = op(q56, d[7]);
    s[h][1] = op(q34, s[h][2]);
    s[h][0] = op(q12, s[h][1]);
    pr[h][0] = d[0];
    pr[h][1] = op(d[0], q12);
    pr[h][2] = op(pr[h][1], q34);
    pr[h][3] = op(pr[h][2], q56);
  }
#pragma unroll
  for (int i = 0; i < 4; i++) {
    W[i] = op(s[0][i], pr[1][i]);       // window from 2i + 1
    W[i + 4] = op(s[1][i], pr[0][i]);   // window from 2i + 9
  }
}

// FAST score m = max(A, -B) of the 16-pixel ring (cv::FAST's cornerScore:
// A = max over the 16 circular 9-arcs of min(v - p), B = min over the arcs of
// max(v - p)) in pixel space: A = v - min_arcs max(p), B = v - max_arcs
// min(p), so no per-pixel differences. Arcs k and k + 1 (k even) share the
// 8-window from k + 1:  min(max arc k, max arc k+1) = max(W[k+1], min(p[k],
// p[k+9])). 98 packed u16 ops for two centres (was 134 with differences).
__device__ __forceinline__ fshort2 fast_m2_regs(const uint2* R) {
  const fushort2 v = as_u2(ring_pair(R, 0, 0));
  fushort2 p[16];
  p[0] = as_u2(ring_pair(R, 3, 0));
  p[1] = as_u2(ring_pair(R, 3, 1));
  p[2] = as_u2(ring_pair(R, 2, 2));
  p[3] = as_u2(ring_pair(R, 1, 3));
  p[4] = as_u2(ring_pair(R, 0, 3));
  p[5] = as_u2(ring_pair(R, -1, 3));
  p[6] = as_u2(ring_pair(R, -2, 2));
  p[7] = as_u2(ring_pair(R, -3, 1));
  p[8] = as_u2(ring_pair(R, -3, 0));
  p[9] = as_u2(ring_pair(R, -3, -1));
  p[10] = as_u2(ring_pair(R, -2, -2));
  p[11] = as_u2(ring_pair(R, -1, -3));
  p[12] = as_u2(ring_pair(R, 0, -3));
  p[13] = as_u2(ring_pair(R, 1, -3));
  p[14] = as_u2(ring_pair(R, 2, -2));
  p[15] = as_u2(ring_pair(R, 3, -1));
  fushort2 Wx[8], Wn[8];
  fast_windows<true>(p, Wx);
  fast_windows<false>(p, Wn);
  // W[i] = window from 2i + 1, shared by arcs 2i and 2i + 1
  fushort2 Ap = pmaxu(Wx[0], pminu(p[0], p[9]));
  fushort2 Bp = pminu(Wn[0], pmaxu(p[0], p[9]));
#pragma unroll
  for (int i = 1; i < 8; i++) {
    const int k = 2 * i;
    Ap = pminu(Ap, pmaxu(Wx[i], pminu(p[k], p[(k + 9) & 15])));
    Bp = pmaxu(Bp, pminu(Wn[i], pmaxu(p[k], p[(k + 9) & 15])));
  }
  const fshort2 zero = {0, 0};
  const fshort2 sv = as_s2(__builtin_bit_cast(uint32_t, v));
  const fshort2 A = sv - as_s2(__builtin_bit_cast(uint32_t, Ap));
  const fshort2 nB = as_s2(__builtin_bit_cast(uint32_t, Bp)) - sv;
  return pmax(pmax(A, nB), zero);
}

// ORBPL_FAST_MM3 (default): the same selections on gfx950's packed 3-input
// v_pk_maximum3_f16 / v_pk_minimum3_f16. A u16 lane holding a pixel value
// 0 .. 255 read as f16 is a subnormal (value x 2^-24), ordered as the
// integers, and IEEE maximum / minimum return one of their inputs bit for bit
// (no NaN can occur, f16 denormals are preserved: the kernel descriptor's
// float_denorm_mode_16_64 is 3), so a 3-input op selects exactly what two
// v_pk_max_u16 / v_pk_min_u16 do. The window extrema fold into 3-input steps,
// the 8-window max/min into the arc step (max3(suffix, prefix, min(p_k,
// p_k+9))) and the arc reduction into 3-input trees: 68 packed ops for two
// centres instead of 98.
#ifndef ORBPL_FAST_MM3
#define ORBPL_FAST_MM3 1
#endif
typedef _Float16 fhalf2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ fhalf2 as_h2(uint32_t v) { return __builtin_bit_cast(fhalf2, v); }
__device__ __forceinline__ fhalf2 hmax(fhalf2 a, fhalf2 b) { return __builtin_elementwise_maximum(a, b); }
__device__ __forceinline__ fhalf2 hmin(fhalf2 a, fhalf2 b) { return __builtin_elementwise_minimum(a, b); }
__device__ __forceinline__ fhalf2 hmax3(fhalf2 a, fhalf2 b, fhalf2 c) { return hmax(hmax(a, b), c); }
__device__ __forceinline__ fhalf2 hmin3(fhalf2 a, fhalf2 b, fhalf2 c) { return hmin(hmin(a, b), c); }

// suffixes from odd starts and prefixes to even ends of both ring halves
// (fast_windows' s / pr) with 3-input ops: 6 per half
template <bool kMax>
__device__ __forceinline__ void fast_sp3(const fhalf2* p, fhalf2 (*s)[4], fhalf2 (*pr)[4]) {
  auto op3 = [](fhalf2 a, fhalf2 b, fhalf2 c) { return kMax ? hmax3(a, b, c) : hmin3(a, b, c); };
#pragma unroll
  for (int h = 0; h < 2; h++) {
    const fhalf2* d = p + 8 * h;
    s[h][3] = d[7];
    s[h][2] = op3(d[5], d[6], d[7]);
    s[h][1] = op3(d[3], d[4], s[h][2]);
    s[h][0] = op3(d[1], d[2], s[h][1]);
    pr[h][0] = d[0];
    pr[h][1] = op3(d[0], d[1], d[2]);
    pr[h][2] = op3(pr[h][1], d[3], d[4]);
    pr[h][3] = op3(pr[h][2], d[5], d[6]);
  }
}

__device__ __forceinline__ fshort2 fast_m2_mm3(const uint2* R) {
  const uint32_t v = ring_pair(R, 0, 0);
  constexpr int kDy[16] = {3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1, 0, 1, 2, 3};
  constexpr int kDx[16] = {0, 1, 2, 3, 3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1};
  fhalf2 p[16];
#pragma unroll
  for (int k = 0; k < 16; k++) p[k] = as_h2(ring_pair(R, kDy[k], kDx[k]));
  fhalf2 sx[2][4], px[2][4], sn[2][4], pn[2][4];
  fast_sp3<true>(p, sx, px);
  fast_sp3<false>(p, sn, pn);
  // arc pair k = 2i, 2i + 1 over the 8-window from 2i + 1: suffix of one half
  // from 2i + 1 (mod 8) and prefix of the other half
  fhalf2 ux[8], un[8];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const int k = 2 * i, h = i < 4 ? 0 : 1, j = i & 3;
    const fhalf2 a = p[k], b = p[(k + 9) & 15];
    ux[i] = hmax3(sx[h][j], px[1 - h][j], hmin(a, b));
    un[i] = hmin3(sn[h][j], pn[1 - h][j], hmax(a, b));
  }
  const fhalf2 Ap = hmin3(hmin3(ux[0], ux[1], ux[2]), hmin3(ux[3], ux[4], ux[5]), hmin(ux[6], ux[7]));
  const fhalf2 Bp = hmax3(hmax3(un[0], un[1], un[2]), hmax3(un[3], un[4], un[5]), hmax(un[6], un[7]));
  const fshort2 zero = {0, 0};
  const fshort2 sv = as_s2(v);
  const fshort2 A = sv - as_s2(__builtin_bit_cast(uint32_t, Ap));
  const fshort2 nB = as_s2(__builtin_bit_cast(uint32_t, Bp)) - sv;
  return pmax(pmax(A, nB), zero);
}

// 8 bytes x-3 .. x+4 of a row from the 3 aligned dwords at byte `off` of a
// wave-uniform base (x-3 = off + o): one 32-bit offset, merged dwordx3 load
__device__ __forceinline__ uint2 load_ring_row(const uint8_t* base, uint32_t off, uint32_t o) {
  const uint8_t* q = base + off;
  const uint32_t w0 = *reinterpret_cast<const uint32_t*>(q);
  const uint32_t w1 = *reinterpret_cast<const uint32_t*>(q + 4);
  const uint32_t w2 = *reinterpret_cast<const uint32_t*>(q + 8);
  return make_uint2(__builtin_amdgcn_alignbyte(w1, w0, o), __builtin_amdgcn_alignbyte(w2, w1, o));
}

// XCD-aware block remap (cdna_hip_programming.md T1): blocks are dealt
// round-robin over the 8 XCDs, so give the blocks that share an XCD a
// contiguous range of the grid (here: the same frames), keeping a frame's
// pyramid re-reads in one XCD's L2. Bijective for any grid size.
__device__ __forceinline__ void xcd_block(int* bx, int* by) {
  const int nx = gridDim.x;
  const int nwg = nx * gridDim.y;
  const int orig = blockIdx.x + nx * blockIdx.y;
  const int xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
  const int wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
  *by = wg / nx;
  *bx = wg - *by * nx;
}

// floor(k / n) by multiply-high: inv = ceil(2^32 / n) for n >= 2 (exact for
// k * n < 2^32), inv = 0 for n == 1.
// (floor((2^32 - 1 + n) / n) = floor((2^32 - 1) / n) + 1: a 32-bit division)
__device__ __forceinline__ uint32_t div_inv(int n) {
  return n > 1 ? 0xFFFFFFFFu / (unsigned)n + 1u : 0u;
}
__device__ __forceinline__ int div_small(int k, uint32_t inv) {
  return inv ? (int)__umulhi((uint32_t)k, inv) : k;
}

// ---------------------------------------------------------------------------
// ComputePyramid (ORBextractor.cc:1107-1132) and the per-level GaussianBlur
// (:1084-1086) in ONE launch. Block (band b, frame f) owns content rows
// [oa, ob) of every level and computes, level after level:
//   1. content rows [na, nb) (own rows plus the halo that the blur and the
//      next level read; host-computed, PyrBand): level 0 = the input image,
//      level l >= 1 = resize(level l-1, INTER_LINEAR) in OpenCV's 8U fixed
//      point (11-bit coefficients, (S>>4)*beta>>16, +2>>2);
//   2. copyMakeBorder(19, REFLECT_101[|ISOLATED]): the 19+19 side pixels of
//      rows [na, nb), then every top/bottom mirror row whose source row lies
//      in [na, nb) (a whole padded row copy);
//   3. the 7x7 sigma=2 blur of the own rows [oa, ob) (pinned P4: out =
//      (sum_v kv sum_u ku I + 2^15) >> 16, k = {18,34,49,54,49,34,18}).
// Resize and blur run as column walks: a thread owns 4 adjacent output
// columns and walks down a row segment, with its resize coefficients (or the
// 7 rows of horizontal blur sums) in registers and the source dwords read
// straight from the just-written level (L1/L2): no LDS staging, three
// barriers per level. Halo rows are computed by both neighbouring bands with
// identical values and every store writes exactly its own bytes, so the
// overlaps are benign.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t byte_of(uint32_t w0, uint32_t w1, uint32_t w2, int p) {
  // byte p (0..11) of the 12-byte little-endian window w0 | w1 | w2
  const uint32_t lo = p < 4 ? w0 : (p < 8 ? w1 : w2);
  return (lo >> (8 * (p & 3))) & 0xFF;
}

// rows per batch of a column walk; each walk keeps two batches of loads in
// flight (registers allow 8 for the blur and 3 for the resize, 2 source
// rows each, within 128 VGPRs: 4 waves per SIMD)
#ifndef ORBPL_PYR_DEPTH
#define ORBPL_PYR_DEPTH 8
#endif
constexpr int kPyrDepth = ORBPL_PYR_DEPTH;        // blur walk
#ifndef ORBPL_PYR_RS_DEPTH
#define ORBPL_PYR_RS_DEPTH 3
#endif
constexpr int kPyrRsDepth = ORBPL_PYR_RS_DEPTH;   // resize walk (2 source rows per row)
// minimum waves per SIMD for k_pyramid (register budget: 4 = 128 VGPRs)
#ifndef ORBPL_PYR_MINW
#define ORBPL_PYR_MINW 4
#endif
// 16-byte loads in flight per thread in the level-0 input copy
#ifndef ORBPL_PYR_COPY_BATCH
#define ORBPL_PYR_COPY_BATCH 8
#endif

// Row segments of a walk (tasks = groups x nseg, rps rows per segment): the
// split with the fewest sequential rows per thread, counting `warm` extra
// rows per segment (the blur's 6 warm-up rows) and idle lanes of the last
// round of tasks. Block-uniform.
__device__ __forceinline__ void walk_split(int groups, int rows, int warm, int* nseg, int* rps) {
  int best = 1, best_cost = 0x7fffffff;
  for (int s = 1; s <= 64 && s <= rows; s++) {
    const int r = (rows + s - 1) / s;
    const int cost = ((groups * s + kPyrThreads - 1) / kPyrThreads) * (r + warm);
    if (cost < best_cost) {
      best_cost = cost;
      best = s;
    }
  }
  *nseg = best;
  *rps = (rows + best - 1) / best;
}

template <bool B>
struct BoolTag {
  static constexpr bool value = B;
};

__device__ __forceinline__ void pyr_resize_rows(const LevelGeom& L, const LevelGeom& S,
                                                const int* __restrict__ rs, uint8_t* fp, int na,
                                                int nb) {
  const int* xofs = rs;
  const int* alpha = rs + L.w;
  const int* yofs = rs + 2 * L.w;
  const int* beta = rs + 2 * L.w + L.h;
  const int groups = (L.w + 3) >> 2;
  int nseg, rps;
  walk_split(groups, nb - na, 2, &nseg, &rps);
  // source dwords and destination bytes as 32-bit offsets from the block's
  // (uniform) level bases
  const uint32_t* src0w = reinterpret_cast<const uint32_t*>(fp + content_off(S, 0, 0));
  const uint32_t spdw = (uint32_t)S.pitch >> 2;
  uint8_t* dst0 = fp + content_off(L, 0, 0);
  for (int task = threadIdx.x; task < groups * nseg; task += kPyrThreads) {
    const int seg = task / groups, gq = task - seg * groups;
    const int ra = na + seg * rps, rb = min(ra + rps, nb);
    const int x = 4 * gq;
    const int d0 = xofs[x] >> 2;                 // first source dword of the group
    // per column: the source pair (sx, sx + 1) as u16x2 by one v_perm from
    // the low (bytes 0-7) or high (bytes 4-11) half of the 12-byte window,
    // weighted by (alpha0, alpha1) in one v_dot2_u32_u16
    uint32_t sel[4];
    bool hiw[4];
    fushort2 cf[4];
    // narrow groups (all 4 pairs within 8 bytes from sx of column x, o = its
    // byte in the first dword; every group at scale factors up to ~2): the
    // window realigned by o (two v_alignbyte per source row) serves all four
    // columns, with no per-column choice of half
    const uint32_t o = (uint32_t)(xofs[x] & 3);
    uint32_t seln[4];
    bool lane_narrow = true;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const int cx = min(x + k, L.w - 1);
      const int p0 = xofs[cx] - 4 * d0;          // byte of sx in the 12-byte window
      hiw[k] = p0 > 6;
      const uint32_t pp = (uint32_t)(hiw[k] ? p0 - 4 : p0);
      sel[k] = pp | (0x0cu << 8) | ((pp + 1) << 16) | (0x0cu << 24);
      const uint32_t pn = (uint32_t)p0 - o;
      lane_narrow = lane_narrow && pn <= 6u;
      seln[k] = pn | (0x0cu << 8) | ((pn + 1) << 16) | (0x0cu << 24);
      if (cx < L.xmax) {
        cf[k] = as_u2((uint32_t)alpha[cx]);      // (alpha0, alpha1), both in [0, 2048]
      } else {
        cf[k] = fushort2{2048, 0};               // sx + 1 >= src width: only sx
      }
    }
    const bool narrow = __ballot(!lane_narrow) == 0ull;   // wave-uniform
    // kPyrRsDepth rows per batch, two batches in flight: the source row
    // indices (yofs) two batches ahead, the source dwords and beta of the next
    // batch, then the current batch's math (rows past rb clamp to rb-1)
    constexpr int D = kPyrRsDepth;
    auto meta = [&](int* sy, int y) {
#pragma unroll
      for (int j = 0; j < D; j++) sy[j] = yofs[min(y + j, rb - 1)];
    };
    auto load = [&](const int* sy, int* bq, uint32_t (*u)[3], uint32_t (*v)[3], int y) {
#pragma unroll
      for (int j = 0; j < D; j++) {
        bq[j] = beta[min(y + j, rb - 1)];
        // uniform base + 32-bit per-lane dword offsets (saddr loads)
        const uint32_t q0 = umul24((uint32_t)min(max(sy[j], 0), S.h - 1), spdw) + (uint32_t)d0;
        const uint32_t q1 = umul24((uint32_t)min(max(sy[j] + 1, 0), S.h - 1), spdw) + (uint32_t)d0;
        ld_dw3(src0w, q0, &u[j][0], &u[j][1], &u[j][2]);
        ld_dw3(src0w, q1, &v[j][0], &v[j][1], &v[j][2]);
      }
    };
    auto work = [&](auto narrow_tag, const int* bq, uint32_t (*u)[3], uint32_t (*v)[3], int y) {
      constexpr bool kNarrow = decltype(narrow_tag)::value;
#pragma unroll
      for (int j = 0; j < D; j++) {
        if (y + j >= rb) break;
        const int b0 = (int)(short)(bq[j] & 0xFFFF), b1 = (int)(short)(bq[j] >> 16);
        uint32_t packed = 0;
        uint32_t ua0 = 0, ua1 = 0, va0 = 0, va1 = 0;
        if constexpr (kNarrow) {
          ua0 = __builtin_amdgcn_alignbyte(u[j][1], u[j][0], o);
          ua1 = __builtin_amdgcn_alignbyte(u[j][2], u[j][1], o);
          va0 = __builtin_amdgcn_alignbyte(v[j][1], v[j][0], o);
          va1 = __builtin_amdgcn_alignbyte(v[j][2], v[j][1], o);
        }
#pragma unroll
        for (int k = 0; k < 4; k++) {
          // alpha1 == 0 at the right edge: the (unused) sx + 1 byte may be border
          uint32_t tu, tv;
          if constexpr (kNarrow) {
            tu = __builtin_amdgcn_perm(ua1, ua0, seln[k]);
            tv = __builtin_amdgcn_perm(va1, va0, seln[k]);
          } else {
            tu = hiw[k] ? __builtin_amdgcn_perm(u[j][2], u[j][1], sel[k])
                        : __builtin_amdgcn_perm(u[j][1], u[j][0], sel[k]);
            tv = hiw[k] ? __builtin_amdgcn_perm(v[j][2], v[j][1], sel[k])
                        : __builtin_amdgcn_perm(v[j][1], v[j][0], sel[k]);
          }
          const int h0 = (int)__builtin_amdgcn_udot2(as_u2(tu), cf[k], 0u, false);
          const int h1 = (int)__builtin_amdgcn_udot2(as_u2(tv), cf[k], 0u, false);
          // beta <= 2048, h >> 4 < 2^16: 24-bit products (v_mul_u32_u24)
          const uint32_t o = (uint32_t)((((int)umul24((uint32_t)b0, (uint32_t)(h0 >> 4)) >> 16) +
                                         ((int)umul24((uint32_t)b1, (uint32_t)(h1 >> 4)) >> 16) + 2) >> 2);
          packed |= o << (8 * k);
        }
        const uint32_t doff = umul24((uint32_t)(y + j), (uint32_t)L.pitch) + (uint32_t)x;
        if (x + 4 <= L.w) {
          st_b4(dst0, doff, packed);
        } else {  // last partial group: the border bytes belong to step 2
          for (int k = 0; k < L.w - x; k++) dst0[doff + k] = (uint8_t)(packed >> (8 * k));
        }
      }
    };
    auto walk = [&](auto narrow_tag) {
      int sa[D], sb[D], ba[D], bb[D];
      uint32_t ua[D][3], va[D][3], ub[D][3], vb[D][3];
      meta(sa, ra);
      meta(sb, ra + D);
      load(sa, ba, ua, va, ra);
      for (int y = ra; y < rb; y += 2 * D) {
        meta(sa, y + 2 * D);
        load(sb, bb, ub, vb, y + D);
        work(narrow_tag, ba, ua, va, y);
        if (y + D >= rb) break;
        meta(sb, y + 3 * D);
        load(sa, ba, ua, va, y + 2 * D);
        work(narrow_tag, bb, ub, vb, y + D);
      }
    };
    if (narrow)
      walk(BoolTag<true>{});
    else
      walk(BoolTag<false>{});
  }
}

// GaussianBlur 7x7, sigma 2, 8U fixed point (cv::GaussianBlur bit-exact
// path): taps 18 34 49 54 49 34 18 (/256) each way, horizontal sums exact
// in u16 (<= 255 * 256), the vertical sum exact in u32, one rounding
// (acc + 2^15) >> 16 (<= 255: no clamp needed).
//
// (b_j, b_j+1) as u16x2 from the 12-byte window w0 | w1 | w2, b_j = byte j+1
template <int j>
__device__ __forceinline__ fushort2 blur_pair(uint32_t w0, uint32_t w1, uint32_t w2) {
  constexpr int i = j + 1;
  if constexpr (i + 1 <= 7)
    return as_u2(__builtin_amdgcn_perm(w1, w0, (uint32_t)(i | (0x0c << 8) | ((i + 1) << 16) | (0x0c << 24))));
  else
    return as_u2(__builtin_amdgcn_perm(w2, w1, (uint32_t)((i - 4) | (0x0c << 8) | ((i - 3) << 16) | (0x0c << 24))));
}

// horizontal 7-tap sums of content columns x .. x+3 from the padded row's
// dwords w0 | w1 | w2 = content columns x-4 .. x+7, packed as 4 x u16
// (packed u16 arithmetic: two columns per instruction)
#ifndef ORBPL_BLUR_DOT4
#define ORBPL_BLUR_DOT4 1
#endif
__device__ __forceinline__ uint2 blur_h4(uint32_t w0, uint32_t w1, uint32_t w2) {
#if ORBPL_BLUR_DOT4
  // one v_dot4_u32_u8 per source dword and output column: column x + j sums
  // bytes j + 1 .. j + 7 of the window with the taps placed at their byte
  // lanes (integer sums: the same values as the packed u16 form below, which
  // needs 9 byte-pair permutes and 14 packed ops per 4 columns, here 10 dot4
  // + 2 packs)
  constexpr uint32_t k0_a = 0x31221200u, k0_b = 0x12223136u;   // j = 0: w0 (-, 18, 34, 49), w1 (54, 49, 34, 18)
  constexpr uint32_t k1_a = 0x22120000u, k1_b = 0x22313631u, k1_c = 0x00000012u;
  constexpr uint32_t k2_a = 0x12000000u, k2_b = 0x31363122u, k2_c = 0x00001222u;
  constexpr uint32_t k3_b = 0x36312212u, k3_c = 0x00122231u;
  const uint32_t h0 = __builtin_amdgcn_udot4(w1, k0_b, __builtin_amdgcn_udot4(w0, k0_a, 0u, false), false);
  const uint32_t h1 = __builtin_amdgcn_udot4(
      w2, k1_c, __builtin_amdgcn_udot4(w1, k1_b, __builtin_amdgcn_udot4(w0, k1_a, 0u, false), false), false);
  const uint32_t h2 = __builtin_amdgcn_udot4(
      w2, k2_c, __builtin_amdgcn_udot4(w1, k2_b, __builtin_amdgcn_udot4(w0, k2_a, 0u, false), false), false);
  const uint32_t h3 = __builtin_amdgcn_udot4(w2, k3_c, __builtin_amdgcn_udot4(w1, k3_b, 0u, false), false);
  // sums <= 255 * 256 < 2^16: pack column pairs as u16x2
  return make_uint2(__builtin_amdgcn_perm(h1, h0, 0x05040100u), __builtin_amdgcn_perm(h3, h2, 0x05040100u));
#else
  const fushort2 P0 = blur_pair<0>(w0, w1, w2), P1 = blur_pair<1>(w0, w1, w2);
  const fushort2 P2 = blur_pair<2>(w0, w1, w2), P3 = blur_pair<3>(w0, w1, w2);
  const fushort2 P4 = blur_pair<4>(w0, w1, w2), P5 = blur_pair<5>(w0, w1, w2);
  const fushort2 P6 = blur_pair<6>(w0, w1, w2), P7 = blur_pair<7>(w0, w1, w2);
  const fushort2 P8 = blur_pair<8>(w0, w1, w2);
  const fushort2 k0 = {18, 18}, k1 = {34, 34}, k2 = {49, 49}, k3 = {54, 54};
  const fushort2 h01 = k0 * (P0 + P6) + k1 * (P1 + P5) + k2 * (P2 + P4) + k3 * P3;
  const fushort2 h23 = k0 * (P2 + P8) + k1 * (P3 + P7) + k2 * (P4 + P6) + k3 * P5;
  return make_uint2(__builtin_bit_cast(uint32_t, h01), __builtin_bit_cast(uint32_t, h23));
#endif
}

// ORBPL_BLUR_VPAIR (default): the vertical taps over ADJACENT-row pairs. The
// horizontal sums of rows r, r+1 of a column packed as u16x2, P_r = (h_r,
// h_r+1), serve three output rows (r+3, r+1, r-1 with tap pairs (18, 34),
// (49, 54), (49, 34)), so each source row costs one v_perm per column
// (P_r+1 from P_r's high half and the new row) and each output row 3
// v_dot2 + 1 v_mad per column: 20 ops per 4 columns instead of the
// symmetric pairing's 12 v_perm + 16 v_dot2 (rows v and 6-v are a new pair for
// every output row). Integer sums, the same values.
#ifndef ORBPL_BLUR_VPAIR
#define ORBPL_BLUR_VPAIR 1
#endif
// horizontal 7-tap sums of content columns x .. x+3, one u32 each (<= 65280)
__device__ __forceinline__ uint4 blur_h4u(uint32_t w0, uint32_t w1, uint32_t w2) {
  constexpr uint32_t k0_a = 0x31221200u, k0_b = 0x12223136u;
  constexpr uint32_t k1_a = 0x22120000u, k1_b = 0x22313631u, k1_c = 0x00000012u;
  constexpr uint32_t k2_a = 0x12000000u, k2_b = 0x31363122u, k2_c = 0x00001222u;
  constexpr uint32_t k3_b = 0x36312212u, k3_c = 0x00122231u;
  uint4 h;
  h.x = __builtin_amdgcn_udot4(w1, k0_b, __builtin_amdgcn_udot4(w0, k0_a, 0u, false), false);
  h.y = __builtin_amdgcn_udot4(w2, k1_c,
                               __builtin_amdgcn_udot4(w1, k1_b, __builtin_amdgcn_udot4(w0, k1_a, 0u, false), false),
                               false);
  h.z = __builtin_amdgcn_udot4(w2, k2_c,
                               __builtin_amdgcn_udot4(w1, k2_b, __builtin_amdgcn_udot4(w0, k2_a, 0u, false), false),
                               false);
  h.w = __builtin_amdgcn_udot4(w2, k3_c, __builtin_amdgcn_udot4(w1, k3_b, 0u, false), false);
  return h;
}
// (h_r, h_r+1) of 4 columns from two rows' sums
__device__ __forceinline__ uint4 blur_pair_rows(uint4 a, uint4 b) {
  constexpr uint32_t kLo = 0x05040100u;   // (a.lo16, b.lo16)
  return make_uint4(__builtin_amdgcn_perm(b.x, a.x, kLo), __builtin_amdgcn_perm(b.y, a.y, kLo),
                    __builtin_amdgcn_perm(b.z, a.z, kLo), __builtin_amdgcn_perm(b.w, a.w, kLo));
}
// P_r+1 from P_r = (h_r, h_r+1) and row r+2's sums
__device__ __forceinline__ uint4 blur_pair_next(uint4 p, uint4 b) {
  constexpr uint32_t kHiLo = 0x05040302u;   // (p.hi16, b.lo16)
  return make_uint4(__builtin_amdgcn_perm(b.x, p.x, kHiLo), __builtin_amdgcn_perm(b.y, p.y, kHiLo),
                    __builtin_amdgcn_perm(b.z, p.z, kHiLo), __builtin_amdgcn_perm(b.w, p.w, kHiLo));
}
// the 4 blurred bytes of output row y from P_y-3, P_y-1, P_y+1 and h_y+3
__device__ __forceinline__ uint32_t blur_vpair4(uint4 pa, uint4 pb, uint4 pc, uint4 h3) {
  const fushort2 ka = {18, 34}, kb = {49, 54}, kc = {49, 34};
  auto col = [&](uint32_t a, uint32_t b, uint32_t c, uint32_t h) __attribute__((always_inline)) {
    uint32_t s = __builtin_amdgcn_udot2(as_u2(a), ka, 1u << 15, false);
    s = __builtin_amdgcn_udot2(as_u2(b), kb, s, false);
    s = __builtin_amdgcn_udot2(as_u2(c), kc, s, false);
    return s + umul24(h, 18u);
  };
  const uint32_t a0 = col(pa.x, pb.x, pc.x, h3.x), a1 = col(pa.y, pb.y, pc.y, h3.y);
  const uint32_t a2 = col(pa.z, pb.z, pc.z, h3.z), a3 = col(pa.w, pb.w, pc.w, h3.w);
  const uint32_t p01 = __builtin_amdgcn_perm(a1, a0, 0x0c0c0602u);   // a0.b2 | a1.b2 << 8
  const uint32_t p23 = __builtin_amdgcn_perm(a3, a2, 0x06020c0cu);   // a2.b2 << 16 | a3.b2 << 24
  return p01 | p23;
}

// vertical 7-tap of one packed word (2 columns) of the ring h[0..6]: rows v
// and 6-v paired into u16x2 (v_perm) and summed with v_dot2_u32_u16
__device__ __forceinline__ void blur_v2(uint32_t h0, uint32_t h1, uint32_t h2, uint32_t h3,
                                        uint32_t h4, uint32_t h5, uint32_t h6, uint32_t* lo,
                                        uint32_t* hi) {
  const fushort2 k0 = {18, 18}, k1 = {34, 34}, k2 = {49, 49};
  const fushort2 kc_lo = {54, 0}, kc_hi = {0, 54};
  constexpr uint32_t kLo = 0x05040100u, kHi = 0x07060302u;   // (a.lo, b.lo), (a.hi, b.hi)
  uint32_t a = __builtin_amdgcn_udot2(as_u2(__builtin_amdgcn_perm(h6, h0, kLo)), k0, 1u << 15, false);
  a = __builtin_amdgcn_udot2(as_u2(__builtin_amdgcn_perm(h5, h1, kLo)), k1, a, false);
  a = __builtin_amdgcn_udot2(as_u2(__builtin_amdgcn_perm(h4, h2, kLo)), k2, a, false);
  a = __builtin_amdgcn_udot2(as_u2(h3), kc_lo, a, false);
  uint32_t b = __builtin_amdgcn_udot2(as_u2(__builtin_amdgcn_perm(h6, h0, kHi)), k0, 1u << 15, false);
  b = __builtin_amdgcn_udot2(as_u2(__builtin_amdgcn_perm(h5, h1, kHi)), k1, b, false);
  b = __builtin_amdgcn_udot2(as_u2(__builtin_amdgcn_perm(h4, h2, kHi)), k2, b, false);
  b = __builtin_amdgcn_udot2(as_u2(h3), kc_hi, b, false);
  *lo = a;
  *hi = b;
}

// the 4 blurred bytes of a ring h[0..6] (byte 2 of each 32-bit sum)
__device__ __forceinline__ uint32_t blur_v4(const uint2* h) {
  uint32_t a0, a1, a2, a3;
  blur_v2(h[0].x, h[1].x, h[2].x, h[3].x, h[4].x, h[5].x, h[6].x, &a0, &a1);
  blur_v2(h[0].y, h[1].y, h[2].y, h[3].y, h[4].y, h[5].y, h[6].y, &a2, &a3);
  const uint32_t p01 = __builtin_amdgcn_perm(a1, a0, 0x0c0c0602u);   // a0.b2 | a1.b2 << 8
  const uint32_t p23 = __builtin_amdgcn_perm(a3, a2, 0x06020c0cu);   // a2.b2 << 16 | a3.b2 << 24
  return p01 | p23;
}

__device__ __forceinline__ void pyr_blur_rows(const LevelGeom& L, const uint8_t* fp, uint8_t* bp,
                                              int oa, int ob) {
  const int G4 = (L.w + 3) >> 2;
  int nseg, rps;
  walk_split(G4, ob - oa, 6, &nseg, &rps);
  for (int task = threadIdx.x; task < G4 * nseg; task += kPyrThreads) {
    const int seg = task / G4, gq = task - seg * G4;
    const int ra = oa + seg * rps, rb = min(ra + rps, ob);
    if (ra >= rb) continue;
    // padded row py holds content column x-4 at byte kContent0 - 4 + x
    // uniform base + 32-bit per-lane offsets (saddr loads: one VGPR per row)
    const uint32_t* col = reinterpret_cast<const uint32_t*>(fp + L.pyr_off);
    const uint32_t c0 = (uint32_t)((kContent0 - 4) / 4 + gq);
    const uint32_t pw = (uint32_t)L.pitch >> 2;
#if ORBPL_BLUR_VPAIR
    // P[k] = P_y-3+k (rows y-3+k, y-2+k) for the next output row y
    uint4 P[5];
    {
      uint4 hp;
#pragma unroll
      for (int v = 0; v < 6; v++) {
        const uint32_t q = umul24((uint32_t)(ra - 3 + v + kEdge), pw) + c0;
        uint32_t a0, a1, a2;
        ld_dw3(col, q, &a0, &a1, &a2);
        const uint4 hv = blur_h4u(a0, a1, a2);
        if (v > 0) P[v - 1] = blur_pair_rows(hp, hv);
        hp = hv;
      }
    }
#else
    uint2 h[7];
#pragma unroll
    for (int v = 0; v < 6; v++) {
      const uint32_t q = umul24((uint32_t)(ra - 3 + v + kEdge), pw) + c0;
      uint32_t a0, a1, a2;
      ld_dw3(col, q, &a0, &a1, &a2);
      h[v + 1] = blur_h4(a0, a1, a2);
    }
#endif
    uint8_t* out = bp + L.boff;                 // uniform; the lane's column 4 gq
    const uint32_t ocol = 4u * (uint32_t)gq;
    // kPyrDepth rows per batch, two batches: the next batch's source dwords
    // are loaded before the current batch's math (rows past rb clamp to rb-1)
    auto load = [&](uint32_t (*w)[3], int y) {
#pragma unroll
      for (int j = 0; j < kPyrDepth; j++) {
        const uint32_t q = umul24((uint32_t)(min(y + j, rb - 1) + 3 + kEdge), pw) + c0;
        ld_dw3(col, q, &w[j][0], &w[j][1], &w[j][2]);
      }
    };
    auto work = [&](uint32_t (*w)[3], int y) {
#pragma unroll
      for (int j = 0; j < kPyrDepth; j++) {
        if (y + j >= rb) break;
#if ORBPL_BLUR_VPAIR
        const uint4 h3 = blur_h4u(w[j][0], w[j][1], w[j][2]);   // row y+j+3
        const uint32_t o = blur_vpair4(P[0], P[2], P[4], h3);
        const uint4 pn = blur_pair_next(P[4], h3);
#pragma unroll
        for (int v = 0; v < 4; v++) P[v] = P[v + 1];
        P[4] = pn;
#else
#pragma unroll
        for (int v = 0; v < 6; v++) h[v] = h[v + 1];
        h[6] = blur_h4(w[j][0], w[j][1], w[j][2]);
        const uint32_t o = blur_v4(h);
#endif
        st_b4(out, umul24((uint32_t)(y + j), (uint32_t)L.bpitch) + ocol, o);
      }
    };
    uint32_t wa[kPyrDepth][3], wb[kPyrDepth][3];
    load(wa, ra);
    for (int y = ra; y < rb; y += 2 * kPyrDepth) {
      load(wb, y + kPyrDepth);
      work(wa, y);
      if (y + kPyrDepth >= rb) break;
      load(wa, y + 2 * kPyrDepth);
      work(wb, y + kPyrDepth);
    }
  }
}

__global__ void __launch_bounds__(kPyrThreads, ORBPL_PYR_MINW) k_pyramid(const uint8_t* __restrict__ img, int stride,
                                                         long long frame_pitch, uint8_t* pyr,
                                                         uint8_t* __restrict__ blur,
                                                         const OrbGeom* __restrict__ g,
                                                         const int* __restrict__ rs_all,
                                                         const PyrBand* __restrict__ bands,
                                                         long long* __restrict__ prof, int l0,
                                                         int l1) {
  const int t = threadIdx.x;
  const int f = blockIdx.y;
  // debug: phase time stamps of block (0, 0) (4 per level after the start)
  const bool stamp = prof && t == 0 && blockIdx.x == 0 && f == 0;
  if (stamp) prof[0] = (long long)wall_clock64();
  const PyrBand& B = bands[blockIdx.x];
  uint8_t* fp = pyr + (long long)f * g->pyr_bytes;
  uint8_t* bp = blur + (long long)f * g->blur_bytes;
  // levels [l0, l1) (one launch per group of levels: the FAST launches of a
  // group's levels run on another stream beside the next group's launch)
  for (int l = l0; l < l1; l++) {
    const LevelGeom& L = g->lv[l];
    const int na = B.na[l], nb = B.nb[l];
    // ---- 1. content rows [na, nb) ----
    if (l == 0) {
      const uint8_t* src = img + (long long)f * frame_pitch;
      const int nv = (L.w + 15) >> 4;
      const uint32_t inv_nv = div_inv(nv);
      const int total = (nb - na) * nv;
      // kCopyBatch 16-byte loads in flight per thread before their stores
      constexpr int kCopyBatch = ORBPL_PYR_COPY_BATCH;
      for (int i0 = t; i0 < total; i0 += kPyrThreads * kCopyBatch) {
        uint4 v[kCopyBatch];
        bool whole[kCopyBatch];
#pragma unroll
        for (int b = 0; b < kCopyBatch; b++) {
          const int i = i0 + b * kPyrThreads;
          const int rr = div_small(i, inv_nv);
          const int r = na + rr, c = (i - rr * nv) * 16;
          const uint8_t* sp = src + (long long)r * stride + c;
          whole[b] = i < total && c + 16 <= L.w && ((reinterpret_cast<uintptr_t>(sp) & 15) == 0);
          v[b] = whole[b] ? *reinterpret_cast<const uint4*>(sp) : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int b = 0; b < kCopyBatch; b++) {
          const int i = i0 + b * kPyrThreads;
          const int rr = div_small(i, inv_nv);
          const int r = na + rr, c = (i - rr * nv) * 16;
          if (whole[b]) *reinterpret_cast<uint4*>(fp + content_off(L, c, r)) = v[b];
        }
        // ragged row ends or an unaligned source: byte copies
#pragma unroll
        for (int b = 0; b < kCopyBatch; b++) {
          const int i = i0 + b * kPyrThreads;
          if (i < total && !whole[b]) {
            const int rr = div_small(i, inv_nv);
            const int r = na + rr, c = (i - rr * nv) * 16;
            uint8_t* d = fp + content_off(L, c, r);
            const uint8_t* sp = src + (long long)r * stride + c;
            const int n = min(16, L.w - c);
            for (int k = 0; k < n; k++) d[k] = sp[k];
          }
        }
      }
    } else {
      pyr_resize_rows(L, g->lv[l - 1], rs_all + L.rs_off, fp, na, nb);
    }
    __syncthreads();
    if (stamp) prof[1 + 4 * l] = (long long)wall_clock64();
    // ---- 2a. side borders of rows [na, nb): thread per (row, side), the 19
    // mirrored bytes (reflect-101: content 19..1 on the left, w-2..w-20 on the
    // right) from aligned dword loads issued together ----
    if (L.w >= kEdge + 2) {
      // row (i >> 1), side (i & 1): padded row and the aligned dword holding
      // the first content byte used (o = its byte in that dword)
      auto side_at = [&](int i, uint8_t** prow, int* o) __attribute__((always_inline)) -> const uint32_t* {
        const int r = na + (i >> 1), side = i & 1;
        *prow = fp + L.pyr_off + (long long)(r + kEdge) * L.pitch;
        const int c0 = side ? L.w - kEdge - 1 : 0;        // first content byte used
        const int a = kContent0 + c0;                     // its byte in the row
        *o = a & 3;
        return reinterpret_cast<const uint32_t*>(*prow + (a & ~3));
      };
      const int ntask = (nb - na) * 2;
      struct Run { uint32_t w[6]; };
      auto side_load = [&](int i) __attribute__((always_inline)) -> Run {
        uint8_t* prow;
        int o;
        const uint32_t* src = side_at(min(i, ntask - 1), &prow, &o);
        Run R;
#pragma unroll
        for (int k = 0; k < 6; k++) R.w[k] = src[k];
        return R;
      };
      auto side_store = [&](int i, Run R) __attribute__((always_inline)) {
        if (i >= ntask) return;
        uint8_t* prow;
        int o;
        side_at(i, &prow, &o);
        // the 20-byte run c0 .. c0+19 realigned to byte 0 (v_alignbyte by o)
        uint32_t A[5];
#pragma unroll
        for (int k = 0; k < 5; k++) A[k] = __builtin_amdgcn_alignbyte(R.w[k + 1], R.w[k], (uint32_t)o);
        auto byte_at = [&](int j) __attribute__((always_inline)) -> uint8_t {
          return (uint8_t)(A[j >> 2] >> (8 * (j & 3)));
        };
        if ((i & 1) == 0) {
#pragma unroll
          for (int px = 0; px < kEdge; px++) prow[kLead + px] = byte_at(kEdge - px);   // content 19 - px
        } else {
#pragma unroll
          for (int k = 0; k < kEdge; k++)                   // content w - 2 - k = c0 + 18 - k
            prow[kLead + L.w + kEdge + k] = byte_at(kEdge - 1 - k);
        }
      };
      // four tasks' loads in flight before their stores
      constexpr int T = kPyrThreads;
      for (int i0 = t; i0 < ntask; i0 += 4 * T) {
        const Run r0 = side_load(i0), r1 = side_load(i0 + T);
        const Run r2 = side_load(i0 + 2 * T), r3 = side_load(i0 + 3 * T);
        side_store(i0, r0);
        side_store(i0 + T, r1);
        side_store(i0 + 2 * T, r2);
        side_store(i0 + 3 * T, r3);
      }
    } else {
      for (int i = t; i < (nb - na) * 2 * kEdge; i += kPyrThreads) {
        const int rr = i / (2 * kEdge), k = i - rr * 2 * kEdge;
        const int r = na + rr;
        const int px = k < kEdge ? k : L.w + k;          // padded column
        const int cx = reflect101_dev(px - kEdge, L.w);
        fp[padded_off(L, px, r + kEdge)] = fp[content_off(L, cx, r)];
      }
    }
    __syncthreads();
    if (stamp) prof[2 + 4 * l] = (long long)wall_clock64();
    // ---- 2b. top / bottom mirror rows with a source row in [na, nb) ----
    {
      const int t0 = max(na, 1), t1 = min(nb, kEdge + 1);               // y = -cy
      const int b0 = max(na, L.h - 1 - kEdge), b1 = min(nb, L.h - 1);   // y = 2h-2-cy
      const int nt = max(0, t1 - t0), nbm = max(0, b1 - b0);
      const int nq = L.pitch >> 4;
      const int ncopy = (nt + nbm) * nq;
      // 16-byte piece i: source (content) and destination (mirror) row offsets
      auto mirror_at = [&](int i, long long* so, long long* dof) __attribute__((always_inline)) {
        const int k = i / nq, q = i - k * nq;
        int cy, py;
        if (k < nt) {
          cy = t0 + k;
          py = kEdge - cy;
        } else {
          cy = b0 + (k - nt);
          py = 2 * L.h - 2 - cy + kEdge;
        }
        *so = L.pyr_off + (long long)(cy + kEdge) * L.pitch + 16 * q;
        *dof = L.pyr_off + (long long)py * L.pitch + 16 * q;
      };
      auto mirror_load = [&](int i) __attribute__((always_inline)) -> uint4 {
        long long so, dof;
        mirror_at(min(i, ncopy - 1), &so, &dof);
        return *reinterpret_cast<const uint4*>(fp + so);
      };
      auto mirror_store = [&](int i, uint4 v) __attribute__((always_inline)) {
        if (i >= ncopy) return;
        long long so, dof;
        mirror_at(i, &so, &dof);
        *reinterpret_cast<uint4*>(fp + dof) = v;
      };
      // four pieces' loads in flight before their stores
      constexpr int T = kPyrThreads;
      for (int i0 = t; i0 < ncopy; i0 += 4 * T) {
        const uint4 v0 = mirror_load(i0), v1 = mirror_load(i0 + T);
        const uint4 v2 = mirror_load(i0 + 2 * T), v3 = mirror_load(i0 + 3 * T);
        mirror_store(i0, v0);
        mirror_store(i0 + T, v1);
        mirror_store(i0 + 2 * T, v2);
        mirror_store(i0 + 3 * T, v3);
      }
    }
    __syncthreads();
    if (stamp) prof[3 + 4 * l] = (long long)wall_clock64();
    // ---- 3. blurred own rows (the next level only reads content rows) ----
    pyr_blur_rows(L, fp, bp, B.oa[l], B.ob[l]);
    if (stamp) prof[4 + 4 * l] = (long long)wall_clock64();
  }
}

// NMS for the centre pair at M[r][q], M[r][q+1]: returns (m_lo, m_hi) in
// *m and the max over each centre's 8 neighbours in *mx.
__device__ __forceinline__ void nms_pair(const uint32_t* M, int ps, int r, int q, fushort2* m,
                                         fushort2* mx) {
  const uint32_t* c = M + r * ps + q;
  *m = as_u2(c[0]);
  fushort2 a = pmaxu(as_u2(c[-1]), as_u2(c[1]));
  a = pmaxu(a, pmaxu(as_u2(c[-ps - 1]), as_u2(c[-ps])));
  a = pmaxu(a, pmaxu(as_u2(c[-ps + 1]), as_u2(c[ps - 1])));
  a = pmaxu(a, pmaxu(as_u2(c[ps]), as_u2(c[ps + 1])));
  *mx = a;
}

__device__ __forceinline__ int wave_incl_scan(int v);

// minimum waves per SIMD for k_fast_cells (register budget); see DESIGN.md
// (6: the MM3 score fit 80 VGPRs without spills; since the DPP neighbours and
// the scalar wave index it takes 71 = 7 waves; 8 fits 63 without spills but
// gains nothing on the headline, profiles/r06/ab/occupancy_fast_pyr_ab.txt)
#ifndef ORBPL_FAST_MINW
#define ORBPL_FAST_MINW 6
#endif
// neighbour pixels of the walk's row from the adjacent lanes by DPP wave
// shifts (1 VALU each) instead of ds_bpermute with per-row lane arithmetic
#ifndef ORBPL_FAST_DPP
#define ORBPL_FAST_DPP 1
#endif
// the ring's next row loaded one row ahead of its use
#ifndef ORBPL_FAST_PREFETCH
#define ORBPL_FAST_PREFETCH 1
#endif
__global__ void __launch_bounds__(256, ORBPL_FAST_MINW) k_fast_cells(const uint8_t* __restrict__ pyr,
                                                    const OrbGeom* __restrict__ g,
                                                    const CellGeom* __restrict__ cells,
                                                    uint32_t* __restrict__ cell_cands,
                                                    int* __restrict__ cell_counts, int ini_th,
                                                    int min_th, int cell0, int cell1) {
  extern __shared__ uint32_t fast_smem[];
  // the wave index as a scalar: the cell, its geometry and the window's row
  // base are then wave-uniform (scalar loads, saddr row loads)
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  int bx, f;
  xcd_block(&bx, &f);
  const int cell = cell0 + bx * 4 + wave;   // cells [cell0, cell1): one group of levels
  if (cell >= cell1) return;
  const CellGeom cg = cells[cell];
  const int slots = g->cell_slots;
  int* cnt_out = cell_counts + (long long)f * g->ncells_total + cell;
  if (cg.x1 == 0) {  // skipped cell (ORBextractor.cc:794-804)
    if (lane == 0) *cnt_out = 0;
    return;
  }
  const int pw = fast_pstride(g->fast_win_w);   // u16 per m-plane row
  const int pw2 = pw >> 1;                      // dwords per row: dword d = pixels (2d, 2d+1)
  uint32_t* M = fast_smem + wave * fast_wave_words(g->fast_win_w, g->fast_win_h);
  // candidate bit masks of detection row r (bit p = column pair p):
  // mask[4 r + j], j = 0 lo / 1 hi pixel at min_th, 2 lo / 3 hi at ini_th
  uint32_t* mask = M + g->fast_win_h * pw2;
  const LevelGeom& L = g->lv[cg.level];
  const int cols = cg.x1 - cg.x0, rows = cg.y1 - cg.y0;
  // zero the window's m (outside the detection region = 0) and the masks
  {
    const int nq = rows * pw2 / 4;
    for (int k = lane; k < nq; k += 64) reinterpret_cast<uint4*>(M)[k] = make_uint4(0, 0, 0, 0);
    for (int k = lane; k < 4 * g->fast_win_h; k += 64) mask[k] = 0;
  }
  __builtin_amdgcn_wave_barrier();
  const int t_ini = max((ini_th < 0 ? 0 : (ini_th > 255 ? 255 : ini_th)) + 1, 2);
  const int t_min = max((min_th < 0 ? 0 : (min_th > 255 ? 255 : min_th)) + 1, 2);
  // ---- m for the detection region rows [3, rows-3), cols [3, cols-3):
  // lane = (column pair p, row segment); each lane walks its rows with the
  // 7 ring rows of its pair in registers, loaded straight from the level.
  // The raw-m NMS (a candidate is a local maximum of m with m >= T; the
  // neighbours' raw m stand in for cv::FAST's thresholded scores, which only
  // differ where m < T <= the centre's) runs in the same walk one row behind:
  // the row above / below come from the lane's own registers, the left / right
  // neighbour pixels from the adjacent lanes. The first and last row of each
  // segment are finished from the m plane in LDS afterwards. ----
  const int dr = rows - 6, dc = cols - 6;
  const int np = (dc + 1) >> 1;
  const uint32_t inv_np = div_inv(np);
  const int npair = (dr > 0 && dc > 0) ? dr * np : 0;
  uint16_t* M16 = reinterpret_cast<uint16_t*>(M);
  int nseg = 1, rps = dr;
  bool any_ini = false;
  if (npair > 0) {
    nseg = max(1, 64 / np);
    rps = (dr + nseg - 1) / nseg;
    const int seg = div_small(lane, inv_np), p = lane - seg * np;
    const bool in_seg = seg < nseg;
    const int ra = in_seg ? seg * rps : 0, rb = in_seg ? min(ra + rps, dr) : 0;
    const int cx = cg.x0 + 3 + 2 * p;                    // content column of the left centre
    const int abase = (cx - 3) & ~3;
    const uint32_t o = (uint32_t)((cx - 3) - abase);
    const uint32_t pitch = (uint32_t)L.pitch;
    // window row w = content row cg.y0 + w; detection row r = window row r + 3;
    // rows as 32-bit byte offsets from the window's (uniform) first row
    const uint8_t* wrow = pyr + (long long)f * g->pyr_bytes + content_off(L, 0, cg.y0);
    const uint32_t acol = (uint32_t)abase;
    const bool has_hi = 2 * p + 1 < dc;
    const bool has_left = p > 0, has_right = p + 1 < np;
    const uint32_t pbit = 1u << p;
    uint2 R[7];
    if (in_seg) {
#pragma unroll
      for (int k = 0; k < 6; k++) R[k + 1] = load_ring_row(wrow, umul24((uint32_t)(ra + k), pitch) + acol, o);
    }
    // rows r-1, r-2 of the walk: packed m, 3-wide row max, centre-excluded max
    uint32_t m1 = 0, rmax1 = 0, rmax2 = 0, cmax1 = 0;
    const int nit = __builtin_amdgcn_readfirstlane(rps);   // the longest segment
#if ORBPL_FAST_PREFETCH
    // the next ring row's dwords are loaded one row ahead
    uint32_t nw0 = 0, nw1 = 0, nw2 = 0;
    auto ring_raw = [&](int row) __attribute__((always_inline)) {
      const uint8_t* q = wrow + (umul24((uint32_t)row, pitch) + acol);
      nw0 = *reinterpret_cast<const uint32_t*>(q);
      nw1 = *reinterpret_cast<const uint32_t*>(q + 4);
      nw2 = *reinterpret_cast<const uint32_t*>(q + 8);
    };
    if (in_seg && ra < rb) ring_raw(ra + 6);
#endif
    for (int i = 0; i < nit; i++) {
      const int r = ra + i;
      const bool act = r < rb;
      uint32_t m = 0;
      if (act) {
#pragma unroll
        for (int k = 0; k < 6; k++) R[k] = R[k + 1];
#if ORBPL_FAST_PREFETCH
        R[6] = make_uint2(__builtin_amdgcn_alignbyte(nw1, nw0, o), __builtin_amdgcn_alignbyte(nw2, nw1, o));
        if (r + 1 < rb) ring_raw(r + 7);
#else
        R[6] = load_ring_row(wrow, umul24((uint32_t)(r + 6), pitch) + acol, o);
#endif
#if ORBPL_FAST_MM3
        const fshort2 m2 = fast_m2_mm3(R);
#else
        const fshort2 m2 = fast_m2_regs(R);
#endif
        const int wr = r + 3;
        const uint32_t lo = (uint32_t)(uint16_t)m2.x;
        const uint32_t hi = has_hi ? (uint32_t)(uint16_t)m2.y : 0u;
        m = lo | (hi << 16);
        const uint32_t mo = umul24((uint32_t)wr, (uint32_t)pw) + 3 + 2 * p;
        M16[mo] = (uint16_t)lo;   // window column x = 3 + 2p
        M16[mo + 1] = (uint16_t)hi;
      }
      // all lanes: neighbour pixels of the same row from the adjacent lanes
#if ORBPL_FAST_DPP
      // DPP wave shifts (lane i <- lane i - 1 / i + 1; lane 0 / 63 read 0)
      const uint32_t lhi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(m >> 16), 0x138, 0xf, 0xf, false);
      const uint32_t rlo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(m & 0xFFFFu), 0x130, 0xf, 0xf, false);
#else
      const uint32_t lhi = (uint32_t)__shfl_up((int)(m >> 16), 1, 64);
      const uint32_t rlo = (uint32_t)__shfl_down((int)(m & 0xFFFFu), 1, 64);
#endif
      if (act) {
        const uint32_t Pl = (has_left ? lhi : 0u) | (m << 16);        // (x-1, x)
        const uint32_t Pr = (m >> 16) | ((has_right ? rlo : 0u) << 16);  // (x+1, x+2)
        const fushort2 cm = pmaxu(as_u2(Pl), as_u2(Pr));
        const uint32_t cmax = __builtin_bit_cast(uint32_t, cm);
        const uint32_t rmax = __builtin_bit_cast(uint32_t, pmaxu(cm, as_u2(m)));
        if (i >= 2) {
          // NMS of row r-1 (interior: rows r-2 and r are this segment's)
          const fushort2 mx = pmaxu(pmaxu(as_u2(rmax2), as_u2(rmax)), as_u2(cmax1));
          const fushort2 mc = as_u2(m1);
          const bool lmax_lo = mc.x > mx.x, lmax_hi = mc.y > mx.y;
          const int row = r - 1;
          uint32_t* mr = mask + 4 * row;
          if (lmax_lo && mc.x >= t_min) atomicOr(mr, pbit);
          if (lmax_hi && mc.y >= t_min) atomicOr(mr + 1, pbit);
          const bool ilo = lmax_lo && mc.x >= t_ini, ihi = lmax_hi && mc.y >= t_ini;
          if (ilo) atomicOr(mr + 2, pbit);
          if (ihi) atomicOr(mr + 3, pbit);
          any_ini |= ilo || ihi;
        }
        rmax2 = rmax1;
        rmax1 = rmax;
        cmax1 = cmax;
        m1 = m;
      }
    }
  }
  __builtin_amdgcn_wave_barrier();
  // ---- segment edge rows (first and last of each segment) from the m plane ----
  if (npair > 0) {
    const int nedge = 2 * nseg * np;
    for (int k = lane; k < nedge; k += 64) {
      const int e = div_small(k, inv_np), p = k - e * np;
      const int sg = e >> 1;
      const int ra = sg * rps, rb = min(ra + rps, dr);
      if (ra >= rb) continue;
      const int row = (e & 1) ? rb - 1 : ra;
      if ((e & 1) && rb - 1 == ra) continue;   // one-row segment: done once
      // rows wr-1, wr, wr+1: dword 1+p = pixels (x-1, x), dword 2+p = (x+1, x+2)
      fushort2 rm[3], cmc = {0, 0}, m = {0, 0};
#pragma unroll
      for (int d = 0; d < 3; d++) {
        const uint32_t* w = M + (row + 2 + d) * pw2 + 1 + p;
        const uint32_t A = w[0], B = w[1];
        const fushort2 cm = pmaxu(as_u2(A), as_u2(B));
        const fushort2 mm = as_u2(__builtin_amdgcn_perm(B, A, 0x05040302u));   // (x, x+1)
        rm[d] = pmaxu(cm, mm);
        if (d == 1) {
          cmc = cm;
          m = mm;
        }
      }
      const fushort2 mx = pmaxu(pmaxu(rm[0], rm[2]), cmc);
      const bool lmax_lo = m.x > mx.x, lmax_hi = m.y > mx.y;
      const uint32_t pbit = 1u << p;
      uint32_t* mr = mask + 4 * row;
      if (lmax_lo && m.x >= t_min) atomicOr(mr, pbit);
      if (lmax_hi && m.y >= t_min) atomicOr(mr + 1, pbit);
      const bool ilo = lmax_lo && m.x >= t_ini, ihi = lmax_hi && m.y >= t_ini;
      if (ilo) atomicOr(mr + 2, pbit);
      if (ihi) atomicOr(mr + 3, pbit);
      any_ini |= ilo || ihi;
    }
  }
  __builtin_amdgcn_wave_barrier();
  // ---- emission in raster order: cv::FAST at ini_th, or at min_th when the
  // cell has no corner at ini_th (ORBextractor.cc:807-817); lane = row ----
  const bool use_ini = __ballot(any_ini) != 0ull;
  const int j0 = use_ini ? 2 : 0;
  uint32_t* out = cell_cands + ((long long)f * g->ncells_total + cell) * slots;
  const int xoff = cg.x0 - kMinBorder, yoff = cg.y0 - kMinBorder;
  uint32_t blo = 0, bhi = 0;
  if (lane < dr && npair > 0) {
    blo = mask[4 * lane + j0];
    bhi = mask[4 * lane + j0 + 1];
  }
  const int cnt = __popc(blo) + __popc(bhi);
  const int incl = wave_incl_scan(cnt);
  const int n = __shfl(incl, 63, 64);
  int pos = incl - cnt;
  const int y = yoff + lane + 3;
  const uint32_t* Mrow = M + (lane + 3) * pw2 + 1;
  uint32_t rem = blo | bhi;
  while (rem) {
    const int p = __builtin_ctz(rem);
    rem &= rem - 1;
    const fushort2 m = as_u2(__builtin_amdgcn_perm(Mrow[p + 1], Mrow[p], 0x05040302u));
    const int x = xoff + 3 + 2 * p;
    if ((blo >> p) & 1u) {
      if (pos < slots) out[pos] = pack_cand(x, y, m.x - 1);
      pos++;
    }
    if ((bhi >> p) & 1u) {
      if (pos < slots) out[pos] = pack_cand(x + 1, y, m.y - 1);
      pos++;
    }
  }
  if (lane == 0) *cnt_out = n < slots ? n : slots;
}

// ---------------------------------------------------------------------------
// Block-wide helpers (256 threads = 4 waves)
// ---------------------------------------------------------------------------
__device__ __forceinline__ int wave_incl_scan(int v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    int u = __shfl_up(v, o, 64);
    if (lane >= o) v += u;
  }
  return v;
}

// Exclusive scan of vals[0..n) in place (n <= 256*kPer); returns the total.
// NT = 64 (a one-wave workgroup): element i in round i / 64 at lane i % 64,
// one wave scan per round and a running offset, no LDS partials or barrier
// (the caller's __syncthreads are then wave barriers).
template <int kPer, int NT = 256>
__device__ int block_excl_scan(int* vals, int n, int* s_wsum) {
  if constexpr (NT == 64) {
    const int lane = threadIdx.x;
    int run = 0;
    for (int base = 0; base < n; base += 64) {
      const int i = base + lane;
      const int v = i < n ? vals[i] : 0;
      const int incl = wave_incl_scan(v);
      if (i < n) vals[i] = run + incl - v;
      run += __shfl(incl, 63, 64);
    }
    __builtin_amdgcn_wave_barrier();
    return run;
  }
  static_assert(NT == 256 || NT == 64, "octree workgroups: 4 waves or 1");
  const int t = threadIdx.x;
  int local[kPer];
  int sum = 0;
#pragma unroll
  for (int k = 0; k < kPer; k++) {
    int i = t * kPer + k;
    local[k] = i < n ? vals[i] : 0;
    sum += local[k];
  }
  int incl = wave_incl_scan(sum);
  const int wave = t >> 6, lane = t & 63;
  if (lane == 63) s_wsum[wave] = incl;
  __syncthreads();
  int wofs = 0, total = 0;
#pragma unroll
  for (int w = 0; w < 4; w++) {
    int s = s_wsum[w];
    if (w < wave) wofs += s;
    total += s;
  }
  int run = wofs + incl - sum;
#pragma unroll
  for (int k = 0; k < kPer; k++) {
    int i = t * kPer + k;
    if (i < n) vals[i] = run;
    run += local[k];
  }
  __syncthreads();
  return total;
}

// ---------------------------------------------------------------------------
// DistributeOctTree (ORBextractor.cc:539-763) for one (frame, level).
//
// The reference keeps a std::list of nodes and pushes children to the front.
// Here the list is an array in list order, rebuilt after every pass:
//   new list = [children of the last processed node (n4..n1 nonempty)] ...
//              [children of the first processed node] ++ [untouched nodes].
// Keys (candidates) carry the index of their node; each pass is one sweep to
// count children (LDS atomics) and one sweep to re-index keys. Phase-2 passes
// divide nodes in descending (size, creation) order and stop at the first
// node after which size >= N (prefix sums over the speculative child counts).
// ---------------------------------------------------------------------------
// Keys' node indices live in LDS (u16) for levels with at most kOctLdsCand
// FAST candidates (every level of a 640x480 frame), else in global memory;
// 8 KB keeps two blocks per CU.
constexpr int kOctLdsCand = 4096;
// first pyramid level whose octree launch runs one-wave workgroups (the
// launch of a level group starting there; ORBPL_OCT_WAVE_FROM overrides)
#ifndef ORBPL_OCT_WAVE_FROM
#define ORBPL_OCT_WAVE_FROM 3
#endif
constexpr int kOctWaveFrom = ORBPL_OCT_WAVE_FROM;

// The node list never exceeds the level's kp_cap = max(N + 3, 4 nIni) (a
// phase-1 pass starts only while size + 3 nexp <= N, phase 2 stops at the
// first size >= N), so the list arrays are sized by kCap = the smallest of
// 256 / 512 / 1024 that holds every level's kp_cap: at 1000 features 27 KB
// of LDS per workgroup (5 per CU) instead of 74 KB (2 per CU).
template <int kCap, int kKn = kOctLdsCand>
struct OctShared {
  uint2 rect[2][kCap];              // (x0 | y0<<16, x1 | y1<<16)
  int cnt[2][kCap];
  int rank[kCap];                   // processing rank of a list entry, -1 = untouched
  int upos[kCap];                   // new position of an untouched entry
  int child[4 * kCap];              // child counts, then child positions
  int exp_pos[kCap];                // expandable children (creation order): list position
  int exp_cnt[kCap];
  int proc[kCap];                   // processing order -> list position (phase 2)
  int scan[kOctMaxList];            // also the cell-count scan (<= 1024 cells)
  int wsum[8];
  int misc[8];
  uint16_t kn[kKn];                 // node of each key when total <= kKn
};

__device__ __forceinline__ uint2 mk_rect(int x0, int y0, int x1, int y1) {
  return make_uint2((uint32_t)x0 | ((uint32_t)y0 << 16), (uint32_t)x1 | ((uint32_t)y1 << 16));
}

__device__ __forceinline__ int child_of(uint2 r, int x, int y) {
  int x0 = r.x & 0xFFFF, y0 = r.x >> 16, x1 = r.y & 0xFFFF, y1 = r.y >> 16;
  int mx = x0 + ((x1 - x0 + 1) >> 1), my = y0 + ((y1 - y0 + 1) >> 1);
  return x < mx ? (y < my ? 0 : 2) : (y < my ? 1 : 3);
}

__device__ __forceinline__ uint2 child_rect(uint2 r, int c) {
  int x0 = r.x & 0xFFFF, y0 = r.x >> 16, x1 = r.y & 0xFFFF, y1 = r.y >> 16;
  int mx = x0 + ((x1 - x0 + 1) >> 1), my = y0 + ((y1 - y0 + 1) >> 1);
  switch (c) {
    case 0: return mk_rect(x0, y0, mx, my);
    case 1: return mk_rect(mx, y0, x1, my);
    case 2: return mk_rect(x0, my, mx, y1);
    default: return mk_rect(mx, my, x1, y1);
  }
}

// debug (ORBPL_OCT_PROFILE): wall-clock ticks of block (level = blockIdx.x,
// frame 0): [8 * level + 0] setup, [+1] passes, [+2] phase-2 passes,
// [+3] retain, [+4] number of passes, [+5] candidates, [+6] final size
__device__ long long g_oct_prof[8 * 16];
__device__ int g_oct_prof_on;

// NT = 256 (4 waves) or 64: the levels with few candidates run as one wave,
// whose block scans are wave scans and whose barriers are wave barriers (a
// pass's fixed cost was its ~16 block barriers and scans)
template <int kCap, int NT = 256>
__global__ void __launch_bounds__(NT) k_octree(const OrbGeom* __restrict__ g,
                                                const uint32_t* __restrict__ cell_cands,
                                                const int* __restrict__ cell_counts,
                                                uint32_t* __restrict__ kcand,
                                                int* __restrict__ knode,
                                                uint32_t* __restrict__ kp_list,
                                                int* __restrict__ kp_count,
                                                int* __restrict__ err_flag, int l0) {
  extern __shared__ char smem_raw[];
  // one-wave workgroups keep the key nodes of up to 2048 candidates in LDS
  // (23 instead of 27 KB at kCap 256: 6 workgroups per CU)
  constexpr int kKn = NT == 64 ? 2048 : kOctLdsCand;
  OctShared<kCap, kKn>& S = *reinterpret_cast<OctShared<kCap, kKn>*>(smem_raw);
  const int level = l0 + blockIdx.x, f = blockIdx.y, t = threadIdx.x;   // levels l0 ..
  const LevelGeom& L = g->lv[level];
  const int N = L.nfeat;
  const bool stamp = g_oct_prof_on && f == 0 && t == 0;
  long long ot[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  long long o0 = stamp ? (long long)wall_clock64() : 0;
  auto lap = [&](int k) {
    if (stamp) {
      const long long o1 = (long long)wall_clock64();
      ot[k] += o1 - o0;
      o0 = o1;
    }
  };
  const int slots = g->cell_slots;
  int* out_count = kp_count + (long long)f * g->nlevels + level;
  uint32_t* out_list = kp_list + (long long)f * g->kp_cap_total + L.kp_base;
  uint32_t* K = kcand + (long long)f * g->cand_cap_total + L.cand_base;
  int* KN = knode + (long long)f * g->cand_cap_total + L.cand_base;

  // ---- 1. gather candidates in cell order (vToDistributeKeys order) ----
  const int ncells = L.ncells;
  const int* ccnt = cell_counts + (long long)f * g->ncells_total + L.cell_base;
  for (int i = t; i < ncells; i += NT) S.scan[i] = ccnt[i];
  __syncthreads();
  const int total = block_excl_scan<4, NT>(S.scan, ncells, S.wsum);
  if (total == 0) {
    if (t == 0) *out_count = 0;
    return;
  }
  const bool kn_lds = total <= kKn;   // block-uniform
  auto kn_get = [&](int k) -> int { return kn_lds ? (int)S.kn[k] : KN[k]; };
  auto kn_set = [&](int k, int v) {
    if (kn_lds) S.kn[k] = (uint16_t)v;
    else KN[k] = v;
  };
  // ---- 2. initial nodes (ORBextractor.cc:543-585), fused with the gather:
  // thread per key position k, its cell = the last cell whose prefix <= k ----
  const int nIni = L.n_ini;
  const float hX = L.hx;
  const int H = L.max_border_y - kMinBorder;
  for (int i = t; i < nIni; i += NT) S.child[i] = 0;
  __syncthreads();
  {
    const uint32_t* cc = cell_cands + ((long long)f * g->ncells_total + L.cell_base) * slots;
    for (int k = t; k < total; k += NT) {
      int lo = 0, hi = ncells - 1;
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (S.scan[mid] <= k) lo = mid;
        else hi = mid - 1;
      }
      const uint32_t c = cc[(long long)lo * slots + (k - S.scan[lo])];
      K[k] = c;
      int idx = (int)((float)cand_x(c) / hX);
      if (idx >= nIni) idx = nIni - 1;
      kn_set(k, idx);
      atomicAdd(&S.child[idx], 1);
    }
  }
  __syncthreads();
  // list = nonempty initial nodes in order
  for (int i = t; i < nIni; i += NT) S.scan[i] = S.child[i] > 0 ? 1 : 0;
  __syncthreads();
  int size = block_excl_scan<4, NT>(S.scan, nIni, S.wsum);
  int cur = 0;
  for (int i = t; i < nIni; i += NT) {
    if (S.child[i] > 0) {
      int p = S.scan[i];
      S.rect[0][p] = mk_rect((int)(hX * (float)i), 0, (int)(hX * (float)(i + 1)), H);
      S.cnt[0][p] = S.child[i];
      S.upos[i] = p;
    }
  }
  __syncthreads();
  for (int k = t; k < total; k += NT) kn_set(k, S.upos[kn_get(k)]);
  // expandable list (for phase 2): empty until a pass creates children
  int nexp = 0;
  bool finish = false;
  bool phase2 = false;
  __syncthreads();

  lap(0);
  while (!finish) {
    const int prevSize = size;
    ot[4]++;
    // ---- choose the nodes to divide and their processing rank ----
    int nproc;  // number of candidate nodes (speculative in phase 2)
    if (!phase2) {
      for (int i = t; i < size; i += NT) S.scan[i] = S.cnt[cur][i] > 1 ? 1 : 0;
      __syncthreads();
      nproc = block_excl_scan<4, NT>(S.scan, size, S.wsum);
      for (int i = t; i < size; i += NT) {
        bool d = S.cnt[cur][i] > 1;
        S.rank[i] = d ? S.scan[i] : -1;
        if (d) S.proc[S.scan[i]] = i;
      }
    } else {
      // sort expandable nodes by (count, seq) descending; seq = creation index
      nproc = nexp;
      for (int i = t; i < size; i += NT) S.rank[i] = -1;
      __syncthreads();
      for (int i = t; i < nexp; i += NT) {
        int ci = S.exp_cnt[i];
        int r = 0;
        for (int j = 0; j < nexp; j++) {
          int cj = S.exp_cnt[j];
          r += (cj > ci) || (cj == ci && j > i);
        }
        S.proc[r] = S.exp_pos[i];
        S.rank[S.exp_pos[i]] = r;
      }
    }
    __syncthreads();
    if (nproc == 0) break;  // nothing divisible: size == prevSize -> finish
    if (4 * nproc > 4 * kCap) {
      if (t == 0) atomicOr(err_flag, 1);
      break;
    }
    for (int i = t; i < 4 * nproc; i += NT) S.child[i] = 0;
    __syncthreads();
    // ---- sweep 1: child counts ----
    for (int k = t; k < total; k += NT) {
      int e = kn_get(k);
      int r = S.rank[e];
      if (r >= 0) {
        uint32_t c = K[k];
        atomicAdd(&S.child[4 * r + child_of(S.rect[cur][e], cand_x(c), cand_y(c))], 1);
      }
    }
    __syncthreads();
    // nonempty children per processed node
    for (int r = t; r < nproc; r += NT) {
      int ne = (S.child[4 * r] > 0) + (S.child[4 * r + 1] > 0) + (S.child[4 * r + 2] > 0) +
               (S.child[4 * r + 3] > 0);
      S.scan[r] = ne;
    }
    __syncthreads();
    int nchild_all = block_excl_scan<4, NT>(S.scan, nproc, S.wsum);  // S.scan = prefix (excl)
    int kproc = nproc;
    if (phase2) {
      // first r with prevSize + sum_{q<=r}(ne_q - 1) >= N
      if (t == 0) S.misc[0] = nproc;
      __syncthreads();
      for (int r = t; r < nproc; r += NT) {
        int ne = (r + 1 < nproc ? S.scan[r + 1] : nchild_all) - S.scan[r];
        int sz = prevSize + (S.scan[r] + ne) - (r + 1);
        if (sz >= N) atomicMin(&S.misc[0], r + 1);
      }
      __syncthreads();
      kproc = S.misc[0];
      for (int i = t; i < size; i += NT)
        if (S.rank[i] >= kproc) S.rank[i] = -1;
      __syncthreads();
    }
    const int nchild = kproc < nproc ? S.scan[kproc] : nchild_all;
    // ---- new positions: children blocks in reverse processing order ----
    const int nxt = cur ^ 1;
    for (int r = t; r < kproc; r += NT) {
      const int pre = S.scan[r];
      const int ne = (r + 1 < nproc ? S.scan[r + 1] : nchild_all) - pre;
      const int off = nchild - pre - ne;
      const int e = S.proc[r];
      const uint2 pr = S.rect[cur][e];
      int above = 0;  // nonempty children with larger index come first (n4..n1)
      for (int c = 3; c >= 0; c--) {
        int cc = S.child[4 * r + c];
        if (cc > 0) {
          int p = off + above;
          above++;
          S.rect[nxt][p] = child_rect(pr, c);
          S.cnt[nxt][p] = cc;
          S.child[4 * r + c] = p;  // now: position
        } else {
          S.child[4 * r + c] = -1;
        }
      }
    }
    // untouched entries keep relative order after the children
    for (int i = t; i < size; i += NT) S.upos[i] = S.rank[i] < 0 ? 1 : 0;
    __syncthreads();
    const int nunt = block_excl_scan<4, NT>(S.upos, size, S.wsum);
    for (int i = t; i < size; i += NT) {
      if (S.rank[i] < 0) {
        int p = nchild + S.upos[i];
        S.rect[nxt][p] = S.rect[cur][i];
        S.cnt[nxt][p] = S.cnt[cur][i];
        S.upos[i] = p;
      }
    }
    const int newSize = nchild + nunt;
    if (newSize > kCap) {
      if (t == 0) atomicOr(err_flag, 2);
      break;
    }
    __syncthreads();
    // ---- sweep 2: re-index keys ----
    for (int k = t; k < total; k += NT) {
      int e = kn_get(k);
      int r = S.rank[e];
      int ne;
      if (r >= 0) {
        uint32_t c = K[k];
        ne = S.child[4 * r + child_of(S.rect[cur][e], cand_x(c), cand_y(c))];
      } else {
        ne = S.upos[e];
      }
      kn_set(k, ne);
    }
    // ---- expandable children in creation order (rank asc, child asc) ----
    for (int r = t; r < kproc; r += NT) {
      int ne = 0;
#pragma unroll
      for (int c = 0; c < 4; c++) {
        int p = S.child[4 * r + c];
        ne += (p >= 0 && S.cnt[nxt][p] > 1) ? 1 : 0;
      }
      S.scan[r] = ne;
    }
    __syncthreads();
    nexp = block_excl_scan<4, NT>(S.scan, kproc, S.wsum);
    for (int r = t; r < kproc; r += NT) {
      int o = S.scan[r];
#pragma unroll
      for (int c = 0; c < 4; c++) {
        int p = S.child[4 * r + c];
        if (p >= 0 && S.cnt[nxt][p] > 1) {
          S.exp_pos[o] = p;
          S.exp_cnt[o] = S.cnt[nxt][p];
          o++;
        }
      }
    }
    __syncthreads();
    cur = nxt;
    size = newSize;
    if (size >= N || size == prevSize) {
      finish = true;
    } else if (!phase2 && size + nexp * 3 > N) {
      phase2 = true;
    }
  }
  lap(1);
  // ---- retain the best key per node (strict >, first in candidate order) ----
  for (int i = t; i < size; i += NT) S.child[i] = 0;
  __syncthreads();
  for (int k = t; k < total; k += NT) {
    uint32_t c = K[k];
    int key = (cand_s(c) << 20) | (kMaxCandPerLevel - k);
    atomicMax(&S.child[kn_get(k)], key);
  }
  __syncthreads();
  const int cap = L.kp_cap;
  for (int i = t; i < size && i < cap; i += NT) {
    int k = kMaxCandPerLevel - (S.child[i] & kMaxCandPerLevel);
    out_list[i] = K[k];
  }
  if (t == 0) {
    if (size > cap) atomicOr(err_flag, 4);
    *out_count = size < cap ? size : cap;
  }
  lap(3);
  ot[5] = total;
  ot[6] = size;
  if (stamp)
    for (int k = 0; k < 8; k++) g_oct_prof[8 * level + k] = ot[k];
}

// ---------------------------------------------------------------------------
// Orientation + descriptor + output, one wave per keypoint slot.
// IC_Angle on the unblurred level, computeOrbDescriptor on the blurred level,
// output rows ordered level by level (ORBextractor.cc:1075-1104).
// ---------------------------------------------------------------------------
// debug (ORBPL_OCT_PROFILE also enables it): phase ticks of frame 0's first
// keypoint wave: [0] slot setup, [1] kp load, [2] IC_Angle, [3] atan2/cos/sin,
// [4] BRIEF tests, [5] stores
__device__ long long g_od_prof[8];

// BRIEF patch staged in LDS: rotated pattern points lie within radius 18.39
// of the keypoint (|bit_pattern_31_| <= 13), so every test reads rows and
// columns ky-18 .. ky+18, kx-18 .. kx+18 of the blurred level. The patch is
// 37 rows of 10 aligned dwords (bytes o .. o+36, o = (kx-18) & 3): 6 wide
// loads per lane that issue with the IC_Angle loads, before the angle is
// known, instead of 8 scattered byte loads (one cache line per lane) after it.
constexpr int kIcR = 15;                             // HALF_PATCH_SIZE
constexpr int kIcRowDw = 9;                          // bytes o .. o+30, o <= 3
constexpr int kIcDw = (2 * kIcR + 1) * kIcRowDw;     // 279
constexpr int kIcLoads = (kIcDw + 63) / 64;          // 5
constexpr int kBriefR = 18;
constexpr int kBriefRows = 2 * kBriefR + 1;
constexpr int kBriefRowDw = 10;
constexpr int kBriefDw = kBriefRows * kBriefRowDw;   // 370
constexpr int kBriefLoads = (kBriefDw + 63) / 64;    // 6

#ifndef ORBPL_OD_MINW
#define ORBPL_OD_MINW 1
#endif

// IC_Angle (ORBextractor.cc:77-108) over one dword of a patch row: pixels
// u0 .. u0+3 of row v; the bytes inside the disc |u| <= um (bytes bq in
// [lo, hi)) masked, then *s0 += their sum and *s1 += their u-weighted sum
// = u0 * sum + sum(bq * pixel), both sums by v_dot4_u32_u8. Integer sums:
// the same m01 / m10 in any order. um < 0 (a lane past the patch) masks all.
__device__ __forceinline__ void ic_dword(uint32_t px, int u0, int um, int* s0, int* s1) {
  const int lo = min(max(-um - u0, 0), 4), hi = min(max(um - u0 + 1, 0), 4);
  // hi > lo: 1 .. 4 bytes, the right shift is at most 24
  const uint32_t m = hi > lo ? (0xFFFFFFFFu >> (8 * (4 - (hi - lo)))) << (8 * lo) : 0u;
  const uint32_t pm = px & m;
  const int a = (int)__builtin_amdgcn_udot4(pm, 0x01010101u, 0u, false);
  const int b = (int)__builtin_amdgcn_udot4(pm, 0x03020100u, 0u, false);
  *s0 += a;
  *s1 += imul24(u0, a) + b;   // |u0| <= 18, a <= 1020
}
__global__ void __launch_bounds__(256, ORBPL_OD_MINW) k_orient_desc(const uint8_t* __restrict__ pyr,
                                                     const uint8_t* __restrict__ blur,
                                                     const OrbGeom* __restrict__ g,
                                                     const uint32_t* __restrict__ kp_list,
                                                     const int* __restrict__ kp_count,
                                                     orbpl_keypoint_dev* __restrict__ out_kps,
                                                     uint8_t* __restrict__ out_desc,
                                                     int kp_pitch, int* __restrict__ out_n,
                                                      int slot0, int slot1, int write_n) {
  __shared__ uint32_t s_patch[4][kBriefDw];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  int bx, f;
  xcd_block(&bx, &f);
  const int slot = slot0 + bx * 4 + wave;   // slots [slot0, slot1): one group of levels
  if (slot >= slot1) return;
  const bool stamp = g_oct_prof_on && f == 0 && slot == 0 && lane == 0;
  long long dt[6] = {0, 0, 0, 0, 0, 0};
  long long d0 = stamp ? (long long)wall_clock64() : 0;
  auto lap = [&](int k) {
    if (stamp) {
      const long long d1 = (long long)wall_clock64();
      dt[k] = d1 - d0;
      d0 = d1;
    }
  };
  int level = 0;
  while (level + 1 < g->nlevels && slot >= g->lv[level + 1].kp_base) level++;
  const LevelGeom& L = g->lv[level];
  const int idx = slot - L.kp_base;
  const int* cnts = kp_count + (long long)f * g->nlevels;
  int offset = 0, total = 0;
  for (int l = 0; l < g->nlevels; l++) {
    int c = cnts[l];
    if (l < level) offset += c;
    total += c;
  }
  // the frame's keypoint count, by the launch of the last level group (all
  // levels' octrees are done by then)
  if (write_n && slot == slot0 && lane == 0) out_n[f] = total < kp_pitch ? total : kp_pitch;
  if (idx >= cnts[level]) return;
  const int opos = offset + idx;
  if (opos >= kp_pitch) return;
  lap(0);
  const uint32_t c = kp_list[(long long)f * g->kp_cap_total + slot];
  const int kx = cand_x(c) + kMinBorder, ky = cand_y(c) + kMinBorder;
  if (stamp) (void)__builtin_amdgcn_readfirstlane(kx);
  lap(1);
  // --- IC_Angle patch loads: rows ky-15 .. ky+15 as 9 aligned dwords each
  // (bytes o .. o+30 from the aligned base, o = address & 3), 5 per lane ---
  const uint8_t* irow0 = pyr + (long long)f * g->pyr_bytes + content_off(L, kx - kIcR, ky - kIcR);
  const int io = (int)(reinterpret_cast<uintptr_t>(irow0) & 3);
  const uint32_t* irow = reinterpret_cast<const uint32_t*>(irow0 - io);
  const int ipdw = L.pitch >> 2;
  uint32_t iv[kIcLoads];
#pragma unroll
  for (int j = 0; j < kIcLoads; j++) {
    const int i = lane + 64 * j;
    const int r = i / kIcRowDw, q = i - r * kIcRowDw;
    iv[j] = i < kIcDw ? irow[r * ipdw + q] : 0u;
  }
  // --- BRIEF patch loads (consumed after the angle) ---
  const int bx0 = kx - kBriefR;
  const uint32_t* prow = reinterpret_cast<const uint32_t*>(
      blur + (long long)f * g->blur_bytes + L.boff + (long long)(ky - kBriefR) * L.bpitch +
      (bx0 & ~3));
  const int pdw = L.bpitch >> 2;
  uint32_t pv[kBriefLoads];
#pragma unroll
  for (int j = 0; j < kBriefLoads; j++) {
    const int i = lane + 64 * j;
    const int r = i / kBriefRowDw, q = i - r * kBriefRowDw;
    pv[j] = i < kBriefDw ? prow[r * pdw + q] : 0u;
  }
  // --- IC_Angle moments: pixel (u, v) of the disc |u| <= umax[|v|]; each
  // lane takes the 4 pixels of its dwords (integer sums: any order) ---
  int m01 = 0, m10 = 0;
#pragma unroll
  for (int j = 0; j < kIcLoads; j++) {
    const int i = lane + 64 * j;
    const int r = i / kIcRowDw, q = i - r * kIcRowDw;
    const int v = r - kIcR;
    const int um = i < kIcDw ? g->umax[v < 0 ? -v : v] : -1;
    const int u0 = 4 * q - io - kIcR;   // u of the dword's byte 0
    int s0 = 0, s1 = 0;
#pragma unroll
    for (int bq = 0; bq < 4; bq++) {
      const int u = u0 + bq;
      const int px = (int)((iv[j] >> (8 * bq)) & 0xFFu);
      const int w = (u <= um && -u <= um) ? px : 0;
      s0 += w;
      s1 += u * w;
    }
    m10 += s1;
    m01 += v * s0;
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    m10 += __shfl_xor(m10, o, 64);
    m01 += __shfl_xor(m01, o, 64);
  }
  lap(2);
  const float angle = fast_atan2_deg((float)m01, (float)m10);
  // --- steered BRIEF on the blurred level ---
  const float factorPI = (float)(3.14159265358979323846 / 180.f);
  float a, b;
  cr_cos_sin(angle * factorPI, &a, &b);
  if (stamp) (void)__builtin_amdgcn_readfirstlane(__float_as_int(a + b));
  lap(3);
  uint32_t* patch = s_patch[wave];
#pragma unroll
  for (int j = 0; j < kBriefLoads; j++) {
    const int i = lane + 64 * j;
    if (i < kBriefDw) patch[i] = pv[j];
  }
  __builtin_amdgcn_wave_barrier();
  // centre byte of the patch: row kBriefR, byte (bx0 & 3) + kBriefR
  const uint8_t* bimg = reinterpret_cast<const uint8_t*>(patch) + kBriefR * 4 * kBriefRowDw +
                        (bx0 & 3) + kBriefR;
  const int step = 4 * kBriefRowDw;
  uint64_t words[4];
#pragma unroll
  for (int r = 0; r < 4; r++) {
    const int tst = r * 64 + lane;
    const int* p = &c_pattern[4 * tst];
    const float x1 = (float)p[0], y1 = (float)p[1], x2 = (float)p[2], y2 = (float)p[3];
    const int v1 = bimg[cv_round(x1 * b + y1 * a) * step + cv_round(x1 * a - y1 * b)];
    const int v2 = bimg[cv_round(x2 * b + y2 * a) * step + cv_round(x2 * a - y2 * b)];
    words[r] = __ballot(v1 < v2);
  }
  lap(4);
  uint8_t* d = out_desc + ((long long)f * kp_pitch + opos) * 32;
  if (lane < 4) {
    uint64_t w = lane == 0 ? words[0] : lane == 1 ? words[1] : lane == 2 ? words[2] : words[3];
    reinterpret_cast<uint64_t*>(d)[lane] = w;
  }
  if (lane == 0) {
    orbpl_keypoint_dev kp;
    float sx = (float)kx, sy = (float)ky;
    if (level != 0) {
      sx = sx * L.scale;
      sy = sy * L.scale;
    }
    kp.x = sx;
    kp.y = sy;
    kp.size = (float)L.scaled_patch;
    kp.angle = angle;
    kp.response = (float)cand_s(c);
    kp.octave = level;
    kp.class_id = -1;
    out_kps[(long long)f * kp_pitch + opos] = kp;
  }
  lap(5);
  if (stamp)
    for (int k = 0; k < 6; k++) g_od_prof[k] = dt[k];
}

// Two keypoints per wave (ORBPL_OD_PAIR): each 32-lane half runs the kernel
// above for its own slot - 9 IC and 12 BRIEF dword loads per lane, the
// moments reduced within the half, 8 rounds of 32 tests whose ballot halves
// are the two descriptors' dwords. The per-keypoint uniform work (level and
// offset search, atan2, the correctly rounded cos / sin, address math) is
// issued once for two keypoints. Same operations per keypoint: bit-exact.
// Measured (tools/gpu_r04_ab.sh, 10 ORB tests green; isolated, 1024 frames):
// 1.465-1.469 -> 1.403-1.409 ms (the kernel stays bound by its patch gathers).
#ifndef ORBPL_OD_PAIR
#define ORBPL_OD_PAIR 1
#endif
constexpr int kIcLoads2 = (kIcDw + 31) / 32;         // 9
constexpr int kBriefLoads2 = (kBriefDw + 31) / 32;   // 12
__global__ void __launch_bounds__(256, ORBPL_OD_MINW) k_orient_desc2(const uint8_t* __restrict__ pyr,
                                                      const uint8_t* __restrict__ blur,
                                                      const OrbGeom* __restrict__ g,
                                                      const uint32_t* __restrict__ kp_list,
                                                      const int* __restrict__ kp_count,
                                                      orbpl_keypoint_dev* __restrict__ out_kps,
                                                      uint8_t* __restrict__ out_desc,
                                                      int kp_pitch, int* __restrict__ out_n,
                                                      int slot0, int slot1, int write_n) {
  __shared__ uint32_t s_patch[8][kBriefDw];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int half = lane >> 5, l32 = lane & 31;
  int bx, f;
  xcd_block(&bx, &f);
  const int slot = slot0 + bx * 8 + wave * 2 + half;   // slots [slot0, slot1)
  const int nlev = g->nlevels;
  bool act = slot < slot1;
  int level = 0;
  if (act)
    while (level + 1 < nlev && slot >= g->lv[level + 1].kp_base) level++;
  const LevelGeom& L = g->lv[level];
  const int idx = slot - L.kp_base;
  const int* cnts = kp_count + (long long)f * nlev;
  int offset = 0, total = 0, mine = 0;
  for (int l = 0; l < nlev; l++) {
    const int c = cnts[l];
    if (l < level) offset += c;
    if (l == level) mine = c;
    total += c;
  }
  if (write_n && slot == slot0 && l32 == 0) out_n[f] = total < kp_pitch ? total : kp_pitch;
  act = act && idx < mine && offset + idx < kp_pitch;
  if (!__any(act)) return;
  const int opos = offset + idx;
  const uint32_t c = act ? kp_list[(long long)f * g->kp_cap_total + slot] : 0u;
  const int kx = act ? cand_x(c) + kMinBorder : kIcR + kBriefR,
            ky = act ? cand_y(c) + kMinBorder : kIcR + kBriefR;
  // IC_Angle patch: rows ky-15 .. ky+15 as 9 aligned dwords each, loaded as
  // 32-bit dword offsets from the frame's (uniform) pyramid base
  const uint32_t* fpyr = reinterpret_cast<const uint32_t*>(pyr + (long long)f * g->pyr_bytes);
  const int ioff = (int)content_off(L, kx - kIcR, ky - kIcR);   // < 2^31 within a frame
  const int io = ioff & 3;                                      // pyr_bytes % 256 == 0
  const uint32_t ibase = (uint32_t)ioff >> 2;
  const uint32_t ipdw = (uint32_t)L.pitch >> 2;
  uint32_t iv[kIcLoads2];
#pragma unroll
  for (int j = 0; j < kIcLoads2; j++) {
    const uint32_t i = (uint32_t)l32 + 32u * j;
    const uint32_t r = div_c16<kIcRowDw>(i), q = i - umul24(r, kIcRowDw);
    iv[j] = (act && i < (uint32_t)kIcDw) ? ld_dw(fpyr, ibase + umul24(r, ipdw) + q) : 0u;
  }
  const int bx0 = kx - kBriefR;
  const uint32_t* fblur = reinterpret_cast<const uint32_t*>(blur + (long long)f * g->blur_bytes);
  const uint32_t pdw = (uint32_t)L.bpitch >> 2;
  const uint32_t pbase =
      (uint32_t)((L.boff + (long long)(ky - kBriefR) * L.bpitch + (bx0 & ~3)) >> 2);
  uint32_t pv[kBriefLoads2];
#pragma unroll
  for (int j = 0; j < kBriefLoads2; j++) {
    const uint32_t i = (uint32_t)l32 + 32u * j;
    const uint32_t r = div_c16<kBriefRowDw>(i), q = i - umul24(r, kBriefRowDw);
    pv[j] = (act && i < (uint32_t)kBriefDw) ? ld_dw(fblur, pbase + umul24(r, pdw) + q) : 0u;
  }
  int m01 = 0, m10 = 0;
#pragma unroll
  for (int j = 0; j < kIcLoads2; j++) {
    const int i = l32 + 32 * j;
    const int r = (int)div_c16<kIcRowDw>((uint32_t)i), q = i - (int)umul24((uint32_t)r, kIcRowDw);
    const int v = r - kIcR;
    const int um = i < kIcDw ? g->umax[v < 0 ? -v : v] : -1;
    int s0 = 0;
    ic_dword(iv[j], 4 * q - io - kIcR, um, &s0, &m10);
    m01 += imul24(v, s0);   // |v| <= 15, s0 <= 1020
  }
#pragma unroll
  for (int o = 16; o >= 1; o >>= 1) {   // within the half
    m10 += __shfl_xor(m10, o, 64);
    m01 += __shfl_xor(m01, o, 64);
  }
  const float angle = fast_atan2_deg((float)m01, (float)m10);
  const float factorPI = (float)(3.14159265358979323846 / 180.f);
  float a, b;
  cr_cos_sin(angle * factorPI, &a, &b);
  uint32_t* patch = s_patch[wave * 2 + half];
#pragma unroll
  for (int j = 0; j < kBriefLoads2; j++) {
    const int i = l32 + 32 * j;
    if (i < kBriefDw) patch[i] = pv[j];
  }
  __builtin_amdgcn_wave_barrier();
  const uint8_t* bimg = reinterpret_cast<const uint8_t*>(patch) + kBriefR * 4 * kBriefRowDw +
                        (bx0 & 3) + kBriefR;
  const int step = 4 * kBriefRowDw;
  uint32_t words[8];
#pragma unroll
  for (int r = 0; r < 8; r++) {
    const float4 P = c_pattern_f[r * 32 + l32];
    const float x1 = P.x, y1 = P.y, x2 = P.z, y2 = P.w;
    // cvRound(y) * step + cvRound(x): the rounded values are integers below
    // 2^5, so the float multiply-add is exact and one conversion remains
    const float fs = (float)step;
    const int v1 = bimg[(int)(__builtin_rintf(x1 * b + y1 * a) * fs + __builtin_rintf(x1 * a - y1 * b))];
    const int v2 = bimg[(int)(__builtin_rintf(x2 * b + y2 * a) * fs + __builtin_rintf(x2 * a - y2 * b))];
    words[r] = (uint32_t)(__ballot(v1 < v2) >> (32 * half));
  }
  if (!act) return;
  uint8_t* d = out_desc + ((long long)f * kp_pitch + opos) * 32;
  if (l32 < 8) {
    uint32_t w = words[0];
#pragma unroll
    for (int r = 1; r < 8; r++) w = l32 == r ? words[r] : w;
    reinterpret_cast<uint32_t*>(d)[l32] = w;
  }
  if (l32 == 0) {
    orbpl_keypoint_dev kp;
    float sx = (float)kx, sy = (float)ky;
    if (level != 0) {
      sx = sx * L.scale;
      sy = sy * L.scale;
    }
    kp.x = sx;
    kp.y = sy;
    kp.size = (float)L.scaled_patch;
    kp.angle = angle;
    kp.response = (float)cand_s(c);
    kp.octave = level;
    kp.class_id = -1;
    out_kps[(long long)f * kp_pitch + opos] = kp;
  }
}

// ---------------------------------------------------------------------------
// Host-side launchers (called by the runtime in orbpl_runtime.cpp)
// ---------------------------------------------------------------------------
hipError_t upload_pattern(hipStream_t s) {
  static float pf[1024];
  static const bool filled = [] {
    for (int i = 0; i < 1024; i++) pf[i] = (float)bit_pattern_31_[i];
    return true;
  }();
  (void)filled;
  const hipError_t e = hipMemcpyToSymbolAsync(HIP_SYMBOL(c_pattern), bit_pattern_31_,
                                              sizeof(bit_pattern_31_), 0, hipMemcpyHostToDevice, s);
  if (e != hipSuccess) return e;
  return hipMemcpyToSymbolAsync(HIP_SYMBOL(c_pattern_f), pf, sizeof(pf), 0, hipMemcpyHostToDevice, s);
}


int read_od_profile(long long* out8) {
  return hipMemcpyFromSymbol(out8, HIP_SYMBOL(g_od_prof), 6 * sizeof(long long)) == hipSuccess ? 0 : -1;
}

int read_octree_profile(long long* out128) {
  return hipMemcpyFromSymbol(out128, HIP_SYMBOL(g_oct_prof), 128 * sizeof(long long)) == hipSuccess
             ? 0 : -1;
}

void launch_pyramid(const OrbGeom& hg, const OrbGeom* dg, const uint8_t* img, int stride,
                    long long frame_pitch, uint8_t* pyr, uint8_t* blur, const int* rs,
                    const PyrBand* bands, int nbands, int batch, long long* prof, int l0, int l1,
                    hipStream_t s) {
  hipLaunchKernelGGL(k_pyramid, dim3(nbands, batch), dim3(kPyrThreads), 0, s, img, stride,
                     frame_pitch, pyr, blur, dg, rs, bands, prof, l0, l1);
}

void launch_fast(const OrbGeom& hg, const OrbGeom* dg, const CellGeom* cells, const uint8_t* pyr,
                 uint32_t* cell_cands, int* cell_counts, int ini_th, int min_th, int batch,
                 int l0, int l1, hipStream_t s) {
  const size_t smem = 4 * 4 * (size_t)fast_wave_words(hg.fast_win_w, hg.fast_win_h);
  const int c0 = hg.lv[l0].cell_base;
  const int c1 = l1 < hg.nlevels ? hg.lv[l1].cell_base : hg.ncells_total;
  if (c1 <= c0) return;
  hipLaunchKernelGGL(k_fast_cells, dim3((c1 - c0 + 3) / 4, batch), dim3(256), smem, s, pyr, dg,
                     cells, cell_cands, cell_counts, ini_th, min_th, c0, c1);
}

void launch_octree(const OrbGeom& hg, const OrbGeom* dg, const uint32_t* cell_cands,
                   const int* cell_counts, uint32_t* kcand, int* knode, uint32_t* kp_list,
                   int* kp_count, int* err_flag, int batch, int l0, int l1, hipStream_t s) {
  set_smem_attr((const void*)k_octree<1024, 256>, sizeof(OctShared<1024>));
  int cap = 0;
  for (int l = 0; l < hg.nlevels; l++) cap = std::max(cap, hg.lv[l].kp_cap);
  if (once_per_device((const void*)&g_oct_prof_on)) {
    const int on = getenv("ORBPL_OCT_PROFILE") ? 1 : 0;
    (void)hipMemcpyToSymbolAsync(HIP_SYMBOL(g_oct_prof_on), &on, sizeof(int), 0,
                                 hipMemcpyHostToDevice, s);
  }
  // levels from ORBPL_OCT_WAVE_FROM on (default 3: the coarse levels, a few
  // hundred candidates each) as one-wave workgroups; 0 = all, nlevels = none
  const char* wf = getenv("ORBPL_OCT_WAVE_FROM");   // read per launch: tests vary it
  const int wave_from = wf ? atoi(wf) : kOctWaveFrom;
  const bool one_wave = l0 >= wave_from;
#define ORBPL_OCT_LAUNCH(CAP)                                                                   \
  if (one_wave)                                                                                 \
    hipLaunchKernelGGL((k_octree<CAP, 64>), dim3(l1 - l0, batch), dim3(64),                    \
                       sizeof(OctShared<CAP, 2048>), s, dg, cell_cands, cell_counts, kcand,     \
                       knode,                                                                   \
                       kp_list, kp_count, err_flag, l0);                                        \
  else                                                                                          \
    hipLaunchKernelGGL((k_octree<CAP, 256>), dim3(l1 - l0, batch), dim3(256),                  \
                       sizeof(OctShared<CAP>), s, dg, cell_cands, cell_counts, kcand, knode,    \
                       kp_list, kp_count, err_flag, l0);
  if (cap <= 256) {
    ORBPL_OCT_LAUNCH(256)
  } else if (cap <= 512) {
    ORBPL_OCT_LAUNCH(512)
  } else {
    if (one_wave) set_smem_attr((const void*)k_octree<1024, 64>, sizeof(OctShared<1024, 2048>));
    ORBPL_OCT_LAUNCH(1024)
  }
#undef ORBPL_OCT_LAUNCH
}

void launch_orient_desc(const OrbGeom& hg, const OrbGeom* dg, const uint8_t* pyr,
                        const uint8_t* blur, const uint32_t* kp_list, const int* kp_count,
                        orbpl_keypoint_dev* out_kps, uint8_t* out_desc, int kp_pitch, int* out_n,
                        int batch, int l0, int l1, hipStream_t s) {
  // keypoint slots of levels [l0, l1); the launch of the last level writes
  // the frames' keypoint counts
  const int s0 = hg.lv[l0].kp_base;
  const int s1 = l1 < hg.nlevels ? hg.lv[l1].kp_base : hg.kp_cap_total;
  const int wn = l1 == hg.nlevels ? 1 : 0;
  if (s1 <= s0) return;
  static const char* pe = getenv("ORBPL_OD_PAIR");
  // the phase-stamp profile (ORBPL_OCT_PROFILE) lives in the one-per-wave kernel
  static const bool pair = (pe ? atoi(pe) != 0 : ORBPL_OD_PAIR) && !getenv("ORBPL_OCT_PROFILE");
  if (pair)
    hipLaunchKernelGGL(k_orient_desc2, dim3((s1 - s0 + 7) / 8, batch), dim3(256), 0, s, pyr, blur,
                       dg, kp_list, kp_count, out_kps, out_desc, kp_pitch, out_n, s0, s1, wn);
  else
    hipLaunchKernelGGL(k_orient_desc, dim3((s1 - s0 + 3) / 4, batch), dim3(256), 0, s, pyr, blur,
                       dg, kp_list, kp_count, out_kps, out_desc, kp_pitch, out_n, s0, s1, wn);
}

}  // namespace orbpl
