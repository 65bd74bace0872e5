// Line-feature kernels (LSD + LBD), shared between lsd_kernels.hip and the
// C-ABI runtime (lsd_runtime.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/orbpl.h"

namespace orbpl {

constexpr int kLsdMaxLines = 4096;    // raw LSD segments kept per frame
constexpr int kLsdMaxCand = 4096;     // refined rectangles awaiting NFA validation per frame
// introsort segments of at most this many elements are finished in LDS, one
// wave each (k_lsd_sort_wave); the global kernel partitions down to it.
// Lines leg at 3072 streams, 2 rounds (profiles/r06/ab/lsd_sort_wave_ab.txt):
// 2048 17.2k / 17.0k, 1024 17.4k / 17.6k, 512 16.9k / 16.6k frames/s
#ifndef ORBPL_SORT_LOCAL_MAX
#define ORBPL_SORT_LOCAL_MAX 1024
#endif
constexpr int kSortLocalMax = ORBPL_SORT_LOCAL_MAX;
constexpr int kSpecLanes = 64;        // speculative regions per round (one wave)
constexpr int kLaneCap = 2048;        // region points a lane can hold (both grows)
// waves per frame of the speculative seed loop at a given batch: 4 for 97-384
// frames (at most half the GPU's ~3072 co-resident seed-loop waves, so a
// second LSD batch - the stereo right images - still fits beside it), else 1.
// LSD probe (ms per batch, 4 / 2 waves vs 1): batch 64 89.8 vs 85.7, 256 86.9
// vs 91.2, 1024 (2 waves) 124.7 vs 138.0, batch 1 equal; but the stereo
// workload's two concurrent 1024-frame LSD batches at 2 waves each
// oversubscribe the GPU (seed loop 128 -> 201 ms per step), so 2 waves are
// not used by default.
#ifndef ORBPL_SPEC_WAVES
#define ORBPL_SPEC_WAVES 0   // 0 = by batch; 1, 2 or 4 forces it (A/B)
#endif
__host__ __device__ inline int lsd_spec_waves(int batch) {
  if (ORBPL_SPEC_WAVES) return ORBPL_SPEC_WAVES;
  return (batch > 96 && batch <= 384) ? 4 : 1;
}
// lane lists to allocate for batches up to B: the largest batch x waves
__host__ __device__ inline long long lsd_spec_lane_frames(int B) {
  const int b4 = B < 384 ? B : 384;
  const long long m1 = (long long)B * lsd_spec_waves(B), m4 = (long long)b4 * lsd_spec_waves(b4);
  return m1 > m4 ? m1 : m4;
}
constexpr int kLineKeep = 80;         // LineExtractor.cpp:24
constexpr int kLsdSortChunk = 256;    // elements per partition chunk
constexpr float kLsdNotdef = -1.0f;   // NOTDEF marker in the degree map

// Per-frame geometry of the LSD path (host-computed, passed by value).
struct LsdGeom {
  int W, H;          // input image
  int sw, sh;        // 0.8-scaled image
  int n;             // (sw-1)*(sh-1) pseudo-ordered pixels
  int gk[7];         // GaussianBlur 8.8 fixed-point kernel (sigma 0.75, 7 taps)
  int ksize;
  double rho;        // gradient threshold quant / sin(prec)
  double prec, p;    // angle tolerance (rad) and its probability
  double log_nt;     // LOG_NT
  int min_reg_size;
  // INTER_LINEAR_EXACT ranges: dx in [rx0, rx1) and dy in [ry0, ry1) interpolate
  int rx0, rx1, ry0, ry1;
  // sort scratch capacities
  int seg_cap, chunk_cap, leaf_cap;
  int mask_cap;   // k_lsd_sort's chunks per level whose stopper masks are kept (sort_masks)
};

// Device scratch of one frame slot (all pointers are per-batch bases; the
// kernels index them with the frame number).
// Seed-loop pixel words: 4x4-pixel tiles of 8-byte words, so that a 3x3
// neighbourhood touches 2.25 128-byte lines on average (row-major float4
// records + separate stamps touched ~7).
__host__ __device__ inline int lsd_sd_tw(int sw) { return (sw + 3) >> 2; }
__host__ __device__ inline long long lsd_sd_words(int sw, int sh) {
  return (long long)lsd_sd_tw(sw) * ((sh + 3) >> 2) * 16;
}
// per frame: the pixel words (lsd_sd_words) followed by the angle-term plane
// in the same tiles: (cos | sin << 32) of the pixel's float angle, the
// region_grow accumulation terms (P2), so a grow step adds a pixel without
// evaluating them on its serial chain
__host__ __device__ inline long long lsd_sd_frame_words(int sw, int sh) {
  return 2 * lsd_sd_words(sw, sh);
}
// A pixel's word and its angle terms side by side: one 16-byte load per
// neighbour in the grow, 4x4-pixel tiles of 256 B.
__host__ __device__ inline int lsd_sd_index(int x, int y, int tw) {
  const int i = ((((y >> 2) * tw) + (x >> 2)) << 4) | ((y & 3) << 2) | (x & 3);
  return 2 * i;
}
// The degree plane (LsdScratch::deg) in 8x4-pixel tiles of 128 B: the NFA
// walk of k_lsd_validate reads a rectangle row by row, and a thin oblique
// rectangle's consecutive rows then share a line (row-major, every row of it
// was a line of its own).
__host__ __device__ inline int lsd_deg_tw(int sw) { return (sw + 7) >> 3; }
__host__ __device__ inline long long lsd_deg_words(int sw, int sh) {
  return (long long)lsd_deg_tw(sw) * ((sh + 3) >> 2) * 32;
}
__host__ __device__ inline int lsd_deg_index(int x, int y, int dtw) {
  return ((((y >> 2) * dtw) + (x >> 3)) << 5) | ((y & 3) << 3) | (x & 7);
}
// offset (u64 words) of a pixel's angle terms from its pixel word
__host__ __device__ inline long long lsd_cs_offset(int sw, int sh) {
  return 1;
}

struct LsdScratch {
  uint8_t* blur;       // W*H
  uint8_t* scaled;     // sw*sh
  float* deg;          // lsd_deg_words per frame (lsd_deg_index tiles), fastAtan2
                       // degrees or kLsdNotdef
  int* q;              // sw*sh, gx^2 + gy^2
  unsigned* maxq;      // 1 per frame
  uint32_t* A;         // n: key << 22 | raster index, sorted in place
  int* Lpos;           // n
  int* Rpos;           // n
  int4* seg0;          // seg_cap (first, last, depth, -)
  int4* seg1;          // seg_cap
  int4* heap;          // seg_cap
  int* seg_i;          // 8 * seg_cap: pivot, choff, nL, nR, K, cut, nch, -
  int* chunk_i;        // 4 * chunk_cap: Lc, Rc, Lpre, Rsuf
  unsigned long long* sort_masks;   // mask_cap * 32 per frame: a level's chunk stopper ballots
  int2* leaves;        // leaf_cap
  uint32_t* reg;       // 3*sw*sh region overflow (point, q, degrees)
  float* lines;        // kLsdMaxLines * 4
  int* nlines;         // 1 per frame
  int* err;            // 1 per frame: capacity overflow flags
  long long* prof;     // optional: 8 cycle counters per frame (phase profile)
  double* cand;        // kLsdMaxCand * 12 per frame: refined rectangles, seed order
  int* ncand;          // 1 per frame
  float* cand_line;    // kLsdMaxCand * 4 per frame: validated segment
  int* cand_ok;        // kLsdMaxCand per frame: log_nfa > log_eps
  uint64_t* sd;        // lsd_sd_words(g) per frame, 4x4-pixel tiles (lsd_sd_index):
                       // low word = the pixel's degrees (float bits), high word =
                       // the speculative seed loop's claim stamp (0 = USED,
                       // 0xFFFFFFFF = unclaimed); written by k_lsd_grad
  uint4* lbuf;         // kSpecLanes * kLaneCap per frame: per-lane region lists
                       // (x | y << 16, degrees, modgrad as a double lo / hi)
  int4* sort_local;    // seg_cap per frame: introsort segments finished in LDS
  int* sort_nlocal;    // 1 per frame
  int* sort_kt;        // 1 per frame: key bound, key < kt => NOTDEF pixel
  const double* lgam;  // log_gamma(i + 1) for i < lgam_n (k_lgamma_table): the
  int lgam_n;          // NFA's three log_gamma terms at integer arguments
  int* sort_nge;       // 1 per frame: elements with key >= kt (the list's
                       // exactly sorted prefix; every later pixel is NOTDEF)
};

// Outputs of LineExtractor::ExtractLineSegment per frame.
struct LineOut {
  orbpl_keyline* kl_all;  // kLsdMaxLines per frame: every detected KeyLine
  orbpl_keyline* kl;      // kLineKeep per frame: the kept KeyLines, sorted
  uint8_t* desc;          // kLineKeep * 32 per frame: LBD rows
  double* coef;           // kLineKeep * 3 per frame
  int* n;                 // kept count per frame
};

// BinaryDescriptor's local (F_l, 3 bands x 7) and global (F_g, 63 rows)
// Gaussian weights, as the floats computeLBD multiplies with.
struct LbdWeights {
  float gL[21];
  float gG[63];
};

void launch_keylines(const LsdGeom& g, const LsdScratch& sc, const LineOut& o, int batch,
                     hipStream_t s);
// the 5x5 blur (g5, ksize 5) and computeSobel fused per tile
void launch_blur_sobel(const LsdGeom& g5, const uint8_t* img, int stride, long long frame_pitch,
                       int16_t* dx, int16_t* dy, int batch, hipStream_t s);
void launch_sobel(int W, int H, const uint8_t* blur5, int16_t* dx, int16_t* dy, int batch,
                  hipStream_t s);
void launch_lbd(int W, int H, const int16_t* dx, const int16_t* dy, const LbdWeights& w,
                const LineOut& o, int batch, hipStream_t s);

void launch_lsd_blur(const LsdGeom& g, const uint8_t* img, int stride, long long frame_pitch,
                     uint8_t* out, int batch, hipStream_t s);
void launch_lsd_resize(const LsdGeom& g, const int* tabs, const uint8_t* blur, uint8_t* scaled,
                       int batch, hipStream_t s);
// fused blur + resize + grad: scaled-image tiles of kPrTW x kPrTH; the
// source span of a tile must fit kPrSC x kPrSR (lsd_prep_fits) and ksize be 7
constexpr int kPrTW = 64, kPrTH = 16, kPrSC = 96, kPrSR = 32, kPrR = 3;
void launch_lsd_prep(const LsdGeom& g, const int* tabs, const uint8_t* img, int stride,
                     long long frame_pitch, uint8_t* scaled, float* deg, int* q, uint64_t* sd,
                     unsigned* maxq, int batch, hipStream_t s);
void launch_lsd_grad(const LsdGeom& g, const uint8_t* scaled, float* deg, int* q, uint64_t* sd,
                     unsigned* maxq, int batch, hipStream_t s);
void launch_lsd_sort(const LsdGeom& g, const LsdScratch& sc, int batch, hipStream_t s);
void launch_lsd_sort_keys(int n, const int* keys, const LsdScratch& sc, hipStream_t s);
// serial = true: the wave-serial seed loop (k_lsd_grow); false: the
// speculative lane-parallel loop (k_lsd_spec). Identical results.
void launch_lsd_grow(const LsdGeom& g, const LsdScratch& sc, int batch, hipStream_t s,
                     bool serial);
size_t lsd_grow_smem(const LsdGeom& g);
void launch_lsd_validate(const LsdGeom& g, const LsdScratch& sc, int batch, hipStream_t s);
// t[i] = log_gamma(i + 1), i < n, with the NFA's own log_gamma (once per context)
void launch_lgamma_table(double* t, int n, hipStream_t s);

// Host runtime (lsd_runtime.cpp): LSD (+ LineExtractor when `out` is set) of
// `batch` frames on stream `s`; lsdx_check reads the device capacity flags.
int lsdx_run(lsdx_ctx* c, const uint8_t* d_imgs, int batch, int stride, int64_t frame_pitch,
             const LineOut* out, hipStream_t s, hipEvent_t ev_mid,
             const hipEvent_t* ev_stage = nullptr);
int lsdx_check(lsdx_ctx* c, int batch);

}  // namespace orbpl
