// Per-frame tracking kernels for gfx950: everything Tracking::TrackWithMotionModel
// (Tracking.cc:1212-1330) runs on the current frame after extraction, for a
// batch of independent streams (one workgroup per stream where the reference
// is sequential inside a frame).
//
//   k_frame_prepare : Frame glue (Frame.cc:135-205 RGB-D constructor body):
//                     UndistortKeyPoints, ComputeStereoFromRGBD, PosInGrid
//   k_predict       : mCurrentFrame.SetPose(mVelocity * mLastFrame.mTcw)
//   k_match_last    : ORBmatcher::SearchByProjection(Frame&, const Frame&, th,
//                     bMono) (ORBmatcher.cc:1710-1879) incl. the rotation
//                     histogram, plus the 2*th retry of TrackWithMotionModel
//   k_pose          : Optimizer::PoseOptimization[WithLines] (Optimizer.cc:
//                     375-619, 2132-2486) — the whole 4 x 10 LM loop on device
//   k_finish        : discard outliers, velocity update (Tracking.cc:479-484),
//                     and the next frame's map points (StereoInitialization-
//                     style keyframe: every keypoint with depth, Tracking.cc:
//                     608-660 / Frame::UnprojectStereo)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <stdint.h>

#include "orbpl_math.h"
#include "track_common.h"
#include "track_kernels.h"
#include "lsd_kernels.h"
#include "orbpl_runtime.h"

namespace orbpl {

// ---------------------------------------------------------------------------
// Frame glue: one thread per keypoint.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_frame_prepare(TrackConsts c, const KeyPointD* __restrict__ kps,
                                                       const int* __restrict__ n_in, int kp_pitch,
                                                       const float* __restrict__ depth,
                                                       long long depth_pitch,
                                                       KeyPointD* __restrict__ kps_un,
                                                       float* __restrict__ depth_out,
                                                       float* __restrict__ uright,
                                                       int* __restrict__ gcell) {
  const int f = blockIdx.y;
  const int i = blockIdx.x * 256 + threadIdx.x;
  const int n = n_in[f];
  if (i >= n) return;
  const long long o = (long long)f * kp_pitch + i;
  KeyPointD k = kps[o];
  KeyPointD u = k;
  if (c.k1 != 0.0f) undistort_point_d(c, k.x, k.y, &u.x, &u.y);
  kps_un[o] = u;
  float d_out = -1.f, ur = -1.f;
  if (depth) {
    const int v = (int)k.y, uu = (int)k.x;
    const float d = depth[(long long)f * depth_pitch + (long long)v * c.width + uu];
    if (d > 0) {
      d_out = d;
      ur = u.x - c.bf / d;
    }
  }
  depth_out[o] = d_out;
  uright[o] = ur;
  const int px = (int)roundf((u.x - c.minX) * c.gridInvW);
  const int py = (int)roundf((u.y - c.minY) * c.gridInvH);
  gcell[o] = (px < 0 || px >= kGridCols || py < 0 || py >= kGridRows) ? -1 : px + kGridCols * py;
}

// ---------------------------------------------------------------------------
// Constant-velocity prediction (Tracking.cc:1228). One thread per stream.
// ---------------------------------------------------------------------------
__global__ void k_predict(StreamState* __restrict__ st, int nstreams) {
  trk_priority();
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= nstreams) return;
  StreamState& S = st[s];
  if (!S.has_last) return;
  if (S.has_velocity) {
    float Twl[16], V[16];
    pose_inverse(S.Tlast2, Twl);
    gemm44(S.Tlast, Twl, V);       // mVelocity = Tcw(t-1) * Twc(t-2)
    gemm44(V, S.Tlast, S.Tcw);     // SetPose(mVelocity * mLastFrame.mTcw)
  } else {
    for (int k = 0; k < 16; k++) S.Tcw[k] = S.Tlast[k];
  }
}

// ---------------------------------------------------------------------------
// SearchByProjection(CurrentFrame, LastFrame): one 256-thread workgroup per
// stream. The current frame's 64x48 grid is rebuilt in LDS (stable counting
// sort = the reference's mGrid cell vectors in index order).
//   Phase A (parallel over last-frame map points): projection, window and the
//     unconstrained best candidate: min (distance, grid-scan order).
//   Phase B (wave 0, ordered): the reference skips candidates already taken by
//     a map point with Observations() > 0 earlier in the loop. Chunks of 64
//     points are accepted at once when no point's best is taken by an earlier
//     one; otherwise the chunk is replayed point by point with re-scans.
//   Phase C: rotation histogram, ComputeThreeMaxima, removal.
// ---------------------------------------------------------------------------
struct MatchArgs {
  // current frame (per stream pitch kp_pitch)
  const KeyPointD* cur_kps_un;
  const uint8_t* cur_desc;
  const float* cur_uright;
  const int* cur_gcell;
  const int* cur_n;
  // last frame
  const KeyPointD* last_kps_un;
  const uint8_t* last_has_mp;
  const uint8_t* last_outlier;
  const float* last_xyz;
  const uint8_t* last_desc;     // map point descriptors
  const int* last_nobs;
  const int* last_n;
  int kp_pitch;
  // poses
  const float* Tcw;             // per stream 16 floats (stride pose_stride floats)
  const float* Tlw;
  int pose_stride;
  // outputs
  int* match;                   // per stream kp_pitch
  int* nmatches;                // per stream (stride nm_stride ints)
  int nm_stride;
  float th;
  int mono;
  int check_ori;
  int retry;                    // TrackWithMotionModel: if nmatches < 20 redo with 2*th
  const StreamState* active;    // optional: skip streams without a last frame
  int prof;                     // debug: phase stamps of stream 0 into g_match_prof
};

// debug (ORBPL_MATCH_PROFILE): wall-clock ticks (100 MHz) of stream 0's
// SearchByProjection: [0] grid, [1] phase A, [2] phase B, [3] phase C, [4] output
__device__ long long g_match_prof[8];

__device__ __forceinline__ int hamming32(const uint8_t* a, const uint8_t* b) {
  const uint4 a0 = *reinterpret_cast<const uint4*>(a);
  const uint4 a1 = *reinterpret_cast<const uint4*>(a + 16);
  const uint4 b0 = *reinterpret_cast<const uint4*>(b);
  const uint4 b1 = *reinterpret_cast<const uint4*>(b + 16);
  return __popc(a0.x ^ b0.x) + __popc(a0.y ^ b0.y) + __popc(a0.z ^ b0.z) + __popc(a0.w ^ b0.w) +
         __popc(a1.x ^ b1.x) + __popc(a1.y ^ b1.y) + __popc(a1.z ^ b1.z) + __popc(a1.w ^ b1.w);
}

// Hamming distance of a descriptor held in registers and one in LDS
__device__ __forceinline__ int hamming_rl(uint4 a0, uint4 a1, const uint4* b) {
  const uint4 b0 = b[0], b1 = b[1];
  return __popc(a0.x ^ b0.x) + __popc(a0.y ^ b0.y) + __popc(a0.z ^ b0.z) + __popc(a0.w ^ b0.w) +
         __popc(a1.x ^ b1.x) + __popc(a1.y ^ b1.y) + __popc(a1.z ^ b1.z) + __popc(a1.w ^ b1.w);
}

// Current-frame descriptors staged in LDS for KMAX <= ORBPL_MATCH_DESC_LDS_MAX
// (32 KB at 1024 keypoints), else read from global memory (L2). Default 0:
// from global memory for every KMAX - the smaller workgroup is placed sooner
// beside the next batch's extraction kernels, and the scan's descriptor reads
// hit L2 (A/B on one box, 1024 streams, two rounds: k_match_last isolated
// 0.70 -> 0.50 ms, headline 124.3k / 125.6k -> 129.0k / 128.8k frames/s,
// tools/gpu_r04_f.sh).
#ifndef ORBPL_MATCH_DESC_LDS_MAX
#define ORBPL_MATCH_DESC_LDS_MAX 0
#endif
__host__ __device__ constexpr bool match_desc_lds(int kmax) { return kmax <= ORBPL_MATCH_DESC_LDS_MAX; }
__host__ __device__ constexpr int match_desc_slots(int kmax) { return match_desc_lds(kmax) ? 2 * kmax : 1; }

struct ProjInfo {
  bool ok;
  float u, v, invzc, radius;
  int minLevel, maxLevel;
  int cx0, cx1, cy0, cy1;
};

__device__ __forceinline__ ProjInfo project_point(const TrackConsts& c, const float* Tc,
                                                  const float* X, int nLastOctave, float th,
                                                  bool bForward, bool bBackward) {
  ProjInfo p;
  p.ok = false;
  float x3Dc[3];
  gemm_R_x_plus_t(Tc, X, x3Dc);
  const float xc = x3Dc[0], yc = x3Dc[1];
  const float invzc = (float)(1.0 / (double)x3Dc[2]);
  if (invzc < 0) return p;
  const float u = c.fx * xc * invzc + c.cx;
  const float v = c.fy * yc * invzc + c.cy;
  if (u < c.minX || u > c.maxX) return p;
  if (v < c.minY || v > c.maxY) return p;
  p.u = u;
  p.v = v;
  p.invzc = invzc;
  p.radius = th * c.scale[nLastOctave];
  if (bForward) {
    p.minLevel = nLastOctave;
    p.maxLevel = -1;
  } else if (bBackward) {
    p.minLevel = 0;
    p.maxLevel = nLastOctave;
  } else {
    p.minLevel = nLastOctave - 1;
    p.maxLevel = nLastOctave + 1;
  }
  const float r = p.radius;
  p.cx0 = max(0, (int)floorf((u - c.minX - r) * c.gridInvW));
  p.cx1 = min(kGridCols - 1, (int)ceilf((u - c.minX + r) * c.gridInvW));
  p.cy0 = max(0, (int)floorf((v - c.minY - r) * c.gridInvH));
  p.cy1 = min(kGridRows - 1, (int)ceilf((v - c.minY + r) * c.gridInvH));
  if (p.cx0 >= kGridCols || p.cx1 < 0 || p.cy0 >= kGridRows || p.cy1 < 0) return p;
  p.ok = true;
  return p;
}

// Frame::GetFeaturesInArea + the best-candidate loop (ORBmatcher.cc:1789-1826).
// Returns (dist << 16) | idx of the first minimum in scan order, or -1.
template <bool kLdsDesc, class SH>
__device__ int scan_best(const SH& S, const TrackConsts& c, const ProjInfo& p,
                         const uint8_t* dMP, const uint8_t* cur_desc, bool use_claims,
                         float mbf) {
  const uint4 m0 = *reinterpret_cast<const uint4*>(dMP);
  const uint4 m1 = *reinterpret_cast<const uint4*>(dMP + 16);
  int bestDist = 256, bestIdx = -1;
  const bool bCheckLevels = (p.minLevel > 0) || (p.maxLevel >= 0);
  const float r = p.radius;
  // cells are numbered column-major (ix * rows + iy), so the reference's
  // inner iy loop over one grid column is one contiguous run of items
  for (int ix = p.cx0; ix <= p.cx1; ix++) {
    const int b = S.cell_start[ix * kGridRows + p.cy0];
    const int e = S.cell_start[ix * kGridRows + p.cy1 + 1];
    for (int q = b; q < e; q++) {
      const int j = S.items[q];
      const int oc = S.oct[j];
      if (bCheckLevels) {
        if (oc < p.minLevel) continue;
        if (p.maxLevel >= 0 && oc > p.maxLevel) continue;
      }
      const float2 xy = S.xy[j];
      const float distx = xy.x - p.u, disty = xy.y - p.v;
      if (!(fabsf(distx) < r && fabsf(disty) < r)) continue;
      if (use_claims && ((S.claimed[j >> 5] >> (j & 31)) & 1u)) continue;
      const float urj = S.ur[j];
      if (urj > 0) {
        const float ur = p.u - mbf * p.invzc;
        const float er = fabsf(ur - urj);
        if (er > p.radius) continue;
      }
      int dist;
      if constexpr (kLdsDesc) dist = hamming_rl(m0, m1, &S.desc[2 * j]);
      else dist = hamming32(dMP, cur_desc + (long long)j * 32);
      if (dist < bestDist) {
        bestDist = dist;
        bestIdx = j;
      }
    }
  }
  return bestIdx < 0 ? -1 : ((bestDist << 16) | bestIdx);
}

constexpr int kTopK = 4;
// k_match_last block size: one block per stream. The kernel takes up to
// kMatchThreads; it launches with kMatchLaunchThreads: in pipelined tracking it
// shares the CUs with the next batch's extraction, and a 4-wave workgroup is
// placed as soon as one extraction workgroup retires where a 16-wave one waits
// for a CU to drain (256 streams: 97.1k frames/s at 256 threads, 91.2k at 1024)
constexpr int kMatchThreads = 1024;
constexpr int kMatchLaunchThreads = 256;

template <int KMAX>
struct MatchShared {
  int cell_start[kGridCols * kGridRows + 1];
  uint16_t items[KMAX];
  float2 xy[KMAX];
  float ur[KMAX];
  float ang[KMAX];
  int8_t oct[KMAX];
  int16_t gc[KMAX];               // grid cell (PosInGrid) or -1
  int top[KMAX * kTopK];          // phase A: best candidates (dist << 16 | idx), sorted;
                                  // during the grid build: per-cell fill counters
  uint8_t ntop[KMAX];             // candidates with dist <= TH_HIGH (saturating)
  int bin[KMAX];                  // accepted -> histogram bin, else -1
  int sel[KMAX];                  // accepted candidate (current-frame index)
  int mpw[KMAX];                  // last writer (last-frame index) per current keypoint
  int fc[KMAX];                   // phase B: first claimer lane per candidate (INT_MAX: none)
  uint32_t claimed[KMAX / 32];
  uint32_t removed[KMAX / 32];
  uint4 desc[match_desc_slots(KMAX)];   // current descriptors (KMAX <= 1024)
  int hist[32];
  int wsum[kMatchThreads / 64];
  int misc[8];
};
static_assert(kMatchMaxKp * kTopK >= kGridCols * kGridRows, "top[] doubles as cell fill counters");

template <int KMAX, int NT>
__global__ void __launch_bounds__(NT) k_match_last(TrackConsts c, MatchArgs a) {
  trk_priority();
  static_assert((kGridCols * kGridRows) % NT == 0 && NT <= kMatchThreads, "cell scan split");
  extern __shared__ char smem_raw[];
  MatchShared<KMAX>& S = *reinterpret_cast<MatchShared<KMAX>*>(smem_raw);
  const int s = blockIdx.x, t = threadIdx.x;
  const int wave = t >> 6, lane = t & 63;
  const bool stamp = a.prof && s == 0 && t == 0;
  long long mt[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  long long m0 = stamp ? (long long)wall_clock64() : 0;
  auto lap = [&](int k) {
    if (stamp) {
      const long long m1 = (long long)wall_clock64();
      mt[k] += m1 - m0;
      m0 = m1;
    }
  };
  if (a.active && !a.active[s].has_last) {
    if (t == 0) a.nmatches[(long long)s * a.nm_stride] = 0;
    for (int i = t; i < a.cur_n[s]; i += NT) a.match[(long long)s * a.kp_pitch + i] = -1;
    return;
  }
  const int n = min(a.cur_n[s], KMAX);
  const int nl = min(a.last_n[s], KMAX);
  const long long cb = (long long)s * a.kp_pitch;
  const KeyPointD* ck = a.cur_kps_un + cb;
  const uint8_t* cdesc = a.cur_desc + cb * 32;
  const float* Tc = a.Tcw + (long long)s * a.pose_stride;
  const float* Tl = a.Tlw + (long long)s * a.pose_stride;
  // ---- current frame into LDS + grid (AssignFeaturesToGrid, Frame.cc:265-287) ----
  for (int i = t; i < kGridCols * kGridRows; i += NT) S.cell_start[i] = 0;
  __syncthreads();
  for (int i = t; i < n; i += NT) {
    const KeyPointD k = ck[i];
    S.xy[i] = make_float2(k.x, k.y);
    S.ang[i] = k.angle;
    S.oct[i] = (int8_t)k.octave;
    S.ur[i] = a.cur_uright[cb + i];
    int g;
    if (a.cur_gcell) {
      g = a.cur_gcell[cb + i];
    } else {  // Frame::PosInGrid (Frame.cc:527-538)
      const int px = (int)roundf((k.x - c.minX) * c.gridInvW);
      const int py = (int)roundf((k.y - c.minY) * c.gridInvH);
      g = (px < 0 || px >= kGridCols || py < 0 || py >= kGridRows) ? -1 : px + kGridCols * py;
    }
    if (g >= 0) g = (g % kGridCols) * kGridRows + g / kGridCols;   // column-major cell
    S.gc[i] = (int16_t)g;
    if (g >= 0) atomicAdd(&S.cell_start[g], 1);
    if constexpr (match_desc_lds(KMAX)) {
      const uint4* dsrc = reinterpret_cast<const uint4*>(cdesc + (long long)i * 32);
      S.desc[2 * i] = dsrc[0];
      S.desc[2 * i + 1] = dsrc[1];
    }
  }
  __syncthreads();
  {  // exclusive scan of the 3072 cell counts (kPer per thread)
    constexpr int kPer = (kGridCols * kGridRows) / NT;
    int loc[kPer];
    int sum = 0;
#pragma unroll
    for (int k = 0; k < kPer; k++) {
      loc[k] = S.cell_start[t * kPer + k];
      sum += loc[k];
    }
    int incl = sum;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      int u = __shfl_up(incl, o, 64);
      if (lane >= o) incl += u;
    }
    if (lane == 63) S.wsum[wave] = incl;
    __syncthreads();
    int base = 0;
    for (int w = 0; w < wave; w++) base += S.wsum[w];
    int run = base + incl - sum;
#pragma unroll
    for (int k = 0; k < kPer; k++) {
      S.cell_start[t * kPer + k] = run;
      S.top[t * kPer + k] = run;  // fill counter
      run += loc[k];
    }
    if (t == NT - 1) S.cell_start[kGridCols * kGridRows] = run;
    __syncthreads();
  }
  // place items (any order), then sort each cell by index: the reference's
  // mGrid[ix][iy] vectors hold indices in increasing order
  for (int i = t; i < n; i += NT) {
    const int g = S.gc[i];
    if (g >= 0) S.items[atomicAdd(&S.top[g], 1)] = (uint16_t)i;
  }
  __syncthreads();
  for (int cell = t; cell < kGridCols * kGridRows; cell += NT) {
    const int b = S.cell_start[cell], e = S.cell_start[cell + 1];
    for (int q = b + 1; q < e; q++) {
      const uint16_t v = S.items[q];
      int r = q - 1;
      while (r >= b && S.items[r] > v) {
        S.items[r + 1] = S.items[r];
        r--;
      }
      S.items[r + 1] = v;
    }
  }
  __syncthreads();
  lap(0);
  // ---- forward/backward motion (ORBmatcher.cc:1724-1744) ----
  float twc[3], tlc[3];
  gemm_neg_Rt_t(Tc, twc);
  gemm_R_x_plus_t(Tl, twc, tlc);
  const bool bForward = tlc[2] > c.mb && !a.mono;
  const bool bBackward = -tlc[2] > c.mb && !a.mono;
  const float mbf = c.bf;
  float th = a.th;
  int nmatches = 0;
  for (int attempt = 0; attempt < 2; attempt++) {
    // ---- phase A: per map point, the first kTopK candidates with distance
    // <= TH_HIGH in (distance, scan order), and how many such candidates exist
    for (int i = t; i < nl; i += NT) {
      int tk[kTopK] = {-1, -1, -1, -1};
      int cnt = 0;
      const long long li = cb + i;
      if (a.last_has_mp[li] && !a.last_outlier[li]) {
        const ProjInfo p = project_point(c, Tc, a.last_xyz + li * 3, a.last_kps_un[li].octave, th,
                                         bForward, bBackward);
        if (p.ok) {
          const uint8_t* dMP = a.last_desc + li * 32;
          const uint4 m0 = *reinterpret_cast<const uint4*>(dMP);
          const uint4 m1 = *reinterpret_cast<const uint4*>(dMP + 16);
          const bool bCheckLevels = (p.minLevel > 0) || (p.maxLevel >= 0);
          const float r = p.radius;
          const float urp = p.u - mbf * p.invzc;
          // column-major cells: one contiguous item run per grid column,
          // in the reference's (ix outer, iy inner) scan order
          for (int ix = p.cx0; ix <= p.cx1; ix++) {
            const int b = S.cell_start[ix * kGridRows + p.cy0];
            const int e = S.cell_start[ix * kGridRows + p.cy1 + 1];
            for (int q = b; q < e; q++) {
              const int j = S.items[q];
              const int oc = S.oct[j];
              if (bCheckLevels) {
                if (oc < p.minLevel) continue;
                if (p.maxLevel >= 0 && oc > p.maxLevel) continue;
              }
              const float2 xy = S.xy[j];
              if (!(fabsf(xy.x - p.u) < r && fabsf(xy.y - p.v) < r)) continue;
              const float urj = S.ur[j];
              if (urj > 0 && fabsf(urp - urj) > p.radius) continue;
              int dist;
              if constexpr (match_desc_lds(KMAX)) dist = hamming_rl(m0, m1, &S.desc[2 * j]);
              else dist = hamming32(dMP, cdesc + (long long)j * 32);
              if (dist > 100) continue;
              cnt++;
              int v = (dist << 16) | j;
              // stable insertion: equal distances keep scan order; once
              // inserted, the displaced entries shift down one place each
              bool ins = false;
#pragma unroll
              for (int q2 = 0; q2 < kTopK; q2++) {
                const int cur = tk[q2];
                if (ins || cur < 0 || (v >> 16) < (cur >> 16)) {
                  tk[q2] = v;
                  v = cur;
                  ins = true;
                  if (v < 0) break;
                }
              }
            }
          }
        }
      }
#pragma unroll
      for (int q2 = 0; q2 < kTopK; q2++) S.top[i * kTopK + q2] = tk[q2];
      S.ntop[i] = (uint8_t)min(cnt, 255);
    }
    for (int i = t; i < n; i += NT) {
      S.mpw[i] = -1;
      S.fc[i] = 0x7fffffff;
    }
    for (int i = t; i < KMAX / 32; i += NT) {
      S.claimed[i] = 0;
      S.removed[i] = 0;
    }
    if (t < 32) S.hist[t] = 0;
    __syncthreads();
    lap(1);
    // ---- phase B (wave 0): the reference's in-order loop, where a candidate
    // taken by an earlier map point with Observations() > 0 is skipped ----
    if (wave == 0) {
      int acc = 0;
      for (int base = 0; base < nl; base += 64) {
        const int i = base + lane;
        const long long li = cb + i;
        const bool valid = i < nl && S.ntop[i] > 0;
        const bool claimer = valid && a.last_nobs[li] > 0;
        const int ntk = valid ? min((int)S.ntop[i], kTopK) : 0;
        bool decided = !valid;
        int p = 0;
        int choice = -1;  // >= 0 candidate, -1 none, -2 needs a full re-scan
        if (i < nl) {
          S.bin[i] = -1;
          S.sel[i] = -1;
        }
        int start = 0;
        while (true) {
          if (!decided && lane >= start) {
            while (p < ntk) {
              const int k = S.top[i * kTopK + p] & 0xFFFF;
              if (!((S.claimed[k >> 5] >> (k & 31)) & 1u)) break;
              p++;
            }
            choice = p < ntk ? (S.top[i * kTopK + p] & 0xFFFF) : (S.ntop[i] > kTopK ? -2 : -1);
          }
          // first undecided lane whose choice an earlier undecided claimer takes,
          // or that needs a re-scan: every undecided claimer posts its lane to
          // its choice (atomicMin), then each lane compares the first poster
          const bool und = !decided && lane >= start;
          const bool cq = und && claimer && choice >= 0;
          if (cq) atomicMin(&S.fc[choice], lane);
          __threadfence_block();
          bool coll = und && choice == -2;
          if (und && choice >= 0 && S.fc[choice] < lane) coll = true;
          __threadfence_block();
          if (cq) S.fc[choice] = 0x7fffffff;
          __threadfence_block();
          const unsigned long long cm = __ballot(coll);
          const int lc = cm ? __ffsll((long long)cm) - 1 : 64;
          if (und && lane < lc) {
            if (choice >= 0) {
              atomicMax(&S.mpw[choice], i);
              if (claimer) atomicOr(&S.claimed[choice >> 5], 1u << (choice & 31));
              float rot = a.last_kps_un[li].angle - S.ang[choice];
              if (rot < 0.0f) rot += 360.0f;
              int b = (int)roundf(rot * (30 / 360.0f));
              if (b == 30) b = 0;
              S.bin[i] = b;
              S.sel[i] = choice;
              acc++;
            }
            decided = true;
          }
          if (lc == 64) break;
          __builtin_amdgcn_wave_barrier();
          if (lane == lc && choice == -2) {
            // all kTopK candidates taken: full re-scan excluding taken ones
            const ProjInfo pj = project_point(c, Tc, a.last_xyz + li * 3, a.last_kps_un[li].octave,
                                              th, bForward, bBackward);
            const int r = scan_best<match_desc_lds(KMAX)>(S, c, pj, a.last_desc + li * 32, cdesc,
                                                          true, mbf);
            if (r >= 0 && (r >> 16) <= 100) {
              const int k = r & 0xFFFF;
              atomicMax(&S.mpw[k], i);
              if (claimer) atomicOr(&S.claimed[k >> 5], 1u << (k & 31));
              float rot = a.last_kps_un[li].angle - S.ang[k];
              if (rot < 0.0f) rot += 360.0f;
              int b = (int)roundf(rot * (30 / 360.0f));
              if (b == 30) b = 0;
              S.bin[i] = b;
              S.sel[i] = k;
              acc++;
            }
            decided = true;
          }
          __builtin_amdgcn_wave_barrier();
          start = lc;
        }
      }
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) acc += __shfl_xor(acc, o, 64);
      if (lane == 0) S.misc[0] = acc;
    }
    __syncthreads();
    lap(2);
    nmatches = S.misc[0];
    // ---- phase C: rotation consistency (ORBmatcher.cc:1850-1876, 2035-2077) ----
    if (a.check_ori) {
      for (int i = t; i < nl; i += NT)
        if (S.bin[i] >= 0) atomicAdd(&S.hist[S.bin[i]], 1);
      __syncthreads();
      if (t == 0) {
        int max1 = 0, max2 = 0, max3 = 0, ind1 = -1, ind2 = -1, ind3 = -1;
        for (int i = 0; i < 30; i++) {
          const int sz = S.hist[i];
          if (sz > max1) {
            max3 = max2; max2 = max1; max1 = sz; ind3 = ind2; ind2 = ind1; ind1 = i;
          } else if (sz > max2) {
            max3 = max2; max2 = sz; ind3 = ind2; ind2 = i;
          } else if (sz > max3) {
            max3 = sz; ind3 = i;
          }
        }
        if (max2 < 0.1f * (float)max1) {
          ind2 = -1; ind3 = -1;
        } else if (max3 < 0.1f * (float)max1) {
          ind3 = -1;
        }
        S.misc[1] = ind1; S.misc[2] = ind2; S.misc[3] = ind3;
        S.misc[4] = 0;
      }
      __syncthreads();
      const int ind1 = S.misc[1], ind2 = S.misc[2], ind3 = S.misc[3];
      int nrem = 0;
      for (int i = t; i < nl; i += NT) {
        const int b = S.bin[i];
        if (b >= 0 && b != ind1 && b != ind2 && b != ind3) {
          const int k = S.sel[i];
          atomicOr(&S.removed[k >> 5], 1u << (k & 31));
          nrem++;
        }
      }
      if (nrem) atomicAdd(&S.misc[4], nrem);
      __syncthreads();
      nmatches -= S.misc[4];
    }
    lap(3);
    if (!(a.retry && nmatches < 20 && attempt == 0)) break;
    th = 2 * a.th;
    __syncthreads();
  }
  for (int i = t; i < n; i += NT) {
    int m = S.mpw[i];
    if (a.check_ori && ((S.removed[i >> 5] >> (i & 31)) & 1u)) m = -1;
    a.match[cb + i] = m;
  }
  if (t == 0) a.nmatches[(long long)s * a.nm_stride] = nmatches;
  lap(4);
  if (stamp)
    for (int k = 0; k < 8; k++) g_match_prof[k] = mt[k];
}

// ---------------------------------------------------------------------------
// Pose-only Levenberg-Marquardt, one workgroup per stream; all of g2o's
// control flow (optimization_algorithm_levenberg.cpp:61-164) runs on device,
// thread 0 solves the 6x6 system and updates the SE3 estimate; H, b and chi2
// are block reductions in double.
// ---------------------------------------------------------------------------
struct Quat { double w, x, y, z; };
struct SE3d { Quat q; double t[3]; };

// Every thread of a k_pose workgroup runs the same LM control on the same
// reduced sums, so the estimate and its rotation are uniform: readfirstlane
// lets them live in scalar registers instead of 32 VGPRs.
__device__ __forceinline__ double uni(double v) {
  const int lo = __builtin_amdgcn_readfirstlane(__double2loint(v));
  const int hi = __builtin_amdgcn_readfirstlane(__double2hiint(v));
  return __hiloint2double(hi, lo);
}
__device__ __forceinline__ void uni(SE3d& T) {
  T.q.w = uni(T.q.w); T.q.x = uni(T.q.x); T.q.y = uni(T.q.y); T.q.z = uni(T.q.z);
  T.t[0] = uni(T.t[0]); T.t[1] = uni(T.t[1]); T.t[2] = uni(T.t[2]);
}
__device__ __forceinline__ void uni(double R[3][3]) {
#pragma unroll
  for (int r = 0; r < 3; r++)
#pragma unroll
    for (int c = 0; c < 3; c++) R[r][c] = uni(R[r][c]);
}

__device__ __forceinline__ void normalize_rotation(Quat& q) {
  if (q.w < 0) { q.w = -q.w; q.x = -q.x; q.y = -q.y; q.z = -q.z; }
  const double n = sqrt(q.w * q.w + q.x * q.x + q.y * q.y + q.z * q.z);
  q.w /= n; q.x /= n; q.y /= n; q.z /= n;
}
__device__ Quat quat_from_R(const double m[3][3]) {
  Quat q;
  double t = m[0][0] + m[1][1] + m[2][2];
  if (t > 0) {
    t = sqrt(t + 1.0);
    q.w = 0.5 * t;
    t = 0.5 / t;
    q.x = (m[2][1] - m[1][2]) * t;
    q.y = (m[0][2] - m[2][0]) * t;
    q.z = (m[1][0] - m[0][1]) * t;
  } else {
    int i = 0;
    if (m[1][1] > m[0][0]) i = 1;
    if (m[2][2] > m[i][i]) i = 2;
    const int j = (i + 1) % 3, k = (j + 1) % 3;
    t = sqrt(m[i][i] - m[j][j] - m[k][k] + 1.0);
    double v[3];
    v[i] = 0.5 * t;
    t = 0.5 / t;
    q.w = (m[k][j] - m[j][k]) * t;
    v[j] = (m[j][i] + m[i][j]) * t;
    v[k] = (m[k][i] + m[i][k]) * t;
    q.x = v[0]; q.y = v[1]; q.z = v[2];
  }
  return q;
}
__device__ __forceinline__ void quat_to_R(const Quat& q, double R[3][3]) {
  const double tx = 2 * q.x, ty = 2 * q.y, tz = 2 * q.z;
  const double twx = tx * q.w, twy = ty * q.w, twz = tz * q.w;
  const double txx = tx * q.x, txy = ty * q.x, txz = tz * q.x;
  const double tyy = ty * q.y, tyz = tz * q.y, tzz = tz * q.z;
  R[0][0] = 1 - (tyy + tzz); R[0][1] = txy - twz; R[0][2] = txz + twy;
  R[1][0] = txy + twz; R[1][1] = 1 - (txx + tzz); R[1][2] = tyz - twx;
  R[2][0] = txz - twy; R[2][1] = tyz + twx; R[2][2] = 1 - (txx + tyy);
}
__device__ __forceinline__ void quat_rotate(const Quat& q, const double v[3], double o[3]) {
  double uv[3] = {q.y * v[2] - q.z * v[1], q.z * v[0] - q.x * v[2], q.x * v[1] - q.y * v[0]};
  uv[0] += uv[0]; uv[1] += uv[1]; uv[2] += uv[2];
  const double c[3] = {q.y * uv[2] - q.z * uv[1], q.z * uv[0] - q.x * uv[2], q.x * uv[1] - q.y * uv[0]};
  o[0] = v[0] + q.w * uv[0] + c[0];
  o[1] = v[1] + q.w * uv[1] + c[1];
  o[2] = v[2] + q.w * uv[2] + c[2];
}
__device__ SE3d se3_exp(const double u[6]) {
  const double w0 = u[0], w1 = u[1], w2 = u[2];
  const double theta = sqrt(w0 * w0 + w1 * w1 + w2 * w2);
  const double O[3][3] = {{0, -w2, w1}, {w2, 0, -w0}, {-w1, w0, 0}};
  double O2[3][3];
  for (int r = 0; r < 3; r++)
    for (int cc = 0; cc < 3; cc++) O2[r][cc] = O[r][0] * O[0][cc] + O[r][1] * O[1][cc] + O[r][2] * O[2][cc];
  double R[3][3], V[3][3];
  if (theta < 0.00001) {
    for (int r = 0; r < 3; r++)
      for (int cc = 0; cc < 3; cc++) {
        R[r][cc] = (r == cc ? 1.0 : 0.0) + O[r][cc] + O2[r][cc];
        V[r][cc] = R[r][cc];
      }
  } else {
    const double a = sin(theta) / theta;
    const double b = (1 - cos(theta)) / (theta * theta);
    const double c3 = (theta - sin(theta)) / (theta * theta * theta);
    for (int r = 0; r < 3; r++)
      for (int cc = 0; cc < 3; cc++) {
        R[r][cc] = (r == cc ? 1.0 : 0.0) + a * O[r][cc] + b * O2[r][cc];
        V[r][cc] = (r == cc ? 1.0 : 0.0) + b * O[r][cc] + c3 * O2[r][cc];
      }
  }
  SE3d s;
  s.q = quat_from_R(R);
  normalize_rotation(s.q);
  for (int r = 0; r < 3; r++) s.t[r] = V[r][0] * u[3] + V[r][1] * u[4] + V[r][2] * u[5];
  return s;
}
__device__ SE3d se3_mul(const SE3d& a, const SE3d& b) {
  SE3d r = a;
  double rt[3];
  quat_rotate(a.q, b.t, rt);
  r.t[0] += rt[0]; r.t[1] += rt[1]; r.t[2] += rt[2];
  Quat q;
  q.w = a.q.w * b.q.w - a.q.x * b.q.x - a.q.y * b.q.y - a.q.z * b.q.z;
  q.x = a.q.w * b.q.x + a.q.x * b.q.w + a.q.y * b.q.z - a.q.z * b.q.y;
  q.y = a.q.w * b.q.y + a.q.y * b.q.w + a.q.z * b.q.x - a.q.x * b.q.z;
  q.z = a.q.w * b.q.z + a.q.z * b.q.w + a.q.x * b.q.y - a.q.y * b.q.x;
  normalize_rotation(q);
  r.q = q;
  return r;
}

struct alignas(16) PoseEdge {
  float obs[4];   // mono: u,v ; stereo: u,v,ur ; line: sx,sy,ex,ey
  float X[6];     // point: Xw ; line: world start, end
  float info;
  int kind;       // 0 mono, 1 stereo, 2 line
  int idx;        // frame index
  int pad;
};

// The fixed part of k_pose's LDS; launch_pose appends per-edge chi2 / level /
// outlier flags for ecap edges and the on-chip edge records (PoseLds).
struct PoseShared {
  double red[4][32];
  double sys[1][28];              // reduced H (upper, row-major), b, robust chi2
  int wsum[8];
  int misc[8];
};

// Edge storage of one stream. Point edges are 32-byte records {u, v, ur,
// invSigma2} {X, Y, Z, index} (kind = ur < 0 ? mono : stereo), line edges
// PoseEdge records. The first pcap point edges and the first lcap line edges
// live in LDS, read by every linearisation, trial and classification pass;
// the rest (frames beyond the block's LDS budget) in the stream's global
// scratch (pose_edge_bytes() per edge slot: points, then lines).
struct PoseLds {
  float* chi2;                    // (float) chi2 of the last computed error (stale
                                  // semantics; only its float is ever compared)
  uint8_t* level;
  uint8_t* out_flag;
  float4* prec;                   // pcap point records (2 float4 each)
  PoseEdge* lrec;                 // lcap line records
  float4* pg;                     // global: point records
  PoseEdge* lg;                   // global: line records
  int pcap, lcap, npts;
};

__device__ __forceinline__ PoseEdge fetch_edge(const PoseLds& V, int k) {
  PoseEdge e;
  if (k < V.npts) {
    float4 A, B;
    if (k < V.pcap) {
      A = V.prec[2 * k];
      B = V.prec[2 * k + 1];
    } else {
      A = V.pg[2 * k];
      B = V.pg[2 * k + 1];
    }
    e.obs[0] = A.x; e.obs[1] = A.y; e.obs[2] = A.z; e.obs[3] = 0;
    e.info = A.w;
    e.X[0] = B.x; e.X[1] = B.y; e.X[2] = B.z;
    e.X[3] = e.X[4] = e.X[5] = 0;
    e.idx = __float_as_int(B.w);
    e.kind = A.z < 0 ? 0 : 1;
    e.pad = 0;
  } else {
    const int j = k - V.npts;
    e = j < V.lcap ? V.lrec[j] : V.lg[j];
  }
  return e;
}

__device__ __forceinline__ PoseEdge fetch_point(const PoseLds& V, int k) {
  float4 A, B;
  if (k < V.pcap) {
    A = V.prec[2 * k];
    B = V.prec[2 * k + 1];
  } else {
    A = V.pg[2 * k];
    B = V.pg[2 * k + 1];
  }
  PoseEdge e;
  e.obs[0] = A.x; e.obs[1] = A.y; e.obs[2] = A.z; e.obs[3] = 0;
  e.info = A.w;
  e.X[0] = B.x; e.X[1] = B.y; e.X[2] = B.z;
  e.X[3] = e.X[4] = e.X[5] = 0;
  e.idx = __float_as_int(B.w);
  e.kind = A.z < 0 ? 0 : 1;
  e.pad = 0;
  return e;
}

__device__ __forceinline__ void store_point(const PoseLds& V, int k, float u, float v, float ur,
                                            float info, const float* X, int idx) {
  const float4 A = make_float4(u, v, ur, info), B = make_float4(X[0], X[1], X[2], __int_as_float(idx));
  float4* d = k < V.pcap ? V.prec : V.pg;
  d[2 * k] = A;
  d[2 * k + 1] = B;
}

struct PoseCam {
  double fx, fy, cx, cy, bf;
  int fixed_line_jac;  // ORBPL_POSE_FIXED_LINE_JAC: analytic line Jacobian
};

__device__ void edge_error(const PoseEdge& e, const PoseCam& c, const SE3d& T, const double R[3][3],
                           double* err) {
  if (e.kind == 2) {
    double nw[3], vw[3];
    const double sp[3] = {e.X[0], e.X[1], e.X[2]}, ep[3] = {e.X[3], e.X[4], e.X[5]};
    nw[0] = sp[1] * ep[2] - sp[2] * ep[1];
    nw[1] = sp[2] * ep[0] - sp[0] * ep[2];
    nw[2] = sp[0] * ep[1] - sp[1] * ep[0];
    for (int k = 0; k < 3; k++) vw[k] = ep[k] - sp[k];
    double Rn[3], Rv[3];
    for (int r = 0; r < 3; r++) {
      Rn[r] = R[r][0] * nw[0] + R[r][1] * nw[1] + R[r][2] * nw[2];
      Rv[r] = R[r][0] * vw[0] + R[r][1] * vw[1] + R[r][2] * vw[2];
    }
    const double* t = T.t;
    const double tRv[3] = {-t[2] * Rv[1] + t[1] * Rv[2], t[2] * Rv[0] - t[0] * Rv[2], -t[1] * Rv[0] + t[0] * Rv[1]};
    const double nc[3] = {Rn[0] + tRv[0], Rn[1] + tRv[1], Rn[2] + tRv[2]};
    const double l0 = c.fy * nc[0], l1 = c.fx * nc[1];
    const double l2 = -c.fy * c.cx * nc[0] + -c.fx * c.cy * nc[1] + c.fx * c.fy * nc[2];
    const double sq = sqrt(l0 * l0 + l1 * l1);
    err[0] = ((double)e.obs[0] * l0 + (double)e.obs[1] * l1 + l2) / sq;
    err[1] = ((double)e.obs[2] * l0 + (double)e.obs[3] * l1 + l2) / sq;
    err[2] = 0;
    return;
  }
  const double X[3] = {e.X[0], e.X[1], e.X[2]};
  double p[3];
  quat_rotate(T.q, X, p);
  p[0] += T.t[0]; p[1] += T.t[1]; p[2] += T.t[2];
  if (e.kind == 0) {
    err[0] = (double)e.obs[0] - (p[0] / p[2] * c.fx + c.cx);
    err[1] = (double)e.obs[1] - (p[1] / p[2] * c.fy + c.cy);
    err[2] = 0;
  } else {
    const float invz = (float)(1.0 / p[2]);
    const double u = p[0] * (double)invz * c.fx + c.cx;
    const double v = p[1] * (double)invz * c.fy + c.cy;
    err[0] = (double)e.obs[0] - u;
    err[1] = (double)e.obs[1] - v;
    err[2] = (double)e.obs[2] - (u - c.bf * (double)invz);
  }
}

__device__ void edge_jacobian(const PoseEdge& e, const PoseCam& c, const SE3d& T,
                              const double R[3][3], double J[3][6]) {
  if (e.kind == 2) {
    double nw[3], vw[3];
    const double sp[3] = {e.X[0], e.X[1], e.X[2]}, ep[3] = {e.X[3], e.X[4], e.X[5]};
    nw[0] = sp[1] * ep[2] - sp[2] * ep[1];
    nw[1] = sp[2] * ep[0] - sp[0] * ep[2];
    nw[2] = sp[0] * ep[1] - sp[1] * ep[0];
    for (int k = 0; k < 3; k++) vw[k] = ep[k] - sp[k];
    double Rn[3], Rv[3];
    for (int r = 0; r < 3; r++) {
      Rn[r] = R[r][0] * nw[0] + R[r][1] * nw[1] + R[r][2] * nw[2];
      Rv[r] = R[r][0] * vw[0] + R[r][1] * vw[1] + R[r][2] * vw[2];
    }
    const double* t = T.t;
    const double tRv[3] = {-t[2] * Rv[1] + t[1] * Rv[2], t[2] * Rv[0] - t[0] * Rv[2], -t[1] * Rv[0] + t[0] * Rv[1]};
    const double nc[3] = {Rn[0] + tRv[0], Rn[1] + tRv[1], Rn[2] + tRv[2]};
    const double l0 = c.fy * nc[0], l1 = c.fx * nc[1];
    const double l2 = -c.fy * c.cx * nc[0] + -c.fx * c.cy * nc[1] + c.fx * c.fy * nc[2];
    const double ln = sqrt(l0 * l0 + l1 * l1);
    if (c.fixed_line_jac) {
      // analytic form (oracle edge_jacobian, ORBPL_POSE_FIXED_LINE_JAC):
      // J_r = dd_r K_line [-[n_c]x | -[v_c]x]
      const double N[2] = {(double)e.obs[0] * l0 + (double)e.obs[1] * l1 + l2,
                           (double)e.obs[2] * l0 + (double)e.obs[3] * l1 + l2};
      const double Sn[3][3] = {{0, -nc[2], nc[1]}, {nc[2], 0, -nc[0]}, {-nc[1], nc[0], 0}};
      const double Sv[3][3] = {{0, -Rv[2], Rv[1]}, {Rv[2], 0, -Rv[0]}, {-Rv[1], Rv[0], 0}};
      const double A[3][3] = {{c.fy, 0, 0}, {0, c.fx, 0}, {-c.fy * c.cx, -c.fx * c.cy, c.fx * c.fy}};
#pragma unroll
      for (int r = 0; r < 2; r++) {
        const double dd0 = ((double)e.obs[2 * r] - (l0 * N[r]) / (ln * ln)) / ln;
        const double dd1 = ((double)e.obs[2 * r + 1] - (l1 * N[r]) / (ln * ln)) / ln;
        const double dd2 = 1.0 / ln;
        double M[3];
#pragma unroll
        for (int k = 0; k < 3; k++) M[k] = dd0 * A[0][k] + dd1 * A[1][k] + dd2 * A[2][k];
#pragma unroll
        for (int k = 0; k < 3; k++) {
          J[r][k] = -(M[0] * Sn[0][k] + M[1] * Sn[1][k] + M[2] * Sn[2][k]);
          J[r][3 + k] = -(M[0] * Sv[0][k] + M[1] * Sv[1][k] + M[2] * Sv[2][k]);
        }
      }
#pragma unroll
      for (int k = 0; k < 6; k++) J[2][k] = 0.0;
      return;
    }
    const double e2 = (double)e.obs[2] * l0 + (double)e.obs[3] * l1 + l2;
    // pinned P7: row 0 = end-point values, row 1 = 0
    const double d0 = ((double)e.obs[2] - (l0 * e2) / (ln * ln)) / ln;
    const double d1 = ((double)e.obs[3] - (l1 * e2) / (ln * ln)) / ln;
    const double M0[3] = {d0 * c.fy + 1.0 * (-c.fy * c.cx), d1 * c.fx + 1.0 * (c.fx * c.cy), 1.0 * (c.fx * c.fy)};
    // D = [-S(Rv) - S(tRv) | -S(Rv)] (rows 0..2 of dLc_ddelta)
    const double S1[3][3] = {{0, -Rv[2], Rv[1]}, {Rv[2], 0, -Rv[0]}, {-Rv[1], Rv[0], 0}};
    const double S2[3][3] = {{0, -tRv[2], tRv[1]}, {tRv[2], 0, -tRv[0]}, {-tRv[1], tRv[0], 0}};
    for (int k = 0; k < 3; k++) {
      J[0][k] = M0[0] * (-1.0 * S1[0][k] - S2[0][k]) + M0[1] * (-1.0 * S1[1][k] - S2[1][k]) +
                M0[2] * (-1.0 * S1[2][k] - S2[2][k]);
      J[0][3 + k] = M0[0] * (-1.0 * S1[0][k]) + M0[1] * (-1.0 * S1[1][k]) + M0[2] * (-1.0 * S1[2][k]);
      J[1][k] = 0.0;
      J[1][3 + k] = 0.0;
      J[2][k] = 0.0;
      J[2][3 + k] = 0.0;
    }
    return;
  }
  const double X[3] = {e.X[0], e.X[1], e.X[2]};
  double p[3];
  quat_rotate(T.q, X, p);
  p[0] += T.t[0]; p[1] += T.t[1]; p[2] += T.t[2];
  const double x = p[0], y = p[1], invz = 1.0 / p[2], invz_2 = invz * invz;
  J[0][0] = x * y * invz_2 * c.fx;
  J[0][1] = -(1 + (x * x * invz_2)) * c.fx;
  J[0][2] = y * invz * c.fx;
  J[0][3] = -invz * c.fx;
  J[0][4] = 0;
  J[0][5] = x * invz_2 * c.fx;
  J[1][0] = (1 + y * y * invz_2) * c.fy;
  J[1][1] = -x * y * invz_2 * c.fy;
  J[1][2] = -x * invz * c.fy;
  J[1][3] = 0;
  J[1][4] = -invz * c.fy;
  J[1][5] = y * invz_2 * c.fy;
  if (e.kind == 1) {
    J[2][0] = J[0][0] - c.bf * y * invz_2;
    J[2][1] = J[0][1] + c.bf * x * invz_2;
    J[2][2] = J[0][2];
    J[2][3] = J[0][3];
    J[2][4] = 0;
    J[2][5] = J[0][5] - c.bf * invz_2;
  } else {
    for (int k = 0; k < 6; k++) J[2][k] = 0;
  }
}

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Reduce NV doubles over the block; result valid in every thread.
template <int NV, int kPoseWaves>
__device__ void block_sum(double* v, PoseShared& S) {
  const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
#pragma unroll
  for (int k = 0; k < NV; k++) v[k] = wave_sum_d(v[k]);
  if (kPoseWaves == 1) return;
  if (lane == 0)
#pragma unroll
    for (int k = 0; k < NV; k++) S.red[wave][k] = v[k];
  __syncthreads();
#pragma unroll
  for (int k = 0; k < NV; k++) {
    double r = S.red[0][k];
#pragma unroll
    for (int w = 1; w < kPoseWaves; w++) r += S.red[w][k];
    v[k] = r;
  }
  __syncthreads();
}

// One halving step of the transposed wave reduction: lanes whose `mask` bit
// is set keep the upper half of v[0..2h), the others the lower half, each
// adding its partner's copy of the half it keeps.
template <int H>
__device__ __forceinline__ void tr_step(double* v, int mask) {
  const bool hi = (threadIdx.x & mask) != 0;
#pragma unroll
  for (int k = 0; k < H; k++) {
    const double send = hi ? v[k] : v[k + H];
    const double keep = hi ? v[k + H] : v[k];
    v[k] = keep + __shfl_xor(send, mask, 64);
  }
}

// Sum 28 per-thread doubles over the block into out[0..28)
// (shared memory). 29 shuffles per wave instead of 28 full butterflies.
template <int kPoseWaves>
__device__ void block_sum28_to(double* v, PoseShared& S, double* out) {
  const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
  tr_step<14>(v, 1);   // index k + 14*b0
  tr_step<7>(v, 2);    // k + 7*b1 + 14*b0, k < 7
  v[7] = 0;
  tr_step<4>(v, 4);    // j = k + 4*b2 (j == 7 is padding)
  tr_step<2>(v, 8);
  tr_step<1>(v, 16);   // j = b4 + 2*b3 + 4*b2
  v[0] += __shfl_xor(v[0], 32, 64);
  const int j = ((lane >> 4) & 1) + 2 * ((lane >> 3) & 1) + 4 * ((lane >> 2) & 1);
  if (lane < 32 && j < 7) S.red[wave][j + 7 * ((lane >> 1) & 1) + 14 * (lane & 1)] = v[0];
  __syncthreads();
  if (t < 28) {
    double r = S.red[0][t];
#pragma unroll
    for (int w = 1; w < kPoseWaves; w++) r += S.red[w][t];
    out[t] = r;
  }
  __syncthreads();
}

__device__ __forceinline__ void huber(double chi, double delta, double dsqr, double* rho0,
                                      double* rho1) {
  if (chi <= dsqr) {
    *rho0 = chi;
    *rho1 = 1.;
  } else {
    const double sq = sqrt(chi);
    *rho0 = 2 * sq * delta - dsqr;
    *rho1 = delta / sq;
  }
}

// A point edge's chi2 at T and its robust value: edge_error's arithmetic for
// kinds 0 / 1 without branches (the mono projection's two divisions issued for
// every edge, the stereo 1 / z taken from the first), so that the unrolled
// trial pass overlaps several edges' dependent FP64 chains.
__device__ __forceinline__ double point_chi2(const PoseEdge& e, const PoseCam& c, const SE3d& T,
                                             bool robust, double dMono, double dsMono,
                                             double dStereo, double dsStereo, double* rho0) {
  const double X[3] = {e.X[0], e.X[1], e.X[2]};
  double p[3];
  quat_rotate(T.q, X, p);
  p[0] += T.t[0]; p[1] += T.t[1]; p[2] += T.t[2];
  const bool mono = e.kind == 0;
  const double q0 = (mono ? p[0] : 1.0) / p[2];
  const double q1 = p[1] / p[2];
  const float invz = (float)q0;
  const double u = mono ? q0 * c.fx + c.cx : p[0] * (double)invz * c.fx + c.cx;
  const double v = mono ? q1 * c.fy + c.cy : p[1] * (double)invz * c.fy + c.cy;
  const double e0 = (double)e.obs[0] - u, e1 = (double)e.obs[1] - v;
  const double e2 = (double)e.obs[2] - (u - c.bf * (double)invz);
  const double info = (double)e.info;
  double x2 = e0 * info * e0;
  x2 += e1 * info * e1;
  const double x3 = x2 + e2 * info * e2;
  x2 = mono ? x2 : x3;
  double r = x2;
  if (robust) {
    const double delta = mono ? dMono : dStereo, dsqr = mono ? dsMono : dsStereo;
    const double sq = sqrt(x2);
    r = x2 <= dsqr ? x2 : 2 * sq * delta - dsqr;
  }
  *rho0 = r;
  return x2;
}

// A point edge's linearisation (edge_error + edge_jacobian for kinds 0 / 1,
// branch-free: 1 / z and the mono quotients all issued), its chi2 and robust
// weight; the caller accumulates H / b in its edge order.
struct PointLin {
  double err[3], J[3][6], x2, w, r0, info;
};
__device__ __forceinline__ void point_lin(const PoseEdge& e, const PoseCam& c, const SE3d& T,
                                          bool robust, double dMono, double dsMono, double dStereo,
                                          double dsStereo, PointLin& o) {
  const double X[3] = {e.X[0], e.X[1], e.X[2]};
  double p[3];
  quat_rotate(T.q, X, p);
  p[0] += T.t[0]; p[1] += T.t[1]; p[2] += T.t[2];
  const bool mono = e.kind == 0;
  const double iz = 1.0 / p[2];
  const double m0 = p[0] / p[2], m1 = p[1] / p[2];
  const float invzf = (float)iz;
  const double u = mono ? m0 * c.fx + c.cx : p[0] * (double)invzf * c.fx + c.cx;
  const double v = mono ? m1 * c.fy + c.cy : p[1] * (double)invzf * c.fy + c.cy;
  o.err[0] = (double)e.obs[0] - u;
  o.err[1] = (double)e.obs[1] - v;
  o.err[2] = mono ? 0.0 : (double)e.obs[2] - (u - c.bf * (double)invzf);
  o.info = (double)e.info;
  double x2 = o.err[0] * o.info * o.err[0];
  x2 += o.err[1] * o.info * o.err[1];
  x2 += o.err[2] * o.info * o.err[2];
  o.x2 = x2;
  o.w = 1.0;
  o.r0 = x2;
  if (robust) {
    const double delta = mono ? dMono : dStereo, dsqr = mono ? dsMono : dsStereo;
    const double sq = sqrt(x2);
    const bool in = x2 <= dsqr;
    o.r0 = in ? x2 : 2 * sq * delta - dsqr;
    o.w = in ? 1.0 : delta / sq;
  }
  const double x = p[0], y = p[1], invz_2 = iz * iz;
  double (&J)[3][6] = o.J;
  J[0][0] = x * y * invz_2 * c.fx;
  J[0][1] = -(1 + (x * x * invz_2)) * c.fx;
  J[0][2] = y * iz * c.fx;
  J[0][3] = -iz * c.fx;
  J[0][4] = 0;
  J[0][5] = x * invz_2 * c.fx;
  J[1][0] = (1 + y * y * invz_2) * c.fy;
  J[1][1] = -x * y * invz_2 * c.fy;
  J[1][2] = -x * iz * c.fy;
  J[1][3] = 0;
  J[1][4] = -iz * c.fy;
  J[1][5] = y * invz_2 * c.fy;
  J[2][0] = mono ? 0.0 : J[0][0] - c.bf * y * invz_2;
  J[2][1] = mono ? 0.0 : J[0][1] + c.bf * x * invz_2;
  J[2][2] = mono ? 0.0 : J[0][2];
  J[2][3] = mono ? 0.0 : J[0][3];
  J[2][4] = 0;
  J[2][5] = mono ? 0.0 : J[0][5] - c.bf * invz_2;
}

__device__ __forceinline__ void accumulate_lin(const PointLin& o, double* acc) {
  acc[27] += o.r0;
  const double wi = o.w * o.info;
#pragma unroll
  for (int i = 0; i < 6; i++) {
    double bi = o.J[0][i] * o.info * o.err[0];
    bi += o.J[1][i] * o.info * o.err[1];
    bi += o.J[2][i] * o.info * o.err[2];
    acc[21 + i] -= o.w * bi;
  }
#pragma unroll
  for (int i = 0; i < 6; i++) {
#pragma unroll
    for (int j = i; j < 6; j++) {
      double h = o.J[0][i] * wi * o.J[0][j];
      h += o.J[1][i] * wi * o.J[1][j];
      h += o.J[2][i] * wi * o.J[2][j];
      acc[6 * i - i * (i - 1) / 2 + (j - i)] += h;
    }
  }
}

// point_lin + accumulate_lin with the Jacobian built one row at a time into
// the accumulators (6 doubles live instead of 18; H / b summed row by row, a
// different order of the same products). Returns chi2; skips the
// accumulation for inactive edges.
template <int>
__device__ __forceinline__ double point_lin_rows(const PoseEdge& e, const PoseCam& c, const SE3d& T,
                                                 bool robust, double dMono, double dsMono,
                                                 double dStereo, double dsStereo, bool on,
                                                 double* acc) {
  const double X[3] = {e.X[0], e.X[1], e.X[2]};
  double p[3];
  quat_rotate(T.q, X, p);
  p[0] += T.t[0]; p[1] += T.t[1]; p[2] += T.t[2];
  const bool mono = e.kind == 0;
  const double iz = 1.0 / p[2];
  const double m0 = p[0] / p[2], m1 = p[1] / p[2];
  const float invzf = (float)iz;
  const double u = mono ? m0 * c.fx + c.cx : p[0] * (double)invzf * c.fx + c.cx;
  const double v = mono ? m1 * c.fy + c.cy : p[1] * (double)invzf * c.fy + c.cy;
  const double e0 = (double)e.obs[0] - u, e1 = (double)e.obs[1] - v;
  const double e2 = mono ? 0.0 : (double)e.obs[2] - (u - c.bf * (double)invzf);
  const double info = (double)e.info;
  double x2 = e0 * info * e0;
  x2 += e1 * info * e1;
  x2 += e2 * info * e2;
  double w = 1.0, r0 = x2;
  if (robust) {
    const double delta = mono ? dMono : dStereo, dsqr = mono ? dsMono : dsStereo;
    const double sq = sqrt(x2);
    const bool in = x2 <= dsqr;
    r0 = in ? x2 : 2 * sq * delta - dsqr;
    w = in ? 1.0 : delta / sq;
  }
  if (!on) return x2;
  acc[27] += r0;
  const double wi = w * info;
  const double x = p[0], y = p[1], invz_2 = iz * iz;
  auto row = [&](const double (&j)[6], double er) {
#pragma unroll
    for (int i = 0; i < 6; i++) acc[21 + i] -= w * (j[i] * info * er);
#pragma unroll
    for (int i = 0; i < 6; i++)
#pragma unroll
      for (int q = i; q < 6; q++) acc[6 * i - i * (i - 1) / 2 + (q - i)] += j[i] * wi * j[q];
  };
  const double j0[6] = {x * y * invz_2 * c.fx, -(1 + (x * x * invz_2)) * c.fx, y * iz * c.fx,
                        -iz * c.fx, 0.0, x * invz_2 * c.fx};
  row(j0, e0);
  {
    const double j1[6] = {(1 + y * y * invz_2) * c.fy, -x * y * invz_2 * c.fy, -x * iz * c.fy, 0.0,
                          -iz * c.fy, y * invz_2 * c.fy};
    row(j1, e1);
  }
  if (!mono) {
    const double j2[6] = {j0[0] - c.bf * y * invz_2, j0[1] + c.bf * x * invz_2, j0[2], j0[3], 0.0,
                          j0[5] - c.bf * invz_2};
    row(j2, e2);
  }
  return x2;
}

__device__ bool solve6(const double A[6][6], const double b[6], double x[6]) {
  // LDL^T without pivoting (pinned P8); fully unrolled so every array index
  // is a compile-time constant (registers, no scratch). One division per
  // pivot (its reciprocal scales the column and the back substitution): the
  // step differs from the oracle's quotients in the last bits only.
  double L[6][6], D[6], rD[6];
  bool ok = true;
#pragma unroll
  for (int j = 0; j < 6; j++) {
    double d = A[j][j];
#pragma unroll
    for (int k = 0; k < j; k++) d -= L[j][k] * L[j][k] * D[k];
    D[j] = d;
    rD[j] = 1.0 / d;
    ok = ok && (d > 0);
#pragma unroll
    for (int i = j + 1; i < 6; i++) {
      double s = A[i][j];
#pragma unroll
      for (int k = 0; k < j; k++) s -= L[i][k] * L[j][k] * D[k];
      L[i][j] = s * rD[j];
    }
  }
  if (!ok) return false;
  double y[6];
#pragma unroll
  for (int i = 0; i < 6; i++) {
    double s = b[i];
#pragma unroll
    for (int k = 0; k < i; k++) s -= L[i][k] * y[k];
    y[i] = s;
  }
#pragma unroll
  for (int i = 5; i >= 0; i--) {
    double s = y[i] * rD[i];
#pragma unroll
    for (int k = i + 1; k < 6; k++) s -= L[k][i] * x[k];
    x[i] = s;
  }
  return true;
}

struct PoseArgs {
  const KeyPointD* kps_un;
  const float* uright;
  const int* match;           // last-frame index per current keypoint, or -1
  const uint8_t* has_mp;      // alternative to match (host API): 1 = edge
  const float* mp_xyz;        // with match: last frame's xyz (per stream kp_pitch*3); else own
  const int* n;
  int kp_pitch;
  // lines (host API only)
  const float* kl_obs;
  const int* kl_octave;
  const uint8_t* has_ml;
  const float* ml_xyz;
  int nl;
  float* Tcw;                 // in/out per stream (stride pose_stride)
  int pose_stride;
  uint8_t* outlier;           // in/out per stream kp_pitch
  uint8_t* line_outlier;      // in/out (host API)
  int* ninliers;              // per stream (stride nm_stride)
  int nm_stride;
  const StreamState* active;
  PoseEdge* edges;            // scratch, per stream kPoseMaxEdges
  // tracker-mode lines (see PoseLaunch)
  const orbpl_keyline* t_kl_un;
  const int* t_lmatch;
  const float* t_ml_xyz;
  const int* t_nl;
  uint8_t* t_loutlier;
  int lpitch;
  int prof;                   // debug: phase stamps of stream 0 into g_pose_prof
  int fixed_line_jac;         // ORBPL_POSE_FIXED_LINE_JAC
  int gate_lm;                // 1: only active[s].lm_active; 2: only trk && trk_go
  const int* list;            // optional: the streams to run (list_n of them)
  const int* list_n;
  int ecap;                   // edges per stream (chi2 / flags in LDS)
  int pcap, lcap;             // point / line edge records in LDS (the rest global)
};

// k_pose's dynamic LDS: PoseShared, chi2 / level / outlier flag per edge,
// pcap point records, lcap line records
__host__ __device__ __forceinline__ size_t pose_lds_bytes(int ecap, int pcap, int lcap) {
  const size_t h = (sizeof(PoseShared) + 15) & ~(size_t)15;
  const size_t f = ((size_t)ecap * 6 + 15) & ~(size_t)15;
  return h + f + (size_t)pcap * 32 + (size_t)lcap * sizeof(PoseEdge);
}

// debug (ORBPL_POSE_PROFILE): accumulated wall-clock ticks (100 MHz) of
// stream 0's pose: [0] edges, [1] linearize+reduce, [2] solve+exp,
// [3] trial errors+reduce, [4] classify, [5] LM iterations, [6] trials
__device__ long long g_pose_prof[8];

__device__ void se3_from_T(const float* T, SE3d& s) {
  double R[3][3];
  for (int r = 0; r < 3; r++)
    for (int cc = 0; cc < 3; cc++) R[r][cc] = T[r * 4 + cc];
  s.q = quat_from_R(R);
  normalize_rotation(s.q);
  s.t[0] = T[3]; s.t[1] = T[7]; s.t[2] = T[11];
}

// kPoseThreads threads per stream (one workgroup per stream), kMinWaves waves
// per SIMD the register budget must allow (1: ~300 VGPRs; 2: 256 and a few
// spills); launch_pose picks both from the streams per CU
template <int kPoseThreads>
__device__ __forceinline__ void pose_stream(const TrackConsts& tc, const PoseArgs& a,
                                            PoseShared& S, PoseLds V, const int s) {
  constexpr int kPoseWaves = kPoseThreads / 64;
  const int t = threadIdx.x;
  // TrackWithMotionModel returns before optimising when no last frame exists
  // or nmatches < 20 after the retry (Tracking.cc:1255-1265).
  // (with lines: also when LineMatcher found < 15, Tracking.cc:1260-1265)
  // TrackLocalMap's pose runs only where TrackWithMotionModel succeeded
  // (the TrackReferenceKeyFrame pose leaves every other stream's count alone:
  // it is the motion model's)
  if (a.gate_lm == 2 && !(a.active[s].trk && a.active[s].trk_go)) return;
  if (a.gate_lm ? (a.gate_lm == 1 ? !a.active[s].lm_active
                                  : !(a.active[s].trk && a.active[s].trk_go))
                : (a.active && (!a.active[s].has_last || a.active[s].nmatches < 20 ||
                                (a.t_kl_un && a.active[s].nlmatches < 15)))) {
    if (t == 0) a.ninliers[(long long)s * a.nm_stride] = 0;
    return;
  }
  const PoseCam c{tc.fx, tc.fy, tc.cx, tc.cy, tc.bf, a.fixed_line_jac};
  const bool stamp = a.prof && s == 0 && t == 0;
  long long pt[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  long long t0 = stamp ? (long long)wall_clock64() : 0;
  auto lap = [&](int k) {
    if (stamp) {
      const long long t1 = (long long)wall_clock64();
      pt[k] += t1 - t0;
      t0 = t1;
    }
  };
  const long long cb = (long long)s * a.kp_pitch;
  const int n = a.n[s];
  uint8_t* outl = a.outlier + cb;
  // ---- edges (Optimizer.cc:2190-2283, 2285-2352), compacted in index order ----
  {
    char* G = reinterpret_cast<char*>(a.edges) + (long long)s * kPoseMaxEdges * (32 + sizeof(PoseEdge));
    V.pg = reinterpret_cast<float4*>(G);
    V.lg = reinterpret_cast<PoseEdge*>(G + kPoseMaxEdges * 32);
  }
  const int wave = t >> 6, lane = t & 63;
  int npts = 0;
  for (int base = 0; base < n; base += kPoseThreads) {
    const int i = base + t;
    int j = -1;
    if (i < n) {
      if (a.match) j = a.match[cb + i];
      else if (a.has_mp[cb + i]) j = i;
    }
    const int flag = j >= 0 ? 1 : 0;
    int incl = flag;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      int u = __shfl_up(incl, o, 64);
      if (lane >= o) incl += u;
    }
    if (lane == 63) S.wsum[wave] = incl;
    __syncthreads();
    int off = npts;
    int tot = 0;
    for (int w = 0; w < kPoseWaves; w++) {
      if (w < wave) off += S.wsum[w];
      tot += S.wsum[w];
    }
    const int k = off + incl - flag;
    if (flag && k < a.ecap) {
      const KeyPointD kp = a.kps_un[cb + i];
      const float ur = a.uright[cb + i];
      store_point(V, k, kp.x, kp.y, ur, tc.inv_sigma2[kp.octave], a.mp_xyz + (cb + j) * 3, i);
      V.level[k] = 0;
      V.out_flag[k] = 0;
      outl[i] = 0;
    }
    npts += tot;
    __syncthreads();
  }
  npts = min(npts, a.ecap);
  V.npts = npts;
  // line edges in line index order: a block-wide prefix over the matched lines
  // (Optimizer.cc:2285-2352)
  int nlines = 0;
  {
    const bool trk = a.t_kl_un != nullptr;
    const long long lb = (long long)s * a.lpitch;
    const int nlc = trk ? a.t_nl[s] : a.nl;
    for (int base = 0; base < nlc; base += kPoseThreads) {
      const int i = base + t;
      int m = -1;
      if (i < nlc) m = trk ? a.t_lmatch[lb + i] : (a.has_ml[i] ? i : -1);
      const int flag = m >= 0 ? 1 : 0;
      int incl = flag;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        int u = __shfl_up(incl, o, 64);
        if (lane >= o) incl += u;
      }
      if (lane == 63) S.wsum[wave] = incl;
      __syncthreads();
      int off = npts + nlines;
      int tot = 0;
      for (int w = 0; w < kPoseWaves; w++) {
        if (w < wave) off += S.wsum[w];
        tot += S.wsum[w];
      }
      const int k = off + incl - flag;
      if (flag && k < a.ecap) {
        if (i < n) outl[i] = 0;  // reference writes mvbOutlier here (Optimizer.cc:2308)
        PoseEdge e;
        e.kind = 2;
        e.idx = i;
        if (trk) {
          const orbpl_keyline kl = a.t_kl_un[lb + i];
          e.obs[0] = kl.startPointX;
          e.obs[1] = kl.startPointY;
          e.obs[2] = kl.endPointX;
          e.obs[3] = kl.endPointY;
          e.info = tc.inv_sigma2[kl.octave];
          const float* X = a.t_ml_xyz + (lb + m) * 6;
          for (int q = 0; q < 6; q++) e.X[q] = X[q];
          V.out_flag[k] = a.t_loutlier[lb + i];
        } else {
          for (int q = 0; q < 4; q++) e.obs[q] = a.kl_obs[4 * i + q];
          e.info = tc.inv_sigma2[a.kl_octave[i]];
          for (int q = 0; q < 6; q++) e.X[q] = a.ml_xyz[6 * i + q];
          V.out_flag[k] = a.line_outlier[i];
        }
        e.pad = 0;
        (k - npts < V.lcap ? V.lrec : V.lg)[k - npts] = e;
        V.level[k] = 0;
      }
      nlines += tot;
      __syncthreads();
    }
    nlines = min(nlines, a.ecap - npts);
    if (t == 0) {
      S.misc[0] = npts + nlines;
      S.misc[2] = nlines;
    }
  }
  __syncthreads();
  lap(0);
  const int ne = S.misc[0];
  nlines = S.misc[2];
  float* Tout = a.Tcw + (long long)s * a.pose_stride;
  if (npts < 3 && nlines < 3) {
    if (t == 0) a.ninliers[(long long)s * a.nm_stride] = 0;
    return;
  }
  // const float deltaMono = sqrt(5.991) (Optimizer.cc:2184-2186): double sqrt
  // rounded to float; RobustKernelHuber::setDelta keeps dsqr as a float.
  const double deltaMono = (double)(float)sqrt(5.991), deltaStereo = (double)(float)sqrt(7.815);
  const double dsqrMono = (double)(float)(deltaMono * deltaMono);
  const double dsqrStereo = (double)(float)(deltaStereo * deltaStereo);
  SE3d T0;
  se3_from_T(Tout, T0);
  int nBadOut = 0;
  bool robust = true;
  for (int round = 0; round < 4; round++) {
    SE3d T = T0;
    uni(T);
    // ---- optimizer.optimize(10) ----
    int nact = 0;
    for (int k = t; k < ne; k += kPoseThreads) nact += V.level[k] == 0;
    {
      double v = nact;
      block_sum<1, kPoseWaves>(&v, S);
      nact = (int)v;
    }
    if (nact > 0) {
      double lambda = 0, ni = 2;
      int nBadLM = 0;
      double x[6] = {0, 0, 0, 0, 0, 0};
      for (int it = 0; it < 10; it++) {
        // computeActiveErrors + buildSystem at T (fused: same estimate)
        double R[3][3];
        quat_to_R(T.q, R);
        uni(R);
        double acc[28];
        for (int k = 0; k < 28; k++) acc[k] = 0;
        int k = t;
#if defined(ORBPL_POSE_ROWS)
        for (; k < npts; k += kPoseThreads) {
          const PoseEdge e = fetch_point(V, k);
          const bool on = V.level[k] == 0;
          const double x2 = point_lin_rows<0>(e, c, T, robust, deltaMono, dsqrMono, deltaStereo,
                                              dsqrStereo, on, acc);
          if (on) V.chi2[k] = (float)x2;
        }
#elif !defined(ORBPL_POSE_LIN1)
        // point edges two at a time (branch-free, this thread's edge order kept)
        for (; k + kPoseThreads < npts; k += 2 * kPoseThreads) {
          PointLin o0, o1;
          const PoseEdge e0 = fetch_point(V, k), e1 = fetch_point(V, k + kPoseThreads);
          const bool on0 = V.level[k] == 0, on1 = V.level[k + kPoseThreads] == 0;
          point_lin(e0, c, T, robust, deltaMono, dsqrMono, deltaStereo, dsqrStereo, o0);
          point_lin(e1, c, T, robust, deltaMono, dsqrMono, deltaStereo, dsqrStereo, o1);
          if (on0) {
            V.chi2[k] = (float)o0.x2;
            accumulate_lin(o0, acc);
          }
          if (on1) {
            V.chi2[k + kPoseThreads] = (float)o1.x2;
            accumulate_lin(o1, acc);
          }
        }
#endif
        for (; k < ne; k += kPoseThreads) {
          const PoseEdge e = fetch_edge(V, k);
          if (V.level[k]) continue;
          double err[3], J[3][6];
          edge_error(e, c, T, R, err);
          // rows beyond the edge's dimension are zero (err[2] = 0 and J row 2
          // = 0 for mono and line edges): adding them leaves every sum exact
          double x2 = err[0] * (double)e.info * err[0];
          x2 += err[1] * (double)e.info * err[1];
          x2 += err[2] * (double)e.info * err[2];
          V.chi2[k] = (float)x2;
          double w = 1.0, r0 = x2;
          if (robust) {
            const bool isMono = e.kind == 0;
            huber(x2, isMono ? deltaMono : deltaStereo, isMono ? dsqrMono : dsqrStereo, &r0, &w);
          }
          acc[27] += r0;
          edge_jacobian(e, c, T, R, J);
          const double info = (double)e.info;
          const double wi = w * info;
#pragma unroll
          for (int i = 0; i < 6; i++) {
            double bi = J[0][i] * info * err[0];
            bi += J[1][i] * info * err[1];
            bi += J[2][i] * info * err[2];
            acc[21 + i] -= w * bi;
          }
#pragma unroll
          for (int i = 0; i < 6; i++) {
#pragma unroll
            for (int j = i; j < 6; j++) {
              double h = J[0][i] * wi * J[0][j];
              h += J[1][i] * wi * J[1][j];
              h += J[2][i] * wi * J[2][j];
              acc[6 * i - i * (i - 1) / 2 + (j - i)] += h;
            }
          }
        }
        lap(7);
        block_sum28_to<kPoseWaves>(acc, S, S.sys[0]);
        lap(1);
        pt[5]++;
        double b[6];
        for (int i = 0; i < 6; i++) b[i] = S.sys[0][21 + i];
        double currentChi = S.sys[0][27];
        const double iniChi = currentChi;
        if (it == 0) {
          double md = 0;
          for (int j = 0, q = 0; j < 6; q += 6 - j, j++) md = fmax(fabs(S.sys[0][q]), md);
          lambda = 1e-5 * md;
          ni = 2;
          nBadLM = 0;
        }
        double rho = 0;
        int qmax = 0;
        do {
          const SE3d backup = T;
          double Hl[6][6];
          {
            const double* sy = S.sys[0];
#pragma unroll
            for (int i = 0; i < 6; i++)
#pragma unroll
              for (int j = i; j < 6; j++) {
                const double v = sy[6 * i - i * (i - 1) / 2 + (j - i)];
                Hl[i][j] = v;
                Hl[j][i] = v;
              }
          }
#pragma unroll
          for (int j = 0; j < 6; j++) Hl[j][j] += lambda;
          const bool ok2 = solve6(Hl, b, x);
          T = se3_mul(se3_exp(x), T);
          uni(T);
          lap(2);
          pt[6]++;
          // computeActiveErrors at the trial estimate
          double R2[3][3];
          quat_to_R(T.q, R2);
          uni(R2);
          double tc2 = 0;
          // point edges four at a time (this thread's edge order kept)
          int k = t;
          for (; k + 3 * kPoseThreads < npts; k += 4 * kPoseThreads) {
            PoseEdge e4[4];
            bool on[4];
            double x4[4], r4[4];
#pragma unroll
            for (int u = 0; u < 4; u++) {
              e4[u] = fetch_point(V, k + u * kPoseThreads);
              on[u] = V.level[k + u * kPoseThreads] == 0;
            }
#pragma unroll
            for (int u = 0; u < 4; u++)
              x4[u] = point_chi2(e4[u], c, T, robust, deltaMono, dsqrMono, deltaStereo, dsqrStereo, &r4[u]);
#pragma unroll
            for (int u = 0; u < 4; u++)
              if (on[u]) {
                V.chi2[k + u * kPoseThreads] = (float)x4[u];
                tc2 += r4[u];
              }
          }
          for (; k < ne; k += kPoseThreads) {
            const PoseEdge e = fetch_edge(V, k);
            if (V.level[k]) continue;
            double err[3];
            edge_error(e, c, T, R2, err);
            double x2 = err[0] * (double)e.info * err[0];
            x2 += err[1] * (double)e.info * err[1];
            if (e.kind == 1) x2 += err[2] * (double)e.info * err[2];
            V.chi2[k] = (float)x2;
            double r0 = x2, w;
            if (robust) {
              const bool isMono = e.kind == 0;
              huber(x2, isMono ? deltaMono : deltaStereo, isMono ? dsqrMono : dsqrStereo, &r0, &w);
            }
            tc2 += r0;
          }
          block_sum<1, kPoseWaves>(&tc2, S);
          lap(3);
          double tempChi = ok2 ? tc2 : 1.7976931348623157e308;
          rho = currentChi - tempChi;
          double scale = 0;
          for (int j = 0; j < 6; j++) scale += x[j] * (lambda * x[j] + b[j]);
          scale += 1e-3;
          rho /= scale;
          if (rho > 0 && isfinite(tempChi)) {
            double al = 1. - pow((2 * rho - 1), 3);
            al = fmin(al, 2. / 3.);
            const double sf = fmax(1. / 3., al);
            lambda *= sf;
            ni = 2;
            currentChi = tempChi;
          } else {
            lambda *= ni;
            ni *= 2;
            T = backup;
            uni(T);
          }
          qmax++;
        } while (rho < 0 && qmax < 10);
#ifdef ORBPL_POSE_TRIALS
        if (s == 0 && t == 0) printf("pose blk0 round %d it %d trials %d rho %g\n", round, it, qmax, rho);
#endif
        if (qmax == 10 || rho == 0) break;
        if ((iniChi - currentChi) * 1e3 < iniChi) nBadLM++;
        else nBadLM = 0;
        if (nBadLM >= 3) break;
      }
    }
    // ---- classify (Optimizer.cc:2387-2470) ----
    double R[3][3];
    quat_to_R(T.q, R);
    uni(R);
    int nbad = 0;
    // point edges four at a time; an edge's outlier flag is kept in out_flag
    // (for points it mirrors mvbOutlier[idx], written here only)
    int k = t;
    for (; k + 3 * kPoseThreads < npts; k += 4 * kPoseThreads) {
      PoseEdge e4[4];
      double x4[4], r4[4];
#pragma unroll
      for (int u = 0; u < 4; u++) e4[u] = fetch_point(V, k + u * kPoseThreads);
#pragma unroll
      for (int u = 0; u < 4; u++)
        x4[u] = point_chi2(e4[u], c, T, false, deltaMono, dsqrMono, deltaStereo, dsqrStereo, &r4[u]);
#pragma unroll
      for (int u = 0; u < 4; u++) {
        const int kk = k + u * kPoseThreads;
        float chi2 = V.chi2[kk];
        if (V.out_flag[kk]) {
          chi2 = (float)x4[u];
          V.chi2[kk] = chi2;
        }
        const bool bad = chi2 > (e4[u].kind == 0 ? 5.991f : 7.815f);
        V.out_flag[kk] = bad;
        outl[e4[u].idx] = bad;
        nbad += bad;
        V.level[kk] = bad ? 1 : 0;
      }
    }
    for (; k < ne; k += kPoseThreads) {
      const PoseEdge e = fetch_edge(V, k);
      const bool was_out = V.out_flag[k] != 0;
      float chi2 = V.chi2[k];
      if (was_out) {
        double err[3];
        edge_error(e, c, T, R, err);
        double x2 = err[0] * (double)e.info * err[0];
        x2 += err[1] * (double)e.info * err[1];
        if (e.kind == 1) x2 += err[2] * (double)e.info * err[2];
        chi2 = (float)x2;
        V.chi2[k] = chi2;
      }
      const float th = e.kind == 0 ? 5.991f : (e.kind == 1 ? 7.815f : 2 * 7.815f);
      const bool bad = chi2 > th;
      V.out_flag[k] = bad;
      if (e.kind != 2) {
        outl[e.idx] = bad;
        nbad += bad;
      }
      V.level[k] = bad ? 1 : 0;
    }
    {
      double v = nbad;
      block_sum<1, kPoseWaves>(&v, S);
      nbad = (int)v;
    }
    nBadOut = nbad;
    lap(4);
    if (round == 2) robust = false;
    // every thread ran the same LM control flow on the same reduced sums, so
    // T is identical in all threads (no broadcast needed)
    if (round == 3 || ne < 10) {
      if (t == 0) {
        double Rf[3][3];
        quat_to_R(T.q, Rf);
        for (int r = 0; r < 3; r++) {
          for (int cc = 0; cc < 3; cc++) Tout[r * 4 + cc] = (float)Rf[r][cc];
          Tout[r * 4 + 3] = (float)T.t[r];
        }
        Tout[12] = 0; Tout[13] = 0; Tout[14] = 0; Tout[15] = 1;
      }
      break;
    }
    __syncthreads();
  }
  for (int k = t; k < ne; k += kPoseThreads) {
    const PoseEdge e = fetch_edge(V, k);
    if (e.kind == 2) {
      if (a.t_kl_un) a.t_loutlier[(long long)s * a.lpitch + e.idx] = V.out_flag[k];
      else a.line_outlier[e.idx] = V.out_flag[k];
    }
  }
  if (t == 0) a.ninliers[(long long)s * a.nm_stride] = npts - nBadOut;
  if (stamp)
    for (int k = 0; k < 8; k++) g_pose_prof[k] = pt[k];
  // (pt[7]: linearize edge loop only; pt[1]: its block reduction)
}

// One workgroup per stream, or (a.list) a small grid looping over the streams
// a list names (the rarely used TrackReferenceKeyFrame pose: a launch of one
// workgroup per stream costs its placement beside the extraction kernels even
// when no stream has work)
template <int kPoseThreads, int kMinWaves>
__global__ void __launch_bounds__(kPoseThreads, kMinWaves) k_pose(TrackConsts tc, PoseArgs a) {
  trk_priority();
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  PoseShared& S = *reinterpret_cast<PoseShared*>(smem_raw);
  PoseLds V;
  {
    char* q = smem_raw + ((sizeof(PoseShared) + 15) & ~(size_t)15);
    V.chi2 = reinterpret_cast<float*>(q);
    V.level = reinterpret_cast<uint8_t*>(q + (size_t)a.ecap * 4);
    V.out_flag = V.level + a.ecap;
    q += ((size_t)a.ecap * 6 + 15) & ~(size_t)15;
    V.prec = reinterpret_cast<float4*>(q);
    V.lrec = reinterpret_cast<PoseEdge*>(q + (size_t)a.pcap * 32);
    V.pcap = a.pcap;
    V.lcap = a.lcap;
  }
  if (a.list) {
    const int n = *a.list_n;
    for (int b = blockIdx.x; b < n; b += gridDim.x) {
      pose_stream<kPoseThreads>(tc, a, S, V, a.list[b]);
      __syncthreads();
    }
  } else {
    pose_stream<kPoseThreads>(tc, a, S, V, blockIdx.x);
  }
}

// ---------------------------------------------------------------------------
// After PoseOptimization: discard outliers (Tracking.cc:1273-1296), velocity
// history, and the next frame's map points (all keypoints with depth,
// UnprojectStereo at the optimised pose, Observations = 1).
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_finish(TrackConsts c, StreamState* __restrict__ st,
                                                const int* __restrict__ n_in, int kp_pitch,
                                                const KeyPointD* __restrict__ kps_un,
                                                const float* __restrict__ depth,
                                                int* __restrict__ match,
                                                uint8_t* __restrict__ outlier,
                                                uint8_t* __restrict__ has_mp,
                                                float* __restrict__ mp_xyz,
                                                int* __restrict__ nobs, LineFinish lf,
                                                int local_map) {
  trk_priority();
  const int s = blockIdx.x, t = threadIdx.x;
  StreamState& S = st[s];
  const int n = n_in[s];
  const long long cb = (long long)s * kp_pitch;
  __shared__ float sT[16];
  __shared__ int s_map, s_lmap;
  if (t < 16) sT[t] = S.Tcw[t];
  if (t == 0) {
    s_map = 0;
    s_lmap = 0;
  }
  __syncthreads();
  float Ow[3];
  gemm_neg_Rt_t(sT, Ow);
  int nmap = 0;
  for (int i = t; i < n; i += 256) {
    const long long o = cb + i;
    if (S.has_last && match[o] >= 0) {
      if (outlier[o]) match[o] = -1;
      else nmap++;
    }
    // next frame's map points: keyframe-style creation (Tracking.cc:625-645)
    const float z = depth[o];
    outlier[o] = 0;
    if (z > 0) {
      const KeyPointD k = kps_un[o];
      const float x3[3] = {(k.x - c.cx) * z * c.invfx, (k.y - c.cy) * z * c.invfy, z};
      float w[3];
      gemm_Rt_x_plus_c(sT, x3, Ow, w);
      mp_xyz[o * 3] = w[0];
      mp_xyz[o * 3 + 1] = w[1];
      mp_xyz[o * 3 + 2] = w[2];
      has_mp[o] = 1;
      nobs[o] = 1;
    } else {
      has_mp[o] = 0;
      nobs[o] = 0;
    }
  }
  if (nmap) atomicAdd(&s_map, nmap);
  if (lf.nl) {
    // lines: outlier discard (Tracking.cc:1298-1314; outliers decrement the
    // count there) and the next frame's map lines (StereoInitialization,
    // Tracking.cc:668-690; the end point is unprojected with the start
    // point's depth, Frame.cc:1192)
    const long long lb = (long long)s * kLineKeep;
    const int nl = lf.nl[s];
    int lmap = 0;
    for (int j = t; j < nl; j += 256) {
      const long long o = lb + j;
      if (S.has_last && lf.lmatch[o] >= 0) {
        if (lf.loutlier[o]) {
          lf.lmatch[o] = -1;
          lmap--;
        } else {
          lmap++;
        }
      }
      lf.loutlier[o] = 0;
      const float zs = lf.dstart[o], ze = lf.dend[o];
      if (zs > 0 && ze > 0) {
        const orbpl_keyline k = lf.kl_un[o];
        const float a3[3] = {(k.startPointX - c.cx) * zs * c.invfx, (k.startPointY - c.cy) * zs * c.invfy, zs};
        const float b3[3] = {(k.endPointX - c.cx) * zs * c.invfx, (k.endPointY - c.cy) * zs * c.invfy, zs};
        gemm_Rt_x_plus_c(sT, a3, Ow, lf.ml_xyz + o * 6);
        gemm_Rt_x_plus_c(sT, b3, Ow, lf.ml_xyz + o * 6 + 3);
        lf.has_ml[o] = 1;
      } else {
        lf.has_ml[o] = 0;
      }
    }
    if (lmap) atomicAdd(&s_lmap, lmap);
  }
  __syncthreads();
  if (t == 0) {
    S.nmatches_map = s_map;
    if (lf.nl) {
      S.nlmatches_map = s_lmap;
      const bool tracked = S.nmatches >= 20 && S.nlmatches >= 15;
      S.ok = S.has_last ? (tracked && (s_map >= 10 || s_lmap >= 15)) : 1;
    } else {
      S.nlmatches_map = 0;
      S.ok = S.has_last ? (S.nmatches >= 20 && s_map >= 10) : 1;
    }
    // TrackReferenceKeyFrame's decision (Tracking.cc:1031)
    if (S.has_last && S.trk) S.ok = S.trk_go && s_map >= 10 && (!lf.nl || s_lmap >= 10);
    // TrackLocalMap runs after a successful TrackWithMotionModel and decides
    // the frame's outcome (Tracking.cc:433-436)
    if (local_map && S.has_last) S.ok = S.ok && S.lm_ok;
    for (int k = 0; k < 16; k++) {
      S.Tlast2[k] = S.Tlast[k];
      S.Tlast[k] = S.Tcw[k];
    }
    S.has_velocity = S.has_last;
    S.has_last = 1;
  }
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
size_t match_smem_bytes() { return sizeof(MatchShared<2048>); }
size_t pose_smem_bytes() { return sizeof(PoseShared); }


void launch_frame_prepare(const TrackConsts& c, const KeyPointD* kps, const int* n, int kp_pitch,
                          const float* depth, long long depth_pitch, KeyPointD* kps_un,
                          float* depth_out, float* uright, int* gcell, int batch, hipStream_t s) {
  hipLaunchKernelGGL(k_frame_prepare, dim3((kp_pitch + 255) / 256, batch), dim3(256), 0, s, c, kps, n,
                     kp_pitch, depth, depth_pitch, kps_un, depth_out, uright, gcell);
}

// u16 depth -> f32, 8 pixels per thread (16-byte loads, 2 x 16-byte stores)
__global__ void __launch_bounds__(256) k_depth_u16(const uint16_t* __restrict__ in,
                                                   float* __restrict__ out, long long n8,
                                                   long long n, float scale) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i < n8) {
    const uint4 v = reinterpret_cast<const uint4*>(in)[i];
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    float4 a, b;
    a.x = (float)(w[0] & 0xFFFFu) * scale;
    a.y = (float)(w[0] >> 16) * scale;
    a.z = (float)(w[1] & 0xFFFFu) * scale;
    a.w = (float)(w[1] >> 16) * scale;
    b.x = (float)(w[2] & 0xFFFFu) * scale;
    b.y = (float)(w[2] >> 16) * scale;
    b.z = (float)(w[3] & 0xFFFFu) * scale;
    b.w = (float)(w[3] >> 16) * scale;
    reinterpret_cast<float4*>(out)[2 * i] = a;
    reinterpret_cast<float4*>(out)[2 * i + 1] = b;
  } else if (i == n8) {
    for (long long k = 8 * n8; k < n; k++) out[k] = (float)in[k] * scale;
  }
}

void launch_depth_u16(const uint16_t* in, float* out, long long n, float scale, hipStream_t s) {
  const long long n8 = n / 8;
  hipLaunchKernelGGL(k_depth_u16, dim3((unsigned)((n8 + 1 + 255) / 256)), dim3(256), 0, s, in, out,
                     n8, n, scale);
}

void launch_predict(StreamState* st, int nstreams, hipStream_t s) {
  hipLaunchKernelGGL(k_predict, dim3((nstreams + 63) / 64), dim3(64), 0, s, st, nstreams);
}

void launch_match_last(const TrackConsts& c, const MatchLaunch& m, int nstreams, hipStream_t s) {
  MatchArgs a;
  a.cur_kps_un = m.cur_kps_un;
  a.cur_desc = m.cur_desc;
  a.cur_uright = m.cur_uright;
  a.cur_gcell = m.cur_gcell;
  a.cur_n = m.cur_n;
  a.last_kps_un = m.last_kps_un;
  a.last_has_mp = m.last_has_mp;
  a.last_outlier = m.last_outlier;
  a.last_xyz = m.last_xyz;
  a.last_desc = m.last_desc;
  a.last_nobs = m.last_nobs;
  a.last_n = m.last_n;
  a.kp_pitch = m.kp_pitch;
  a.Tcw = m.Tcw;
  a.Tlw = m.Tlw;
  a.pose_stride = m.pose_stride;
  a.match = m.match;
  a.nmatches = m.nmatches;
  a.nm_stride = m.nm_stride;
  a.th = m.th;
  a.mono = m.mono;
  a.check_ori = m.check_ori;
  a.retry = m.retry;
  a.active = m.active;
  static const int prof = getenv("ORBPL_MATCH_PROFILE") ? 1 : 0;
  a.prof = prof;
  // threads per frame (ORBPL_MATCH_NT overrides, A/B runs)
  const char* nt_env = getenv("ORBPL_MATCH_NT");   // read per launch: tests vary it
  const int nt = nt_env ? atoi(nt_env) : kMatchLaunchThreads;
#define ORBPL_MATCH_LAUNCH(KM, NTH)                                                          \
  if ((KM == 1024) == (m.kp_pitch <= 1024) && nt == NTH) {                                   \
    set_smem_attr((const void*)k_match_last<KM, NTH>, sizeof(MatchShared<KM>));             \
    hipLaunchKernelGGL((k_match_last<KM, NTH>), dim3(nstreams), dim3(NTH),                  \
                       sizeof(MatchShared<KM>), s, c, a);                                    \
    return;                                                                                  \
  }
  ORBPL_MATCH_LAUNCH(1024, 1024)
  ORBPL_MATCH_LAUNCH(1024, 512)
  ORBPL_MATCH_LAUNCH(1024, 256)
  ORBPL_MATCH_LAUNCH(1024, 128)
  ORBPL_MATCH_LAUNCH(2048, 1024)
  ORBPL_MATCH_LAUNCH(2048, 512)
  ORBPL_MATCH_LAUNCH(2048, 256)
  ORBPL_MATCH_LAUNCH(2048, 128)
#undef ORBPL_MATCH_LAUNCH
  set_smem_attr((const void*)k_match_last<2048, 1024>, sizeof(MatchShared<2048>));
  hipLaunchKernelGGL((k_match_last<2048, 1024>), dim3(nstreams), dim3(1024), sizeof(MatchShared<2048>), s,
                     c, a);
}

int read_match_profile(long long* out8) {
  return hipMemcpyFromSymbol(out8, HIP_SYMBOL(g_match_prof), 8 * sizeof(long long)) == hipSuccess ? 0 : -1;
}

int read_pose_profile(long long* out8) {
  return hipMemcpyFromSymbol(out8, HIP_SYMBOL(g_pose_prof), 8 * sizeof(long long)) == hipSuccess ? 0 : -1;
}

void launch_pose(const TrackConsts& c, const PoseLaunch& p, int nstreams, hipStream_t s) {
  PoseArgs a;
  a.kps_un = p.kps_un;
  a.uright = p.uright;
  a.match = p.match;
  a.has_mp = p.has_mp;
  a.mp_xyz = p.mp_xyz;
  a.n = p.n;
  a.kp_pitch = p.kp_pitch;
  a.kl_obs = p.kl_obs;
  a.kl_octave = p.kl_octave;
  a.has_ml = p.has_ml;
  a.ml_xyz = p.ml_xyz;
  a.nl = p.nl;
  a.Tcw = p.Tcw;
  a.pose_stride = p.pose_stride;
  a.outlier = p.outlier;
  a.line_outlier = p.line_outlier;
  a.ninliers = p.ninliers;
  a.nm_stride = p.nm_stride;
  a.active = p.active;
  a.edges = p.edges;
  a.t_kl_un = p.t_kl_un;
  a.t_lmatch = p.t_lmatch;
  a.t_ml_xyz = p.t_ml_xyz;
  a.t_nl = p.t_nl;
  a.t_loutlier = p.t_loutlier;
  a.lpitch = p.lpitch;
  a.fixed_line_jac = p.fixed_line_jac;
  a.gate_lm = p.gate_lm;
  a.list = p.list;
  a.list_n = p.list_n;
  static const int prof = getenv("ORBPL_POSE_PROFILE") ? 1 : 0;
  a.prof = prof;
  // threads per stream by streams per CU: the widest workgroup while every
  // stream gets its own CU (lowest latency per stream), then narrower ones so
  // that more streams share a CU at one wave per SIMD. At 512 / 1024 streams:
  // 128x1 0.50 / 0.96 ms, 64x1 0.70 / 0.72, 128x2 0.72 / 0.84, 64x2 0.74 / 1.08
  // (isolated; "threads x waves per SIMD"). ORBPL_POSE_CFG="threads,waves"
  // overrides (A/B runs).
  const int cus = device_cu_count();
  int nt = 256, mw = 1;
  if (nstreams > cus) nt = 128;
  if (nstreams > 2 * cus) nt = 64;   // (2 waves per SIMD measured slower at 512 / 1024)
  static const char* cfg = getenv("ORBPL_POSE_CFG");
  if (cfg) sscanf(cfg, "%d,%d", &nt, &mw);
  const int grid = p.list ? (nstreams < kListGrid ? nstreams : kListGrid) : nstreams;
  // LDS: the CU's 160 KiB shared by the workgroups it holds at once (by the
  // grid and the one-wave-per-SIMD register budget); within a workgroup's
  // share every edge's chi2 / flags, the line records, then as many point
  // records as fit. ORBPL_POSE_LDS=bytes overrides the share (A/B runs).
  const int nlmax = p.t_kl_un ? p.lpitch : p.nl;
  a.ecap = std::min(kPoseMaxEdges, p.kp_pitch + nlmax);
  {
    const int maxb = std::max(1, 4 * mw / std::max(1, nt / 64));
    const int bpc = std::min(maxb, std::max(1, (grid + cus - 1) / cus));
    // (capped at 16 KiB: in the pipelined tracker the pose workgroups are
    // placed beside extraction workgroups, and a larger share delays them
    // more than the on-chip records save: 40 KiB -4.5 %, 0 -2.5 % end to end)
    long budget = std::min(163840L / bpc, 16384L);
    static const char* lds_env = getenv("ORBPL_POSE_LDS");
    if (lds_env) budget = std::min(163840L, atol(lds_env));
    const long fixed = (long)pose_lds_bytes(a.ecap, 0, 0);
    a.lcap = fixed + (long)nlmax * (long)sizeof(PoseEdge) <= budget ? nlmax : 0;
    const long room = budget - fixed - (long)a.lcap * (long)sizeof(PoseEdge);
    a.pcap = (int)std::max(0L, std::min((long)std::min(p.kp_pitch, a.ecap), room / 32));
  }
  const size_t smem = pose_lds_bytes(a.ecap, a.pcap, a.lcap);
#define ORBPL_POSE_LAUNCH(NT, MW)                                                 \
  if (nt == NT && mw == MW) {                                                      \
    set_smem_attr((const void*)k_pose<NT, MW>, 163840);                           \
    hipLaunchKernelGGL((k_pose<NT, MW>), dim3(grid), dim3(NT), smem, s, c, a);     \
    return;                                                                        \
  }
  ORBPL_POSE_LAUNCH(256, 1)
  ORBPL_POSE_LAUNCH(128, 1)
  ORBPL_POSE_LAUNCH(64, 1)
  ORBPL_POSE_LAUNCH(256, 2)
  ORBPL_POSE_LAUNCH(128, 2)
  ORBPL_POSE_LAUNCH(64, 2)
#undef ORBPL_POSE_LAUNCH
  set_smem_attr((const void*)k_pose<64, 1>, 163840);
  hipLaunchKernelGGL((k_pose<64, 1>), dim3(grid), dim3(64), smem, s, c, a);
}

void launch_finish(const TrackConsts& c, StreamState* st, const int* n, int kp_pitch,
                   const KeyPointD* kps_un, const float* depth, int* match, uint8_t* outlier,
                   uint8_t* has_mp, float* mp_xyz, int* nobs, const LineFinish& lf, int nstreams,
                   hipStream_t s, int local_map) {
  hipLaunchKernelGGL(k_finish, dim3(nstreams), dim3(256), 0, s, c, st, n, kp_pitch, kps_un, depth,
                     match, outlier, has_mp, mp_xyz, nobs, lf, local_map);
}

}  // namespace orbpl

namespace orbpl {
size_t pose_edge_bytes() { return 32 + sizeof(PoseEdge); }
}  // namespace orbpl
