// Tracking::SearchLocalPoints on gfx950 (restated in oracle/track_oracle.cpp):
//   k_in_frustum   : Frame::IsInFrustum(MapPoint*, viewCosLimit) (Frame.cc:345-401)
//                    + MapPoint::PredictScale (MapPoint.cc:416-431), thread per point
//   k_match_local  : ORBmatcher::SearchByProjection(Frame&, const vector<MapPoint*>&,
//                    th) (ORBmatcher.cc:72-183), one workgroup per frame:
//     index build   - the grid keypoints as records sorted by (octave, column,
//                     row, index) in LDS, one range per (octave, column)
//     phase A       - every map point in parallel: its first 4 candidates in
//                     (distance, grid-scan position) order, whose first two
//                     are the reference's running best / second, with the
//                     keypoints already holding a map point with
//                     Observations() > 0 skipped
//     phase B       - wave 0, map points in order: a point's outcome can only
//                     change if its best or second candidate is claimed by an
//                     earlier accepted point (removing any other candidate
//                     leaves the running top-2 unchanged), so chunks of 64 are
//                     decided at once up to the first such collision; lanes
//                     whose candidates committed points claimed take the next
//                     unclaimed entries of their list (a new scan when it runs
//                     out), all together; the last writer of a
//                     keypoint wins, as F.mvpMapPoints[bestIdx] = pMP does
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "lsd_math.h"
#include "track_common.h"
#include "track_kernels.h"
#include "orbpl_runtime.h"

namespace orbpl {

__global__ void __launch_bounds__(256) k_in_frustum(TrackConsts c, float log_scale, InFrustumArgs a) {
  trk_priority();
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (a.n_arr) {  // batched: stream blockIdx.y
    const int b = blockIdx.y;
    const long long o = (long long)b * a.pitch;
    a.n = a.n_arr[b];
    a.Tcw += (long long)b * a.pose_stride;
    a.xyz += o * 3;
    a.normal += o * 3;
    a.min_dist += o;
    a.max_dist += o;
    a.in_view += o;
    a.proj_x += o;
    a.proj_y += o;
    a.proj_xr += o;
    a.level += o;
    a.view_cos += o;
  }
  if (i >= a.n) return;
  a.in_view[i] = 0;
  a.proj_x[i] = 0.f;
  a.proj_y[i] = 0.f;
  a.proj_xr[i] = 0.f;
  a.view_cos[i] = 0.f;
  a.level[i] = -1;
  const float* T = a.Tcw;
  const float P[3] = {a.xyz[3 * i], a.xyz[3 * i + 1], a.xyz[3 * i + 2]};
  float Pc[3];
  gemm_R_x_plus_t(T, P, Pc);
  if (Pc[2] < 0.0f) return;
  const float invz = 1.0f / Pc[2];
  const float u = c.fx * Pc[0] * invz + c.cx;
  const float v = c.fy * Pc[1] * invz + c.cy;
  if (u < c.minX || u > c.maxX) return;
  if (v < c.minY || v > c.maxY) return;
  float Ow[3];
  gemm_neg_Rt_t(T, Ow);
  const float PO[3] = {P[0] - Ow[0], P[1] - Ow[1], P[2] - Ow[2]};
  // cv::norm (P16): double squares, one rounding
  const float dist =
      (float)sqrt((double)PO[0] * PO[0] + (double)PO[1] * PO[1] + (double)PO[2] * PO[2]);
  // GetMin/MaxDistanceInvariance (MapPoint.cc:387-397): 0.8f / 1.2f times the
  // raw mfMinDistance / mfMaxDistance the arrays hold
  if (dist < 0.8f * a.min_dist[i] || dist > 1.2f * a.max_dist[i]) return;
  // Mat::dot (P16): float products, double sum
  double dot = 0;
#pragma unroll
  for (int k = 0; k < 3; k++) dot += (double)(float)(PO[k] * a.normal[3 * i + k]);
  const float vc = (float)(dot / (double)dist);
  if (vc < a.view_cos_limit) return;
  const float ratio = a.max_dist[i] / dist;   // PredictScale: mfMaxDistance / dist (MapPoint.cc:421)
  int ns = (int)ceilf((float)lsdm::log_((double)ratio) / log_scale);  // P15
  if (ns < 0) ns = 0;
  else if (ns >= c.nlevels) ns = c.nlevels - 1;
  a.in_view[i] = 1;
  a.proj_x[i] = u;
  a.proj_xr[i] = u - c.bf * invz;
  a.proj_y[i] = v;
  a.level[i] = ns;
  a.view_cos[i] = vc;
}

namespace {

constexpr int kLocalThreads = 1024;   // widest build: the index build and phase A; wave 0 runs phase B
constexpr int kLevelCols = kMaxLevelsT * kGridCols;   // (octave, grid column) ranges

// The current frame's keypoints in LDS for up to kLocalKp keypoints: 140 KB at
// 2048 (one workgroup per CU), 71 KB at 1024 (two per CU: the 1000-feature
// configurations). The keypoints in the grid are held as records sorted by
// (octave, column, row, index): the candidates of one octave in one grid
// column are one contiguous range, in the reference's scan order.
// ORBPL_LOCAL_DESC_LDS: the current descriptors staged in LDS (1) or read
// from global memory (0, the default: L2-resident, 32 KB less LDS per
// workgroup at 1024 keypoints; A/B on one box, two rounds: k_match_local
// isolated 0.228 -> 0.160 ms, headline within noise, tools/gpu_r04_g.sh)
#ifndef ORBPL_LOCAL_DESC_LDS
#define ORBPL_LOCAL_DESC_LDS 0
#endif
template <int kLocalKp>
struct LocalShared {
  uint4 desc[ORBPL_LOCAL_DESC_LDS ? kLocalKp * 2 : 1];   // current descriptors (32 B rows)
  float4 rec[kLocalKp];              // sorted records: x, y, uRight, bits(column | row | index)
  int mw[kLocalKp];                  // last writer (map point index) per keypoint
  int own[kLocalKp];                 // phase B: (round << 6) | (63 - lane) of the round's
                                     // first claimer per keypoint
  uint32_t skey[kLocalKp];           // sort keys: octave << 23 | scan key
  uint16_t list[4 * kLocalKp];       // in-view map points of a window, by predicted level
  uint16_t lc_start[kLevelCols + 1]; // first record of each (octave, column)
  int8_t oct[kLocalKp];
  uint32_t claimed[kLocalKp / 32];   // holds a map point with Observations() > 0
  int lvl_cnt[kMaxLevelsT];
  int lvl_pos[kMaxLevelsT];
};

struct Top2 {
  int bd, bi, bl;   // best distance, index, level
  int sd, si, sl;   // second distance, index of the candidate that set it, level
};

// The reference's running best / second pair (ORBmatcher.cc:128-145, strict
// comparisons) is the first two candidates in (distance, scan position) order:
// the best is the earliest candidate of minimal distance, the second the
// earliest other candidate of the next distance (or of the same one). Claims
// only remove candidates, so the pair under later claims is the first two
// unclaimed entries of that order. GetFeaturesInArea scans grid columns, then
// rows, then the cell's keypoints in index order (Frame.cc:406-441), so the
// scan position of a keypoint is its scan key column << 17 | row << 11 | index.
// The scan keeps the first kTopK entries of (distance, scan key) order as
// entry = distance << 23 | scan key (all ones = empty: no candidate has
// distance 255 and row 63); bit 31 of the last entry flags more candidates than
// the list holds.
constexpr int kTopK = 4;
constexpr uint32_t kEmpty = 0xFFFFFFFFu;
constexpr uint32_t kMore = 0x80000000u;

struct TopList {
  uint32_t e[kTopK];
};

__device__ __forceinline__ int hamming32l(const uint8_t* a, const uint8_t* b) {
  const uint4 a0 = *reinterpret_cast<const uint4*>(a);
  const uint4 a1 = *reinterpret_cast<const uint4*>(a + 16);
  const uint4 b0 = *reinterpret_cast<const uint4*>(b);
  const uint4 b1 = *reinterpret_cast<const uint4*>(b + 16);
  return __popc(a0.x ^ b0.x) + __popc(a0.y ^ b0.y) + __popc(a0.z ^ b0.z) + __popc(a0.w ^ b0.w) +
         __popc(a1.x ^ b1.x) + __popc(a1.y ^ b1.y) + __popc(a1.z ^ b1.z) + __popc(a1.w ^ b1.w);
}

// the wave's LDS operations so far are complete and the compiler moves no
// memory access across (one wave: LDS executes its operations in order). Unlike
// a workgroup fence it does not wait for the wave's outstanding global loads
// (phase B's next-chunk prefetch).
__device__ __forceinline__ void lds_wave_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

template <int KP>
__device__ __forceinline__ bool is_claimed(const LocalShared<KP>& S, int j) {
  return (S.claimed[j >> 5] >> (j & 31)) & 1u;
}

// GetFeaturesInArea(x, y, r*scale, level-1, level) + the candidate loop
// (ORBmatcher.cc:96-160) against the current claims. The cell window of
// GetFeaturesInArea holds every keypoint that passes the exact |dx|, |dy| < r
// test (PosInGrid rounds, the window floors / ceils), so the scan visits the
// window's columns of the two octaves only and keeps the scan order by key.
template <int KP>
__device__ TopList local_scan(const LocalShared<KP>& S, const TrackConsts& c, const LocalArgs& a,
                              int i) {
  TopList t;
#pragma unroll
  for (int k = 0; k < kTopK; k++) t.e[k] = kEmpty;
  int cnt = 0;
  const int lev = a.level[i];
  float r = (a.view_cos[i] > 0.998) ? 2.5f : 4.0f;
  if (a.th != 1.0) r *= a.th;
  const float rad = r * c.scale[lev];
  const float x = a.proj_x[i], y = a.proj_y[i], xr = a.proj_xr[i];
  const int cx0 = max(0, (int)floorf((x - c.minX - rad) * c.gridInvW));
  const int cx1 = min(kGridCols - 1, (int)ceilf((x - c.minX + rad) * c.gridInvW));
  const int cy0 = max(0, (int)floorf((y - c.minY - rad) * c.gridInvH));
  const int cy1 = min(kGridRows - 1, (int)ceilf((y - c.minY + rad) * c.gridInvH));
  if (cx0 >= kGridCols || cx1 < 0 || cy0 >= kGridRows || cy1 < 0) return t;
  const uint4* dp = reinterpret_cast<const uint4*>(a.mp_desc + (long long)i * 32);
  const uint4 m0 = dp[0], m1 = dp[1];
  // octaves lev-1 and lev (bCheckLevels always holds: maxLevel = lev >= 0)
  for (int L = max(lev - 1, 0); L <= lev; L++) {
    const int id0 = L * kGridCols;
    int k = S.lc_start[id0 + cx0];
    const int kend = S.lc_start[id0 + cx1 + 1];
    while (k < kend) {
      const float4 R = S.rec[k++];
      const uint32_t w = __float_as_uint(R.w);
      const int row = (int)((w >> 11) & 63);
      if (row < cy0 || row > cy1) continue;
      if (!(fabsf(R.x - x) < rad && fabsf(R.y - y) < rad)) continue;
      const int j = (int)(w & 2047);
      if (is_claimed(S, j)) continue;
      if (R.z > 0 && fabsf(xr - R.z) > rad) continue;
#if ORBPL_LOCAL_DESC_LDS
      const uint4 c0 = S.desc[2 * j], c1 = S.desc[2 * j + 1];
#else
      const uint4* cd = reinterpret_cast<const uint4*>(a.desc + (long long)j * 32);
      const uint4 c0 = cd[0], c1 = cd[1];
#endif
      const uint32_t dist = __popc(m0.x ^ c0.x) + __popc(m0.y ^ c0.y) + __popc(m0.z ^ c0.z) +
                            __popc(m0.w ^ c0.w) + __popc(m1.x ^ c1.x) + __popc(m1.y ^ c1.y) +
                            __popc(m1.z ^ c1.z) + __popc(m1.w ^ c1.w);
      if (dist >= 256) continue;   // never below the initial 256 of either slot
      cnt++;
      // sorted insert: the list stays ascending in (distance, scan key)
      uint32_t v = (dist << 23) | (w & 0x7FFFFFu);
#pragma unroll
      for (int q = 0; q < kTopK; q++) {
        const uint32_t eq = t.e[q];
        const bool lt = v < eq;
        t.e[q] = lt ? v : eq;
        v = lt ? eq : v;
      }
    }
  }
  if (cnt > kTopK) t.e[kTopK - 1] |= kMore;
  return t;
}

// the first two unclaimed entries; *full = the list cannot decide (fewer than
// two unclaimed entries while candidates beyond the kept ones exist)
template <int KP>
__device__ __forceinline__ Top2 pick2(const LocalShared<KP>& S, const TopList& t, bool* full) {
  // the claim words and octaves of all entries first (independent LDS reads,
  // one round trip), then the choice in registers
  uint32_t cw[kTopK];
  int ol[kTopK];
#pragma unroll
  for (int k = 0; k < kTopK; k++) {
    const int j = t.e[k] == kEmpty ? 0 : (int)(t.e[k] & 2047);
    cw[k] = S.claimed[j >> 5];
    ol[k] = S.oct[j];
  }
  Top2 r{256, -1, -1, 256, -1, -1};
  int found = 0;
#pragma unroll
  for (int k = 0; k < kTopK; k++) {
    const uint32_t ek = t.e[k];
    const int j = (int)(ek & 2047);
    const bool use = ek != kEmpty && found < 2 && !((cw[k] >> (j & 31)) & 1u);
    const int d = (int)((ek >> 23) & 255);
    if (use && found == 0) {
      r.bi = j; r.bd = d; r.bl = ol[k];
    } else if (use) {
      r.si = j; r.sd = d; r.sl = ol[k];
    }
    found += use;
  }
  const uint32_t last = t.e[kTopK - 1];
  *full = found < 2 && last != kEmpty && (last & kMore);
  return r;
}

}  // namespace

template <int kLocalKp, int NT>
__global__ void __launch_bounds__(NT) k_match_local(TrackConsts c, LocalArgs a) {
  trk_priority();
  if (a.n_arr) {  // batched: stream blockIdx.x
    const int b = blockIdx.x;
    const long long ko = (long long)b * a.kp_pitch, mo = (long long)b * a.mp_pitch;
    a.n = a.n_arr[b];
    a.nmp = a.nmp_arr[b];
    a.kps_un += ko;
    a.desc += ko * 32;
    a.uright += ko;
    if (a.cur_nobs) a.cur_nobs += ko;
    a.match += ko;
    a.in_view += mo;
    a.proj_x += mo;
    a.proj_y += mo;
    a.proj_xr += mo;
    a.level += mo;
    a.view_cos += mo;
    a.mp_desc += mo * 32;
    if (a.mp_nobs) a.mp_nobs += mo;
    a.scratch += mo;
    a.nmatches += (long long)b * a.nm_stride;
  }
  extern __shared__ char smem_local[];
  LocalShared<kLocalKp>& S = *reinterpret_cast<LocalShared<kLocalKp>*>(smem_local);
  const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
  const int n = min(a.n, kLocalKp);
#ifdef ORBPL_LOCAL_PROF
  long long tp0 = wall_clock64(), tp1 = 0, tp2 = 0;
#endif
  // ---- keypoint index (AssignFeaturesToGrid with PosInGrid, Frame.cc:265-287, 527-538) ----
  for (int i = t; i < kLocalKp / 32; i += NT) S.claimed[i] = 0;
#if ORBPL_LOCAL_DESC_LDS
  {
    const uint4* d = reinterpret_cast<const uint4*>(a.desc);
    for (int i = t; i < 2 * n; i += NT) S.desc[i] = d[i];
  }
#endif
  __syncthreads();
  for (int i = t; i < kLocalKp; i += NT) {
    uint32_t key = kEmpty;
    if (i < n) {
      const KeyPointD k = a.kps_un[i];
      S.oct[i] = (int8_t)k.octave;
      S.mw[i] = -1;
      S.own[i] = 0;
      const int px = (int)roundf((k.x - c.minX) * c.gridInvW);
      const int py = (int)roundf((k.y - c.minY) * c.gridInvH);
      if (px >= 0 && px < kGridCols && py >= 0 && py < kGridRows && k.octave >= 0 &&
          k.octave < kMaxLevelsT)
        key = (uint32_t)k.octave << 23 | (uint32_t)px << 17 | (uint32_t)py << 11 | (uint32_t)i;
      if (a.cur_nobs && a.cur_nobs[i] > 0) atomicOr(&S.claimed[i >> 5], 1u << (i & 31));
    }
    S.skey[i] = key;
  }
  __syncthreads();
  // bitonic sort of the keys (the padding sorts last)
  for (int size = 2; size <= kLocalKp; size <<= 1)
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int p = t; p < kLocalKp / 2; p += NT) {
        const int lo = 2 * p - (p & (stride - 1)), hi = lo + stride;
        const uint32_t u = S.skey[lo], v = S.skey[hi];
        if ((u > v) == ((lo & size) == 0)) {
          S.skey[lo] = v;
          S.skey[hi] = u;
        }
      }
      __syncthreads();
    }
  for (int k = t; k < kLocalKp; k += NT) {
    const uint32_t key = S.skey[k];
    const int cur = key == kEmpty ? kLevelCols : (int)(key >> 17);
    const int prev = k == 0 ? -1 : (S.skey[k - 1] == kEmpty ? kLevelCols : (int)(S.skey[k - 1] >> 17));
    for (int id = prev + 1; id <= cur; id++) S.lc_start[id] = (uint16_t)k;
    if (k == kLocalKp - 1)
      for (int id = cur + 1; id <= kLevelCols; id++) S.lc_start[id] = (uint16_t)kLocalKp;
    if (key != kEmpty) {
      const int j = (int)(key & 2047);
      const KeyPointD kp = a.kps_un[j];
      S.rec[k] = make_float4(kp.x, kp.y, a.uright[j], __uint_as_float(key & 0x7FFFFFu));
    }
  }
  __syncthreads();
#ifdef ORBPL_LOCAL_PROF
  tp1 = wall_clock64();
#endif
  // ---- phase A: windows of in-view map points, grouped by predicted level
  // (similar scan lengths per wave) ----
  constexpr int kList = 4 * kLocalKp;
  for (int base = 0; base < a.nmp; base += kList) {
    const int m = min(kList, a.nmp - base);
    if (t < kMaxLevelsT) S.lvl_cnt[t] = 0;
    __syncthreads();
    for (int i = t; i < m; i += NT)
      if (a.in_view[base + i]) atomicAdd(&S.lvl_cnt[a.level[base + i]], 1);
    __syncthreads();
    if (t == 0) {
      int run = 0;
      for (int l = 0; l < kMaxLevelsT; l++) {
        S.lvl_pos[l] = run;
        run += S.lvl_cnt[l];
      }
      S.lvl_cnt[0] = run;   // the window's in-view count
    }
    __syncthreads();
    const int nlist = S.lvl_cnt[0];
    for (int i = t; i < m; i += NT)
      if (a.in_view[base + i]) S.list[atomicAdd(&S.lvl_pos[a.level[base + i]], 1)] = (uint16_t)i;
    __syncthreads();
    for (int p = t; p < nlist; p += NT) {
      const int i = base + S.list[p];
      const TopList r = local_scan(S, c, a, i);
      a.scratch[i] = make_int4((int)r.e[0], (int)r.e[1], (int)r.e[2], (int)r.e[3]);
    }
    __syncthreads();
  }
#ifdef ORBPL_LOCAL_PROF
  tp2 = wall_clock64();
  int prof_rounds = 0, prof_rescans = 0;
#endif
  // ---- phase B (wave 0, map point order) ----
  // Rounds over a chunk of 64 map points. A lane whose best or second
  // candidate was claimed by a committed point rescans against the committed
  // claims (all stale lanes of the chunk in parallel); the round's claimers
  // then stamp their keypoint in S.own, a lane whose best or second candidate
  // carries a stamp of an earlier lane collides, and the chunk commits in
  // order up to the first collision. The colliding lane is stale in the next
  // round (its candidate is now claimed) and so is rescanned, which makes
  // every lane's committed outcome the one of the sequential loop.
  if (wave == 0) {
    int acc = 0, round = 0;
    // the next chunk's lists, in-view flags and Observations() are loaded one
    // chunk ahead (their latency overlaps the current chunk's rounds)
    int4 nv = make_int4(0, 0, 0, 0);
    int nin = 0, nnobs = 0;
    if (lane < a.nmp) {
      nv = a.scratch[lane];
      nin = a.in_view[lane];
      nnobs = a.mp_nobs ? a.mp_nobs[lane] : 1;
    }
    for (int base = 0; base < a.nmp; base += 64) {
      const int i = base + lane;
      TopList lst;
#pragma unroll
      for (int k = 0; k < kTopK; k++) lst.e[k] = kEmpty;
      if (i < a.nmp && nin) {
        lst.e[0] = (uint32_t)nv.x;
        lst.e[1] = (uint32_t)nv.y;
        lst.e[2] = (uint32_t)nv.z;
        lst.e[3] = (uint32_t)nv.w;
      }
      const int nobs = i < a.nmp ? nnobs : 0;
      if (i + 64 < a.nmp) {
        nv = a.scratch[i + 64];
        nin = a.in_view[i + 64];
        nnobs = a.mp_nobs ? a.mp_nobs[i + 64] : 1;
      }
      // the pair under the claims of the earlier chunks
      bool full;
      Top2 r = pick2(S, lst, &full);
      if (full) {
        lst = local_scan(S, c, a, i);
        r = pick2(S, lst, &full);
      }
      bool decided = !(i < a.nmp && r.bi >= 0);
      while (true) {
        round++;
#ifdef ORBPL_LOCAL_PROF
        prof_rounds++;
#endif
        const bool stale =
            !decided && ((int)is_claimed(S, max(r.bi, 0)) | (int)(r.si >= 0 && is_claimed(S, max(r.si, 0))));
        if (stale) {
          // the pair under the committed claims: from the kept list, or a new
          // scan when the list runs out
          r = pick2(S, lst, &full);
          if (full) {
#ifdef ORBPL_LOCAL_PROF
            prof_rescans++;
#endif
            lst = local_scan(S, c, a, i);
            r = pick2(S, lst, &full);
          }
          if (r.bi < 0) decided = true;
        }
        const bool accept = !decided && r.bd <= 100 && !(r.bl == r.sl && r.bd > a.nnratio * r.sd);
        const bool claimer = accept && nobs > 0;
        const int key = (round << 6) | (63 - lane);
        if (claimer) atomicMax(&S.own[r.bi], key);
        lds_wave_sync();
        // both stamps read at once (index 0 stands in for a missing candidate)
        const int ob = S.own[max(r.bi, 0)], os = S.own[max(r.si, 0)];
        const bool coll = !decided && (((ob >> 6) == round && 63 - (ob & 63) < lane) ||
                                       (r.si >= 0 && (os >> 6) == round && 63 - (os & 63) < lane));
        const unsigned long long cm = __ballot(coll);
        const int lc = cm ? __ffsll((long long)cm) - 1 : 64;
        if (!decided && lane < lc) {
          if (accept) {
            atomicMax(&S.mw[r.bi], i);
            if (claimer) atomicOr(&S.claimed[r.bi >> 5], 1u << (r.bi & 31));
            acc++;
          }
          decided = true;
        }
        if (lc == 64) break;
        lds_wave_sync();
      }
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) acc += __shfl_xor(acc, o, 64);
    if (lane == 0) *a.nmatches = acc;
#ifdef ORBPL_LOCAL_PROF
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) prof_rescans += __shfl_xor(prof_rescans, o, 64);
    if (lane == 0 && blockIdx.x % 128 == 0)
      printf("local blk %d n %d nmp %d grid %lld A %lld B %lld rounds %d rescans %d acc %d\n",
             (int)blockIdx.x, n, a.nmp, tp1 - tp0, tp2 - tp1, wall_clock64() - tp2, prof_rounds,
             prof_rescans, acc);
#endif
  }
  __syncthreads();
  for (int i = t; i < n; i += NT) a.match[i] = S.mw[i];
}

void launch_in_frustum(const TrackConsts& c, float log_scale, const InFrustumArgs& a,
                       hipStream_t s, int nstreams) {
  const long long n = a.n_arr ? a.pitch : a.n;
  if (n <= 0) return;
  hipLaunchKernelGGL(k_in_frustum, dim3((unsigned)((n + 255) / 256), a.n_arr ? nstreams : 1),
                     dim3(256), 0, s, c, log_scale, a);
}

void launch_match_local(const TrackConsts& c, const LocalArgs& a, hipStream_t s, int nstreams) {
  const int cap = a.n_arr ? a.kp_pitch : a.n;   // keypoints a frame can hold
  // threads per frame: narrower workgroups are placed sooner beside the next
  // batch's extraction and pack more frames per CU once frames outnumber CUs
  // (256 / 1024 streams: 512 threads 98.2k / 116.9k frames/s, 256 threads
  // 97.6k / 120.8k, 1024 threads 97.2k / 114.3k). ORBPL_LOCAL_NT overrides.
  const char* nt_env = getenv("ORBPL_LOCAL_NT");   // read per launch: tests vary it
  int nt = nstreams > device_cu_count() ? 256 : 512;
  if (nt_env) nt = atoi(nt_env);
#define ORBPL_LOCAL_LAUNCH(KP, NTH)                                                              \
  if ((KP == 1024) == (cap <= 1024) && nt == NTH) {                                             \
    set_smem_attr((const void*)k_match_local<KP, NTH>, sizeof(LocalShared<KP>));               \
    hipLaunchKernelGGL((k_match_local<KP, NTH>), dim3(a.n_arr ? nstreams : 1), dim3(NTH),      \
                       sizeof(LocalShared<KP>), s, c, a);                                       \
    return;                                                                                     \
  }
  ORBPL_LOCAL_LAUNCH(1024, 1024)
  ORBPL_LOCAL_LAUNCH(1024, 512)
  ORBPL_LOCAL_LAUNCH(1024, 256)
  ORBPL_LOCAL_LAUNCH(2048, 1024)
  ORBPL_LOCAL_LAUNCH(2048, 512)
  ORBPL_LOCAL_LAUNCH(2048, 256)
#undef ORBPL_LOCAL_LAUNCH
  set_smem_attr((const void*)k_match_local<2048, kLocalThreads>, sizeof(LocalShared<2048>));
  hipLaunchKernelGGL((k_match_local<2048, kLocalThreads>), dim3(a.n_arr ? nstreams : 1), dim3(kLocalThreads),
                     sizeof(LocalShared<2048>), s, c, a);
}


// ---------------------------------------------------------------------------
// ORBmatcher::SearchByBoW(KeyFrame*, Frame&, vector<MapPoint*>&)
// (ORBmatcher.cc:247-410). Features sharing a vocabulary node are compared
// only with each other and a frame feature is claimed only by keyframe
// features of its own node, so nodes are independent: both feature lists are
// sorted by (node, index) in LDS (bitonic), every common node is walked by
// one thread in the reference's order, then the rotation histogram.
// ---------------------------------------------------------------------------
namespace {
constexpr int kBowMax = 2048;
__device__ void bitonic_sort(uint32_t* a, int n) {
  for (int k = 2; k <= n; k <<= 1)
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < n; i += blockDim.x) {
        const int l = i ^ j;
        if (l > i) {
          const uint32_t x = a[i], y = a[l];
          if (((i & k) == 0) ? (x > y) : (x < y)) {
            a[i] = y;
            a[l] = x;
          }
        }
      }
      __syncthreads();
    }
}
}  // namespace

// LDS of one SearchByBoW instance for frames of up to CAP features: both
// sorted key lists, each keyframe feature's four best frame candidates, the
// claims and rotation bins.
template <int CAP>
struct BowShared {
  uint32_t skf[CAP], sf[CAP];
  alignas(16) uint32_t cand[CAP][4];   // by sorted keyframe position: (dist << 11 | iF), ascending
  int16_t smatch[CAP];     // frame feature -> claiming keyframe feature, -1
  int8_t sbin[CAP];        // rotation bin of a claimed frame feature, -1
  int hist[32];
  int s_n, s_ind[3];
};

__device__ __forceinline__ int hamming32(const uint4 k0, const uint4 k1, const uint4 f0,
                                         const uint4 f1) {
  return __popc(k0.x ^ f0.x) + __popc(k0.y ^ f0.y) + __popc(k0.z ^ f0.z) + __popc(k0.w ^ f0.w) +
         __popc(k1.x ^ f1.x) + __popc(k1.y ^ f1.y) + __popc(k1.z ^ f1.z) + __popc(k1.w ^ f1.w);
}

// [fb, fe) of the frame features of `node` in the sorted list sf (sentinels
// 0xFFFFFFFF sort above every node: node ids are < 2^21 - 1)
template <int CAP>
__device__ __forceinline__ void frame_run(const uint32_t* sf, uint32_t node, int* fb, int* fe) {
  int lo = 0, hi = CAP;
  while (lo < hi) {
    const int m = (lo + hi) >> 1;
    if ((sf[m] >> 11) < node) lo = m + 1;
    else hi = m;
  }
  int e = lo, h2 = CAP;
  while (e < h2) {
    const int m = (e + h2) >> 1;
    if ((sf[m] >> 11) <= node) e = m + 1;
    else h2 = m;
  }
  *fb = lo;
  *fe = e;
}

// The body (ORBmatcher.cc:247-410). Nodes are independent (a frame feature is
// claimed only by keyframe features of its own node); within a node the
// reference walks the keyframe features in index order, each taking the best
// (and second-best) distance over the node's frame features not yet claimed.
//   1. both FeatureVectors sorted by (node, index) in LDS;
//   2. every keyframe feature (all lanes) computes its four smallest
//      (distance, frame index) keys over its node's frame run, the frame
//      descriptors read from L2 in parallel;
//   3. one lane per node replays the reference's in-order claims from those
//      lists: the first two unclaimed entries are the best and second-best
//      distances (ties keep index order, as the strict `<` of the reference);
//      only when three of a truncated list are claimed does the lane rescan
//      the run exactly;
//   4. the rotation histogram and its top-3 cut.
// fdl (LDS, 2 uint4 per feature) optionally stages the frame's descriptors.
template <int CAP, int NT>
__device__ void match_bow_body(const BowArgs& a, BowShared<CAP>& B, const uint4* fdl) {
  const int t = threadIdx.x;
  const int nkf = min(a.nkf, CAP), nf = min(a.nf, CAP);
  // key = node << 11 | index; features without a node sort last
  for (int i = t; i < CAP; i += NT) {
    B.skf[i] = (i < nkf && a.kf_node[i] >= 0) ? ((uint32_t)a.kf_node[i] << 11) | (uint32_t)i : 0xFFFFFFFFu;
    B.sf[i] = (i < nf && a.f_node[i] >= 0) ? ((uint32_t)a.f_node[i] << 11) | (uint32_t)i : 0xFFFFFFFFu;
    B.smatch[i] = -1;
    B.sbin[i] = -1;
  }
  if (t < 32) B.hist[t] = 0;
  if (t == 0) B.s_n = 0;
  __syncthreads();
  // the padding sorts last: sorting the next power of two above the counts
  // leaves the same runs
  int ns = 64;
  while (ns < nkf || ns < nf) ns <<= 1;
  bitonic_sort(B.skf, ns);
  bitonic_sort(B.sf, ns);
  const uint4* fd = reinterpret_cast<const uint4*>(a.f_desc);
  const uint4* kd = reinterpret_cast<const uint4*>(a.kf_desc);
  // 2. candidate lists, one keyframe feature per lane
  for (int p = t; p < nkf; p += NT) {
    const uint32_t key = B.skf[p];
    uint32_t c0 = 0xFFFFFFFFu, c1 = c0, c2 = c0, c3 = c0;
    if (key != 0xFFFFFFFFu && a.kf_valid[key & 0x7FF]) {
      const int iKF = (int)(key & 0x7FF);
      int fb, fe;
      frame_run<CAP>(B.sf, key >> 11, &fb, &fe);
      const uint4 k0 = kd[2 * iKF], k1 = kd[2 * iKF + 1];
#pragma unroll 4
      for (int r = fb; r < fe; r++) {
        const uint32_t iF = B.sf[r] & 0x7FF;
        const uint4 f0 = fdl ? fdl[2 * iF] : fd[2 * iF];
        const uint4 f1 = fdl ? fdl[2 * iF + 1] : fd[2 * iF + 1];
        const int d = hamming32(k0, k1, f0, f1);
        // a distance of 256 never beats the reference's initial 256
        const uint32_t k = d < 256 ? ((uint32_t)d << 11) | iF : 0xFFFFFFFFu;
        // sorted insertion (frame indices ascend along the run: ties keep order)
        c3 = min(c3, max(c2, k));
        c2 = min(c2, max(c1, k));
        c1 = min(c1, max(c0, k));
        c0 = min(c0, k);
      }
    }
    B.cand[p][0] = c0;
    B.cand[p][1] = c1;
    B.cand[p][2] = c2;
    B.cand[p][3] = c3;
  }
  __syncthreads();
  // 3. in-order claims, one lane per keyframe node run
  int nm = 0;
  for (int p = t; p < nkf; p += NT) {
    const uint32_t key = B.skf[p];
    if (key == 0xFFFFFFFFu) continue;
    const uint32_t node = key >> 11;
    if (p > 0 && (B.skf[p - 1] >> 11) == node) continue;   // not the run's first
    int fb, fe;
    frame_run<CAP>(B.sf, node, &fb, &fe);
    if (fb == fe) continue;
    for (int q = p; q < nkf && B.skf[q] != 0xFFFFFFFFu && (B.skf[q] >> 11) == node; q++) {
      const int iKF = (int)(B.skf[q] & 0x7FF);
      if (!a.kf_valid[iKF]) continue;
      const uint4 cv = *reinterpret_cast<const uint4*>(B.cand[q]);
      const uint32_t cl[4] = {cv.x, cv.y, cv.z, cv.w};
      int bestDist1 = 256, bestIdxF = -1, bestDist2 = 256, found = 0;
#pragma unroll
      for (int k = 0; k < 4; k++) {
        if (cl[k] == 0xFFFFFFFFu || found == 2) continue;
        const int iF = (int)(cl[k] & 0x7FF);
        if (B.smatch[iF] >= 0) continue;
        if (found == 0) {
          bestDist1 = (int)(cl[k] >> 11);
          bestIdxF = iF;
        } else {
          bestDist2 = (int)(cl[k] >> 11);
        }
        found++;
      }
      if (found < 2 && cl[3] != 0xFFFFFFFFu && fe - fb > 4) {
        // the list was cut at four: the rest of the run decides, exactly
        const uint4 k0 = kd[2 * iKF], k1 = kd[2 * iKF + 1];
        bestDist1 = 256;
        bestIdxF = -1;
        bestDist2 = 256;
        for (int r = fb; r < fe; r++) {
          const int iF = (int)(B.sf[r] & 0x7FF);
          if (B.smatch[iF] >= 0) continue;
          const int dist = hamming32(k0, k1, fdl ? fdl[2 * iF] : fd[2 * iF],
                                     fdl ? fdl[2 * iF + 1] : fd[2 * iF + 1]);
          if (dist < bestDist1) {
            bestDist2 = bestDist1;
            bestDist1 = dist;
            bestIdxF = iF;
          } else if (dist < bestDist2) {
            bestDist2 = dist;
          }
        }
      }
      if (bestDist1 <= 50 && static_cast<float>(bestDist1) < a.nnratio * static_cast<float>(bestDist2)) {
        B.smatch[bestIdxF] = (int16_t)iKF;
        if (a.check_ori) {
          float rot = a.kf_angle[(long long)iKF * a.kf_angle_stride] -
                      a.f_angle[(long long)bestIdxF * a.f_angle_stride];
          if (rot < 0.0f) rot += 360.0f;
          int bin = (int)roundf(rot * (30 / 360.0f));
          if (bin == 30) bin = 0;
          B.sbin[bestIdxF] = (int8_t)bin;
          atomicAdd(&B.hist[bin], 1);
        }
        nm++;
      }
    }
  }
  if (nm) atomicAdd(&B.s_n, nm);
  __syncthreads();
  // 4. rotation consistency (ORBmatcher.cc:2035-2077, :386-404)
  if (a.check_ori) {
    if (t == 0) {
      int max1 = 0, max2 = 0, max3 = 0, ind1 = -1, ind2 = -1, ind3 = -1;
      for (int i = 0; i < 30; i++) {
        const int sz = B.hist[i];
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
      B.s_ind[0] = ind1; B.s_ind[1] = ind2; B.s_ind[2] = ind3;
    }
    __syncthreads();
    int rem = 0;
    for (int j = t; j < nf; j += NT) {
      const int b = B.sbin[j];
      if (b >= 0 && b != B.s_ind[0] && b != B.s_ind[1] && b != B.s_ind[2]) {
        B.smatch[j] = -1;
        rem++;
      }
    }
    if (rem) atomicSub(&B.s_n, rem);
    __syncthreads();
  }
  for (int j = t; j < nf; j += NT) a.match[j] = B.smatch[j];
  if (t == 0) *a.nmatches = B.s_n;
}

__global__ void __launch_bounds__(256) k_match_bow(BowArgs a) {
  trk_priority();
  __shared__ BowShared<kBowMax> B;
  extern __shared__ uint4 bow_fdl[];
  const int nf = min(a.nf, kBowMax);
  const uint4* d = reinterpret_cast<const uint4*>(a.f_desc);
  for (int i = threadIdx.x; i < 2 * nf; i += 256) bow_fdl[i] = d[i];
  // (the body's first barrier orders these stores before any read)
  match_bow_body<kBowMax, 256>(a, B, bow_fdl);
}

void launch_match_bow(const BowArgs& a, hipStream_t s) {
  const size_t smem = (size_t)2 * sizeof(uint4) * (size_t)min(max(a.nf, 0), kBowMax);
  // the dynamic part only (static BowShared + this stay within the CU's 160 KiB)
  set_smem_attr((const void*)k_match_bow, (size_t)2 * sizeof(uint4) * kBowMax);
  hipLaunchKernelGGL(k_match_bow, dim3(1), dim3(256), smem, s, a);
}

// TrackReferenceKeyFrame's ORBmatcher(0.7, true).SearchByBoW(pKF, F)
// (Tracking.cc:947-952) for every stream with st[s].trk: the reference
// keyframe's FeatureVector / map points / descriptors against the current
// frame's. The frame's descriptors stay in global memory (L2): the launch runs
// every step beside the next batch's extraction, so its LDS is kept small.
template <int CAP>
__device__ __forceinline__ void trk_bow_stream(const TrkArgs& a, BowShared<CAP>& B, const int s) {
  StreamState& S = a.st[s];
  if (!S.trk) return;
  const long long cb = (long long)s * a.kp_pitch;
  BowArgs b;
  b.nkf = a.last_n[s];
  b.kf_node = a.last_feat_node + cb;
  b.kf_valid = a.last_has_mp + cb;
  b.kf_desc = a.last_desc + cb * 32;
  b.kf_angle = &a.last_kps_un[cb].angle;
  b.kf_angle_stride = (int)(sizeof(KeyPointD) / sizeof(float));
  b.nf = a.n[s];
  b.f_node = a.feat_node + cb;
  b.f_desc = a.desc + cb * 32;
  b.f_angle = &a.kps_un[cb].angle;
  b.f_angle_stride = (int)(sizeof(KeyPointD) / sizeof(float));
  b.nnratio = 0.7f;
  b.check_ori = 1;
  b.match = a.match + cb;
  b.nmatches = &S.nmatches;
  match_bow_body<CAP, 256>(b, B, nullptr);
}

// one workgroup per stream, or (a.list) a grid looping over the listed
// streams (the map model's TrackReferenceKeyFrame streams)
template <int CAP>
__global__ void __launch_bounds__(256) k_trk_bow(TrkArgs a) {
  trk_priority();
  __shared__ BowShared<CAP> B;
  if (a.list) {
    const int n = *a.list_n;
    for (int b = blockIdx.x; b < n; b += gridDim.x) {
      trk_bow_stream<CAP>(a, B, a.list[b]);
      __syncthreads();
    }
  } else {
    trk_bow_stream<CAP>(a, B, blockIdx.x);
  }
}

void launch_trk_bow(const TrkArgs& a, int nstreams, hipStream_t s) {
  // a listed launch: one workgroup per stream up to kTrkGrid (the list is on
  // the device; an empty list costs every workgroup one load)
  static const int env_grid = getenv("ORBPL_TRK_GRID") ? atoi(getenv("ORBPL_TRK_GRID")) : 0;
  const int cap_grid = env_grid > 0 ? env_grid : kTrkGrid;
  const int grid = a.list ? (nstreams < cap_grid ? nstreams : cap_grid) : nstreams;
  if (a.kp_pitch <= 1024)
    hipLaunchKernelGGL(k_trk_bow<1024>, dim3(grid), dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL(k_trk_bow<kBowMax>, dim3(grid), dim3(256), 0, s, a);
}

}  // namespace orbpl
