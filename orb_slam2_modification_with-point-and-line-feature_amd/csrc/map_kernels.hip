// Tracking::Track's map bookkeeping on gfx950 for the batched tracker
// (ORBPL_TRACK_MAP; restated in oracle/map_oracle.cpp, pinned P23-P25):
//   k_map_begin         : the step's frame id and tracking path, UpdateLastFrame
//                         (Tracking.cc:1044-1210: the last frame re-posed from
//                         its reference keyframe, temporal VO points / lines
//                         from depth) and the constant-velocity prediction
//   k_map_resolve_motion: TrackWithMotionModel's matches as map elements and its
//                         outlier discard (Tracking.cc:1273-1329); the streams
//                         that go on to TrackReferenceKeyFrame get their
//                         reference keyframe staged as a frame
//   k_map_trk_merge     : TrackReferenceKeyFrame's BoW / line matches as map
//                         elements, the 15 / 10 gates (Tracking.cc:942-990)
//   k_map_resolve_trk   : its discard (Tracking.cc:999-1031)
//   k_map_local         : UpdateLocalKeyFrames / UpdateLocalPoints /
//                         UpdateLocalLines (Tracking.cc:1867-2040) over the
//                         covisibility graph, SearchLocalPoints' marks
//   k_map_assemble      : the local matches as map elements, the second pose's
//                         inputs
//   k_map_finish        : TrackLocalMap's decision, the state, the velocity,
//                         the VO cleanup, NeedNewKeyFrame, CreateNewKeyFrame +
//                         ProcessNewKeyFrame + UpdateConnections, the outlier
//                         cleanup, the relative pose; StereoInitialization and
//                         the LOST / reset rules
// One 256-thread block per stream. The matching and the poses reuse the
// batched matcher and k_pose kernels on the arrays these kernels prepare.
#include <hip/hip_runtime.h>

#include "line_common.h"
#include "lsd_kernels.h"
#include "map_kernels.h"
#include "track_common.h"

namespace orbpl {

namespace {

constexpr int kT = 256;
constexpr int kNotInit = 0, kOK = 1, kLost = 2;

__device__ __forceinline__ int block_sum(int v, int* wsum) {
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  if (lane == 0) wsum[wave] = v;
  __syncthreads();
  const int r = wsum[0] + wsum[1] + wsum[2] + wsum[3];
  __syncthreads();
  return r;
}

// position of this thread's flagged element among the block's flagged ones
// (thread order); the block's total in *total
__device__ __forceinline__ int block_prefix(bool flag, int* wsum, int* total) {
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const unsigned long long m = __ballot(flag);
  if (lane == 0) wsum[wave] = __popcll(m);
  __syncthreads();
  int off = 0, tot = 0;
  for (int w = 0; w < 4; w++) {
    if (w < wave) off += wsum[w];
    tot += wsum[w];
  }
  __syncthreads();
  *total = tot;
  return off + __popcll(m & ((1ull << lane) - 1ull));
}

// ascending bitonic sort of P (a power of two) keys in LDS
__device__ void bitonic_sort(unsigned long long* keys, int P) {
  for (int k = 2; k <= P; k <<= 1)
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < P; i += kT) {
        const int ixj = i ^ j;
        if (ixj > i) {
          const unsigned long long a = keys[i], b = keys[ixj];
          const bool up = (i & k) == 0;
          if ((a > b) == up) {
            keys[i] = b;
            keys[ixj] = a;
          }
        }
      }
      __syncthreads();
    }
}

// libstdc++'s std::sort (introsort, median-of-3 pivot to first, unguarded
// partition, heap sort below the depth limit, final insertion sort) of (key,
// idx) records by key ascending: the reference's std::sort of its line
// depth lists (Tracking.cc:1161-1165, 1676-1680), whose tie order depends on
// the algorithm. One thread; n <= kLineKeep.
struct LRec {
  float k;
  int i;
};
__device__ inline bool lless(const LRec& a, const LRec& b) { return a.k < b.k; }

__device__ void stl_push_heap(LRec* f, int hole, int top, LRec v) {
  int parent = (hole - 1) / 2;
  while (hole > top && lless(f[parent], v)) {
    f[hole] = f[parent];
    hole = parent;
    parent = (hole - 1) / 2;
  }
  f[hole] = v;
}
__device__ void stl_adjust_heap(LRec* f, int hole, int len, LRec v) {
  const int top = hole;
  int second = hole;
  while (second < (len - 1) / 2) {
    second = 2 * (second + 1);
    if (lless(f[second], f[second - 1])) second--;
    f[hole] = f[second];
    hole = second;
  }
  if ((len & 1) == 0 && second == (len - 2) / 2) {
    second = 2 * (second + 1);
    f[hole] = f[second - 1];
    hole = second - 1;
  }
  stl_push_heap(f, hole, top, v);
}
__device__ void stl_heap_sort(LRec* f, int n) {
  if (n < 2) return;
  for (int parent = (n - 2) / 2;; parent--) {
    stl_adjust_heap(f, parent, n, f[parent]);
    if (parent == 0) break;
  }
  for (int last = n; last > 1;) {
    --last;
    const LRec v = f[last];
    f[last] = f[0];
    stl_adjust_heap(f, 0, last, v);
  }
}
__device__ void stl_move_median_to_first(LRec* r, LRec* a, LRec* b, LRec* c) {
  LRec* m;
  if (lless(*a, *b)) {
    if (lless(*b, *c)) m = b;
    else if (lless(*a, *c)) m = c;
    else m = a;
  } else if (lless(*a, *c)) {
    m = a;
  } else if (lless(*b, *c)) {
    m = c;
  } else {
    m = b;
  }
  const LRec t = *r;
  *r = *m;
  *m = t;
}
// stk: 3 x 32 ints of LDS for the explicit stack (one thread sorts; an LDS
// stack keeps the caller kernels' register and scratch budget)
__device__ void stl_sort(LRec* f, int n, int* stk) {
  if (n < 2) return;
  int lg = 0;
  while ((1 << (lg + 1)) <= n) lg++;
  // explicit stack for the right-hand recursion of __introsort_loop
  int* st_lo = stk;
  int* st_hi = stk + 32;
  int* st_d = stk + 64;
  int sp = 0;
  st_lo[sp] = 0; st_hi[sp] = n; st_d[sp] = 2 * lg; sp++;
  while (sp > 0) {
    sp--;
    const int lo = st_lo[sp];
    int hi = st_hi[sp], depth = st_d[sp];
    while (hi - lo > 16) {
      if (depth == 0) {
        stl_heap_sort(f + lo, hi - lo);
        break;
      }
      --depth;
      const int mid = lo + (hi - lo) / 2;
      stl_move_median_to_first(f + lo, f + lo + 1, f + mid, f + hi - 1);
      int a = lo + 1, b = hi;
      const LRec piv = f[lo];
      while (true) {
        while (lless(f[a], piv)) ++a;
        --b;
        while (lless(piv, f[b])) --b;
        if (!(a < b)) break;
        const LRec t = f[a];
        f[a] = f[b];
        f[b] = t;
        ++a;
      }
      // __introsort_loop(cut, last, depth); last = cut
      st_lo[sp] = a; st_hi[sp] = hi; st_d[sp] = depth; sp++;
      hi = a;
    }
  }
  // __final_insertion_sort
  auto linear_insert = [&](int i) {
    const LRec v = f[i];
    int j = i - 1;
    int last = i;
    while (lless(v, f[j])) {
      f[last] = f[j];
      last = j;
      --j;
    }
    f[last] = v;
  };
  auto insertion_sort = [&](int lo, int hi) {
    for (int i = lo + 1; i < hi; i++) {
      if (lless(f[i], f[lo])) {
        const LRec v = f[i];
        for (int j = i; j > lo; j--) f[j] = f[j - 1];
        f[lo] = v;
      } else {
        linear_insert(i);
      }
    }
  };
  if (n > 16) {
    insertion_sort(0, 16);
    for (int i = 16; i < n; i++) linear_insert(i);
  } else {
    insertion_sort(0, n);
  }
}

__device__ inline void unproject_f(const TrackConsts& c, const float* T, const float* Ow, float u,
                                   float v, float z, float* w) {
  const float x3[3] = {(u - c.cx) * z * c.invfx, (v - c.cy) * z * c.invfy, z};
  gemm_Rt_x_plus_c(T, x3, Ow, w);
}

__device__ inline int popc32(const uint8_t* a, const uint8_t* b) {
  const uint4* p = reinterpret_cast<const uint4*>(a);
  const uint4* q = reinterpret_cast<const uint4*>(b);
  int d = 0;
#pragma unroll
  for (int k = 0; k < 2; k++) {
    const uint4 x = p[k], y = q[k];
    d += __popc(x.x ^ y.x) + __popc(x.y ^ y.y) + __popc(x.z ^ y.z) + __popc(x.w ^ y.w);
  }
  return d;
}

__device__ inline void copy32(uint8_t* d, const uint8_t* s) {
  reinterpret_cast<uint4*>(d)[0] = reinterpret_cast<const uint4*>(s)[0];
  reinterpret_cast<uint4*>(d)[1] = reinterpret_cast<const uint4*>(s)[1];
}

// pool / temporal element accessors of stream s
struct Pools {
  const MapArgs& a;
  int s;
  long long cb, lb, mb, lmb;
  __device__ Pools(const MapArgs& a_, int s_)
      : a(a_), s(s_), cb((long long)s_ * a_.kp_pitch), lb((long long)s_ * kLineKeep),
        mb((long long)s_ * a_.mpc), lmb((long long)s_ * a_.mlc) {}
  __device__ int mp_nobs(int m) const { return m >= 0 ? a.mp_nobs[mb + m] : 0; }
  __device__ int ml_nobs(int m) const { return m >= 0 ? a.ml_nobs[lmb + m] : 0; }
  // world position of a point element: pool, or temporal at last-frame slot
  __device__ void mp_xyz(int m, float* o) const {
    if (m >= 0) {
      const float4 p = a.mp_pos[mb + m];
      o[0] = p.x; o[1] = p.y; o[2] = p.z;
    } else {
      const float* q = a.l_mp_xyz + (cb + (-2 - m)) * 3;
      o[0] = q[0]; o[1] = q[1]; o[2] = q[2];
    }
  }
  __device__ void ml_xyz(int m, float* o) const {
    const float* q = m >= 0 ? a.ml_pos + (lmb + m) * 6 : a.l_ml_xyz + (lb + (-2 - m)) * 6;
    for (int k = 0; k < 6; k++) o[k] = q[k];
  }
  __device__ long long kfb(int k) const { return (long long)s * a.kfc + k; }
};

// MapPoint::UpdateNormalAndDepth (MapPoint.cc:344-385) with P25's float sums
__device__ void update_normal_depth(const TrackConsts& c, const MapArgs& a, const Pools& P,
                                    int p) {
  const long long g = P.mb + p;
  const int nob = a.mp_nob[g];
  if (nob == 0) return;
  const float4 X = a.mp_pos[g];
  float nrm[3] = {0.f, 0.f, 0.f};
  const uint32_t* ob = a.mp_obs + g * a.kfc;
  for (int k = 0; k < nob; k++) {
    const float* Ow = a.kf_Ow + P.kfb(ob[k] >> 16) * 4;
    const float d[3] = {X.x - Ow[0], X.y - Ow[1], X.z - Ow[2]};
    const float inv = (float)(1.0 / sqrt((double)d[0] * d[0] + (double)d[1] * d[1] + (double)d[2] * d[2]));
    for (int q = 0; q < 3; q++) nrm[q] = nrm[q] + d[q] * inv;
  }
  // the reference keyframe = the creating one = the first observation
  const int rk = ob[0] >> 16, ridx = ob[0] & 0xffff;
  const float* Ow = a.kf_Ow + P.kfb(rk) * 4;
  const float PC[3] = {X.x - Ow[0], X.y - Ow[1], X.z - Ow[2]};
  const float dist = (float)sqrt((double)PC[0] * PC[0] + (double)PC[1] * PC[1] + (double)PC[2] * PC[2]);
  const int level = a.kf_kp[P.kfb(rk) * a.kp_pitch + ridx].octave;
  const float mx = dist * c.scale[level];
  const float mn = mx / c.scale[c.nlevels - 1];
  a.mp_dist[g] = make_float2(mn, mx);
  const float fn = (float)nob;
  a.mp_nrm[g] = make_float4(nrm[0] / fn, nrm[1] / fn, nrm[2] / fn, 0.f);
}

// MapPoint::ComputeDistinctiveDescriptors (MapPoint.cc:256-321): the
// observation descriptor with the least median distance to the others
// (first on ties); dscr: this thread's kMapMaxKF distances. With one or two
// observations the median index is 0 (the distance to itself), so the first
// observation's descriptor wins without a distance. The row's descriptors are
// fetched four at a time (independent loads in flight together).
__device__ void compute_distinctive(const MapArgs& a, const Pools& P, int p, uint16_t* dscr) {
  const long long g = P.mb + p;
  const int nob = a.mp_nob[g];
  if (nob == 0) return;
  const uint32_t* ob = a.mp_obs + g * a.kfc;
  auto dptr = [&](uint32_t o) {
    return reinterpret_cast<const uint4*>(a.kf_desc +
                                          (P.kfb(o >> 16) * a.kp_pitch + (o & 0xffff)) * 32);
  };
  int bi = 0;
  if (nob > 2) {
    const int med = (int)(0.5 * (double)(nob - 1));
    int best = 0x7fffffff;
    for (int i = 0; i < nob; i++) {
      const uint4* di = dptr(ob[i]);
      const uint4 x0 = di[0], x1 = di[1];
      for (int j0 = 0; j0 < nob; j0 += 4) {
        uint32_t o[4];
#pragma unroll
        for (int q = 0; q < 4; q++) o[q] = j0 + q < nob ? ob[j0 + q] : ob[0];
        uint4 y[8];
#pragma unroll
        for (int q = 0; q < 4; q++) {
          const uint4* dj = dptr(o[q]);
          y[2 * q] = dj[0];
          y[2 * q + 1] = dj[1];
        }
#pragma unroll
        for (int q = 0; q < 4; q++) {
          const int j = j0 + q;
          if (j >= nob) break;
          const uint4 u = y[2 * q], v = y[2 * q + 1];
          const int d = __popc(x0.x ^ u.x) + __popc(x0.y ^ u.y) + __popc(x0.z ^ u.z) +
                        __popc(x0.w ^ u.w) + __popc(x1.x ^ v.x) + __popc(x1.y ^ v.y) +
                        __popc(x1.z ^ v.z) + __popc(x1.w ^ v.w);
          dscr[j] = (uint16_t)(i == j ? 0 : d);
        }
      }
      // insertion sort of the row, then its median entry
      for (int x = 1; x < nob; x++) {
        const uint16_t v = dscr[x];
        int y = x - 1;
        while (y >= 0 && dscr[y] > v) {
          dscr[y + 1] = dscr[y];
          y--;
        }
        dscr[y + 1] = v;
      }
      if ((int)dscr[med] < best) {
        best = dscr[med];
        bi = i;
      }
    }
  }
  copy32(a.mp_desc + g * 32, reinterpret_cast<const uint8_t*>(dptr(ob[bi])));
}

// KeyFrame::UpdateBestCovisibles (KeyFrame.cc:139-158): every connection,
// weight descending, ties by id descending (P24). wrow / ks: this thread's
// LDS scratch (kfc ints / bytes) for the row and the sorted ids.
__device__ void update_best_covisibles(const MapArgs& a, const Pools& P, int k, int* wrow,
                                       uint8_t* ks) {
  const int* w = a.kf_w + P.kfb(k) * a.kfc;
  uint8_t* ord = a.kf_ord + P.kfb(k) * a.kfc;
  for (int j = 0; j < a.kfc; j++) wrow[j] = w[j];
  int n = 0;
  for (int j = 0; j < a.kfc; j++)
    if (wrow[j] > 0) ks[n++] = (uint8_t)j;
  // ascending (weight, id), then reversed
  for (int x = 1; x < n; x++) {
    const int v = ks[x];
    int y = x - 1;
    while (y >= 0 && (wrow[ks[y]] > wrow[v] || (wrow[ks[y]] == wrow[v] && ks[y] > v))) {
      ks[y + 1] = ks[y];
      y--;
    }
    ks[y + 1] = (uint8_t)v;
  }
  for (int x = 0; x < n; x++) ord[x] = ks[n - 1 - x];
  a.kf_nord[P.kfb(k)] = n;
}

// KeyFrame::AddConnection (KeyFrame.cc:124-137)
__device__ void add_connection(const MapArgs& a, const Pools& P, int k, int other, int w,
                               int* wrow, uint8_t* ks) {
  int* wk = a.kf_w + P.kfb(k) * a.kfc;
  if (wk[other] == w) return;
  wk[other] = w;
  update_best_covisibles(a, P, k, wrow, ks);
}

}  // namespace

// ---------------------------------------------------------------------------
__global__ void k_map_reset(MapArgs a, const float* T0, int nstreams) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= nstreams) return;
  MapState m{};
  for (int k = 0; k < 16; k++) m.T0[k] = T0 ? T0[s * 16 + k] : (k % 5 == 0 ? 1.f : 0.f);
  m.ref_kf = -1;
  m.last_ref_kf = -1;
  m.last_frame_id = -1;
  a.ms[s] = m;
}

__global__ void __launch_bounds__(kT) k_map_begin(TrackConsts c, MapArgs a) {
  trk_priority();
  __shared__ unsigned long long keys[kMatchMaxKp];
  __shared__ LRec lrec[kLineKeep];
  __shared__ int sstk[96];
  __shared__ float sTl[16];
  __shared__ int s_flag[3];
  __shared__ int s_cut;
  __shared__ int wsum[4];
  const int s = blockIdx.x, t = threadIdx.x;
  MapState& M = a.ms[s];
  StreamState& S = a.st[s];
  const Pools P(a, s);
  if (s == 0 && t == 0) *a.trk_count = 0;
  if (t == 0) {
    const int fid = M.next_id++;
    M.frame_id = fid;
    M.state0 = M.state;
    S.nmatches = S.ninliers = S.nmatches_map = S.ok = 0;
    S.nlmatches = S.nlmatches_map = 0;
    S.lm_active = S.lm_nlocal = S.lm_nllocal = S.lm_wiped = S.lm_ninl = 0;
    S.lm_inl = S.lm_linl = S.lm_ok = 0;
    S.trk = S.trk_go = S.trk_nlm = S.trk_wiped = 0;
    for (int k = 0; k < kMapOut; k++) S.map_out[k] = 0;
    M.n_tp = M.n_tl = 0;
    M.n_local_mp = M.n_local_ml = 0;
    const bool okst = M.state == kOK;
    const bool trk_first = okst && a.refkf && (!M.has_velocity || fid < 2);
    const bool motion = okst && !trk_first;
    M.trk_first = trk_first;
    M.motion = motion;
    S.has_last = motion ? 1 : 0;
    s_flag[0] = motion;
    s_flag[1] = motion && M.last_kf_frame != M.last_frame_id;   // UpdateLastFrame creates
    if (motion) {
      float Tl[16];
      gemm44(M.Tcr, a.kf_T + P.kfb(M.last_ref_kf) * 16, Tl);   // Tlr * Trw
      for (int k = 0; k < 16; k++) {
        sTl[k] = Tl[k];
        S.Tlast[k] = Tl[k];
      }
      if (M.has_velocity) gemm44(M.V, Tl, S.Tcw);
      else
        for (int k = 0; k < 16; k++) S.Tcw[k] = Tl[k];   // no vocabulary: zero velocity (pinned)
    }
    s_cut = 0x7fffffff;
  }
  __syncthreads();
  // a fresh current frame: no map points / lines, no outliers
  const int n = a.n[s], nl = a.lines ? a.nl[s] : 0;
  for (int i = t; i < n; i += kT) {
    a.mpid[P.cb + i] = -1;
    a.outlier[P.cb + i] = 0;
    a.match[P.cb + i] = -1;
  }
  for (int j = t; j < nl; j += kT) {
    a.mlid[P.lb + j] = -1;
    a.loutlier[P.lb + j] = 0;
    a.lmatch[P.lb + j] = -1;
  }
  if (!s_flag[0]) return;
  // ---- the last frame as the matchers read it (its map points / lines) ----
  const int ln = a.l_n[s], lnl = a.lines ? a.l_nl[s] : 0;
  for (int i = t; i < ln; i += kT) {
    const long long o = P.cb + i;
    const int m = a.l_mpid[o];
    a.l_has_mp[o] = m >= 0;
    a.l_nobs[o] = P.mp_nobs(m);
    if (m >= 0) {
      float x[3];
      P.mp_xyz(m, x);
      for (int q = 0; q < 3; q++) a.l_mp_xyz[o * 3 + q] = x[q];
      copy32(a.l_mp_desc + o * 32, a.mp_desc + (P.mb + m) * 32);
    }
  }
  for (int j = t; j < lnl; j += kT) {
    const long long o = P.lb + j;
    const int m = a.l_mlid[o];
    a.l_has_ml[o] = m >= 0;
    if (m >= 0) {
      float x[6];
      P.ml_xyz(m, x);
      for (int q = 0; q < 6; q++) a.l_ml_xyz[o * 6 + q] = x[q];
      copy32(a.l_ml_desc + o * 32, a.ml_desc + (P.lmb + m) * 32);
    }
  }
  if (!s_flag[1]) return;
  // ---- UpdateLastFrame: temporal points, depth ascending (then index) ----
  int Pn = 1;
  while (Pn < ln) Pn <<= 1;
  int nv = 0;
  for (int i = t; i < Pn; i += kT) {
    unsigned long long k = ~0ull;
    if (i < ln) {
      const float z = a.l_depth[P.cb + i];
      if (z > 0) {
        k = ((unsigned long long)__float_as_uint(z) << 32) | (unsigned)i;
        nv++;
      }
    }
    keys[i] = k;
  }
  nv = block_sum(nv, wsum);
  if (nv == 0) return;   // "if(vDepthIdx.empty()) return;" (lines included)
  bitonic_sort(keys, Pn);
  const float thd = c.th_depth;
  for (int j = t; j < nv; j += kT) {
    const float z = __uint_as_float((unsigned)(keys[j] >> 32));
    if (z > thd && j + 1 > 100) atomicMin(&s_cut, j);
  }
  __syncthreads();
  const int last = min(s_cut, nv - 1);
  int ntp = 0;
  for (int j = t; j <= last; j += kT) {
    const int i = (int)(keys[j] & 0xffffffffu);
    const long long o = P.cb + i;
    if (a.l_mpid[o] != -1) continue;   // a map point (Observations() >= 1)
    const float z = __uint_as_float((unsigned)(keys[j] >> 32));
    const KeyPointD kp = a.l_kps_un[o];
    float Ow[3], w[3];
    gemm_neg_Rt_t(sTl, Ow);
    unproject_f(c, sTl, Ow, kp.x, kp.y, z, w);
    a.l_mpid[o] = -2 - i;
    a.l_has_mp[o] = 1;
    a.l_nobs[o] = 0;
    for (int q = 0; q < 3; q++) a.l_mp_xyz[o * 3 + q] = w[q];
    copy32(a.l_mp_desc + o * 32, a.l_desc + o * 32);
    ntp++;
  }
  ntp = block_sum(ntp, wsum);
  if (t == 0) M.n_tp = ntp;
  if (!a.lines) return;
  // ---- temporal lines: std::sort by max end-point depth (thread 0 decides
  // from LDS, the lines are made in parallel) ----
  __shared__ uint8_t lmake[kLineKeep];
  if (t < kLineKeep) lmake[t] = 0;
  if (t < lnl) {
    const long long o = P.lb + t;
    const float zs = a.l_dstart[o], ze = a.l_dend[o];
    lrec[t] = LRec{(zs > 0 && ze > 0) ? fmaxf(zs, ze) : -1.f, a.l_mlid[o] == -1 ? t : -1 - t};
  }
  __syncthreads();
  if (t == 0) {
    int m = 0;
    for (int j = 0; j < lnl; j++)
      if (lrec[j].k >= 0) lrec[m++] = lrec[j];
    stl_sort(lrec, m, sstk);
    int nlines = 0, ntl = 0;
    for (int q = 0; q < m; q++) {
      if (lrec[q].i >= 0) {   // no map line at this line
        lmake[lrec[q].i] = 1;
        ntl++;
      }
      nlines++;
      if (lrec[q].k > thd && nlines > 45) break;
    }
    M.n_tl = ntl;
  }
  __syncthreads();
  if (t < lnl && lmake[t]) {
    const long long o = P.lb + t;
    float Ow[3];
    gemm_neg_Rt_t(sTl, Ow);
    const orbpl_keyline k = a.l_kl_un[o];
    const float zs = a.l_dstart[o];
    float* x = a.l_ml_xyz + o * 6;
    unproject_f(c, sTl, Ow, k.startPointX, k.startPointY, zs, x);
    unproject_f(c, sTl, Ow, k.endPointX, k.endPointY, zs, x + 3);   // Frame.cc:1192
    copy32(a.l_ml_desc + o * 32, a.l_ldesc + o * 32);
    a.l_mlid[o] = -2 - t;
    a.l_has_ml[o] = 1;
  }
}

// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(kT) k_map_resolve_motion(MapArgs a) {
  trk_priority();
  __shared__ int wsum[4];
  __shared__ int s_trk;
  const int s = blockIdx.x, t = threadIdx.x;
  MapState& M = a.ms[s];
  StreamState& S = a.st[s];
  const Pools P(a, s);
  const int fid = M.frame_id;
  const int n = a.n[s], nl = a.lines ? a.nl[s] : 0;
  if (M.state0 != kOK) {
    if (t == 0) a.trk_nml[s] = 0;
    return;
  }
  bool motion_ok = false;
  if (M.motion) {
    for (int i = t; i < n; i += kT) {
      const int m = a.match[P.cb + i];
      a.mpid[P.cb + i] = m >= 0 ? a.l_mpid[P.cb + m] : -1;
    }
    for (int j = t; j < nl; j += kT) {
      const int m = a.lmatch[P.lb + j];
      a.mlid[P.lb + j] = m >= 0 ? a.l_mlid[P.lb + m] : -1;
    }
    const bool posed = S.nmatches >= 20 && (!a.lines || S.nlmatches >= 15);
    int nmap = 0, lnmap = 0;
    if (posed) {
      for (int i = t; i < n; i += kT) {
        const long long o = P.cb + i;
        const int m = a.mpid[o];
        if (m == -1) continue;
        if (a.outlier[o]) {
          a.mpid[o] = -1;
          a.outlier[o] = 0;
          if (m >= 0) a.mp_seen[P.mb + m] = fid;
        } else if (P.mp_nobs(m) > 0) {
          nmap++;
        }
      }
      for (int j = t; j < nl; j += kT) {
        const long long o = P.lb + j;
        const int m = a.mlid[o];
        if (m == -1) continue;
        if (a.loutlier[o]) {
          a.mlid[o] = -1;
          a.loutlier[o] = 0;
          if (m >= 0) a.ml_seen[P.lmb + m] = fid;
          lnmap--;
        } else if (P.ml_nobs(m) > 0) {
          lnmap++;
        }
      }
    }
    nmap = block_sum(nmap, wsum);
    lnmap = block_sum(lnmap, wsum);
    motion_ok = posed && (a.lines ? (nmap >= 10 || lnmap >= 15) : nmap >= 10);
    if (t == 0) {
      S.nmatches_map = nmap;
      S.nlmatches_map = lnmap;
    }
  }
  if (t == 0) {
    S.ok = motion_ok;
    s_trk = a.refkf && (M.trk_first || (M.motion && !motion_ok));
    S.trk = s_trk;
    a.trk_nml[s] = 0;
    if (s_trk) a.trk_list[atomicAdd(a.trk_count, 1)] = s;
  }
  __syncthreads();
  if (!s_trk) return;
  // ---- TrackReferenceKeyFrame: the reference keyframe staged as a frame ----
  const int kf = M.ref_kf;
  const long long kb = P.kfb(kf);
  const int N = a.kf_N[kb], NL = a.lines ? a.kf_NL[kb] : 0;
  for (int i = t; i < N; i += kT) {
    const long long src = kb * a.kp_pitch + i, o = P.cb + i;
    const int m = a.kf_mp[src];
    a.r_kps_un[o] = a.kf_kp[src];
    copy32(a.r_desc + o * 32, a.kf_desc + src * 32);
    a.r_mpid[o] = m;
    a.r_has_mp[o] = m >= 0;
    a.r_node[o] = a.kf_node[src];
    if (m >= 0) {
      const float4 X = a.mp_pos[P.mb + m];
      a.r_mp_xyz[o * 3] = X.x;
      a.r_mp_xyz[o * 3 + 1] = X.y;
      a.r_mp_xyz[o * 3 + 2] = X.z;
    }
  }
  for (int j = t; j < NL; j += kT) {
    const long long src = kb * kLineKeep + j, o = P.lb + j;
    const int m = a.kf_ml[src];
    a.r_mlid[o] = m;
    a.r_has_ml[o] = m >= 0;
    if (m >= 0) {
      for (int q = 0; q < 6; q++) a.r_ml_xyz[o * 6 + q] = a.ml_pos[(P.lmb + m) * 6 + q];
      copy32(a.r_ml_desc + o * 32, a.ml_desc + (P.lmb + m) * 32);
    }
  }
  // the frame's current line assignments (the motion model's after its
  // discard) and their observation counts for the keyframe line search
  for (int j = t; j < nl; j += kT) {
    const int m = a.mlid[P.lb + j];
    a.trk_cur_nobs[P.lb + j] = m != -1 ? P.ml_nobs(m) : 0;
  }
  for (int i = t; i < n; i += kT) a.match[P.cb + i] = -1;
  if (t == 0) {
    a.r_n[s] = N;
    if (a.lines) a.r_nl[s] = NL;
    a.trk_nml[s] = NL;
    for (int k = 0; k < 16; k++) S.Tcw[k] = S.Tlast[k];   // SetPose(mLastFrame.mTcw)
    S.nmatches = 0;
    S.ninliers = 0;
    S.nmatches_map = S.nlmatches_map = 0;
    S.trk_go = S.trk_nlm = S.trk_wiped = 0;
  }
}

__device__ static void pose_inputs(const MapArgs& a, const Pools& P, int n, int nl) {
  for (int i = threadIdx.x; i < n; i += kT) {
    const long long o = P.cb + i;
    const int m = a.mpid[o];
    a.m2[o] = m != -1 ? i : -1;
    if (m != -1) P.mp_xyz(m, a.pxyz + o * 3);
  }
  for (int j = threadIdx.x; j < nl; j += kT) {
    const long long o = P.lb + j;
    const int m = a.mlid[o];
    a.lm2[o] = m != -1 ? j : -1;
    if (m != -1) P.ml_xyz(m, a.lpxyz + o * 6);
  }
}

__global__ void __launch_bounds__(kT) k_map_trk_merge(MapArgs a) {
  trk_priority();
  __shared__ int s_go;
  const int s = blockIdx.x, t = threadIdx.x;
  StreamState& S = a.st[s];
  if (!S.trk) return;
  const Pools P(a, s);
  const int n = a.n[s], nl = a.lines ? a.nl[s] : 0;
  // LineMatcher(0.7).SearchByProjection(F, RefKF): its relaxed retry cleared
  // every assignment first; its matches replace the ones they hit
  const bool wiped = a.lines && S.trk_wiped;
  for (int j = t; j < nl; j += kT) {
    const long long o = P.lb + j;
    int m = wiped ? -1 : a.mlid[o];
    const int r = a.trk_lm[o];
    if (r >= 0) m = a.r_mlid[P.lb + r];
    a.mlid[o] = m;
  }
  if (t == 0) {
    if (a.lines) S.nlmatches = S.trk_nlm;
    s_go = S.nmatches >= 15 && (!a.lines || S.trk_nlm >= 10);
    S.trk_go = s_go;
  }
  __syncthreads();
  if (!s_go) return;
  // mCurrentFrame.mvpMapPoints = vpMapPointMatches
  for (int i = t; i < n; i += kT) {
    const int r = a.match[P.cb + i];
    a.mpid[P.cb + i] = r >= 0 ? a.r_mpid[P.cb + r] : -1;
  }
  __syncthreads();
  pose_inputs(a, P, n, nl);
}

__global__ void __launch_bounds__(kT) k_map_resolve_trk(MapArgs a) {
  trk_priority();
  __shared__ int wsum[4];
  const int s = blockIdx.x, t = threadIdx.x;
  MapState& M = a.ms[s];
  StreamState& S = a.st[s];
  const Pools P(a, s);
  if (M.state0 != kOK) {
    if (t == 0) S.lm_active = 0;
    return;
  }
  if (S.trk) {
    bool ok = false;
    if (S.trk_go) {
      const int fid = M.frame_id;
      const int n = a.n[s], nl = a.lines ? a.nl[s] : 0;
      int nmap = 0, lnmap = 0;
      for (int i = t; i < n; i += kT) {
        const long long o = P.cb + i;
        const int m = a.mpid[o];
        if (m == -1) continue;
        if (a.outlier[o]) {
          a.mpid[o] = -1;
          a.outlier[o] = 0;
          if (m >= 0) a.mp_seen[P.mb + m] = fid;
        } else if (P.mp_nobs(m) > 0) {
          nmap++;
        }
      }
      for (int j = t; j < nl; j += kT) {
        const long long o = P.lb + j;
        const int m = a.mlid[o];
        if (m == -1) continue;
        if (a.loutlier[o]) {
          a.mlid[o] = -1;
          a.loutlier[o] = 0;
          if (m >= 0) a.ml_seen[P.lmb + m] = fid;
          lnmap--;
        } else if (P.ml_nobs(m) > 0) {
          lnmap++;
        }
      }
      nmap = block_sum(nmap, wsum);
      lnmap = block_sum(lnmap, wsum);
      ok = nmap >= 10 && (!a.lines || lnmap >= 10);
      if (t == 0) {
        S.nmatches_map = nmap;
        S.nlmatches_map = lnmap;
      }
    }
    if (t == 0) S.ok = ok;
  }
  __syncthreads();
  if (t == 0) S.lm_active = S.ok ? 1 : 0;   // TrackLocalMap runs if bOK
}

// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(kT) k_map_local(MapArgs a) {
  trk_priority();
  __shared__ int cnt[kMapMaxKF];
  __shared__ int wsum[4];
  const int s = blockIdx.x, t = threadIdx.x;
  MapState& M = a.ms[s];
  const StreamState& S = a.st[s];
  const Pools P(a, s);
  if (!S.lm_active) {
    if (t == 0) {
      a.l_count[s] = 0;
      if (a.lines) a.ll_count[s] = 0;
    }
    return;
  }
  const int fid = M.frame_id;
  const int n = a.n[s], nl = a.lines ? a.nl[s] : 0;
  const int nkf = M.n_kf;
  if (t < kMapMaxKF) cnt[t] = 0;
  __syncthreads();
  // ---- UpdateLocalKeyFrames: keyframes observing the frame's points ----
  for (int i = t; i < n; i += kT) {
    const int m = a.mpid[P.cb + i];
    if (m < 0) continue;   // temporal points have no observations
    const long long g = P.mb + m;
    const int nob = a.mp_nob[g];
    const uint32_t* ob = a.mp_obs + g * a.kfc;
    for (int k = 0; k < nob; k++) atomicAdd(&cnt[ob[k] >> 16], 1);
  }
  __syncthreads();
  if (t == 0) {
    bool any = false;
    for (int k = 0; k < nkf; k++) any |= cnt[k] > 0;
    if (any) {
      unsigned long long mark = 0;
      int mx = 0, kmax = -1, nloc = 0;
      for (int k = 0; k < nkf; k++) {
        if (cnt[k] <= 0) continue;
        if (cnt[k] > mx) {
          mx = cnt[k];
          kmax = k;
        }
        M.local_kf[nloc++] = k;
        mark |= 1ull << k;
      }
      const int n0 = nloc;
      for (int q = 0; q < n0; q++) {
        if (nloc > 80) break;
        const int k = M.local_kf[q];
        const long long kb = P.kfb(k);
        const int nn = min(10, a.kf_nord[kb]);
        for (int b = 0; b < nn; b++) {
          const int nb = a.kf_ord[kb * a.kfc + b];
          if (!((mark >> nb) & 1ull)) {
            M.local_kf[nloc++] = nb;
            mark |= 1ull << nb;
            break;
          }
        }
        unsigned long long ch = a.kf_child[kb];
        while (ch) {
          const int cidx = __ffsll((long long)ch) - 1;
          ch &= ch - 1;
          if (!((mark >> cidx) & 1ull)) {
            M.local_kf[nloc++] = cidx;
            mark |= 1ull << cidx;
            break;
          }
        }
        const int par = a.kf_parent[kb];
        if (par >= 0 && !((mark >> par) & 1ull)) {
          M.local_kf[nloc++] = par;
          mark |= 1ull << par;
          break;
        }
      }
      M.n_local_kf = nloc;
      M.ref_kf = kmax;
    }
  }
  // ---- SearchLocalPoints / SearchLocalLines: the frame's own elements are
  // seen (not searched again); Observations() of each keypoint's point ----
  for (int i = t; i < n; i += kT) {
    const int m = a.mpid[P.cb + i];
    if (m >= 0) a.mp_seen[P.mb + m] = fid;
    a.cur_nobs[P.cb + i] = m != -1 ? P.mp_nobs(m) : 0;
  }
  for (int j = t; j < nl; j += kT) {
    const int m = a.mlid[P.lb + j];
    if (m >= 0) a.ml_seen[P.lmb + m] = fid;
    a.cur_nobs_l[P.lb + j] = m != -1 ? P.ml_nobs(m) : 0;
  }
  __syncthreads();
  // ---- UpdateLocalPoints / UpdateLocalLines: the local keyframes' elements
  // in keyframe then index order, each once; the seen ones are not matched
  // (mbTrackInView false), so they are left out of the searched list ----
  const int nloc = M.n_local_kf;
  int np = 0, nlp = 0;
  for (int q = 0; q < nloc; q++) {
    const long long kb = P.kfb(M.local_kf[q]);
    const int N = a.kf_N[kb];
    for (int c0 = 0; c0 < N; c0 += kT) {
      const int i = c0 + t;
      int p = -1;
      if (i < N) {
        p = a.kf_mp[kb * a.kp_pitch + i];
        if (p >= 0 && a.mp_tref[P.mb + p] == fid) p = -1;
      }
      const bool f = p >= 0 && a.mp_seen[P.mb + p] != fid;
      __syncthreads();
      if (p >= 0) a.mp_tref[P.mb + p] = fid;
      int tot = 0;
      const int pos = np + block_prefix(f, wsum, &tot);
      if (f && pos < a.lp) {
        const long long d = (long long)s * a.lp + pos, g = P.mb + p;
        const float4 X = a.mp_pos[g], Nv = a.mp_nrm[g];
        const float2 D = a.mp_dist[g];
        a.l_xyz[d * 3] = X.x; a.l_xyz[d * 3 + 1] = X.y; a.l_xyz[d * 3 + 2] = X.z;
        a.l_nrm[d * 3] = Nv.x; a.l_nrm[d * 3 + 1] = Nv.y; a.l_nrm[d * 3 + 2] = Nv.z;
        a.l_dmin[d] = D.x;   // mfMinDistance, mfMaxDistance: k_in_frustum applies
        a.l_dmax[d] = D.y;   // GetMin/MaxDistanceInvariance's 0.8f / 1.2f itself
        copy32(a.l_ldesc_pts + d * 32, a.mp_desc + g * 32);
        a.l_id[d] = p;
      }
      np += tot;
      __syncthreads();
    }
    if (!a.lines) continue;
    const int NL = a.kf_NL[kb];
    for (int c0 = 0; c0 < NL; c0 += kT) {
      const int j = c0 + t;
      int l = -1;
      if (j < NL) {
        l = a.kf_ml[kb * kLineKeep + j];
        if (l >= 0 && a.ml_tref[P.lmb + l] == fid) l = -1;
      }
      const bool f = l >= 0 && a.ml_seen[P.lmb + l] != fid;
      __syncthreads();
      if (l >= 0) a.ml_tref[P.lmb + l] = fid;
      int tot = 0;
      const int pos = nlp + block_prefix(f, wsum, &tot);
      if (f && pos < a.llp) {
        const long long d = (long long)s * a.llp + pos, g = P.lmb + l;
        for (int k = 0; k < 6; k++) a.ll_xyz[d * 6 + k] = a.ml_pos[g * 6 + k];
        copy32(a.ll_desc + d * 32, a.ml_desc + g * 32);
        a.ll_id[d] = l;
      }
      nlp += tot;
      __syncthreads();
    }
  }
  if (t == 0) {
    if (np > a.lp || nlp > a.llp) M.err |= 4;
    np = min((long long)np, a.lp);
    nlp = min((long long)nlp, a.llp);
    a.l_count[s] = np;
    if (a.lines) a.ll_count[s] = nlp;
    M.n_local_mp = np;
    M.n_local_ml = nlp;
  }
}

__global__ void __launch_bounds__(kT) k_map_assemble(MapArgs a) {
  trk_priority();
  const int s = blockIdx.x, t = threadIdx.x;
  const StreamState& S = a.st[s];
  if (!S.lm_active) return;
  const Pools P(a, s);
  const int n = a.n[s], nl = a.lines ? a.nl[s] : 0;
  for (int i = t; i < n; i += kT) {
    const int r = a.lm_match[P.cb + i];
    if (r >= 0) a.mpid[P.cb + i] = a.l_id[(long long)s * a.lp + r];
  }
  const bool wiped = a.lines && S.lm_wiped;
  for (int j = t; j < nl; j += kT) {
    const long long o = P.lb + j;
    int m = wiped ? -1 : a.mlid[o];
    const int r = a.llm_match[o];
    if (r >= 0) m = a.ll_id[(long long)s * a.llp + r];
    a.mlid[o] = m;
  }
  __syncthreads();
  pose_inputs(a, P, n, nl);
}

// ---------------------------------------------------------------------------
// KeyFrame(Frame&) (KeyFrame.cc:28-58): the frame's data into slot kf
__device__ static void write_keyframe(const MapArgs& a, const Pools& P, int kf, const float* T,
                                      int fid, int n, int nl) {
  const int t = threadIdx.x;
  const long long kb = P.kfb(kf);
  if (t < 16) a.kf_T[kb * 16 + t] = T[t];
  if (t == 0) {
    float Ow[3];
    gemm_neg_Rt_t(T, Ow);
    for (int q = 0; q < 3; q++) a.kf_Ow[kb * 4 + q] = Ow[q];
    a.kf_Ow[kb * 4 + 3] = 0.f;
    a.kf_N[kb] = n;
    a.kf_NL[kb] = nl;
    a.kf_frame[kb] = fid;
    a.kf_nord[kb] = 0;
    a.kf_parent[kb] = -1;
    a.kf_first[kb] = 1;
    a.kf_child[kb] = 0ull;
  }
  for (int j = t; j < a.kfc; j += kT) {
    a.kf_w[kb * a.kfc + j] = 0;
    a.kf_w[P.kfb(j) * a.kfc + kf] = 0;
  }
  for (int i = t; i < n; i += kT) {
    const long long src = P.cb + i, d = kb * a.kp_pitch + i;
    a.kf_mp[d] = a.mpid[src];
    a.kf_kp[d] = a.kps_un[src];
    a.kf_ur[d] = a.uright[src];
    copy32(a.kf_desc + d * 32, a.desc + src * 32);
    a.kf_node[d] = a.vocab ? a.feat_node[src] : -1;
  }
  for (int j = t; j < nl; j += kT) {
    const long long src = P.lb + j, d = kb * kLineKeep + j;
    a.kf_ml[d] = a.mlid[src];
    copy32(a.kf_ldesc + d * 32, a.ldesc + src * 32);
    a.kf_ds[d] = a.dstart[src];
    a.kf_de[d] = a.dend[src];
  }
}

// a new map point of keyframe kf at keypoint i: its pool id into the
// keyframe and the frame (the point itself is built by k_map_kf_points)
__device__ static void mark_new_point(const MapArgs& a, const Pools& P, int p, int kf, int i) {
  a.kf_mp[P.kfb(kf) * a.kp_pitch + i] = p;
  a.mpid[P.cb + i] = p;
}

__device__ static void new_line(const TrackConsts& c, const MapArgs& a, const Pools& P, int l,
                                int kf, int j, const float* T) {
  const long long g = P.lmb + l, src = P.lb + j;
  const orbpl_keyline k = a.kl_un[src];
  const float zs = a.dstart[src], ze = a.dend[src];
  float Ow[3];
  gemm_neg_Rt_t(T, Ow);
  unproject_f(c, T, Ow, k.startPointX, k.startPointY, zs, a.ml_pos + g * 6);
  unproject_f(c, T, Ow, k.endPointX, k.endPointY, zs, a.ml_pos + g * 6 + 3);   // Frame.cc:1192
  // MapLine::AddObservation (one observation: its descriptor is the row's)
  a.ml_nobs[g] = (zs >= 0 && ze >= 0) ? 2 : 1;
  copy32(a.ml_desc + g * 32, a.ldesc + src * 32);
  a.ml_seen[g] = -1;
  a.ml_tref[g] = -1;
  a.kf_ml[P.kfb(kf) * kLineKeep + j] = l;
  a.mlid[src] = l;
}

__global__ void __launch_bounds__(kT) k_map_finish(TrackConsts c, MapArgs a) {
  trk_priority();
  __shared__ unsigned long long keys[kMatchMaxKp];
  __shared__ LRec lrec[kLineKeep];
  __shared__ int lpool[kLineKeep];   // the pool slot a line's new map line takes, -1 none
  __shared__ int sstk[96];
  __shared__ float sT[16];
  __shared__ int wsum[4];
  __shared__ int s_i[8];
  const int s = blockIdx.x, t = threadIdx.x;
  MapState& M = a.ms[s];
  StreamState& S = a.st[s];
  const Pools P(a, s);
  const int fid = M.frame_id;
  const int n = a.n[s], nl = a.lines ? a.nl[s] : 0;
  const int state0 = M.state0;
  if (t == 0) M.new_kf = -1;
  // ================= not initialised: StereoInitialization ================
  if (state0 == kNotInit) {
    const bool init = n > 500;
    if (t < 16) sT[t] = M.T0[t];
    __syncthreads();
    if (init) {
      write_keyframe(a, P, 0, sT, fid, n, nl);
      __syncthreads();
      int base = 0;
      for (int c0 = 0; c0 < n; c0 += kT) {
        const int i = c0 + t;
        const float z = i < n ? a.depth[P.cb + i] : 0.f;
        const bool f = z > 0;
        int tot = 0;
        const int pos = base + block_prefix(f, wsum, &tot);
        if (f && pos < a.mpc) mark_new_point(a, P, pos, 0, i);
        base += tot;
      }
      __syncthreads();
      // a map line per line with both end-point depths, in line order
      {
        const bool f = t < nl && a.dstart[P.lb + t] > 0 && a.dend[P.lb + t] > 0;
        int tot = 0;
        const int pos = block_prefix(f, wsum, &tot);
        if (f && pos < a.mlc) new_line(c, a, P, pos, 0, t, sT);
        if (t == 0) s_i[4] = (int)min((long long)tot, a.mlc);
      }
      __syncthreads();
      if (t == 0) {
        const int nml = s_i[4];
        M.n_kf = 1;
        M.n_mp = (int)min((long long)base, a.mpc);
        M.n_ml = nml;
        M.new_kf = 0;
        M.kf_mp_base = 0;
        if (base > a.mpc) M.err |= 2;
        M.state = kOK;
        M.last_kf_frame = fid;
        M.ref_kf = 0;
        M.n_local_kf = 1;
        M.local_kf[0] = 0;
        M.has_velocity = 0;
        float Twr[16];
        pose_inverse(sT, Twr);
        gemm44(sT, Twr, M.Tcr);
        S.ok = 1;
        S.map_out[0] = 2;
      }
    } else if (t == 0) {
      S.ok = 0;
    }
    if (t < 16) S.Tcw[t] = sT[t];
  } else if (state0 == kLost) {
    // ================= LOST: Relocalization fails (P23) ================
    if (t == 0) {
      float T[16];
      gemm44(M.Tcr, a.kf_T + P.kfb(M.last_ref_kf) * 16, T);
      for (int k = 0; k < 16; k++) S.Tcw[k] = T[k];
      S.ok = 0;
      M.state = kLost;
    }
  } else {
    // ================= tracked: TrackLocalMap's decision ================
    bool ok = false;
    if (S.lm_active) {
      int inl = 0, linl = 0;
      for (int i = t; i < n; i += kT) {
        const long long o = P.cb + i;
        const int m = a.mpid[o];
        inl += m != -1 && !a.outlier[o] && P.mp_nobs(m) > 0;
        // STEREO: an outlier's map point leaves the frame (Tracking.cc:1374-1377)
        if (a.stereo && m != -1 && a.outlier[o]) a.mpid[o] = -1;
      }
      for (int j = t; j < nl; j += kT) {
        const long long o = P.lb + j;
        const int m = a.mlid[o];
        linl += m != -1 && !a.loutlier[o] && P.ml_nobs(m) > 0;
        if (a.stereo && m != -1 && a.loutlier[o]) a.mlid[o] = -1;   // :1398-1401
      }
      inl = block_sum(inl, wsum);
      linl = block_sum(linl, wsum);
      ok = !(fid < a.max_frames && inl + linl < 60) && !(inl < 30 && linl < 20);
      if (t == 0) {
        S.lm_inl = inl;
        S.lm_linl = linl;
        S.lm_ok = ok;
        s_i[0] = inl;
      }
    }
    if (t == 0) {
      S.ok = ok;
      M.state = ok ? kOK : kLost;
    }
    if (t < 16) sT[t] = S.Tcw[t];
    __syncthreads();
    if (ok) {
      if (t == 0) {
        float LastTwc[16];
        pose_inverse(S.Tlast, LastTwc);
        gemm44(sT, LastTwc, M.V);   // mVelocity = Tcw * LastTwc
        M.has_velocity = 1;
        S.map_out[4] = M.n_tp;
        S.map_out[11] = M.n_tl;
      }
      // ---- clean VO matches: temporal elements leave the frame ----
      for (int i = t; i < n; i += kT) {
        const long long o = P.cb + i;
        const int m = a.mpid[o];
        if (m != -1 && P.mp_nobs(m) < 1) {
          a.outlier[o] = 0;
          a.mpid[o] = -1;
        }
      }
      for (int j = t; j < nl; j += kT) {
        const long long o = P.lb + j;
        const int m = a.mlid[o];
        if (m != -1 && P.ml_nobs(m) < 1) {
          a.loutlier[o] = 0;
          a.mlid[o] = -1;
        }
      }
      __syncthreads();
      // ---- NeedNewKeyFrame (P23: Local Mapping idle, never stopped) ----
      const int nKFs = M.n_kf;
      const int nMinObs = nKFs <= 2 ? 2 : 3;
      const long long rb = P.kfb(M.ref_kf);
      const int rN = a.kf_N[rb];
      int nref = 0, ntc = 0, nntc = 0;
      for (int i = t; i < rN; i += kT) {
        const int p = a.kf_mp[rb * a.kp_pitch + i];
        nref += p >= 0 && a.mp_nobs[P.mb + p] >= nMinObs;
      }
      for (int i = t; i < n; i += kT) {
        const long long o = P.cb + i;
        const float z = a.depth[o];
        if (z > 0 && z < c.th_depth) {
          if (a.mpid[o] != -1 && !a.outlier[o]) ntc++;
          else nntc++;
        }
      }
      nref = block_sum(nref, wsum);
      ntc = block_sum(ntc, wsum);
      nntc = block_sum(nntc, wsum);
      const int inl = s_i[0];
      bool need = true;
      if (fid < a.max_frames && nKFs > a.max_frames) need = false;
      const bool close = ntc < 100 && nntc > 70;
      float thRefRatio = 0.75f;
      if (nKFs < 2) thRefRatio = 0.4f;
      const bool c1a = fid >= M.last_kf_frame + a.max_frames;
      const bool c1b = fid >= M.last_kf_frame + 0;   // && bLocalMappingIdle
      const bool c1c = inl < nref * 0.25 || close;
      const bool c2 = (inl < nref * thRefRatio || close) && inl > 15;
      need = need && (c1a || c1b || c1c) && c2;
      if (need && nKFs >= a.kfc) {
        need = false;
        if (t == 0) M.err |= 1;
      }
      if (need) {
        // ==== CreateNewKeyFrame ====
        const int kf = nKFs;
        write_keyframe(a, P, kf, sT, fid, n, nl);
        __syncthreads();
        // new points: depth ascending (then index), all close ones and at
        // least the 100 closest (Tracking.cc:1592-1655)
        int Pn = 1;
        while (Pn < n) Pn <<= 1;
        int nv = 0;
        for (int i = t; i < Pn; i += kT) {
          unsigned long long k = ~0ull;
          if (i < n) {
            const float z = a.depth[P.cb + i];
            if (z > 0) {
              k = ((unsigned long long)__float_as_uint(z) << 32) | (unsigned)i;
              nv++;
            }
          }
          keys[i] = k;
        }
        if (t == 0) s_i[1] = 0x7fffffff;
        nv = block_sum(nv, wsum);
        bitonic_sort(keys, Pn);
        for (int j = t; j < nv; j += kT) {
          const float z = __uint_as_float((unsigned)(keys[j] >> 32));
          if (z > c.th_depth && j + 1 > 100) atomicMin(&s_i[1], j);
        }
        __syncthreads();
        const int last = nv > 0 ? min(s_i[1], nv - 1) : -1;
        int base = M.n_mp;
        for (int c0 = 0; c0 <= last; c0 += kT) {
          const int j = c0 + t;
          int i = -1;
          if (j <= last) i = (int)(keys[j] & 0xffffffffu);
          const bool f = i >= 0 && a.mpid[P.cb + i] == -1;
          int tot = 0;
          const int pos = base + block_prefix(f, wsum, &tot);
          if (f && pos < a.mpc) mark_new_point(a, P, pos, kf, i);
          base += tot;
        }
        __syncthreads();
        // new lines: std::sort by the larger end-point depth, all close ones
        // and at least 45 (Tracking.cc:1660-1730); thread 0 decides from LDS,
        // the lines are created in parallel
        if (t < kLineKeep) lpool[t] = -1;
        if (t < nl) {
          const long long o = P.lb + t;
          const float zs = a.dstart[o], ze = a.dend[o];
          lrec[t] = LRec{(zs > 0 && ze > 0) ? fmaxf(zs, ze) : -1.f, a.mlid[o] == -1 ? t : -1 - t};
        }
        __syncthreads();
        if (t == 0) {
          if (base > a.mpc) M.err |= 2;
          M.kf_mp_base = M.n_mp;
          M.new_kf = kf;
          M.n_mp = (int)min((long long)base, a.mpc);
          int m = 0;
          for (int j = 0; j < nl; j++)
            if (lrec[j].k >= 0) lrec[m++] = lrec[j];   // in line order, as the reference's vector
          stl_sort(lrec, m, sstk);
          int nlines = 0, nml = M.n_ml;
          for (int q = 0; q < m; q++) {
            if (lrec[q].i >= 0) {   // no map line at this line yet
              if (nml < a.mlc) lpool[lrec[q].i] = nml++;
              else M.err |= 2;
            }
            nlines++;
            if (lrec[q].k > c.th_depth && nlines > 45) break;
          }
          M.n_ml = nml;
          M.n_kf = kf + 1;
          M.ref_kf = kf;
          M.last_kf_frame = fid;
          S.map_out[0] = 1;
        }
        __syncthreads();
        if (t < nl && lpool[t] >= 0) new_line(c, a, P, lpool[t], kf, t, sT);
        __syncthreads();
        // LocalMapping::ProcessNewKeyFrame and UpdateConnections follow in
        // k_map_kf_points / k_map_connect
      }
      // ---- outliers leave the frame (Tracking.cc:548-555; lines by the
      // point flags, replicated) ----
      for (int i = t; i < n; i += kT) {
        const long long o = P.cb + i;
        if (a.mpid[o] != -1 && a.outlier[o]) a.mpid[o] = -1;
      }
      for (int j = t; j < nl; j += kT) {
        const long long o = P.lb + j;
        if (a.mlid[o] != -1 && j < n && a.outlier[P.cb + j]) a.mlid[o] = -1;
      }
    }
    __syncthreads();
    // relative pose to the frame's reference keyframe (Tracking.cc:580-587)
    if (t == 0) {
      float Twr[16];
      pose_inverse(a.kf_T + P.kfb(M.ref_kf) * 16, Twr);
      gemm44(sT, Twr, M.Tcr);
      if (S.lm_active) {
        S.map_out[8] = M.n_local_kf;
        S.map_out[9] = M.n_local_mp;
        S.map_out[10] = M.n_local_ml;
      }
    }
  }
  __syncthreads();
  if (t == 0) {
    // reset soon after initialisation (Tracking.cc:558-568)
    const bool reset_now = M.state == kLost && M.n_kf <= 5;
    if (reset_now) {
      M.state = kNotInit;
      M.n_kf = M.n_mp = M.n_ml = 0;
      M.has_velocity = 0;
      M.n_local_kf = 0;
      M.ref_kf = -1;
    }
    S.map_out[1] = M.n_kf;
    S.map_out[2] = M.n_mp;
    S.map_out[3] = M.n_ml;
    S.map_out[5] = S.trk;
    S.map_out[6] = reset_now ? 0 : M.ref_kf;   // the oracle's record of a reset step: 0
    S.map_out[7] = M.state;
    for (int k = 0; k < 16; k++) S.Tlast[k] = S.Tcw[k];
    M.last_ref_kf = M.ref_kf;
    M.last_frame_id = fid;
  }
}

// LocalMapping::ProcessNewKeyFrame's per-point work (LocalMapping.cc:186-240,
// P23) for the keyframe k_map_finish inserted, and the construction of its new
// map points (MapPoint(x3D, pKF, pMap) + AddObservation +
// ComputeDistinctiveDescriptors + UpdateNormalAndDepth, Tracking.cc:1592-1655):
// one thread per keypoint of the keyframe, grid (keypoints / 64, streams), so
// the points' dependent gathers overlap across many waves.
__global__ void __launch_bounds__(64) k_map_kf_points(TrackConsts c, MapArgs a) {
  trk_priority();
  __shared__ uint16_t dscr[64][kMapMaxKF];
  const int s = blockIdx.y;
  const MapState& M = a.ms[s];
  const int kf = M.new_kf;
  if (kf < 0) return;
  const Pools P(a, s);
  const long long kb = P.kfb(kf);
  const int i = blockIdx.x * 64 + threadIdx.x;
  if (i >= a.kf_N[kb]) return;
  const long long d = kb * a.kp_pitch + i;
  const int p = a.kf_mp[d];
  if (p < 0) return;
  const long long g = P.mb + p;
  if (p >= M.kf_mp_base) {
    // a new point from the keyframe's depth
    float T[16];
    for (int q = 0; q < 16; q++) T[q] = a.kf_T[kb * 16 + q];
    const float Ow[3] = {a.kf_Ow[kb * 4], a.kf_Ow[kb * 4 + 1], a.kf_Ow[kb * 4 + 2]};
    const KeyPointD kp = a.kf_kp[d];
    float w[3];
    unproject_f(c, T, Ow, kp.x, kp.y, a.depth[P.cb + i], w);
    a.mp_pos[g] = make_float4(w[0], w[1], w[2], 0.f);
    a.mp_obs[g * a.kfc] = ((uint32_t)kf << 16) | (uint32_t)i;
    a.mp_nob[g] = 1;
    a.mp_nobs[g] = a.kf_ur[d] >= 0 ? 2 : 1;
    a.mp_seen[g] = -1;
    a.mp_tref[g] = -1;
    copy32(a.mp_desc + g * 32, a.kf_desc + d * 32);   // one observation: its descriptor
    update_normal_depth(c, a, P, p);
    return;
  }
  // a tracked point: AddObservation, UpdateNormalAndDepth, ComputeDistinctiveDescriptors
  const int nob = a.mp_nob[g];
  if (nob > 0 && (int)(a.mp_obs[g * a.kfc + nob - 1] >> 16) == kf) return;   // IsInKeyFrame
  a.mp_obs[g * a.kfc + nob] = ((uint32_t)kf << 16) | (uint32_t)i;
  a.mp_nob[g] = nob + 1;
  a.mp_nobs[g] += a.kf_ur[d] >= 0 ? 2 : 1;
  update_normal_depth(c, a, P, p);
  compute_distinctive(a, P, p, dscr[threadIdx.x]);
}

// KeyFrame::UpdateConnections (KeyFrame.cc:363-452) of the inserted keyframe:
// covisibility counts over its points' observations, the connected keyframes'
// ordered lists (thread k updates keyframe k), its own list and parent.
// Dynamic LDS: 5 x kfc x kfc bytes of per-thread scratch.
__global__ void __launch_bounds__(kT) k_map_connect(MapArgs a) {
  trk_priority();
  extern __shared__ int cscr[];
  __shared__ int cnt[kMapMaxKF];
  __shared__ int pw[kMapMaxKF], pk[kMapMaxKF];
  __shared__ int s_i[2];
  const int s = blockIdx.x, t = threadIdx.x;
  const MapState& M = a.ms[s];
  const int kf = M.new_kf;
  if (kf <= 0) return;   // the initial keyframe has no other keyframe to connect to
  const Pools P(a, s);
  const long long kb = P.kfb(kf);
  const int N = a.kf_N[kb];
  if (t < kMapMaxKF) cnt[t] = 0;
  __syncthreads();
  for (int i = t; i < N; i += kT) {
    const int p = a.kf_mp[kb * a.kp_pitch + i];
    if (p < 0) continue;
    const long long g = P.mb + p;
    const int nob = a.mp_nob[g];
    for (int k = 0; k < nob; k++) {
      const int o = a.mp_obs[g * a.kfc + k] >> 16;
      if (o != kf) atomicAdd(&cnt[o], 1);
    }
  }
  __syncthreads();
  // the connection decision (thread 0), then every connected keyframe k
  // updates its own list on thread k (independent rows)
  if (t == 0) {
    int nmax = 0, kmax = -1, np = 0;
    for (int k = 0; k < kf; k++) {
      if (cnt[k] <= 0) continue;
      if (cnt[k] > nmax) {
        nmax = cnt[k];
        kmax = k;
      }
      np += cnt[k] >= 15;
    }
    s_i[0] = kmax;   // -1: no covisible keyframe (no connection at all)
    s_i[1] = np;
  }
  __syncthreads();
  const int kmax = s_i[0], npass = s_i[1];
  if (kmax < 0) return;
  if (t < kf && (cnt[t] >= 15 || (npass == 0 && t == kmax))) {
    int* wrow = cscr + t * a.kfc;
    uint8_t* ks = reinterpret_cast<uint8_t*>(cscr + a.kfc * a.kfc) + t * a.kfc;
    add_connection(a, P, t, kf, cnt[t], wrow, ks);
  }
  if (t == 0) {
    int np = 0;
    for (int k = 0; k < kf; k++)
      if (cnt[k] >= 15) {
        pw[np] = cnt[k];
        pk[np++] = k;
      }
    if (np == 0) {
      pw[np] = cnt[kmax];
      pk[np++] = kmax;
    }
    // sort (weight, id) ascending, the ordered list is its reverse
    for (int x = 1; x < np; x++) {
      const int vw = pw[x], vk = pk[x];
      int y = x - 1;
      while (y >= 0 && (pw[y] > vw || (pw[y] == vw && pk[y] > vk))) {
        pw[y + 1] = pw[y];
        pk[y + 1] = pk[y];
        y--;
      }
      pw[y + 1] = vw;
      pk[y + 1] = vk;
    }
    int* wk = a.kf_w + kb * a.kfc;
    for (int k = 0; k < kf; k++) wk[k] = cnt[k];
    uint8_t* ord = a.kf_ord + kb * a.kfc;
    for (int x = 0; x < np; x++) ord[x] = (uint8_t)pk[np - 1 - x];
    a.kf_nord[kb] = np;
    if (a.kf_first[kb]) {
      const int par = ord[0];
      a.kf_parent[kb] = par;
      a.kf_child[P.kfb(par)] |= 1ull << kf;
      a.kf_first[kb] = 0;
    }
  }
}

// ---------------------------------------------------------------------------
void launch_map_reset(const MapArgs& a, const float* T0, int nstreams, hipStream_t s) {
  hipLaunchKernelGGL(k_map_reset, dim3((nstreams + 255) / 256), dim3(256), 0, s, a, T0, nstreams);
}
// mVelocity = cv::Mat() for the masked streams (what Tracking holds after its
// initialisation or a relocalisation): their next frame runs
// TrackReferenceKeyFrame (Tracking.cc:324-338). ms: map trackers, else st.
__global__ void k_clear_velocity(MapState* ms, StreamState* st, const uint8_t* mask, int n) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n || !mask[s]) return;
  if (ms) ms[s].has_velocity = 0;
  else st[s].has_velocity = 0;
}
void launch_clear_velocity(MapState* ms, StreamState* st, const uint8_t* mask, int nstreams,
                           hipStream_t s) {
  hipLaunchKernelGGL(k_clear_velocity, dim3((nstreams + 255) / 256), dim3(256), 0, s, ms, st, mask,
                     nstreams);
}
void launch_map_begin(const TrackConsts& c, const MapArgs& a, int nstreams, hipStream_t s) {
  hipLaunchKernelGGL(k_map_begin, dim3(nstreams), dim3(kT), 0, s, c, a);
}
void launch_map_resolve_motion(const MapArgs& a, int nstreams, hipStream_t s) {
  hipLaunchKernelGGL(k_map_resolve_motion, dim3(nstreams), dim3(kT), 0, s, a);
}
void launch_map_trk_merge(const MapArgs& a, int nstreams, hipStream_t s) {
  hipLaunchKernelGGL(k_map_trk_merge, dim3(nstreams), dim3(kT), 0, s, a);
}
void launch_map_resolve_trk(const MapArgs& a, int nstreams, hipStream_t s) {
  hipLaunchKernelGGL(k_map_resolve_trk, dim3(nstreams), dim3(kT), 0, s, a);
}
void launch_map_local(const MapArgs& a, int nstreams, hipStream_t s) {
  hipLaunchKernelGGL(k_map_local, dim3(nstreams), dim3(kT), 0, s, a);
}
void launch_map_assemble(const MapArgs& a, int nstreams, hipStream_t s) {
  hipLaunchKernelGGL(k_map_assemble, dim3(nstreams), dim3(kT), 0, s, a);
}
void launch_map_finish(const TrackConsts& c, const MapArgs& a, int nstreams, hipStream_t s) {
  hipLaunchKernelGGL(k_map_finish, dim3(nstreams), dim3(kT), 0, s, c, a);
  hipLaunchKernelGGL(k_map_kf_points, dim3((a.kp_pitch + 63) / 64, nstreams), dim3(64), 0, s, c, a);
  hipLaunchKernelGGL(k_map_connect, dim3(nstreams), dim3(kT), (size_t)5 * a.kfc * a.kfc, s, a);
}

}  // namespace orbpl
