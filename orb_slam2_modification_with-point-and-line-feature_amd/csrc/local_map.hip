// Tracking::TrackLocalMap on gfx950 for the batched tracker
// (ORBPL_TRACK_LOCAL_MAP; restated in oracle/line_track_oracle.cpp
// track_local_map / push_local_kf, defined local map P18):
//   k_lm_gather   : TrackWithMotionModel's outlier discard counts and success
//                   (Tracking.cc:1273-1329), the mnLastFrameSeen marks
//                   (every map point / line the motion model matched) and the
//                   ordered compaction of the local map (the last kLocalKFs
//                   keyframes, most recent first, index order) into per-stream
//                   lists for IsInFrustum / SearchByProjection
//   k_lm_assemble : every match of the frame (motion-model inliers + local
//                   matches; lines after the local matcher's optional wipe)
//                   as per-keypoint / per-line world positions for the second
//                   PoseOptimizationWithLines
//   k_lm_count    : mnMatchesInliers / mnLineMatchesInliers and the decision
//                   (Tracking.cc:1396-1419)
//   k_lm_push     : the frame joins the local map as the newest keyframe with
//                   MapPoint::UpdateNormalAndDepth's normal and distances
// One 256-thread block per stream; the matching itself reuses the batched
// k_in_frustum / k_match_local / k_line_in_frustum / k_line_match_list.
#include <hip/hip_runtime.h>

#include "line_common.h"
#include "lsd_kernels.h"
#include "track_common.h"
#include "track_kernels.h"

namespace orbpl {

namespace {

// ordered block compaction: position of this thread's flagged element
// (base + exclusive prefix over the block), the block total in *total
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

}  // namespace

__global__ void __launch_bounds__(256) k_lm_gather(LocalMapArgs a) {
  trk_priority();
  __shared__ uint32_t seen[kMatchMaxKp / 32];
  __shared__ uint32_t seen_l[(kLineKeep + 31) / 32];
  __shared__ int wsum[4];
  const int s = blockIdx.x, t = threadIdx.x;
  StreamState& S = a.st[s];
  const int K = a.kp_pitch;
  const long long cb = (long long)s * K, lb = (long long)s * kLineKeep;
  const int n = a.n[s], nl = a.lines ? a.nl[s] : 0;
  for (int w = t; w < kMatchMaxKp / 32; w += 256) seen[w] = 0;
  if (t < (kLineKeep + 31) / 32) seen_l[t] = 0;
  __syncthreads();
  // ---- TrackWithMotionModel's discard counts and success (as k_finish) ----
  int nmap = 0, lnmap = 0;
  for (int i = t; i < n; i += 256) {
    const int j = a.match[cb + i];
    const bool inl = j >= 0 && !a.outlier[cb + i];
    a.cur_nobs[cb + i] = inl ? 1 : 0;
    if (j >= 0) {
      atomicOr(&seen[j >> 5], 1u << (j & 31));   // mnLastFrameSeen (inliers and outliers)
      nmap += inl;
    }
  }
  for (int i = t; i < nl; i += 256) {
    const int j = a.lmatch[lb + i];
    const bool inl = j >= 0 && !a.loutlier[lb + i];
    a.cur_nobs_l[lb + i] = inl ? 1 : 0;
    if (j >= 0) {
      atomicOr(&seen_l[j >> 5], 1u << (j & 31));
      lnmap += inl ? 1 : -1;    // outliers decrement (Tracking.cc:1306)
    }
  }
  nmap = block_sum(nmap, wsum);
  lnmap = block_sum(lnmap, wsum);
  const bool tracked = S.nmatches >= 20 && (!a.lines || S.nlmatches >= 15);
  const bool motion_ok =
      S.has_last && (S.trk ? (S.trk_go && nmap >= 10 && (!a.lines || lnmap >= 10))
                           : (tracked && (a.lines ? (nmap >= 10 || lnmap >= 15) : nmap >= 10)));
  if (t == 0) {
    S.lm_active = motion_ok ? 1 : 0;
    S.lm_nlocal = S.lm_nllocal = S.lm_wiped = S.lm_ninl = S.lm_inl = S.lm_linl = 0;
    S.lm_ok = 0;
  }
  int np = 0, nlp = 0;
  if (motion_ok) {
    // ---- local map points: keyframes most recent first, index order ----
    for (int k = 0; k < a.nslots; k++) {
      const int slot = (a.head - k + a.K) % a.K;
      const long long rb = ((long long)s * a.K + slot) * K;
      const int cnt = a.r_n[s * a.K + slot];
      for (int c0 = 0; c0 < cnt; c0 += 256) {
        const int i = c0 + t;
        const bool f = i < cnt && a.r_has[rb + i] && !(k == 0 && ((seen[i >> 5] >> (i & 31)) & 1u));
        int tot = 0;
        const int pos = np + block_prefix(f, wsum, &tot);
        if (f) {
          const long long d = (long long)s * a.lp + pos, src = rb + i;
          for (int q = 0; q < 3; q++) {
            a.l_xyz[d * 3 + q] = a.r_xyz[src * 3 + q];
            a.l_nrm[d * 3 + q] = a.r_nrm[src * 3 + q];
          }
          a.l_dmin[d] = a.r_dmin[src];
          a.l_dmax[d] = a.r_dmax[src];
          const uint4* sd = reinterpret_cast<const uint4*>(a.r_desc + src * 32);
          uint4* dd = reinterpret_cast<uint4*>(a.l_desc + d * 32);
          dd[0] = sd[0];
          dd[1] = sd[1];
        }
        np += tot;
      }
    }
    // ---- local map lines ----
    if (a.lines) {
      for (int k = 0; k < a.nslots; k++) {
        const int slot = (a.head - k + a.K) % a.K;
        const long long rb = ((long long)s * a.K + slot) * kLineKeep;
        const int cnt = a.rl_n[s * a.K + slot];
        for (int c0 = 0; c0 < cnt; c0 += 256) {
          const int i = c0 + t;
          const bool f =
              i < cnt && a.rl_has[rb + i] && !(k == 0 && ((seen_l[i >> 5] >> (i & 31)) & 1u));
          int tot = 0;
          const int pos = nlp + block_prefix(f, wsum, &tot);
          if (f) {
            const long long d = (long long)s * a.llp + pos, src = rb + i;
            for (int q = 0; q < 6; q++) a.ll_xyz[d * 6 + q] = a.rl_xyz[src * 6 + q];
            const uint4* sd = reinterpret_cast<const uint4*>(a.rl_desc + src * 32);
            uint4* dd = reinterpret_cast<uint4*>(a.ll_desc + d * 32);
            dd[0] = sd[0];
            dd[1] = sd[1];
          }
          nlp += tot;
        }
      }
    }
  }
  if (t == 0) {
    a.l_n[s] = np;
    if (a.lines) a.ll_n[s] = nlp;
  }
}

__global__ void __launch_bounds__(256) k_lm_assemble(LocalMapArgs a) {
  trk_priority();
  const int s = blockIdx.x, t = threadIdx.x;
  const StreamState& S = a.st[s];
  const int K = a.kp_pitch;
  const long long cb = (long long)s * K, lb = (long long)s * kLineKeep;
  const int n = a.n[s], nl = a.lines ? a.nl[s] : 0;
  const bool act = S.lm_active != 0;
  for (int i = t; i < n; i += 256) {
    const int j = a.match[cb + i];
    const int m = act ? a.lm_match[cb + i] : -1;
    const float* src = nullptr;
    if (act && j >= 0 && !a.outlier[cb + i]) src = a.last_xyz + (cb + j) * 3;
    else if (m >= 0) src = a.l_xyz + ((long long)s * a.lp + m) * 3;
    a.match2[cb + i] = src ? i : -1;
    if (src)
      for (int q = 0; q < 3; q++) a.xyz2[(cb + i) * 3 + q] = src[q];
    a.outlier2[cb + i] = 0;
  }
  const bool wiped = S.lm_wiped != 0;
  for (int i = t; i < nl; i += 256) {
    const int j = a.lmatch[lb + i];
    const int m = act ? a.llm_match[lb + i] : -1;
    const float* src = nullptr;
    if (act && !wiped && j >= 0 && !a.loutlier[lb + i]) src = a.last_lxyz + (lb + j) * 6;
    else if (m >= 0) src = a.ll_xyz + ((long long)s * a.llp + m) * 6;
    a.lmatch2[lb + i] = src ? i : -1;
    if (src)
      for (int q = 0; q < 6; q++) a.lxyz2[(lb + i) * 6 + q] = src[q];
    a.loutlier2[lb + i] = 0;
  }
}

__global__ void __launch_bounds__(256) k_lm_count(LocalMapArgs a, int frame_id) {
  trk_priority();
  __shared__ int wsum[4];
  const int s = blockIdx.x, t = threadIdx.x;
  StreamState& S = a.st[s];
  const int K = a.kp_pitch;
  const long long cb = (long long)s * K, lb = (long long)s * kLineKeep;
  const int n = a.n[s], nl = a.lines ? a.nl[s] : 0;
  int inl = 0, linl = 0;
  for (int i = t; i < n; i += 256) inl += a.match2[cb + i] >= 0 && !a.outlier2[cb + i];
  for (int i = t; i < nl; i += 256) linl += a.lmatch2[lb + i] >= 0 && !a.loutlier2[lb + i];
  inl = block_sum(inl, wsum);
  linl = block_sum(linl, wsum);
  if (t == 0 && S.lm_active) {
    S.lm_inl = inl;
    S.lm_linl = linl;
    // mnLastRelocFrameId = 0, mMaxFrames = 30 (Tracking.cc:1410-1418)
    S.lm_ok = !(frame_id < 30 && inl + linl < 60) && !(inl < 30 && linl < 20);
  }
}

__global__ void __launch_bounds__(256) k_lm_push(TrackConsts c, LocalMapArgs a) {
  trk_priority();
  __shared__ float sT[16];
  const int s = blockIdx.x, t = threadIdx.x;
  const StreamState& S = a.st[s];
  const int K = a.kp_pitch;
  const long long cb = (long long)s * K, lb = (long long)s * kLineKeep;
  const int n = a.n[s], nl = a.lines ? a.nl[s] : 0;
  if (t < 16) sT[t] = S.Tlast[t];   // the frame's final pose (k_finish)
  __syncthreads();
  float Ow[3];
  gemm_neg_Rt_t(sT, Ow);
  const long long rb = ((long long)s * a.K + a.push_slot) * K;
  for (int i = t; i < n; i += 256) {
    const uint8_t h = a.has_mp[cb + i];
    a.r_has[rb + i] = h;
    const uint4* sd = reinterpret_cast<const uint4*>(a.desc + (cb + i) * 32);
    uint4* dd = reinterpret_cast<uint4*>(a.r_desc + (rb + i) * 32);
    dd[0] = sd[0];
    dd[1] = sd[1];
    if (!h) continue;
    const float X[3] = {a.mp_xyz[(cb + i) * 3], a.mp_xyz[(cb + i) * 3 + 1], a.mp_xyz[(cb + i) * 3 + 2]};
    const float PO[3] = {X[0] - Ow[0], X[1] - Ow[1], X[2] - Ow[2]};
    const double nd = sqrt((double)PO[0] * PO[0] + (double)PO[1] * PO[1] + (double)PO[2] * PO[2]);
    const float inv = (float)(1.0 / nd);
    const float dist = (float)nd;
    const float maxd = dist * c.scale[a.kps_un[cb + i].octave];
    const float mind = maxd / c.scale[c.nlevels - 1];
    for (int q = 0; q < 3; q++) {
      a.r_xyz[(rb + i) * 3 + q] = X[q];
      a.r_nrm[(rb + i) * 3 + q] = PO[q] * inv;
    }
    a.r_dmax[rb + i] = maxd;   // mfMaxDistance / mfMinDistance: k_in_frustum applies
    a.r_dmin[rb + i] = mind;   // the 1.2f / 0.8f of GetMax/MinDistanceInvariance
  }
  if (t == 0) a.r_n[s * a.K + a.push_slot] = n;
  if (a.lines) {
    const long long rlb = ((long long)s * a.K + a.push_slot) * kLineKeep;
    for (int i = t; i < nl; i += 256) {
      a.rl_has[rlb + i] = a.has_ml[lb + i];
      for (int q = 0; q < 6; q++) a.rl_xyz[(rlb + i) * 6 + q] = a.ml_xyz[(lb + i) * 6 + q];
      const uint4* sd = reinterpret_cast<const uint4*>(a.ldesc + (lb + i) * 32);
      uint4* dd = reinterpret_cast<uint4*>(a.rl_desc + (rlb + i) * 32);
      dd[0] = sd[0];
      dd[1] = sd[1];
    }
    if (t == 0) a.rl_n[s * a.K + a.push_slot] = nl;
  }
}

// ---------------------------------------------------------------------------
// Tracking::TrackReferenceKeyFrame (Tracking.cc:942-1032) for the streams
// that need it (ORBPL_TRACK_REFKF, P22; restated in oracle/line_track_oracle.cpp
// lvo_step): the first frame without a velocity and every frame whose motion
// model failed, against the last frame as the reference keyframe.
//   k_trk_prep  : TrackWithMotionModel's outcome (as k_lm_gather), the
//                 decision, SetPose(mLastFrame.mTcw), fresh point matches /
//                 outlier flags, the frame's line assignments kept for the
//                 keyframe line search (the motion model's, outliers removed)
//   k_trk_bow   : ORBmatcher(0.7, true).SearchByBoW(pKF, F) per stream (the
//                 SearchByBoW kernel's body on the stream's FeatureVectors)
//   k_trk_merge : the keyframe line search's matches over the kept
//                 assignments (all cleared when its relaxed retry ran), the
//                 15 / 10 match gates of the pose
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_trk_prep(TrkArgs a) {
  trk_priority();
  __shared__ int wsum[4];
  const int s = blockIdx.x, t = threadIdx.x;
  StreamState& S = a.st[s];
  const int K = a.kp_pitch;
  const long long cb = (long long)s * K, lb = (long long)s * kLineKeep;
  const int n = a.n[s], nl = a.lines ? a.nl[s] : 0;
  const bool tracked = S.nmatches >= 20 && (!a.lines || S.nlmatches >= 15);
  int nmap = 0, lnmap = 0;
  for (int i = t; i < n; i += 256) nmap += a.match[cb + i] >= 0 && !a.outlier[cb + i];
  for (int j = t; j < nl; j += 256)
    if (a.lmatch[lb + j] >= 0) lnmap += a.loutlier[lb + j] ? -1 : 1;
  nmap = block_sum(nmap, wsum);
  lnmap = block_sum(lnmap, wsum);
  const bool mm_ok = S.has_velocity && tracked &&
                     (a.lines ? (nmap >= 10 || lnmap >= 15) : nmap >= 10);
  const bool trk = S.has_last && !mm_ok;
  __syncthreads();
  if (t == 0) {
    S.trk = trk ? 1 : 0;
    S.trk_go = 0;
    if (trk) {
      for (int k = 0; k < 16; k++) S.Tcw[k] = S.Tlast[k];
      S.ninliers = 0;
      S.nmatches = 0;
    }
    a.nml[s] = trk && a.lines ? a.last_nl[s] : 0;
  }
  if (!trk) return;
  for (int i = t; i < n; i += 256) {
    a.match[cb + i] = -1;
    a.outlier[cb + i] = 0;
  }
  for (int j = t; j < nl; j += 256) {
    const int m = a.lmatch[lb + j];
    // the motion model's assignments after its outlier discard (none when it
    // did not run: no velocity)
    const int keep = (S.has_velocity && m >= 0 && !(tracked && a.loutlier[lb + j])) ? m : -1;
    a.lcur[lb + j] = keep;
    a.cur_nobs_l[lb + j] = keep >= 0 ? 1 : 0;
    a.loutlier[lb + j] = 0;
  }
}

__global__ void __launch_bounds__(256) k_trk_merge(TrkArgs a) {
  trk_priority();
  const int s = blockIdx.x, t = threadIdx.x;
  StreamState& S = a.st[s];
  if (!S.trk) return;
  const long long lb = (long long)s * kLineKeep;
  const int nl = a.lines ? a.nl[s] : 0;
  const bool wiped = a.lines && S.trk_wiped;
  for (int j = t; j < nl; j += 256) {
    const int c = a.lcur[lb + j];
    a.lmatch[lb + j] = (!wiped && c >= 0) ? c : a.tlm[lb + j];
  }
  if (t == 0) {
    if (a.lines) S.nlmatches = S.trk_nlm;
    S.trk_go = S.nmatches >= 15 && (!a.lines || S.trk_nlm >= 10);
  }
}

void launch_trk_prep(const TrkArgs& a, int nstreams, hipStream_t s) {
  hipLaunchKernelGGL(k_trk_prep, dim3(nstreams), dim3(256), 0, s, a);
}
void launch_trk_merge(const TrkArgs& a, int nstreams, hipStream_t s) {
  hipLaunchKernelGGL(k_trk_merge, dim3(nstreams), dim3(256), 0, s, a);
}

void launch_lm_gather(const LocalMapArgs& a, int nstreams, hipStream_t s) {
  hipLaunchKernelGGL(k_lm_gather, dim3(nstreams), dim3(256), 0, s, a);
}
void launch_lm_assemble(const LocalMapArgs& a, int nstreams, hipStream_t s) {
  hipLaunchKernelGGL(k_lm_assemble, dim3(nstreams), dim3(256), 0, s, a);
}
void launch_lm_count(const LocalMapArgs& a, int frame_id, int nstreams, hipStream_t s) {
  hipLaunchKernelGGL(k_lm_count, dim3(nstreams), dim3(256), 0, s, a, frame_id);
}
void launch_lm_push(const TrackConsts& c, const LocalMapArgs& a, int nstreams, hipStream_t s) {
  hipLaunchKernelGGL(k_lm_push, dim3(nstreams), dim3(256), 0, s, c, a);
}

}  // namespace orbpl
