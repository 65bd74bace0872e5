// Shared host/device definitions for the per-frame tracking kernels
// (frame glue, ORBmatcher::SearchByProjection, pose-only LM, map update).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace orbpl {

// Issue priority of the tracking-stream kernels' waves. In the pipelined step
// they share SIMDs with the next frame's extraction waves (k_fast_cells is
// VALU-bound), and the instruction arbiter picks by priority, then age: a
// tracking wave that arrives while extraction waves hold the SIMD is the
// youngest and gets the leftover issue slots, so its serial chain (k_pose's
// LM iterations, the matchers' per-keypoint loops) stretches to the length
// of the extraction kernel beside it. s_setprio raises it above them (0-3).
#ifndef ORBPL_TRK_PRIO
#define ORBPL_TRK_PRIO 3
#endif
__device__ __forceinline__ void trk_priority() {
  if constexpr (ORBPL_TRK_PRIO > 0) __builtin_amdgcn_s_setprio(ORBPL_TRK_PRIO);
}

constexpr int kGridCols = 64;   // FRAME_GRID_COLS (Frame.h:41)
constexpr int kGridRows = 48;   // FRAME_GRID_ROWS (Frame.h:40)
constexpr int kMaxLevelsT = 16;

// Camera + Frame constants fixed at the first frame (Frame.cc:180-203).
struct TrackConsts {
  float fx, fy, cx, cy;
  float k1, k2, p1, p2, k3;
  float bf, mb, th_depth;
  float invfx, invfy;
  float minX, maxX, minY, maxY;   // ComputeImageBounds
  float gridInvW, gridInvH;       // mfGridElementWidthInv / HeightInv
  int width, height;
  int nlevels;
  float scale[kMaxLevelsT];       // mvScaleFactors
  float inv_sigma2[kMaxLevelsT];  // mvInvLevelSigma2
};

// Device keypoint record (cv::KeyPoint layout).
struct KeyPointD {
  float x, y, size, angle, response;
  int octave, class_id;
};

// cv::undistortPoints for one point (OpenCV 3.4 cvUndistortPointsInternal,
// TermCriteria(COUNT, 5), R = I, P = K). Plain double +,-,*,/ only.
__host__ __device__ inline void undistort_point_d(const TrackConsts& c, float px, float py,
                                                  float* ox, float* oy) {
  const double fx = c.fx, fy = c.fy, cx = c.cx, cy = c.cy;
  const double k0 = c.k1, k1 = c.k2, k2 = c.p1, k3 = c.p2, k4 = c.k3;
  const double k5 = 0, k6 = 0, k7 = 0, k8 = 0, k9 = 0, k10 = 0, k11 = 0;
  const double ifx = 1. / fx, ify = 1. / fy;
  double x = px, y = py;
  x = (x - cx) * ifx;
  y = (y - cy) * ify;
  const double x0 = x, y0 = y;
  for (int j = 0; j < 5; j++) {
    double r2 = x * x + y * y;
    double icdist = (1 + ((k7 * r2 + k6) * r2 + k5) * r2) / (1 + ((k4 * r2 + k1) * r2 + k0) * r2);
    double deltaX = 2 * k2 * x * y + k3 * (r2 + 2 * x * x) + k8 * r2 + k9 * r2 * r2;
    double deltaY = k2 * (r2 + 2 * y * y) + 2 * k3 * x * y + k10 * r2 + k11 * r2 * r2;
    x = (x0 - deltaX) * icdist;
    y = (y0 - deltaY) * icdist;
  }
  double xx = fx * x + 0.0 * y + cx;
  double yy = 0.0 * x + fy * y + cy;
  double ww = 1. / (0.0 * x + 0.0 * y + 1.0);
  *ox = (float)(xx * ww);
  *oy = (float)(yy * ww);
}

// Pinned P6: cv::Mat float (3x3)*(3x1) [+ c] = double accumulation of the
// exact float products, one rounding to float. T is a row-major 4x4 pose.
__host__ __device__ inline void gemm_R_x_plus_t(const float* T, const float* x, float* out) {
  for (int r = 0; r < 3; r++) {
    double s = (double)T[r * 4] * x[0];
    s += (double)T[r * 4 + 1] * x[1];
    s += (double)T[r * 4 + 2] * x[2];
    out[r] = (float)(s + (double)T[r * 4 + 3]);
  }
}

// -R^T t (Frame::GetCameraCenter / mOw, twc in SearchByProjection)
__host__ __device__ inline void gemm_neg_Rt_t(const float* T, float* out) {
  for (int r = 0; r < 3; r++) {
    double s = (double)T[0 * 4 + r] * T[3];
    s += (double)T[1 * 4 + r] * T[7];
    s += (double)T[2 * 4 + r] * T[11];
    out[r] = (float)(s * -1.0);
  }
}

// R^T x + c  (mRwc * x3Dc + mOw in Frame::UnprojectStereo)
__host__ __device__ inline void gemm_Rt_x_plus_c(const float* T, const float* x, const float* c,
                                                 float* out) {
  for (int r = 0; r < 3; r++) {
    double s = (double)T[0 * 4 + r] * x[0];
    s += (double)T[1 * 4 + r] * x[1];
    s += (double)T[2 * 4 + r] * x[2];
    out[r] = (float)(s + (double)c[r]);
  }
}

// 4x4 float gemm A*B (double accumulation, one rounding)
__host__ __device__ inline void gemm44(const float* A, const float* B, float* C) {
  for (int r = 0; r < 4; r++)
    for (int c = 0; c < 4; c++) {
      double s = (double)A[r * 4] * B[c];
      s += (double)A[r * 4 + 1] * B[4 + c];
      s += (double)A[r * 4 + 2] * B[8 + c];
      s += (double)A[r * 4 + 3] * B[12 + c];
      C[r * 4 + c] = (float)s;
    }
}

// Inverse of a rigid pose as Tracking builds LastTwc (Tracking.cc:~480):
// rotation transposed, translation = camera centre -R^T t.
__host__ __device__ inline void pose_inverse(const float* T, float* Ti) {
  float ow[3];
  gemm_neg_Rt_t(T, ow);
  for (int r = 0; r < 3; r++) {
    for (int c = 0; c < 3; c++) Ti[r * 4 + c] = T[c * 4 + r];
    Ti[r * 4 + 3] = ow[r];
  }
  Ti[12] = 0; Ti[13] = 0; Ti[14] = 0; Ti[15] = 1;
}

// Per-stream scalar state of the tracker (device).
struct StreamState {
  float Tcw[16];       // current frame pose (predicted, then optimised)
  float Tlast[16];     // last frame pose
  float Tlast2[16];    // frame before last (for the constant-velocity model)
  int has_last;        // last frame exists
  int has_velocity;    // mVelocity is set
  int nmatches;        // SearchByProjection result (after retry)
  int ninliers;        // PoseOptimization return value
  int nmatches_map;    // inliers after discarding outliers
  int ok;              // TrackWithMotionModel success
  int nlmatches;       // LineMatcher::SearchByProjection result (lines enabled)
  int nlmatches_map;   // line inliers minus outliers (Tracking.cc:1298-1314)
  // TrackLocalMap (ORBPL_TRACK_LOCAL_MAP)
  int lm_active;       // TrackWithMotionModel succeeded: the local map step runs
  int lm_nlocal;       // SearchLocalPoints matches
  int lm_nllocal;      // SearchLocalLines matches (every passing pair counts)
  int lm_wiped;        // the line matcher's relaxed retry cleared the line assignments
  int lm_ninl;         // second PoseOptimization's return value
  int lm_inl;          // mnMatchesInliers
  int lm_linl;         // mnLineMatchesInliers
  int lm_ok;           // TrackLocalMap's decision
  // TrackReferenceKeyFrame (ORBPL_TRACK_REFKF, P22)
  int trk;             // this step tracks against the reference keyframe
  int trk_go;          // enough BoW / line matches: the pose ran
  int trk_nlm;         // reference-keyframe line matches
  int trk_wiped;       // that line search's relaxed retry cleared the assignments
  // map model (ORBPL_TRACK_MAP, map_kernels.h): keyframe created (1, 2 = the
  // initial one), keyframes, map points, map lines, temporal points,
  // TrackReferenceKeyFrame ran, reference keyframe, tracking state, local
  // keyframes, local map points, local map lines, temporal lines
  int map_out[12];
};

}  // namespace orbpl
