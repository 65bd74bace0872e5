// Launchers of the tracking kernels (track_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "track_common.h"

namespace orbpl {

constexpr int kMatchMaxKp = 2048;    // keypoints per frame the matcher handles
constexpr int kPoseMaxEdges = 2304;  // point + line edges per frame

struct PoseEdge;

struct MatchLaunch {
  const KeyPointD* cur_kps_un;
  const uint8_t* cur_desc;
  const float* cur_uright;
  const int* cur_gcell;
  const int* cur_n;
  const KeyPointD* last_kps_un;
  const uint8_t* last_has_mp;
  const uint8_t* last_outlier;
  const float* last_xyz;
  const uint8_t* last_desc;
  const int* last_nobs;
  const int* last_n;
  int kp_pitch;
  const float* Tcw;
  const float* Tlw;
  int pose_stride;
  int* match;
  int* nmatches;
  int nm_stride;
  float th;
  int mono;
  int check_ori;
  int retry;
  const StreamState* active;
};

struct PoseLaunch {
  const KeyPointD* kps_un;
  const float* uright;
  const int* match;
  const uint8_t* has_mp;
  const float* mp_xyz;
  const int* n;
  int kp_pitch;
  const float* kl_obs;
  const int* kl_octave;
  const uint8_t* has_ml;
  const float* ml_xyz;
  int nl;
  float* Tcw;
  int pose_stride;
  uint8_t* outlier;
  uint8_t* line_outlier;
  int* ninliers;
  int nm_stride;
  const StreamState* active;
  PoseEdge* edges;
};

size_t match_smem_bytes();
size_t pose_smem_bytes();
size_t pose_edge_bytes();

void launch_frame_prepare(const TrackConsts& c, const KeyPointD* kps, const int* n, int kp_pitch,
                          const float* depth, long long depth_pitch, KeyPointD* kps_un,
                          float* depth_out, float* uright, int* gcell, int batch, hipStream_t s);
void launch_predict(StreamState* st, int nstreams, hipStream_t s);
void launch_match_last(const TrackConsts& c, const MatchLaunch& m, int nstreams, hipStream_t s);
void launch_pose(const TrackConsts& c, const PoseLaunch& p, int nstreams, hipStream_t s);
void launch_finish(const TrackConsts& c, StreamState* st, const int* n, int kp_pitch,
                   const KeyPointD* kps_un, const float* depth, int* match, uint8_t* outlier,
                   uint8_t* has_mp, float* mp_xyz, int* nobs, int nstreams, hipStream_t s);

}  // namespace orbpl
