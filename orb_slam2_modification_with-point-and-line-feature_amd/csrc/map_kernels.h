// The reference's map model on the device for the batched tracker
// (ORBPL_TRACK_MAP; restated in oracle/map_oracle.cpp): per stream a keyframe
// table, a map point pool and a map line pool in HBM, and the kernels of
// Tracking::Track that read and write them (map_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "track_common.h"
#include "track_kernels.h"

namespace orbpl {

constexpr int kMapMaxKF = 64;         // keyframes per stream (child sets are 64-bit masks)
constexpr int kMapOut = 12;           // map counters per step (StreamState.map_out)

// Per-stream scalar map state (device).
struct MapState {
  int state;            // 0 not initialised, 1 OK, 2 LOST (Tracking::eTrackingState)
  int n_kf, n_mp, n_ml; // keyframes, map points, map lines in the pools
  int ref_kf;           // mpReferenceKF
  int last_ref_kf;      // mLastFrame.mpReferenceKF
  int last_kf_frame;    // mnLastKeyFrameId
  int last_frame_id;    // mLastFrame.mnId
  int frame_id;         // mCurrentFrame.mnId of this step
  int next_id;          // Frame::nNextId
  int has_velocity;     // !mVelocity.empty()
  int motion;           // this step runs TrackWithMotionModel
  int trk_first;        // this step starts with TrackReferenceKeyFrame
  int state0;           // the state at the start of the step
  int n_tp, n_tl;       // temporal points / lines of UpdateLastFrame
  int n_local_kf;       // mvpLocalKeyFrames (persists across steps)
  int n_local_mp, n_local_ml;
  int err;              // capacity overflow (keyframes / points / lines)
  int new_kf;           // keyframe inserted this step (-1 none): k_map_kf_points / k_map_connect
  int kf_mp_base;       // its first new map point (the pool ids from here on are new)
  int local_kf[kMapMaxKF];
  float V[16];          // mVelocity
  float Tcr[16];        // mlRelativeFramePoses.back()
  float T0[16];         // pose of the initialising frame
};

// Device pointers of the map model and of the frames it reads / writes. Per
// stream s: keyframe arrays at s * kfc (* kp_pitch / kLineKeep / kfc), pools
// at s * mpc / s * mlc, frame arrays at s * kp_pitch / s * kLineKeep.
struct MapArgs {
  MapState* ms;
  StreamState* st;
  int kfc, kp_pitch;
  long long mpc, mlc;
  int lines, refkf, vocab;
  int stereo;              // System::STEREO: TrackLocalMap drops outlier matches (Tracking.cc:1374-1377)
  int max_frames;          // mMaxFrames = Camera.fps (Tracking.cc:81-87; TUM 30, KITTI 10)
  // keyframes
  float* kf_T;            // [kfc][16]
  float* kf_Ow;           // [kfc][4]
  int* kf_N;
  int* kf_NL;
  int* kf_frame;
  int* kf_mp;             // [kfc][K] mvpMapPoints (pool id / -1)
  KeyPointD* kf_kp;       // [kfc][K] mvKeysUn
  float* kf_ur;           // [kfc][K] mvuRight
  uint8_t* kf_desc;       // [kfc][K][32]
  int* kf_node;           // [kfc][K] FeatureVector node
  int* kf_ml;             // [kfc][80] mvpMapLines
  uint8_t* kf_ldesc;      // [kfc][80][32]
  float* kf_ds;           // [kfc][80] mvDepthLineStart
  float* kf_de;           // [kfc][80] mvDepthLineEnd
  int* kf_w;              // [kfc][kfc] mConnectedKeyFrameWeights (0 = none)
  uint8_t* kf_ord;        // [kfc][kfc] mvpOrderedConnectedKeyFrames
  int* kf_nord;
  int* kf_parent;         // -1 = none
  int* kf_first;          // mbFirstConnection
  unsigned long long* kf_child;   // mspChildrens as a bit set
  // map points
  float4* mp_pos;         // xyz, pad
  float4* mp_nrm;         // mNormalVector, pad
  float2* mp_dist;        // mfMinDistance, mfMaxDistance
  uint8_t* mp_desc;       // [32]
  int* mp_nobs;           // nObs
  int* mp_nob;            // observation count
  uint32_t* mp_obs;       // [kfc] kf << 16 | keypoint, keyframe order
  int* mp_seen;           // mnLastFrameSeen
  int* mp_tref;           // mnTrackReferenceForFrame
  // map lines
  float* ml_pos;          // [6]
  uint8_t* ml_desc;
  int* ml_nobs;
  int* ml_seen;
  int* ml_tref;
  // current frame C
  const int* n;
  const KeyPointD* kps_un;
  const float* depth;
  const float* uright;
  const uint8_t* desc;
  const int* feat_node;
  int* match;             // matcher output (index into the last / reference frame)
  uint8_t* outlier;       // mvbOutlier
  int* mpid;              // mvpMapPoints: pool id, -1, or -2 - j (temporal at last-frame slot j)
  const int* nl;
  const orbpl_keyline* kl_un;
  const float* dstart;
  const float* dend;
  const uint8_t* ldesc;
  int* lmatch;
  uint8_t* loutlier;
  int* mlid;
  // the last frame L: its final assignments and the view the matchers read
  const int* l_n;
  const KeyPointD* l_kps_un;
  const float* l_depth;
  const uint8_t* l_desc;
  int* l_mpid;
  uint8_t* l_has_mp;
  float* l_mp_xyz;
  uint8_t* l_mp_desc;
  int* l_nobs;
  const int* l_nl;
  const orbpl_keyline* l_kl_un;
  const float* l_dstart;
  const float* l_dend;
  const uint8_t* l_ldesc;
  int* l_mlid;
  uint8_t* l_has_ml;
  float* l_ml_xyz;
  uint8_t* l_ml_desc;
  // the reference keyframe staged as a frame (TrackReferenceKeyFrame)
  int* r_n;
  KeyPointD* r_kps_un;
  uint8_t* r_desc;
  uint8_t* r_has_mp;
  float* r_mp_xyz;
  int* r_node;
  int* r_mpid;
  int* r_nl;
  uint8_t* r_has_ml;
  float* r_ml_xyz;
  uint8_t* r_ml_desc;
  int* r_mlid;
  // TrackReferenceKeyFrame line search
  int* trk_cur_nobs;      // Observations() of each current line's map line
  int* trk_lm;            // its matches (reference keyframe line index)
  int* trk_nml;           // lines to search per stream (0: not tracked by it)
  int* trk_list;          // the streams that run TrackReferenceKeyFrame this step
  int* trk_count;         // (k_map_resolve_motion appends; k_map_begin clears)
  // pose inputs in current-frame index space
  int* m2;                // i when the keypoint has a map point, else -1
  float* pxyz;            // its position
  int* lm2;
  float* lpxyz;
  // local map lists (capacity lp / llp per stream)
  long long lp, llp;
  float* l_xyz;
  float* l_nrm;
  float* l_dmin;
  float* l_dmax;
  uint8_t* l_ldesc_pts;   // local map point descriptors [32]
  int* l_count;
  int* l_id;
  float* ll_xyz;
  uint8_t* ll_desc;
  int* ll_count;
  int* ll_id;
  int* cur_nobs;          // Observations() of the point at each keypoint
  int* cur_nobs_l;
  const int* lm_match;    // k_match_local output
  const int* llm_match;   // local line matcher output
};

void launch_map_reset(const MapArgs& a, const float* T0, int nstreams, hipStream_t s);
void launch_map_begin(const TrackConsts& c, const MapArgs& a, int nstreams, hipStream_t s);
void launch_clear_velocity(MapState* ms, StreamState* st, const uint8_t* mask, int nstreams,
                           hipStream_t s);
void launch_map_resolve_motion(const MapArgs& a, int nstreams, hipStream_t s);
void launch_map_trk_merge(const MapArgs& a, int nstreams, hipStream_t s);
void launch_map_resolve_trk(const MapArgs& a, int nstreams, hipStream_t s);
void launch_map_local(const MapArgs& a, int nstreams, hipStream_t s);
void launch_map_assemble(const MapArgs& a, int nstreams, hipStream_t s);
void launch_map_finish(const TrackConsts& c, const MapArgs& a, int nstreams, hipStream_t s);

}  // namespace orbpl
