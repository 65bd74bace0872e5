// Launchers of the tracking kernels (track_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "orb_geom.h"
#include "track_common.h"
#include "../../include/orbpl.h"

namespace orbpl {

constexpr int kMatchMaxKp = 2048;    // keypoints per frame the matcher handles
// per-step entries of orbpl_tracker_timings / _line_timings / _lsd_timings /
// _stereo_timings / _kernel_timings (orbpl_tracker_timing_counts reports them)
constexpr int kTimingStages = 11;
constexpr int kLineTimingStages = 3;
constexpr int kLsdTimingStages = 7;
constexpr int kStereoTimingStages = 4;
constexpr int kKernelTimingStages = 4;   // orbpl_tracker_kernel_timings
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
  // tracker-mode lines (per stream, pitch lpitch): current undistorted
  // KeyLines, their matched last-frame line, the last frame's map lines
  const orbpl_keyline* t_kl_un;
  const int* t_lmatch;
  const float* t_ml_xyz;
  const int* t_nl;
  uint8_t* t_loutlier;
  int lpitch;
  int fixed_line_jac;           // ORBPL_POSE_FIXED_LINE_JAC (analytic line Jacobian)
  const int* list = nullptr;    // optional device list of streams to run (list_n of them): a
  const int* list_n = nullptr;  // grid of kListGrid workgroups loops over it
  int gate_lm;                  // 1: run only streams with active[s].lm_active (TrackLocalMap)
                                // 2: only active[s].trk && trk_go (TrackReferenceKeyFrame)
};

// Workgroups of a launch over a device stream list (rare per-stream work such
// as TrackReferenceKeyFrame): small enough to place quickly beside the
// extraction kernels when the list is empty
constexpr int kListGrid = 256;
// k_trk_bow's listed launch: workgroups looping over the listed streams. The
// launch runs every step beside the next batch's extraction, mostly with an
// empty list: 1024 workgroups cost ~0.4 ms of placement per step there
// (rocprof, 1024 streams), 256 keep the empty launch at a few us.
constexpr int kTrkGrid = 256;

// Per-frame line buffers of the tracker (kLineKeep lines per stream).
struct LineTrackArgs {
  const int* nl;                 // lines per stream (current frame)
  const orbpl_keyline* kl;       // KeyLines as extracted (distorted)
  orbpl_keyline* kl_un;          // UndistortKeyLines
  const float* depth;            // depth images
  long long depth_pitch;
  float* dstart;                 // mvDepthLineStart (-1 = none)
  float* dend;                   // mvDepthLineEnd
  float* ur_start;               // optional (host API): start.x - bf / depth, -1 = none
  float* ur_end;
  int* lmatch;                   // matched last-frame line, -1 = none
  uint8_t* loutlier;             // mvbLineOutlier
  const uint8_t* desc;           // current LBD rows
  const int* last_nl;
  const orbpl_keyline* last_kl_un;
  const uint8_t* last_has_ml;
  const uint8_t* last_loutlier;
  const float* last_ml_xyz;      // 6 floats per line: world start, end
  const uint8_t* last_desc;
};

// Stereo line depths (P17): left lines kl (the tracker's kl_un; rectified)
// and right KeyLines kr of the same pair, kLineKeep per stream.
struct StereoLineArgs {
  const int* nl;
  const orbpl_keyline* kl;
  const uint8_t* desc;
  const int* nr;
  const orbpl_keyline* kr;
  const uint8_t* desc_r;
  float* dstart;
  float* dend;
};
void launch_stereo_lines(const TrackConsts& c, const StereoLineArgs& a, int nstreams,
                         hipStream_t s);

// LineMatcher local-map / reference-keyframe overloads (any number of map lines).
struct LineListArgs {
  const float* Tcw;              // 16 floats
  int ncur;
  const orbpl_keyline* cur_kl_un;
  const uint8_t* cur_desc;
  const int* cur_nobs;           // optional: Observations() of the map line already at each line
  int nml;
  const uint8_t* valid;          // mbTrackInView / mvpMapLines[i] != NULL
  const float* ml_xyz6;
  const uint8_t* ml_desc;
  orbpl_keyline* proj_kl;        // scratch, nml entries
  int* proj_src;                 // scratch, nml entries
  int* match;                    // per current line: map line index or -1 (unchanged / wiped)
  int* nmatches;
  int* wiped;                    // 1 when the relaxed retry ran (all assignments cleared first)
  int refkf;                     // batched reference-keyframe overload: no nToMatch gate
  // batched (tracker TrackLocalMap): block s reads ncur_arr[s] / nml_arr[s]
  // and offsets the current-line arrays by s * cur_pitch, the map-line
  // arrays and scratch by s * ml_pitch, Tcw by s * pose_stride, the outputs
  // nmatches / wiped by s * nm_stride. NULL ncur_arr = one frame.
  const int* ncur_arr;
  const int* nml_arr;
  long long cur_pitch;
  long long ml_pitch;
  int pose_stride;
  int nm_stride;
  const int* list = nullptr;     // optional (batched): the streams to run, list_n of them
  const int* list_n = nullptr;
};
void launch_line_match_list(const TrackConsts& c, const LineListArgs& a, hipStream_t s,
                            int nstreams = 1);
// the reference's harness overloads (k_line_pairs, line_track.hip): one frame
struct LinePairArgs {
  const float* Tcw;              // 16 floats
  int mode;                      // 0: LineMatcher.cpp:272-487, 1: :954-1170
  int ncur;
  const orbpl_keyline* cur_kl_un;
  const uint8_t* cur_desc;
  const int* cur_nobs;           // optional
  int nml;
  const uint8_t* valid;
  const orbpl_keyline* base_kl;  // mode 0: the last frame's KeyLines (optional)
  const float* ml_xyz6;
  const uint8_t* ml_desc;
  const int* ml_nobs;            // optional: Observations() of each map line
  orbpl_keyline* proj_kl;        // nml entries
  int* proj_src;
  int* nproj;
  unsigned* okbits;              // ncur x ceil(nml / 32) words of scratch
  int* pairs;                    // (i, j) pairs, pair_cap of them
  int pair_cap;
  int* npairs;
  int* match;
  int* nmatches;
  int* wiped;
};
void launch_line_pairs(const TrackConsts& c, const LinePairArgs& a, hipStream_t s);
void launch_line_bf_knn(int nq, const uint8_t* qdesc, int nt, const uint8_t* tdesc, int* out,
                        int* nm, hipStream_t s);
void launch_line_in_frustum(const float* Tcw, int n, const float* xyz6, uint8_t* in_view,
                            hipStream_t s);
// batched: stream b = blockIdx.y tests n_arr[b] lines at xyz6 + b * pitch * 6
void launch_line_in_frustum_batched(const float* Tcw, int pose_stride, const int* n_arr,
                                    long long pitch, const float* xyz6, uint8_t* in_view,
                                    int nstreams, hipStream_t s);

void launch_line_prepare(const TrackConsts& c, const LineTrackArgs& a, int nstreams,
                         hipStream_t s);
void launch_line_match(const TrackConsts& c, const LineTrackArgs& a, StreamState* st,
                       int nstreams, hipStream_t s);

// Frame::IsInFrustum for a list of map points (match_local.hip).
struct InFrustumArgs {
  int n;
  const float* Tcw;
  const float* xyz;        // n x 3 world positions
  const float* normal;     // n x 3 mean viewing directions
  const float* min_dist;   // mfMinDistance (the kernel applies GetMinDistanceInvariance's 0.8f)
  const float* max_dist;   // mfMaxDistance (the kernel applies GetMaxDistanceInvariance's 1.2f)
  float view_cos_limit;
  uint8_t* in_view;        // mbTrackInView
  float* proj_x;           // mTrackProjX
  float* proj_y;
  float* proj_xr;
  int* level;              // mnTrackScaleLevel
  float* view_cos;         // mTrackViewCos
  // batched (tracker TrackLocalMap): stream b = blockIdx.y reads n_arr[b]
  // points at offset b * pitch of every array and Tcw + b * pose_stride
  const int* n_arr;
  long long pitch;
  int pose_stride;
};

// ORBmatcher::SearchByProjection(Frame&, const vector<MapPoint*>&, th).
struct LocalArgs {
  const KeyPointD* kps_un;
  const uint8_t* desc;
  const float* uright;
  int n;
  const int* cur_nobs;     // Observations() of the map point already at a keypoint (0: none)
  int nmp;
  const uint8_t* in_view;
  const float* proj_x;
  const float* proj_y;
  const float* proj_xr;
  const int* level;
  const float* view_cos;
  const uint8_t* mp_desc;
  const int* mp_nobs;
  float th;
  float nnratio;
  int* match;              // per keypoint: last local map point assigned, -1
  int* nmatches;
  int4* scratch;           // nmp entries
  // batched (tracker TrackLocalMap): block b reads n_arr[b] / nmp_arr[b],
  // offsets the keypoint arrays by b * kp_pitch, the map point arrays and
  // scratch by b * mp_pitch, nmatches by b * nm_stride; mp_nobs NULL = 1
  const int* n_arr;
  const int* nmp_arr;
  long long kp_pitch;
  long long mp_pitch;
  int nm_stride;
};

// ORBmatcher::SearchByBoW(KeyFrame*, Frame&) with per-feature node ids.
// TrackReferenceKeyFrame over the batch (ORBPL_TRACK_REFKF, local_map.hip)
struct TrkArgs {
  StreamState* st;
  int kp_pitch;
  int lines;
  // current frame (after the motion model's matching / pose)
  const int* n;
  int* match;
  uint8_t* outlier;
  const int* nl;
  int* lmatch;
  uint8_t* loutlier;
  const KeyPointD* kps_un;
  const uint8_t* desc;
  const int* feat_node;
  // the reference keyframe = the last frame
  const int* last_n;
  const int* last_nl;
  const KeyPointD* last_kps_un;
  const uint8_t* last_desc;
  const uint8_t* last_has_mp;
  const int* last_feat_node;
  // scratch
  int* lcur;        // the frame's line assignments before the search [S][kLineKeep]
  int* cur_nobs_l;  // Observations() of those (1 / 0)
  int* tlm;         // the reference-keyframe line search's matches
  int* nml;         // per stream: the keyframe's lines to search (0 = stream not tracked by it)
  const int* list = nullptr;     // optional: the streams to run (k_trk_bow), list_n of them
  const int* list_n = nullptr;
};
void launch_trk_prep(const TrkArgs& a, int nstreams, hipStream_t s);
void launch_trk_bow(const TrkArgs& a, int nstreams, hipStream_t s);
void launch_trk_merge(const TrkArgs& a, int nstreams, hipStream_t s);

struct BowArgs {
  int nkf;
  const int* kf_node;
  const uint8_t* kf_valid;
  const uint8_t* kf_desc;
  const float* kf_angle;
  int nf;
  const int* f_node;
  const uint8_t* f_desc;
  const float* f_angle;
  float nnratio;
  int check_ori;
  int* match;
  int* nmatches;
  int kf_angle_stride = 1, f_angle_stride = 1;   // floats between consecutive angles
};
void launch_match_bow(const BowArgs& a, hipStream_t s);

// Frame::ComputeStereoMatches (stereo.hip).
struct StereoArgs {
  // Batched: frame f = blockIdx.x reads counts n_arr[f] / nr_arr[f] (or n /
  // nr when NULL), keypoint rows at f * kp_pitch (kl, dl, kr, dr, uright,
  // depth, sad), pyramids at f * pyr_pitch, entries at f * entry_cap.
  const int* n_arr;
  const int* nr_arr;
  long long kp_pitch;
  long long pyr_pitch;
  int n;
  const KeyPointD* kl;           // left mvKeys
  const uint8_t* dl;
  int nr;
  const KeyPointD* kr;           // right mvKeysRight
  const uint8_t* dr;
  const uint8_t* pyrL;           // one frame's padded pyramids (orbx layout)
  const uint8_t* pyrR;
  LevelGeom lv[8];
  float scale[8];
  float inv_scale[8];
  int nrows;
  float mb, mbf;
  float* uright;                 // mvuRight (-1: none)
  float* depth;                  // mvDepth
  int* sad;                      // scratch n
  uint16_t* entries;             // scratch: row band entries
  int entry_cap;
  int* err;
};
void launch_stereo(const StereoArgs& a, int batch, hipStream_t s);

void launch_in_frustum(const TrackConsts& c, float log_scale, const InFrustumArgs& a,
                       hipStream_t s, int nstreams = 1);
void launch_match_local(const TrackConsts& c, const LocalArgs& a, hipStream_t s,
                        int nstreams = 1);

size_t match_smem_bytes();
size_t pose_smem_bytes();
size_t pose_edge_bytes();

void launch_frame_prepare(const TrackConsts& c, const KeyPointD* kps, const int* n, int kp_pitch,
                          const float* depth, long long depth_pitch, KeyPointD* kps_un,
                          float* depth_out, float* uright, int* gcell, int batch, hipStream_t s);
void launch_predict(StreamState* st, int nstreams, hipStream_t s);
// GrabImageRGBD's imDepth.convertTo(CV_32F, mDepthMapFactor) (Tracking.cc:234-235):
// depth = float(v) * scale, scale = 1.0f / DepthMapFactor (pinned P21)
void launch_depth_u16(const uint16_t* in, float* out, long long n, float scale, hipStream_t s);
void launch_match_last(const TrackConsts& c, const MatchLaunch& m, int nstreams, hipStream_t s);
void launch_pose(const TrackConsts& c, const PoseLaunch& p, int nstreams, hipStream_t s);
// debug: stream 0 phase ticks of the last k_pose launch (ORBPL_POSE_PROFILE)
int read_pose_profile(long long* out8);
// debug: stream 0 phase ticks of the last k_match_last launch (ORBPL_MATCH_PROFILE)
int read_match_profile(long long* out8);
// TrackLocalMap for the batched tracker (local_map.hip). Per stream s:
// keypoint arrays at s * kp_pitch, line arrays at s * kLineKeep, the ring of
// the last K keyframes at (s * K + slot) * kp_pitch (lines: * kLineKeep), the
// gathered local lists at s * lp (lines: s * llp).
struct LocalMapArgs {
  StreamState* st;
  int kp_pitch;
  int lines;
  // current frame: motion-model matches / outliers, map after k_finish
  const int* n;
  const int* match;
  const uint8_t* outlier;
  const int* nl;
  const int* lmatch;
  const uint8_t* loutlier;
  const KeyPointD* kps_un;
  const uint8_t* desc;
  const uint8_t* ldesc;
  const uint8_t* has_mp;
  const float* mp_xyz;
  const uint8_t* has_ml;
  const float* ml_xyz;
  // last frame's map (motion-model matches point into it)
  const float* last_xyz;
  const float* last_lxyz;
  // keyframe ring
  int K, nslots, head, push_slot;
  float* r_xyz;
  float* r_nrm;
  float* r_dmin;
  float* r_dmax;
  uint8_t* r_has;
  uint8_t* r_desc;
  int* r_n;
  float* rl_xyz;
  uint8_t* rl_has;
  uint8_t* rl_desc;
  int* rl_n;
  // gathered local lists
  long long lp, llp;
  float* l_xyz;
  float* l_nrm;
  float* l_dmin;
  float* l_dmax;
  uint8_t* l_desc;
  int* l_n;
  float* ll_xyz;
  uint8_t* ll_desc;
  int* ll_n;
  int* cur_nobs;
  int* cur_nobs_l;
  // local search results
  const int* lm_match;
  const int* llm_match;
  // the second pose's inputs / outputs
  int* match2;
  float* xyz2;
  int* lmatch2;
  float* lxyz2;
  uint8_t* outlier2;
  uint8_t* loutlier2;
};
void launch_lm_gather(const LocalMapArgs& a, int nstreams, hipStream_t s);
void launch_lm_assemble(const LocalMapArgs& a, int nstreams, hipStream_t s);
void launch_lm_count(const LocalMapArgs& a, int frame_id, int nstreams, hipStream_t s);
void launch_lm_push(const TrackConsts& c, const LocalMapArgs& a, int nstreams, hipStream_t s);

// Line part of k_finish (all NULL when lines are disabled).
struct LineFinish {
  const int* nl;
  int* lmatch;
  uint8_t* loutlier;
  const float* dstart;
  const float* dend;
  const orbpl_keyline* kl_un;
  uint8_t* has_ml;
  float* ml_xyz;
};

void launch_finish(const TrackConsts& c, StreamState* st, const int* n, int kp_pitch,
                   const KeyPointD* kps_un, const float* depth, int* match, uint8_t* outlier,
                   uint8_t* has_mp, float* mp_xyz, int* nobs, const LineFinish& lf, int nstreams,
                   hipStream_t s, int local_map = 0);

}  // namespace orbpl
