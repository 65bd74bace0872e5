/*
 * orbpl.h — C-ABI of the MI355X-native ORB-SLAM2 point+line front-end.
 *
 * Every entry point is plain C: pointers + sizes, int status return
 * (0 = ok, < 0 = error, see ORBPL_ERR_*), caller-owned output buffers.
 * No torch / OpenCV / Eigen types cross this boundary. Each function names
 * the reference interface it replaces (file:line in
 * wolfcanli/ORB_SLAM2_Modification_with-point-and-line-feature).
 *
 * Threading: a handle (orbx_ctx / orbpl_tracker) owns one HIP stream on one
 * device and must be used by one host thread at a time — the same contract as
 * one ORB_SLAM2::ORBextractor instance per thread (Frame.cc:152-155).
 */
#ifndef ORBPL_H
#define ORBPL_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ORBPL_OK 0
#define ORBPL_ERR_ARG (-1)       /* bad argument / unsupported geometry      */
#define ORBPL_ERR_CAPACITY (-2)  /* caller buffer or internal cap too small  */
#define ORBPL_ERR_HIP (-3)       /* HIP runtime error (message: orbpl_last_error) */
#define ORBPL_ERR_NODEVICE (-4)  /* no HIP device visible                    */
#define ORBPL_ERR_OVERFLOW (-5)  /* kernel-side capacity overflow flag set   */

/* Mirror of cv::KeyPoint (28 bytes): pt.x, pt.y, size, angle, response,
 * octave, class_id. */
typedef struct orbpl_keypoint {
  float x, y, size, angle, response;
  int32_t octave, class_id;
} orbpl_keypoint;

/* Mirror of cv::line_descriptor::KeyLine (opencv_contrib 3.4, 68 bytes),
 * the element type of Frame::mvKeyLines (Frame.h, LineExtractor.h:27). */
typedef struct orbpl_keyline {
  float angle;
  int32_t class_id;
  int32_t octave;
  float pt_x, pt_y;
  float response;
  float size;
  float startPointX, startPointY, endPointX, endPointY;
  float sPointInOctaveX, sPointInOctaveY, ePointInOctaveX, ePointInOctaveY;
  float lineLength;
  int32_t numOfPixels;
} orbpl_keyline;

/* ORBextractor(int nfeatures, float scaleFactor, int nlevels, int iniThFAST,
 * int minThFAST) — ORBextractor.h:52-53, values from the settings YAML
 * (Tracking.cc:113-125; Examples/RGB-D/TUM1.yaml: 1000, 1.2, 8, 20, 7). */
typedef struct orbpl_orb_params {
  int32_t nfeatures;
  float scale_factor;
  int32_t nlevels;
  int32_t ini_th_fast;
  int32_t min_th_fast;
} orbpl_orb_params;

/* Last error message of the calling thread (static storage). */
const char* orbpl_last_error(void);
/* Number of visible HIP devices. */
int orbpl_device_count(int* n);
/* Hardware queues as recorded when the library was loaded (no HIP call):
 * queues = GPU_MAX_HW_QUEUES the HIP runtime runs with; runtime_started = 1
 * when the runtime was already up (another HIP user came first, so the
 * library changed nothing); set_by_library = 1 when the library filled in
 * the variable (it was unset, or ORBPL_HW_QUEUES asked). lsd_split_1024 = 1
 * when a 1024-stream lines tracker would split its LSD batch (needs >= 8
 * queues; ORBPL_LSD_SPLIT=0/1 overrides). Any pointer may be NULL. */
int orbpl_hw_queue_state(int* queues, int* runtime_started, int* set_by_library,
                         int* lsd_split_1024);
/* Library build tag ("orbpl gfx950 r4").
 * r4: orbpl_frame_is_in_frustum takes the RAW mfMinDistance / mfMaxDistance
 *     (MapPoint::GetMinDistance / GetMaxDistance) and applies the 0.8f / 1.2f
 *     of GetMin/MaxDistanceInvariance itself; r3 callers that pass the
 *     pre-scaled invariance values must switch to the raw ones.
 * r3: orbpl_tracker_timings writes 11 floats per step,
 *     orbpl_tracker_stereo_timings 4 (r1: 9 and 2); size the buffers from
 *     orbpl_tracker_timing_counts. */
const char* orbpl_version(void);

/* Device memory plumbing for hosts without their own GPU allocator (the
 * reference's C++ Tracking, ctypes tests, bench). Synchronous copies. */
int orbpl_dev_malloc(int device, int64_t bytes, void** out);
int orbpl_dev_free(int device, void* ptr);
/* page-locked host memory (hipHostMalloc): the source of asynchronous
 * host-to-device frame copies (orbpl_tracker_step_host) */
int orbpl_host_alloc(int64_t bytes, void** out);
int orbpl_host_free(void* ptr);
int orbpl_memcpy_htod(int device, void* dst, const void* src, int64_t bytes);
int orbpl_memcpy_dtoh(int device, void* dst, const void* src, int64_t bytes);
int orbpl_memset_d(int device, void* dst, int value, int64_t bytes);
int orbpl_device_synchronize(int device);

/* ------------------------------------------------------------------------
 * ORB extraction  — replaces ORB_SLAM2::ORBextractor (include/ORBextractor.h,
 * src/ORBextractor.cc:410-1132).
 * ---------------------------------------------------------------------- */
typedef struct orbx_ctx orbx_ctx;

/* ORBextractor::ORBextractor (ORBextractor.cc:410). width/height fix the
 * image geometry; max_batch frames can be extracted per launch. */
int orbx_create(const orbpl_orb_params* params, int width, int height, int max_batch,
                int device, orbx_ctx** out);
int orbx_destroy(orbx_ctx* ctx);

/* GetLevels / GetScaleFactors / GetInverseScaleFactors / GetScaleSigmaSquares
 * / GetInverseScaleSigmaSquares (ORBextractor.h:60-78). Arrays have nlevels
 * entries; any pointer may be NULL. */
int orbx_get_scale_info(const orbx_ctx* ctx, int* nlevels, float* scale, float* inv_scale,
                        float* sigma2, float* inv_sigma2);
/* Per-level content size and keypoint budget (mnFeaturesPerLevel). */
int orbx_get_level_info(const orbx_ctx* ctx, int* w, int* h, int* nfeatures_per_level);
/* Maximum keypoints one frame can produce (size for kps/desc buffers). */
int orbx_max_keypoints(const orbx_ctx* ctx);
/* Device-free geometry query (no HIP call): per-level sizes and budgets that
 * orbx_create would use, and the per-frame keypoint capacity. Arrays have
 * params->nlevels entries; any pointer may be NULL. */
int orbx_describe(const orbpl_orb_params* params, int width, int height, int* lw, int* lh,
                  int* nfeatures_per_level, float* scale, int* max_keypoints);

/* ORBextractor::operator()(image, mask, keypoints, descriptors)
 * (ORBextractor.cc:1043-1105). Host buffers in and out; synchronous.
 * kps[cap], desc[cap*32] (row i = descriptor of kps[i]); *n = keypoint count.
 * Empty image (NULL or 0 size) returns ORBPL_OK with *n = 0. */
int orbx_extract(orbx_ctx* ctx, const uint8_t* img, int width, int height, int stride,
                 orbpl_keypoint* kps, uint8_t* desc, int cap, int* n);

/* Batched, device-resident form (throughput path). d_imgs: batch frames of
 * width x height u8 in device memory, frame f at d_imgs + f*frame_pitch with
 * row stride `stride`. Outputs are device buffers: d_kps[batch*kp_pitch],
 * d_desc[batch*kp_pitch*32], d_n[batch]. Asynchronous on the ctx stream. */
int orbx_extract_batch_device(orbx_ctx* ctx, const uint8_t* d_imgs, int batch, int stride,
                              int64_t frame_pitch, orbpl_keypoint* d_kps, uint8_t* d_desc,
                              int kp_pitch, int32_t* d_n);

/* The public mvImagePyramid (ORBextractor.h:83; read by Frame.cc:895-1002):
 * copy level `level` of frame `frame` of the last extraction to host. With
 * padded != 0 the (w+38)x(h+38) bordered buffer is returned, else the w x h
 * content; blurred != 0 returns the GaussianBlur(7x7, 2) working image. */
int orbx_get_pyramid(orbx_ctx* ctx, int frame, int level, int padded, int blurred, uint8_t* out,
                     int out_cap, int* w, int* h);

/* Debug/parity: pre-octree FAST candidates (vToDistributeKeys,
 * ORBextractor.cc:820-825) of frame 0 of the last extraction, concatenated by
 * level as (x, y, response) float triples relative to minBorder. */
int orbx_get_candidates(orbx_ctx* ctx, float* xyr, int cap, int* level_counts, int* total);

/* Wait for the ctx stream; returns ORBPL_ERR_OVERFLOW if a kernel reported a
 * capacity overflow since the last call. */
int orbx_synchronize(orbx_ctx* ctx);
/* Device-side timing of the last orbx_extract*: per-stage milliseconds
 * (pyramid, blur, fast, octree, desc) measured with hipEvents on the ctx
 * stream. */
int orbx_last_stage_ms(const orbx_ctx* ctx, float* ms5);
/* Debug: k_pyramid phase times (ns) of block (band 0, frame 0) in the last
 * launch, 4 per level (content, side borders, mirror rows, blur); needs
 * ORBPL_PYR_PROFILE in the environment when the context is created. */
int orbx_debug_pyr_profile(orbx_ctx* ctx, long long* out, int cap, int* n);
/* Debug: k_octree per-level block of frame 0 in the last launch (ORBPL_OCT_PROFILE
 * set before the first launch): 8 values per level (setup ns, pass loop ns, 0,
 * retain ns, passes, candidates, final list size, 0), 16 levels. */
int orbx_debug_octree_profile(orbx_ctx* ctx, long long* out128);


/* ------------------------------------------------------------------------
 * Camera / Frame glue — Frame constructors (Frame.cc:135-205): undistortion
 * (UndistortKeyPoints :737-764, cv::undistortPoints 5 iterations), image
 * bounds (ComputeImageBounds :847-885), RGB-D depth association
 * (ComputeStereoFromRGBD :1065-1117) and the 64x48 grid (PosInGrid :527-538).
 * ---------------------------------------------------------------------- */
typedef struct orbpl_camera {
  float fx, fy, cx, cy;        /* Camera.fx/fy/cx/cy                          */
  float k1, k2, p1, p2, k3;    /* Camera.k1..k3 (OpenCV order)                */
  float bf;                    /* mbf = Camera.bf                             */
  float th_depth;              /* mThDepth = bf * ThDepth / fx (Tracking.cc:134-138) */
  int32_t width, height;
} orbpl_camera;

/* Tracking::Tracking's settings (Tracking.cc:53-147) read from the
 * reference's OpenCV FileStorage YAML files (Examples/RGB-D/TUM1.yaml:8-55):
 * the flat "Key.name: value" subset, with OpenCV 3.4's FileNode conversions
 * (a missing key reads 0). sensor: System::eSensor. cam.th_depth = mbf *
 * ThDepth / fx for stereo / RGB-D (0 monocular); fps 0 -> 30 and max_frames
 * = mMaxFrames (orbpl_tracker_set_fps takes fps); depth_map_factor =
 * mDepthMapFactor = 1 / DepthMapFactor (1 when |DepthMapFactor| < 1e-5 or
 * not RGB-D); cam.width / height from Camera.width / height when present
 * (the reference takes them from the images). */
#define ORBPL_SENSOR_MONOCULAR 0
#define ORBPL_SENSOR_STEREO 1
#define ORBPL_SENSOR_RGBD 2
typedef struct orbpl_settings {
  orbpl_orb_params orb;
  orbpl_camera cam;
  float fps;
  int32_t max_frames;
  float depth_map_factor;      /* mDepthMapFactor (1 / DepthMapFactor)       */
  float depth_map_factor_setting;  /* DepthMapFactor as read (orbpl_tracker_step_host) */
  int32_t rgb;                 /* Camera.RGB */
} orbpl_settings;
int orbpl_settings_load(const char* path, int sensor, orbpl_settings* out);

#define ORBPL_GRID_COLS 64     /* FRAME_GRID_COLS (Frame.h:41) */
#define ORBPL_GRID_ROWS 48     /* FRAME_GRID_ROWS (Frame.h:40) */

/* Per-frame glue on the GPU. Inputs: raw keypoints kps[n] from orbx_extract,
 * optional depth image (float metres, width x height, row stride = width;
 * NULL for monocular: depth/uright = -1). Outputs (caller-owned, n entries):
 * kps_un (mvKeysUn), depth (mvDepth), uright (mvuRight), grid_cell
 * (gx + 64*gy, -1 if PosInGrid fails). bounds[4] = mnMinX, mnMaxX, mnMinY,
 * mnMaxY. */
int orbpl_frame_prepare(const orbpl_camera* cam, const orbpl_keypoint* kps, int n,
                        const float* depth, orbpl_keypoint* kps_un, float* depth_out,
                        float* uright_out, int32_t* grid_cell, float* bounds);

/* ------------------------------------------------------------------------
 * ORBmatcher::SearchByProjection(Frame& CurrentFrame, const Frame& LastFrame,
 * float th, bool bMono)  (ORBmatcher.cc:1710-1879), with ORBmatcher(0.9, true)
 * as Tracking::TrackWithMotionModel builds it (Tracking.cc:1216).
 * ---------------------------------------------------------------------- */
typedef struct orbpl_match_current {
  int32_t n;
  const float* Tcw;            /* 4x4 row-major (mTcw, predicted pose)        */
  const orbpl_keypoint* kps_un;/* mvKeysUn                                    */
  const uint8_t* desc;         /* mDescriptors, n x 32                        */
  const float* uright;         /* mvuRight                                    */
} orbpl_match_current;

typedef struct orbpl_match_last {
  int32_t n;
  const float* Tcw;            /* LastFrame.mTcw                              */
  const orbpl_keypoint* kps_un;/* LastFrame.mvKeysUn (angle, octave used)     */
  const uint8_t* has_mp;       /* LastFrame.mvpMapPoints[i] != NULL           */
  const uint8_t* outlier;      /* LastFrame.mvbOutlier                        */
  const float* mp_xyz;         /* pMP->GetWorldPos(), n x 3                   */
  const uint8_t* mp_desc;      /* pMP->GetDescriptor(), n x 32                */
  const int32_t* mp_nobs;      /* pMP->Observations()                         */
} orbpl_match_last;

/* match[i] = index j of the last-frame map point assigned to current keypoint
 * i (CurrentFrame.mvpMapPoints[i] = LastFrame.mvpMapPoints[j]) or -1.
 * *nmatches = the function's return value. */
int orbm_search_by_projection_last(const orbpl_camera* cam, const float* scale_factors,
                                   int nlevels, const orbpl_match_current* cur,
                                   const orbpl_match_last* last, float th, int mono,
                                   int check_orientation, int32_t* match, int* nmatches);

/* Frame::ComputeStereoMatches (Frame.cc:886-1063) for a stereo pair whose
 * left / right images were extracted by `left` / `right` (batch frame
 * `frame`; their pyramids are the reference's mvImagePyramid): uRight and
 * depth per left keypoint (-1: none). kl / kr = mvKeys / mvKeysRight as
 * returned by orbx_extract. n, nr <= 4096, image height <= 1024. */
int orbpl_stereo_matches(const orbpl_camera* cam, orbx_ctx* left, orbx_ctx* right, int frame,
                         const orbpl_keypoint* kl, const uint8_t* dl, int n,
                         const orbpl_keypoint* kr, const uint8_t* dr, int nr, float* uright,
                         float* depth);

/* ------------------------------------------------------------------------
 * Tracking::SearchLocalPoints pieces (TrackLocalMap)
 * ---------------------------------------------------------------------- */
/* Frame::IsInFrustum(MapPoint*, view_cos_limit) (Frame.cc:345-401) for n map
 * points (world xyz, normal, and the raw mfMinDistance / mfMaxDistance: the
 * range test applies GetMin/MaxDistanceInvariance's 0.8f / 1.2f, MapPoint.cc:
 * 387-397, and PredictScale's ratio is mfMaxDistance / dist, MapPoint.cc:
 * 416-431); outputs the mTrack* fields:
 * in_view (mbTrackInView), proj_x/y, proj_xr (u - bf/z), level
 * (mnTrackScaleLevel, -1 when not in view), view_cos (mTrackViewCos).
 * scale_factor = ORBextractor scale factor (mfLogScaleFactor = logf of it). */
int orbpl_frame_is_in_frustum(const orbpl_camera* cam, float scale_factor, int nlevels,
                              const float* Tcw, int n, const float* xyz, const float* normal,
                              const float* min_dist, const float* max_dist, float view_cos_limit,
                              uint8_t* in_view, float* proj_x, float* proj_y, float* proj_xr,
                              int32_t* level, float* view_cos);
/* ORBmatcher(nnratio).SearchByProjection(F, vpLocalMapPoints, th)
 * (ORBmatcher.cc:72-183): radius RadiusByViewingCos(view_cos) (x th when
 * th != 1) x scale[level], levels [level-1, level], best and second by
 * Hamming, TH_HIGH 100, ratio test only when both are on the same level.
 * cur_nobs[i] = Observations() of the map point already at keypoint i (0 or
 * NULL: none); keypoints holding one with Observations() > 0 are skipped, as
 * are keypoints claimed during the call. match[i] = index of the last local
 * map point assigned to keypoint i in this call (the reference overwrites
 * F.mvpMapPoints[i]), -1 = unchanged. *nmatches = return value. */
int orbm_search_by_projection_local(const orbpl_camera* cam, const float* scale_factors,
                                    int nlevels, const orbpl_match_current* cur, int nmp,
                                    const uint8_t* in_view, const float* proj_x,
                                    const float* proj_y, const float* proj_xr,
                                    const int32_t* level, const float* view_cos,
                                    const uint8_t* mp_desc, const int32_t* mp_nobs,
                                    const int32_t* cur_nobs, float th, float nnratio,
                                    int32_t* match, int* nmatches);

/* ---- DBoW2 ORB vocabulary (ORBVocabulary = TemplatedVocabulary<FORB::
 * TDescriptor, FORB>, Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h) ---- */
typedef struct orbv_vocab orbv_vocab;
/* TemplatedVocabulary::loadFromTextFile (TemplatedVocabulary.h:1338-1420),
 * System.cc:65: "k L scoring weighting" then one node per line (parent,
 * isLeaf, 32 descriptor bytes, weight). A line without tokens (the one after a
 * final '\n') makes no node (pinned P19). Host-only; word ids follow the
 * isLeaf lines in node order. */
int orbv_load_text(const char* path, orbv_vocab** out);
/* The same vocabulary from flat node arrays (node 0 = root, parent[i] < i):
 * a rank's copy of the vocabulary rank 0 loaded and broadcast. */
int orbv_create(int k, int L, int scoring, int weighting, int n_nodes, const int32_t* parent,
                const uint8_t* leaf_flag, const uint8_t* desc, const double* weight,
                orbv_vocab** out);
int orbv_destroy(orbv_vocab* v);
/* out6 = k, L, scoring, weighting, n_nodes, n_words */
int orbv_info(const orbv_vocab* v, int* out6);
/* the flat node arrays orbv_create takes (n_nodes entries; desc 32 B rows) */
int orbv_export(const orbv_vocab* v, int32_t* parent, uint8_t* leaf_flag, uint8_t* desc,
                double* weight);
/* copy the tree to `device` (CSR children, descriptors, words, weights) */
int orbv_upload(orbv_vocab* v, int device);
/* TemplatedVocabulary::transform(features, BowVector, FeatureVector, levelsup)
 * (TemplatedVocabulary.h:1127-1205, 1226-1262) as Frame::ComputeBoW calls it
 * (Frame.cc:730, levelsup 4): the BowVector as bow_n (word, value) pairs in
 * word order, the FeatureVector as the node (at level L - levelsup) of every
 * feature, -1 for a stopped word (weight 0). n <= 4096; bow buffers >= n. */
int orbv_transform(orbv_vocab* v, int device, const uint8_t* desc, int n, int levelsup,
                   uint32_t* bow_words, double* bow_vals, int* bow_n, int32_t* feat_node);
/* The same for nframes device-resident frames: frame f's descriptors at
 * d_desc + f * desc_pitch * 32 (d_n[f] of them, <= max_n <= 4096); outputs
 * per frame at f * out_pitch (feature word / weight / node, BowVector), the
 * BowVector length in d_bow_n[f]; d_err bit 1 = a frame above 4096 features.
 * `stream` = a hipStream_t (NULL: the vocabulary's own stream). */
int orbv_transform_batch_device(orbv_vocab* v, const uint8_t* d_desc, int64_t desc_pitch,
                                const int* d_n, int nframes, int max_n, int levelsup,
                                int32_t* d_feat_node, int32_t* d_feat_word, double* d_feat_weight,
                                uint32_t* d_bow_words, double* d_bow_vals, int* d_bow_n,
                                int64_t out_pitch, int* d_err, void* stream);

/* ORBmatcher(nnratio, checkOri).SearchByBoW(pKF, F, vpMapPointMatches)
 * (ORBmatcher.cc:247-410). The DBoW2 FeatureVectors are passed as one
 * vocabulary node id per feature (-1: none; ids < 2^21 - 1): features meet
 * only within a node, keyframe features in index order, a frame feature taken
 * earlier in the call is skipped; TH_LOW 50 and best < nnratio * second; then
 * the 30-bin rotation check (kf_angle = mvKeysUn, f_angle = mvKeys). kf_valid
 * = the keyframe's map point exists and is not bad. match[j] = keyframe
 * feature index whose map point goes to frame feature j, or -1. n <= 2048. */
int orbm_search_by_bow(int nkf, const int32_t* kf_node, const uint8_t* kf_valid,
                       const uint8_t* kf_desc, const float* kf_angle, int nf, const int32_t* f_node,
                       const uint8_t* f_desc, const float* f_angle, float nnratio, int check_ori,
                       int32_t* match, int* nmatches);

/* ------------------------------------------------------------------------
 * Optimizer::PoseOptimization / PoseOptimizationWithLines
 * (Optimizer.cc:375-619, 2132-2486): 4 rounds x 10 Levenberg-Marquardt
 * iterations on one SE3 vertex, Huber kernel in rounds 0-2, chi2 outlier
 * re-labelling after each round. Point edge i exists if has_mp[i]; it is
 * monocular if uright[i] < 0 else stereo. Line edge j exists if has_ml[j].
 * ---------------------------------------------------------------------- */
typedef struct orbpl_pose_problem {
  int32_t n;                   /* points: N                                   */
  const orbpl_keypoint* kps_un;
  const float* uright;
  const uint8_t* has_mp;
  const float* mp_xyz;         /* n x 3                                       */
  int32_t nl;                  /* lines: NL (0 for PoseOptimization)          */
  const float* kl_obs;         /* nl x 4: startX, startY, endX, endY (mvKeyLinesUn) */
  const int32_t* kl_octave;    /* nl                                          */
  const uint8_t* has_ml;       /* nl                                          */
  const float* ml_xyz;         /* nl x 6: world start, world end              */
  const float* inv_sigma2;     /* mvInvLevelSigma2, nlevels                   */
  int32_t nlevels;
} orbpl_pose_problem;

/* Tcw: in = pFrame->mTcw, out = optimised pose (4x4 row-major float).
 * outlier[n] / line_outlier[nl]: in = pFrame->mvbOutlier / mvbLineOutlier,
 * out = after the call. *n_inliers = return value of the reference
 * (nInitialCorrespondences - nBad, 0 if < 3 correspondences). */
int orbpl_pose_optimization(const orbpl_camera* cam, const orbpl_pose_problem* prob, float* Tcw,
                            uint8_t* outlier, uint8_t* line_outlier, int* n_inliers);
/* Pose options. ORBPL_POSE_FIXED_LINE_JAC: the analytic EdgeLineOnlyPose
 * Jacobian ("--fixed-line-jacobian") instead of the
 * reference's as-written one (types_line_expmap.h:138-152: row 0 overwritten
 * by the end point, row 1 uninitialised -> 0 (pinned P7), +fx*cy in dI_dLc,
 * R*v in place of n_c in dLc_ddelta): de_i/dl = ((x_i - l0 N_i/ln^2)/ln,
 * (y_i - l1 N_i/ln^2)/ln, 1/ln), l = K_line n_c, dn_c/d(w,u) =
 * [-[n_c]x | -[v_c]x] under g2o's left update exp(d) * T. */
#define ORBPL_POSE_FIXED_LINE_JAC 1
int orbpl_pose_optimization_ex(const orbpl_camera* cam, const orbpl_pose_problem* prob, int flags,
                               float* Tcw, uint8_t* outlier, uint8_t* line_outlier,
                               int* n_inliers);


/* ------------------------------------------------------------------------
 * Batched RGB-D tracker: the per-frame hot path of Tracking::Track for
 * n_streams independent camera streams on one device, one
 * TrackWithMotionModel step per call (Tracking.cc:1212-1330):
 *   Frame(RGB-D) extraction + glue -> constant-velocity prediction ->
 *   SearchByProjection(cur, last, th=15, retry 2*th if < 20) ->
 *   PoseOptimization -> discard outliers -> velocity update.
 * Every frame then acts as the keyframe of the next one: its keypoints with
 * depth become map points (StereoInitialization-style, Tracking.cc:608-660);
 * local mapping / loop closing are out of scope.
 * ---------------------------------------------------------------------- */
typedef struct orbpl_tracker orbpl_tracker;

int orbpl_tracker_create(const orbpl_orb_params* orb, const orbpl_camera* cam, int n_streams,
                         int device, orbpl_tracker** out);
/* Tracker flags. ORBPL_TRACK_LINES: the point-and-line variant of the
 * reference's RGB-D tracking (Tracking.cc:1210-1320 with mbUseLines):
 * LineExtractor per frame (lsdx_*), UndistortKeyLines + line depths,
 * LineMatcher::SearchByProjection against the last frame's map lines,
 * PoseOptimization with line edges, line outlier discard and map lines. */
#define ORBPL_TRACK_LINES 1
/* ORBPL_TRACK_STEREO: the reference's stereo tracking (Tracking::GrabImageStereo,
 * Tracking.cc:180-208): Frame(imLeft, imRight) runs ORB on both images
 * concurrently (Frame.cc:88-91), UndistortKeyPoints, ComputeStereoMatches
 * (Frame.cc:886-1063) for depth / uRight; SearchByProjection uses th = 7
 * (Tracking.cc:1238-1241). Images up to 1024 rows.
 * ORBPL_TRACK_STEREO | ORBPL_TRACK_LINES (BASELINE configs[3], a DEFINED mode:
 * the reference's stereo Frame extracts no lines but PoseOptimizationWithLines
 * loops over NL, Optimizer.cc:2287-2303): LineExtractor on both images, line
 * end-point depths from the best LBD match on the right image whose line
 * passes the angle / length / row-overlap / disparity tests,
 * then the RGB-D line path (line matching, line edges, map lines). */
#define ORBPL_TRACK_STEREO 2
/* ORBPL_TRACK_LOCAL_MAP: Tracking::TrackLocalMap after TrackWithMotionModel
 * (Tracking.cc:1332-1420): the local map is the map points / lines of the last
 * 4 frames (every tracked frame is a keyframe) minus those the
 * frame already holds or rejected; SearchLocalPoints (IsInFrustum 0.5,
 * ORBmatcher(0.8).SearchByProjection th 3 RGB-D / 1 stereo, 5 for the first
 * frames), SearchLocalLines (LineMatcher(0.8) local-map overload with its
 * relaxed retry), a second PoseOptimizationWithLines over all matches and the
 * mnMatchesInliers / mnLineMatchesInliers decision. */
#define ORBPL_TRACK_LOCAL_MAP 4
/* ORBPL_TRACK_FIXED_LINE_JAC: PoseOptimizationWithLines with the analytic line
 * Jacobian (ORBPL_POSE_FIXED_LINE_JAC) in every tracker pose. */
#define ORBPL_TRACK_FIXED_LINE_JAC 8
/* ORBPL_TRACK_REFKF: Tracking::Track's choice between TrackWithMotionModel
 * and TrackReferenceKeyFrame (Tracking.cc:324-338, 942-1032; needs a
 * vocabulary, orbpl_tracker_set_vocabulary): the first frame after the
 * initial one (no velocity) and every frame whose motion-model tracking
 * fails are tracked against the reference keyframe (the last frame, P18) by
 * ORBmatcher(0.7, true).SearchByBoW + LineMatcher's reference-keyframe
 * overload from the pose of the last frame, then PoseOptimizationWithLines
 * and the outlier discard; success = 10 map inliers (and, with lines, a
 * line count of 10 after the reference's outlier decrement). Pinned P22. */
#define ORBPL_TRACK_REFKF 16
/* ORBPL_TRACK_MAP: Tracking::Track with the reference's map model
 * (Tracking.cc:283-599; RGB-D streams): StereoInitialization (> 500 keypoints:
 * the first keyframe, a map point per keypoint with depth, a map line per line
 * with both end-point depths), UpdateLastFrame's temporal VO points / lines,
 * TrackWithMotionModel against the last frame's map points / lines,
 * TrackReferenceKeyFrame against the reference keyframe (with
 * ORBPL_TRACK_REFKF and a vocabulary), TrackLocalMap over the covisibility
 * graph (UpdateLocalKeyFrames / UpdateLocalPoints / UpdateLocalLines,
 * SearchLocalPoints / SearchLocalLines, the second pose), NeedNewKeyFrame,
 * CreateNewKeyFrame and LocalMapping::ProcessNewKeyFrame (observations,
 * distinctive descriptors, normals, UpdateConnections), the LOST state and the
 * reset of a map with <= 5 keyframes. Per stream a keyframe table (32 by
 * default; ORBPL_MAP_KF in the environment at creation, 2..64) and point / line
 * pools of keyframes x keypoint capacity / x 80 in HBM: with F keyframe slots
 * and K keypoints per frame about F*K*(160 + 4*F) + F*80*112 bytes per stream
 * (the observation table grows with F^2: K = 1000 gives ~9.5 MB at F = 32,
 * ~27 MB at F = 64, i.e. ~10 / ~28 GB for 1024 streams). A stream whose map
 * needs a keyframe beyond its F slots declines it and raises capacity flag 1
 * (orbpl_tracker_get_map_errors): size F above the keyframes a run inserts
 * (at most one per step). Pinned P23-P25
 * (DESIGN.md): LocalMapping = its ProcessNewKeyFrame run synchronously,
 * Relocalization fails; pointer-ordered containers in keyframe id order.
 * Replaces ORBPL_TRACK_LOCAL_MAP (its P18 local map). With ORBPL_TRACK_STEREO
 * the same Track() on stereo frames (orbpl_tracker_step_stereo: depths from
 * ComputeStereoMatches, line depths P17) with the reference's STEREO branches:
 * motion-model radius 7, local-map radius 1, outlier matches dropped after
 * TrackLocalMap's pose (Tracking.cc:1238-1241, 1374-1401, 1801-1809). */
#define ORBPL_TRACK_MAP 32
int orbpl_tracker_create_ex(const orbpl_orb_params* orb, const orbpl_camera* cam, int n_streams,
                            int device, int flags, orbpl_tracker** out);
int orbpl_tracker_destroy(orbpl_tracker* tr);
/* Forget all stream state; the next step initialises every stream with pose
 * Tcw0 (n_streams x 16 floats row-major, NULL = identity). */
int orbpl_tracker_reset(orbpl_tracker* tr, const float* Tcw0);
/* mVelocity = cv::Mat() for every stream s with mask[s] != 0 (n_streams
 * bytes): the state Tracking holds after its initialisation or a
 * relocalisation, so the stream's next step runs TrackReferenceKeyFrame
 * instead of TrackWithMotionModel (Tracking.cc:324-338; with
 * ORBPL_TRACK_REFKF and a vocabulary; without them the next prediction uses
 * zero velocity). Waits for the tracker's queued steps. Used to time and test
 * TrackReferenceKeyFrame under load. */
int orbpl_tracker_clear_velocity(orbpl_tracker* tr, const uint8_t* mask);
/* Camera.fps of the settings (ORBPL_TRACK_MAP trackers): mMaxFrames = fps,
 * 0 -> 30 (Tracking.cc:81-87), read by NeedNewKeyFrame and TrackLocalMap's
 * recent-relocalisation test. Default 30 (TUM); KITTI's settings say 10. */
int orbpl_tracker_set_fps(orbpl_tracker* tr, float fps);
/* One step for all streams. d_gray: n_streams frames of width*height u8;
 * d_depth: n_streams frames of width*height float metres (device memory,
 * contiguous). Asynchronous on the tracker's stream. */
int orbpl_tracker_step(orbpl_tracker* tr, const uint8_t* d_gray, const float* d_depth);
/* Stereo step (ORBPL_TRACK_STEREO trackers): d_left / d_right hold n_streams
 * rectified frames of width*height u8 each (device memory, contiguous). */
int orbpl_tracker_step_stereo(orbpl_tracker* tr, const uint8_t* d_left, const uint8_t* d_right);
/* Tracking::GrabImageRGBD from host buffers (Tracking.cc:225-248): n_streams
 * gray frames and n_streams 16-bit depth maps (TUM PNG depth, raw units),
 * copied asynchronously on the tracker's copy stream into one of 3 device
 * slots (pinned memory from orbpl_host_alloc makes the copy overlap the
 * previous steps' kernels), depth converted as imDepth.convertTo(CV_32F,
 * 1.0f / depth_map_factor) (pinned P21: float(v) * (1.0f / factor); TUM:
 * DepthMapFactor 5000), then the step. The host buffers may be reused after
 * the next orbpl_tracker_synchronize. */
int orbpl_tracker_step_host(orbpl_tracker* tr, const uint8_t* h_gray, const uint16_t* h_depth,
                            float depth_map_factor);
int orbpl_tracker_synchronize(orbpl_tracker* tr);
/* on != 0: extraction of step t+1 may overlap matching/pose of step t (two
 * HIP streams, three frame buffers). Results are identical either way. */
int orbpl_tracker_set_pipelined(orbpl_tracker* tr, int on);
/* Results of the last step, per stream (any pointer may be NULL):
 * Tcw (16 floats), keypoints, SearchByProjection matches, PoseOptimization
 * inliers, map matches after outlier removal. */
int orbpl_tracker_get_state(orbpl_tracker* tr, float* Tcw, int* nkeypoints, int* nmatches,
                            int* ninliers, int* nmatches_map);
/* hipEvent times of the last step (ms): extract, glue, match, pose, finish. */
int orbpl_tracker_stage_ms(orbpl_tracker* tr, float* ms5);
/* Per-kernel device times (ms, hipEvents on the tracker stream) of the last
 * min(max_steps, 64) steps, 11 per step: pyramid (+ borders + blur, one
 * launch), blur (0), fast, octree, orient+desc, glue+predict, match, pose,
 * finish, local_map (TrackLocalMap: gather, IsInFrustum, local point and line
 * search, second pose, counts; 0 without ORBPL_TRACK_LOCAL_MAP), bow
 * (KeyFrame::ComputeBoW; 0 without a vocabulary). Stereo matching counts in
 * glue. */
int orbpl_tracker_timings(orbpl_tracker* tr, int max_steps, float* ms, int* n_steps);
int orbpl_tracker_timings_reset(orbpl_tracker* tr);
/* Floats per step written by orbpl_tracker_timings, _line_timings,
 * _lsd_timings, _stereo_timings and _kernel_timings (in that order): 11, 3, 7,
 * 4, 4. A caller sizes its buffers max_steps x these. */
int orbpl_tracker_timing_counts(int* counts5);
/* Frames one launch of the extraction kernels (pyramid, FAST, octree,
 * orient+desc) and of the LSD kernels processes. Both equal the stream count
 * unless the tracker splits that batch into two offset halves on two streams
 * (ORBPL_ORB_SPLIT=1; ORBPL_LSD_SPLIT, by default from 1024 streams when the
 * HIP runtime has GPU_MAX_HW_QUEUES >= 8): then the first half's, whose
 * launches the stage timings above bracket. lsd_frames is 0 without lines. */
int orbpl_tracker_launch_frames(const orbpl_tracker* tr, int* orb_frames, int* lsd_frames);
/* Per-kernel device times (ms) of the last min(max_steps, 64) steps, 4 per
 * step, each launch bracketed by its own hipEvents on the tracking stream:
 * k_pose of TrackWithMotionModel, k_pose of TrackReferenceKeyFrame (0 without
 * ORBPL_TRACK_REFKF), k_pose of TrackLocalMap and k_match_local (0 without
 * ORBPL_TRACK_LOCAL_MAP). Summed per kernel they give a kernel's GPU time per
 * step across the stages it runs in. */
int orbpl_tracker_kernel_timings(orbpl_tracker* tr, int max_steps, float* ms, int* n_steps);
/* Debug (ORBPL_POSE_PROFILE set): stream 0's PoseOptimization phase times of
 * the last step in ns (edges, linearize reduction, solve+exp, trial errors,
 * classify), the LM iteration / trial counts, the linearize edge loop (ns). */
int orbpl_tracker_debug_pose_profile(orbpl_tracker* tr, long long* out8);
/* Debug (ORBPL_MATCH_PROFILE set): stream 0's last-frame SearchByProjection
 * phase times of the last step in ns (grid, candidates, ordered claims,
 * rotation check, output). */
int orbpl_tracker_debug_match_profile(orbpl_tracker* tr, long long* out5);
/* Per-stream frame outputs of the last step (host copies, kp_cap entries per
 * stream, see orbpl_tracker_kp_capacity): undistorted keypoints, descriptors,
 * match (last-frame index per keypoint or -1), outlier flags. */
int orbpl_tracker_kp_capacity(const orbpl_tracker* tr);
int orbpl_tracker_get_frame(orbpl_tracker* tr, int stream, orbpl_keypoint* kps_un, uint8_t* desc,
                            int32_t* match, uint8_t* outlier, int* n);
/* Tracking outcome of the last step per stream: ok (TrackWithMotionModel's
 * return), lines of the frame, LineMatcher matches (every passing pair
 * counts, as in the reference), line map matches after outlier discard
 * (outliers decrement, Tracking.cc:1306). Line counts are 0 without lines. */
int orbpl_tracker_get_status(orbpl_tracker* tr, int* ok, int* nlines, int* line_matches,
                             int* line_nmatches_map);
/* Line outputs of the last step (kLineKeep = 80 entries per stream):
 * undistorted KeyLines, LBD rows, matched last-frame line (-1 none), outlier
 * flags. ORBPL_TRACK_LINES trackers only. */
int orbpl_tracker_get_lines(orbpl_tracker* tr, int stream, orbpl_keyline* kl_un, uint8_t* desc,
                            int32_t* lmatch, uint8_t* loutlier, int* n);
/* Line stage device times (ms) of the last min(max_steps, 64) steps, 3 per
 * step: LSD, KeyLines + LBD + UndistortKeyLines, line SearchByProjection. */
int orbpl_tracker_line_timings(orbpl_tracker* tr, int max_steps, float* ms, int* n_steps);
/* Per-step history of every stream, recorded on the device by D2D copies at
 * the end of each step (no host synchronisation inside a step): the next
 * max_steps steps after the call are kept (0 = off; a new call clears it).
 * get_history returns stream `stream`'s first min(max_steps, recorded) steps:
 * Tcw (16 floats per step) and 12 counts per step in the oracle's order:
 * nkeypoints, nmatches, ninliers, nmatches_map, ok, nlines, line_matches,
 * line_nmatches_map, then the TrackLocalMap counts (0 when it did not run):
 * local matches, mnMatchesInliers, local line matches, mnLineMatchesInliers. */
int orbpl_tracker_set_history(orbpl_tracker* tr, int max_steps);
int orbpl_tracker_get_history(orbpl_tracker* tr, int stream, int max_steps, float* Tcw,
                              int* counts12, int* n_steps);
/* ORBPL_TRACK_MAP trackers: the recorded steps' 24 counts per step in the
 * oracle's order (oracle_map_step): the 12 of get_history, then keyframe
 * created (1, 2 = the initial one), keyframes, map points, map lines,
 * temporal points, TrackReferenceKeyFrame ran, reference keyframe (-1 none),
 * state (0 not initialised, 1 OK, 2 LOST), local keyframes, local map points
 * searched, local map lines searched, temporal lines. */
int orbpl_tracker_get_map_history(orbpl_tracker* tr, int stream, int max_steps, int* counts24,
                                  int* n_steps);
/* ORBPL_TRACK_MAP trackers: capacity flags of each stream's map since the last
 * reset (1 keyframe table full: NeedNewKeyFrame declined; 2 point / line pool
 * full; 4 local list full); 0 = the map matches the reference's. */
int orbpl_tracker_get_map_errors(orbpl_tracker* tr, int* err);
/* ORBPL_TRACK_MAP trackers, one stream's map after the last step (host copies):
 * keyframes (n_kf; per keyframe its spanning-tree parent (-1 none), the number
 * of ordered connections and the first `cap` of them (GetVectorCovisibleKeyFrames
 * order, -1 padded)); map points (n_mp; the first `cap`: Observations(),
 * GetDescriptor(), world position, GetNormal(), [mfMinDistance,
 * mfMaxDistance]); map lines (n_ml; Observations(), descriptor, end points).
 * Any output pointer may be NULL. */
int orbpl_tracker_get_map_keyframes(orbpl_tracker* tr, int stream, int* parent, int* ord, int cap,
                                    int* nord, int* n_kf);
int orbpl_tracker_get_map_points(orbpl_tracker* tr, int stream, int cap, int* nobs, uint8_t* desc,
                                 float* xyz, float* normal, float* dist2, int* n_mp);
int orbpl_tracker_get_map_lines(orbpl_tracker* tr, int stream, int cap, int* nobs, uint8_t* desc,
                                float* pos6, int* n_ml);
/* KeyFrame::ComputeBoW (KeyFrame.cc:67; every tracked frame is a keyframe,
 * P18) with `voc` (uploaded to the tracker's device; not owned, must outlive
 * the tracker or be unset with NULL): each step transforms the frame's
 * descriptors on the extraction stream (levelsup: Frame::ComputeBoW's 4). */
int orbpl_tracker_set_vocabulary(orbpl_tracker* tr, orbv_vocab* voc, int levelsup);
/* the last step's BowVector / FeatureVector of one stream (buffers of the
 * tracker's keypoint capacity); n = its keypoints */
int orbpl_tracker_get_bow(orbpl_tracker* tr, int stream, uint32_t* bow_words, double* bow_vals,
                          int* bow_n, int32_t* feat_node, int* n);
/* per stream: 1 when the last step ran TrackReferenceKeyFrame (ORBPL_TRACK_REFKF) */
int orbpl_tracker_get_trk(orbpl_tracker* tr, int* trk);
/* TrackLocalMap outcome of the last step per stream (ORBPL_TRACK_LOCAL_MAP; 0
 * where it did not run): SearchLocalPoints matches, mnMatchesInliers,
 * SearchLocalLines matches (every passing pair counts), mnLineMatchesInliers. */
int orbpl_tracker_get_local_stats(orbpl_tracker* tr, int* local_matches, int* local_inliers,
                                  int* local_line_matches, int* local_line_inliers);
/* LSD / LineExtractor kernel times (ms) of the last min(max_steps, 64) steps,
 * 7 per step (line stream): k_lsd_blur + k_lsd_resize + k_lsd_grad, the
 * pseudo-ordering sort (k_lsd_sort + k_lsd_sort_local), the seed loop
 * (k_lsd_spec), NFA validation + compaction, KeyLines (k_keylines), blur5 +
 * Sobel + LBD, UndistortKeyLines + line depths. */
int orbpl_tracker_lsd_timings(orbpl_tracker* tr, int max_steps, float* ms, int* n_steps);
/* Stereo stage device times (ms) of the last min(max_steps, 64) steps, 4 per
 * step: right-image ORB extraction, ComputeStereoMatches (KeyFrame::ComputeBoW
 * is the bow entry of orbpl_tracker_timings), and with
 * ORBPL_TRACK_LINES the right-image LineExtractor and the stereo line depths
 * (k_stereo_lines); 0 without lines. */
int orbpl_tracker_stereo_timings(orbpl_tracker* tr, int max_steps, float* ms, int* n_steps);

/* ------------------------------------------------------------------------
 * Line tracking, single frame, host pointers (n <= 80 = LineExtractor's cap)
 * ---------------------------------------------------------------------- */
/* Frame::UndistortKeyLines (Frame.cc:769-845) + the line part of
 * ComputeStereoFromRGBD (Frame.cc:1090-1116): undistorted key lines, depth
 * at the distorted end points (-1 = none; imDepth.at<float>(int(v), int(u))
 * on the row-major image) and uRight = x_un - bf / depth (-1 = none). depth
 * may be NULL (no depth: all -1). */
int orbpl_line_frame_prepare(const orbpl_camera* cam, const orbpl_keyline* kl, int n,
                             const float* depth, orbpl_keyline* kl_un, float* dstart, float* dend,
                             float* ur_start, float* ur_end);
/* LineMatcher(0.9, true).SearchByProjection(CurrentFrame, LastFrame)
 * (LineMatcher.cpp:72-269): last-frame map lines (has_ml, outlier flags,
 * world start/end xyz x6, LBD rows) projected with Tcw and Liang-Barsky
 * clipped to the image bounds; every (projected, current) pair passing
 * LineMatching counts, the last passing one wins; one relaxed retry when
 * matches / ncur < 0.2. match[j] = last-frame index or -1. */
int orbl_search_by_projection_last(const orbpl_camera* cam, const float* Tcw, int ncur,
                                   const orbpl_keyline* cur_kl_un, const uint8_t* cur_desc,
                                   int nlast, const orbpl_keyline* last_kl_un,
                                   const uint8_t* has_ml, const uint8_t* last_outlier,
                                   const float* ml_xyz6, const uint8_t* last_desc, int32_t* match,
                                   int* nmatches);

/* Frame::IsInFrustum(MapLine*) (Frame.cc:403-430): in_view unless both
 * world end points (xyz6 = start, end) are behind the camera. */
int orbl_frame_is_in_frustum(const float* Tcw, int n, const float* xyz6, uint8_t* in_view);
/* LineMatcher::SearchByProjection(F, vpLocalMapLines) (LineMatcher.cpp:755-952,
 * valid = mbTrackInView) and SearchByProjection(F, RefKF) (:527-721, valid =
 * mvpMapLines[i] != NULL): any number of map lines (world xyz6, LBD rows).
 * Current lines whose map line has Observations() > 0 (cur_nobs, NULL: none)
 * are skipped in the first pass. match[j] = map line index assigned to
 * current line j, -1 = unchanged; *wiped = 1 when the relaxed retry ran, which
 * first clears every F.mvpMapLines entry (-1 then means NULL). */
int orbl_search_by_projection_list(const orbpl_camera* cam, const float* Tcw, int ncur,
                                   const orbpl_keyline* cur_kl_un, const uint8_t* cur_desc,
                                   const int32_t* cur_nobs, int nml, const uint8_t* valid,
                                   const float* ml_xyz6, const uint8_t* ml_desc, int32_t* match,
                                   int* nmatches, int* wiped);
/* The reference's harness overloads, which also return new_kls (the
 * projected, clipped KeyLines, appended by the caller) and match_indices
 * (every passing (projected i, current j) pair; the relaxed retry clears
 * them): mode 0 = SearchByProjection(Frame&, const Frame&, new_kls,
 * match_indices) (include/LineMatcher.h:51, LineMatcher.cpp:272-487, called by
 * Test/LastFrameProjection.cpp:293): projected KeyLines are copies of
 * base_kl[i] (LastFrame.mvKeyLinesUn) rebuilt by UpdateKeyLineData,
 * Observations() > 0 is tested per pair on the map line current line j holds
 * at that moment (cur_nobs initially, ml_nobs of a map line a pass assigned),
 * retry when matches * 1.0 / NL < 0.2; mode 1 = SearchByProjection(Frame&,
 * const vector<MapLine*>&, new_kls, match_indices) (LineMatcher.h:66,
 * LineMatcher.cpp:954-1170, Test/LocalMapProjectionTest.cpp:334): fresh
 * (zeroed) KeyLines, the Observations() skip per current line, retry when
 * matches <= 0.2 NL. valid = mvpMapLines[i] && !mvbLineOutlier[i] && !isBad()
 * (mode 0) / mbTrackInView && !isBad() (mode 1). Outputs: proj_kl / proj_src
 * (nml capacity; *nproj), pairs as int (i, j) (pair_cap capacity; *npairs =
 * the full count), match[j] = map line assigned by the final pass or -1,
 * *wiped = 1 when the retry ran (every assignment cleared first). cur_nobs,
 * base_kl and ml_nobs may be NULL. (LineMatcher.h:59 declares a reference-
 * keyframe variant the reference never defines.) */
int orbl_search_by_projection_pairs(const orbpl_camera* cam, const float* Tcw, int mode, int ncur,
                                    const orbpl_keyline* cur_kl_un, const uint8_t* cur_desc,
                                    const int32_t* cur_nobs, int nml, const uint8_t* valid,
                                    const orbpl_keyline* base_kl, const float* ml_xyz6,
                                    const uint8_t* ml_desc, const int32_t* ml_nobs,
                                    orbpl_keyline* proj_kl, int32_t* proj_src, int* nproj,
                                    int32_t* pairs, int pair_cap, int* npairs, int32_t* match,
                                    int* nmatches, int* wiped);
/* SearchByProjection(Frame&, KeyFrame*, vector<MapLine*>& vpMapLineMatches)
 * (LineMatcher.h:56, LineMatcher.cpp:492-525): cv::BFMatcher(NORM_HAMMING)
 * knnMatch(keyframe line descriptors = queries, current line descriptors =
 * train, k = 2) and best / second < 0.75 (float): out[j] = the last query
 * whose best train line is j, or -1; *nmatches counts every passing query.
 * Ties go to the lower train index; a query with fewer than two train lines
 * has no match (pinned: the reference reads past the end). nq <= 256. */
int orbl_match_bf_knn(int nq, const uint8_t* qdesc, int nt, const uint8_t* tdesc, int32_t* out,
                      int* nmatches);

/* ------------------------------------------------------------------------
 * Hamming distance — ORBmatcher::DescriptorDistance (ORBmatcher.cc:2083-2103)
 * ---------------------------------------------------------------------- */
int orbpl_descriptor_distance(const uint8_t* a32, const uint8_t* b32);

/* ------------------------------------------------------------------------
 * Line features: LineExtractor::ExtractLineSegment (LineExtractor.cpp:12-74)
 *   LSDDetector::detect(img, keylines, 1, 1)   -> lsdx_detect*
 * One lsdx_ctx per (device, image geometry, max batch); asynchronous on its
 * own HIP stream.
 * ---------------------------------------------------------------------- */
typedef struct lsdx_ctx lsdx_ctx;

int lsdx_create(int width, int height, int max_batch, int device, lsdx_ctx** out);
int lsdx_destroy(lsdx_ctx* ctx);
/* LineSegmentDetector::detect (LSD_REFINE_ADV, scale 0.8) on one host image:
 * segments (x1, y1, x2, y2) in detection order. ORBPL_ERR_CAPACITY if more
 * than cap segments (n_out holds the count). */
int lsdx_detect(lsdx_ctx* ctx, const uint8_t* img, int width, int height, int stride,
                float* lines, int cap, int* n_out);
/* The same for `batch` device-resident frames (frame f at d_imgs + f*frame_pitch). */
int lsdx_detect_batch_device(lsdx_ctx* ctx, const uint8_t* d_imgs, int batch, int stride,
                             int64_t frame_pitch);
int lsdx_synchronize(lsdx_ctx* ctx);
/* LineExtractor::ExtractLineSegment(img, key_lines, line_descriptor,
 * keyline_coefficients) (LineExtractor.cpp:12-74): LSD, KeyLines sorted by
 * response and cut to the 80 longest when more were found, LBD descriptors
 * (32 bytes per row, rows follow the KeyLine order), normalised homogeneous
 * line coefficients (3 doubles per line). */
int lsdx_extract(lsdx_ctx* ctx, const uint8_t* img, int width, int height, int stride,
                 orbpl_keyline* keylines, uint8_t* desc, double* coef, int cap, int* n_out);
int lsdx_extract_batch_device(lsdx_ctx* ctx, const uint8_t* d_imgs, int batch, int stride,
                              int64_t frame_pitch);
int lsdx_get_keylines(lsdx_ctx* ctx, int frame, orbpl_keyline* keylines, uint8_t* desc,
                      double* coef, int cap, int* n_out);
/* Device buffers of the last extraction: frame f's lines start at
 * f*80 KeyLines / f*80*32 bytes / f*80*3 doubles; d_n[f] is the count. */
int lsdx_device_outputs(lsdx_ctx* ctx, orbpl_keyline** d_keylines, uint8_t** d_desc,
                        double** d_coef, int32_t** d_n);
int lsdx_get_lines(lsdx_ctx* ctx, int frame, float* lines, int cap, int* n_out);
/* Intermediate stages of the last run (parity tests): 0.8-scaled 8-bit image
 * (sw*sh), fastAtan2 degrees per pixel (-1 = NOTDEF), pseudo-ordered pixels
 * (x | y << 16, (sw-1)*(sh-1) entries). Any pointer may be NULL. */
int lsdx_get_stages(lsdx_ctx* ctx, int frame, uint8_t* scaled, float* deg, uint32_t* order,
                    int* sw, int* sh, int* n_order);
/* Test hook: the device replica of std::sort(records, key greater) on keys
 * in [0, 1023]; perm receives the record indices in sorted order. */
int orbpl_test_introsort(const int32_t* keys, int n, int32_t* perm);
/* Debug: batch-mean shader-clock counters of the LSD seed loop of the last
 * run. Speculative loop (default): growing cycles, rounds, speculative
 * regions, total cycles, fit + refinement cycles, validate + commit
 * cycles, critical-path grow steps | cooperative regions << 40, rectangles
 * passed to NFA validation. Wave-serial loop: growing cycles, fit +
 * refinement cycles, 0, total cycles, region pixels, prefetches, prefetch
 * cycles, rectangles. */
int lsdx_debug_profile(lsdx_ctx* ctx, long long* out8);
/* on != 0: run the wave-serial seed loop (one region at a time, the direct
 * restatement) instead of the speculative lane-parallel one. Both give the
 * same lines; the switch exists for testing and measurement. */
int lsdx_set_serial_grow(lsdx_ctx* ctx, int on);


#ifdef __cplusplus
}
#endif

#endif /* ORBPL_H */
