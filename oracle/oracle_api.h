// ORACLE — test infrastructure only (see orb_oracle.cpp header).
#pragma once
#include <stdint.h>
#include "../include/orbpl.h"  // ABI structs only (orbpl_keypoint, orbpl_orb_params)

#ifdef __cplusplus
extern "C" {
#endif
int oracle_orb_level_sizes(const orbpl_orb_params* p, int w, int h, int* lw, int* lh,
                           int* nfeat_per_level, float* scale, float* inv_scale);
int oracle_orb_pyramid(const orbpl_orb_params* p, const uint8_t* img, int w, int h, int stride,
                       uint8_t* out, int blurred);
int oracle_orb_candidates(const orbpl_orb_params* p, const uint8_t* img, int w, int h, int stride,
                          float* out_xyr, int cap, int* level_counts);
int oracle_orb_extract(const orbpl_orb_params* p, const uint8_t* img, int w, int h, int stride,
                       orbpl_keypoint* kps, uint8_t* desc, int cap, int* n_out, int* level_counts);
float oracle_fast_atan2(float y, float x);
int oracle_frame_prepare(const orbpl_camera* cam, const orbpl_keypoint* kps, int n,
                         const float* depth, orbpl_keypoint* kps_un, float* depth_out,
                         float* uright, int32_t* grid_cell, float* bounds);
int oracle_search_by_projection_last(const orbpl_camera* cam, const float* scale_factors,
                                     int nlevels, const orbpl_match_current* cur,
                                     const orbpl_match_last* last, float th, int mono,
                                     int check_ori, int32_t* match, int* nmatches_out);
int oracle_frame_is_in_frustum(const orbpl_camera* cam, float log_scale_factor, int nlevels,
                               const float* Tcw, int n, const float* xyz, const float* normal,
                               const float* min_dist, const float* max_dist, float view_cos_limit,
                               uint8_t* in_view, float* proj_x, float* proj_y, float* proj_xr,
                               int32_t* level, float* view_cos);
int oracle_search_by_projection_local(const orbpl_camera* cam, const float* scale_factors,
                                      int nlevels, const orbpl_match_current* cur, int nmp,
                                      const uint8_t* in_view, const float* proj_x,
                                      const float* proj_y, const float* proj_xr,
                                      const int32_t* level, const float* view_cos,
                                      const uint8_t* mp_desc, const int32_t* mp_nobs,
                                      const int32_t* cur_nobs, float th, float nnratio,
                                      int32_t* match, int* nmatches_out);
/* DBoW2 vocabulary (bow_oracle.cpp) */
void* oracle_voc_load_text(const char* path);
int oracle_voc_transform(void* h, const uint8_t* desc, int n, int levelsup, uint32_t* bow_words,
                         double* bow_vals, int* bow_n, int32_t* feat_node, int32_t* feat_word,
                         double* feat_weight);
int oracle_search_by_bow(int nkf, const int32_t* kf_node, const uint8_t* kf_valid,
                         const uint8_t* kf_desc, const float* kf_angle, int nf,
                         const int32_t* f_node, const uint8_t* f_desc, const float* f_angle,
                         float nnratio, int check_ori, int32_t* match, int* nmatches_out);
int oracle_stereo_matches(const orbpl_camera* cam, const float* scale, const float* inv_scale,
                          int nlevels, const int32_t* lw, const int32_t* lh, const uint8_t* pyrL,
                          const uint8_t* pyrR, const orbpl_keypoint* kl, const uint8_t* dl, int n,
                          const orbpl_keypoint* kr, const uint8_t* dr, int nr, float* uright,
                          float* depth);
int oracle_pose_optimization(const orbpl_camera* cam, const orbpl_pose_problem* P, float* Tcw,
                             uint8_t* outlier, uint8_t* line_outlier, int* n_inliers);
/* flags: ORBPL_POSE_FIXED_LINE_JAC (orbpl.h) = analytic line Jacobian */
int oracle_pose_optimization_ex(const orbpl_camera* cam, const orbpl_pose_problem* P, int flags,
                                float* Tcw, uint8_t* outlier, uint8_t* line_outlier,
                                int* n_inliers);
void* oracle_vo_create(const orbpl_orb_params* orb, const orbpl_camera* cam, int n_streams);
void oracle_vo_destroy(void* h);
int oracle_vo_reset(void* h, const float* Tcw0);
int oracle_vo_step(void* h, int stream, const uint8_t* gray, const float* depth, float* Tcw_out,
                   int* out5);
/* line features (lsd_oracle.cpp) */
int oracle_lsd_traffic(const uint8_t* img, int W, int H, long long* out18);
int oracle_lsd_detect(const uint8_t* img, int W, int H, float* lines, int cap, int* n_out);
int oracle_lsd_stages(const uint8_t* img, int W, int H, uint8_t* scaled, double* angles,
                      uint32_t* order, int* sw, int* sh, int* n_order);
int oracle_line_extract(const uint8_t* img, int W, int H, orbpl_keyline* kl_out, uint8_t* desc,
                        double* coef, int cap, int* n_out, int* n_detected);
double oracle_lsdm(int fn, double x, double y);
int oracle_math_probe(int on);
int oracle_math_probe_read(long long* calls, long long* differ, long long* max_ulp);
int oracle_line_iterator_count(int W, int H, float x1, float y1, float x2, float y2);
int oracle_introsort_perm(const int* keys, int n, int* perm);
/* line tracking (line_track_oracle.cpp) */
void oracle_undistort_point(const orbpl_camera* c, float px, float py, float* ox, float* oy);
void oracle_image_bounds(const orbpl_camera* c, float* b4);
int oracle_line_frame_prepare(const orbpl_camera* cam, const orbpl_keyline* kl, int nl,
                              const float* depth, orbpl_keyline* kl_un, float* dstart, float* dend,
                              float* ur_start, float* ur_end);
int oracle_line_search_by_projection_last(const orbpl_camera* cam, const float* Tcw, int ncur,
                                          const orbpl_keyline* cur_kl_un, const uint8_t* cur_desc,
                                          int nlast, const orbpl_keyline* last_kl_un,
                                          const uint8_t* has_ml, const uint8_t* last_outlier,
                                          const float* ml_xyz6, const uint8_t* last_desc,
                                          int32_t* match, int* nmatches_out);
int oracle_line_search_by_projection_list(const orbpl_camera* cam, const float* Tcw, int ncur,
                                          const orbpl_keyline* cur_kl_un, const uint8_t* cur_desc,
                                          const int32_t* cur_nobs, int nml, const uint8_t* valid,
                                          const float* ml_xyz6, const uint8_t* ml_desc,
                                          int32_t* match, int* nmatches_out, int* wiped);
int oracle_line_search_pairs(const orbpl_camera* cam, const float* Tcw, int mode, int ncur,
                             const orbpl_keyline* cur_kl_un, const uint8_t* cur_desc,
                             const int32_t* cur_nobs, int nml, const uint8_t* valid,
                             const orbpl_keyline* base_kl, const float* ml_xyz6,
                             const uint8_t* ml_desc, const int32_t* ml_nobs,
                             orbpl_keyline* proj_kl, int32_t* proj_src, int* nproj,
                             int32_t* pairs, int pair_cap, int* npairs, int32_t* match,
                             int* nmatches_out, int* wiped);
int oracle_line_match_bf_knn(int nq, const uint8_t* qdesc, int nt, const uint8_t* tdesc,
                             int32_t* out, int* nmatches_out);
int oracle_stereo_line_depths(const orbpl_camera* cam, const orbpl_keyline* kl,
                              const uint8_t* desc, int nl, const orbpl_keyline* kr,
                              const uint8_t* desc_r, int nr, float* dstart, float* dend);
int oracle_line_is_in_frustum(const float* Tcw, int n, const float* xyz6, uint8_t* in_view);
void* oracle_lvo_create(const orbpl_orb_params* orb, const orbpl_camera* cam, int n_streams,
                        int use_lines);
/* flags: ORBPL_TRACK_* bits (orbpl.h) | 1 << 16 (ORB || lines on two host threads) */
void* oracle_lvo_create_ex(const orbpl_orb_params* orb, const orbpl_camera* cam, int n_streams,
                           int flags);
void oracle_lvo_destroy(void* h);
int oracle_lvo_reset(void* h, const float* Tcw0);
int oracle_lvo_step(void* h, int stream, const uint8_t* gray, const float* depth, float* Tcw_out,
                    int* out8);
int oracle_lvo_local_stats(void* h, int stream, int* out4);
int oracle_lvo_step_stereo(void* h, int stream, const uint8_t* left, const uint8_t* right,
                           float* Tcw_out, int* out8);
/* Tracking::Track with the map model (map_oracle.cpp) */
void* oracle_map_create(const orbpl_orb_params* orb, const orbpl_camera* cam, int n_streams,
                        int flags);
void oracle_map_destroy(void* h);
int oracle_map_reset(void* h, const float* Tcw0);
int oracle_map_clear_velocity(void* h, int stream);
int oracle_map_step_stereo(void* h, int stream, const uint8_t* left, const uint8_t* right,
                           float* Tcw_out, int* out24);
int oracle_map_set_fps(void* h, float fps);
/* the last step's stage times (ms): ORB, LineExtractor, join wait, whole step */
int oracle_map_stage_times(void* h, double* out4);
int oracle_map_set_vocabulary(void* h, void* voc);
int oracle_map_step(void* h, int stream, const uint8_t* gray, const float* depth, float* Tcw_out,
                    int* out24);
int oracle_map_keyframes(void* h, int stream, int* parent, int* ord, int cap, int* nord);
int oracle_map_points(void* h, int stream, int* nobs, uint8_t* desc, float* xyz, int cap);
int oracle_map_points_geom(void* h, int stream, float* nrm, float* dist2, int cap);
int oracle_map_lines(void* h, int stream, int* nobs, uint8_t* desc, float* pos6, int cap);
#ifdef __cplusplus
}
#endif
