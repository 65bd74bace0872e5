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
/* Library build tag (e.g. "orbpl gfx950 r1"). */
const char* orbpl_version(void);

/* Device memory plumbing for hosts without their own GPU allocator (the
 * reference's C++ Tracking, ctypes tests, bench). Synchronous copies. */
int orbpl_dev_malloc(int device, int64_t bytes, void** out);
int orbpl_dev_free(int device, void* ptr);
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

/* ------------------------------------------------------------------------
 * Hamming distance — ORBmatcher::DescriptorDistance (ORBmatcher.cc:2083-2103)
 * ---------------------------------------------------------------------- */
int orbpl_descriptor_distance(const uint8_t* a32, const uint8_t* b32);

#ifdef __cplusplus
}
#endif

#endif /* ORBPL_H */
