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
#ifdef __cplusplus
}
#endif
