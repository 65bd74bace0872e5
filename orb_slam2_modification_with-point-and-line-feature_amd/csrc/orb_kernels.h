// Kernel launchers of the ORB extraction pipeline (orb_extract.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <vector>

#include "orb_geom.h"

namespace orbpl {

// Device-side mirror of orbpl_keypoint / cv::KeyPoint (28 bytes).
struct orbpl_keypoint_dev {
  float x, y, size, angle, response;
  int octave, class_id;
};

hipError_t upload_pattern(hipStream_t s);
// debug: k_octree phase ticks per level of frame 0 (ORBPL_OCT_PROFILE)
int read_octree_profile(long long* out128);
int read_od_profile(long long* out8);

// Padded pyramid + borders + blurred levels [l0, l1) of `batch` frames
// (k_pyramid; level l0 > 0 reads level l0 - 1 of an earlier launch);
// bands = the nbands-band partition (pyr_band_base(nbands) in the table).
void launch_pyramid(const OrbGeom& hg, const OrbGeom* dg, const uint8_t* img, int stride,
                    long long frame_pitch, uint8_t* pyr, uint8_t* blur, const int* rs,
                    const PyrBand* bands, int nbands, int batch, long long* prof, int l0, int l1,
                    hipStream_t s);
// FAST cells of levels [l0, l1)
void launch_fast(const OrbGeom& hg, const OrbGeom* dg, const CellGeom* cells, const uint8_t* pyr,
                 uint32_t* cell_cands, int* cell_counts, int ini_th, int min_th, int batch,
                 int l0, int l1, hipStream_t s);
void launch_octree(const OrbGeom& hg, const OrbGeom* dg, const uint32_t* cell_cands,
                   const int* cell_counts, uint32_t* kcand, int* knode, uint32_t* kp_list,
                   int* kp_count, int* err_flag, int batch, int l0, int l1, hipStream_t s);
void launch_orient_desc(const OrbGeom& hg, const OrbGeom* dg, const uint8_t* pyr,
                        const uint8_t* blur, const uint32_t* kp_list, const int* kp_count,
                        orbpl_keypoint_dev* out_kps, uint8_t* out_desc, int kp_pitch, int* out_n,
                        int batch, int l0, int l1, hipStream_t s);

// Host geometry (orb_geom.cpp). Returns 0 or an ORBPL_ERR_* code with a
// message in *err.
struct OrbHostGeom {
  OrbGeom g;
  std::vector<CellGeom> cells;
  std::vector<int> rs;           // resize tables for all levels >= 1
  std::vector<PyrBand> bands;    // k_pyramid row bands for B = 1, 2, 4, 8 (15 entries)
  std::vector<float> scale, inv_scale, sigma2, inv_sigma2;
};
int build_orb_geometry(int nfeatures, float scale_factor, int nlevels, int W, int H,
                       OrbHostGeom* out, const char** err);

}  // namespace orbpl
