// Geometry shared by the host runtime and the ORB kernels. Computed once per
// extractor configuration on the host (orb_geom.cpp) with the reference's
// formulas (ORBextractor.cc:410-470, 765-847, 1107-1132) and uploaded.
#pragma once
#include <stdint.h>

namespace orbpl {

constexpr int kMaxLevels = 16;
constexpr int kEdge = 19;          // EDGE_THRESHOLD (ORBextractor.cc:74)
constexpr int kMinBorder = 16;     // EDGE_THRESHOLD - 3 (ORBextractor.cc:773)
// Padded row py of a level starts kLead bytes into its pitch, so that content
// column 0 (padded column 19) sits at byte 32: content rows are 16-B aligned.
constexpr int kLead = 13;
constexpr int kContent0 = kLead + 19;  // = 32
constexpr int kOctMaxList = 1024;  // octree list capacity per (frame, level)
constexpr int kMaxCandPerLevel = (1 << 20) - 1;

struct LevelGeom {
  int w, h;            // content size
  int pw, ph;          // padded size (w + 38, h + 38)
  int pitch;           // padded row pitch in bytes (multiple of 16)
  int pad0;
  long long pyr_off;   // byte offset of the padded level inside one frame's pyramid
  float scale;         // mvScaleFactor[level]
  int nfeat;           // mnFeaturesPerLevel[level]
  int ncols, nrows;    // FAST cell grid (ORBextractor.cc:784-785)
  int wcell, hcell;    // cell size (ORBextractor.cc:786-787)
  int cell_base;       // first cell index of this level in the frame's cell array
  int ncells;          // ncols * nrows
  int max_border_x, max_border_y;  // cols-16, rows-16 (ORBextractor.cc:775-776)
  int n_ini;           // DistributeOctTree initial nodes (ORBextractor.cc:543)
  float hx;            // initial node width (ORBextractor.cc:545)
  int kp_cap;          // keypoint list capacity for this level
  int kp_base;         // offset of this level's list in the frame's list array
  int cand_base;       // offset in the frame's compacted-candidate scratch
  int cand_cap;        // ncells * cell_slots
  int rs_off;          // offset of the resize tables (levels >= 1) in ints
  int xmax;            // first dx whose sx + 1 >= src width (OpenCV resize)
  int scaled_patch;    // (int)(PATCH_SIZE * scale)  (ORBextractor.cc:837)
  int pad2, pad3;
  int bpitch;          // blurred level row pitch (content only, multiple of 16)
  int pad1;
  long long boff;      // byte offset of the blurred level inside one frame's blurred buffer
};

// One FAST window (ORBextractor.cc:789-806): [x0,x1) x [y0,y1) in level
// content coordinates; level index; x1 == 0 marks a skipped cell.
struct CellGeom {
  int16_t x0, y0, x1, y1;
  int16_t level, pad;
};

struct OrbGeom {
  int nlevels;
  int W, H;
  int ncells_total;
  int kp_cap_total;    // sum of kp_cap (per-frame list array size)
  int cand_cap_total;  // sum of cand_cap
  int cell_slots;      // max corners a FAST window can emit: ceil(dw/2)*ceil(dh/2)
  int fast_win_w;      // largest FAST window (x1 - x0) over all cells
  int fast_win_h;      // largest FAST window (y1 - y0)
  long long pyr_bytes; // bytes of one frame's padded pyramid
  long long blur_bytes;  // bytes of one frame's blurred (content-only) pyramid
  int umax[16];        // IC_Angle circular patch row extents (ORBextractor.cc:454-469)
  LevelGeom lv[kMaxLevels];
};

// k_pyramid (fused pyramid + borders + blur): one block per (row band,
// frame). Band b owns content rows [oa, ob) of every level and computes rows
// [na, nb) (own rows plus the halo that the blur and the next level read).
#ifndef ORBPL_PYR_THREADS
#define ORBPL_PYR_THREADS 256
#endif
constexpr int kPyrThreads = ORBPL_PYR_THREADS;   // k_pyramid block (A/B builds override)
constexpr int kPyrMaxBands = 8;      // bands for B = 1, 2, 4, 8 are precomputed
struct PyrBand {
  int na[kMaxLevels], nb[kMaxLevels];
  int oa[kMaxLevels], ob[kMaxLevels];
};
// index of the first band of the B-band partition in the band table
__host__ __device__ inline int pyr_band_base(int B) { return B - 1; }

// Byte offsets (within one frame's padded pyramid) of a content pixel and of
// a padded pixel.
__host__ __device__ inline long long content_off(const LevelGeom& L, int x, int y) {
  return L.pyr_off + (long long)(y + kEdge) * L.pitch + kContent0 + x;
}
__host__ __device__ inline long long padded_off(const LevelGeom& L, int px, int py) {
  return L.pyr_off + (long long)py * L.pitch + kLead + px;
}

// Candidate packing: x (12 bits) | y (12 bits) << 12 | score (8 bits) << 24,
// coordinates relative to minBorder (the reference's vToDistributeKeys frame).
__host__ __device__ inline uint32_t pack_cand(int x, int y, int s) {
  return (uint32_t)x | ((uint32_t)y << 12) | ((uint32_t)s << 24);
}
__host__ __device__ inline int cand_x(uint32_t c) { return (int)(c & 0xFFF); }
__host__ __device__ inline int cand_y(uint32_t c) { return (int)((c >> 12) & 0xFFF); }
__host__ __device__ inline int cand_s(uint32_t c) { return (int)(c >> 24); }

}  // namespace orbpl
