// ============================================================================
// ORACLE — TEST INFRASTRUCTURE ONLY. NOT PART OF THE PRODUCT PATH.
//
// CPU restatement of the reference's per-frame line tracking:
//   Frame::UndistortKeyLines            /root/reference/src/Frame.cc:769-845
//   Frame::ComputeStereoFromRGBD (lines) Frame.cc:1090-1116
//   LineMatcher::SearchByProjection(Frame&, const Frame&)  LineMatcher.cpp:72-269
//     LiangBarsky :1389-1460, LineMatching :1463-1504, LineOverLap :1508-1559,
//     ReprojectionError :1579-1596, UpdateKeyLineData :1601-1624,
//     DescriptorDistance :20-39, thresholds LineMatcher.h:94-98
//   Frame::UnprojectStereoLineStart/End  Frame.cc:1176-1204 (the end point uses
//     mvDepthLineStart, as the reference does)
// Pinned semantics as in lsd_oracle.cpp (P2, P10-P12) plus:
//   P14 depth lookups imDepth.at<float>(int(v), int(u)) read the row-major
//       buffer at v*W + u; an index outside [0, W*H) reads as no depth.
// ============================================================================
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

#include "pinned_math.h"
#include "oracle_api.h"

namespace line_track {

static int popcnt_dist(const uint8_t* a, const uint8_t* b) {
  int d = 0;
  for (int i = 0; i < 32; i++) d += __builtin_popcount((unsigned)(a[i] ^ b[i]));
  return d;
}

static float atan2f_pinned(float y, float x) { return (float)pmath::atan2_((double)y, (double)x); }

// fields recomputed from the end points (UpdateKeyLineData / UndistortKeyLines)
static void refresh_keyline(orbpl_keyline& kl, int W, int H) {
  kl.pt_x = (kl.endPointX + kl.startPointX) / 2;
  kl.pt_y = (kl.endPointY + kl.startPointY) / 2;
  const double dx = (double)(kl.startPointX - kl.endPointX), dy = (double)(kl.startPointY - kl.endPointY);
  kl.lineLength = float(std::sqrt(dx * dx + dy * dy));
  kl.numOfPixels = oracle_line_iterator_count(W, H, kl.startPointX, kl.startPointY, kl.endPointX,
                                              kl.endPointY);
  kl.angle = atan2f_pinned(kl.endPointY - kl.startPointY, kl.endPointX - kl.startPointX);
  kl.size = (kl.endPointX - kl.startPointX) * (kl.endPointY - kl.startPointY);
  kl.response = kl.lineLength / (float)std::max(W, H);
}

static bool liang_barsky(const double line[4], double out[4], const float bounds[4]) {
  const double sx = line[0], sy = line[1], ex = line[2], ey = line[3];
  double p[4], q[4];
  p[0] = sx - ex;
  p[1] = ex - sx;
  p[2] = sy - ey;
  p[3] = ey - sy;
  q[0] = sx - bounds[0];
  q[1] = bounds[2] - sx;
  q[2] = sy - bounds[1];
  q[3] = bounds[3] - sy;
  if (p[0] == 0) {
    if (q[0] <= 0 || q[2] <= 0) return false;
  }
  if (p[2] == 0) {
    if (q[2] >= 0 || q[3] >= 0) return false;
  }
  double u[4];
  for (int i = 0; i < 4; i++) u[i] = q[i] / p[i];
  double u_min = 0, u_max = 1;
  for (int i = 0; i < 4; i++) {
    if (p[i] < 0) {
      if (u_min < u[i]) u_min = u[i];
    } else {
      if (u_max > u[i]) u_max = u[i];
    }
  }
  if (u_max >= u_min) {
    out[0] = sx + std::round(u_min * (ex - sx));
    out[1] = sy + std::round(u_min * (ey - sy));
    out[2] = sx + std::round(u_max * (ex - sx));
    out[3] = sy + std::round(u_max * (ey - sy));
    return true;
  }
  return false;
}

static bool line_overlap(const orbpl_keyline& a, const orbpl_keyline& b, double th) {
  const double d1_x = std::abs(a.startPointX - a.endPointX);
  const double d2_x = std::abs(b.startPointX - b.endPointX);
  const double min_x = std::min(std::min(a.startPointX, a.endPointX), std::min(b.startPointX, b.endPointX));
  const double max_x = std::max(std::max(a.startPointX, a.endPointX), std::max(b.startPointX, b.endPointX));
  const double d1_y = std::abs(a.startPointY - a.endPointY);
  const double d2_y = std::abs(b.startPointY - b.endPointY);
  const double min_y = std::min(std::min(a.startPointY, a.endPointY), std::min(b.startPointY, b.endPointY));
  const double max_y = std::max(std::max(a.startPointY, a.endPointY), std::max(b.startPointY, b.endPointY));
  if (d1_x == 0 || d2_x == 0) {
    if ((d1_y + d2_y - max_y + min_y) / std::min(d1_y, d2_y) >= th) return true;
  }
  if (d1_y == 0 || d2_y == 0) {
    if ((d1_x + d2_x - max_x + min_x) / std::min(d1_x, d2_x) >= th) return true;
  }
  if ((d1_x + d2_x - max_x + min_x) / std::min(d1_x, d2_x) >= th) {
    if (d1_y + d2_y + min_y >= max_y) return true;
    if (max_y - min_y - d1_y - d2_y < 0.3 * std::min(d1_y, d2_y)) return true;
  } else if ((d1_x + d2_x - max_x + min_x) / std::min(d1_x, d2_x) < th &&
             (max_x - min_x - d1_x - d2_x) < 0.3 * std::min(d1_x, d2_x)) {
    if ((d1_y + d2_y - max_y + min_y) / std::min(d1_y, d2_y) >= th) return true;
  }
  return false;
}

static double reprojection_error(const orbpl_keyline& l1, const orbpl_keyline& l2) {
  const double s1[3] = {l1.startPointX, l1.startPointY, 1}, e1[3] = {l1.endPointX, l1.endPointY, 1};
  const double c0 = s1[1] * e1[2] - s1[2] * e1[1];
  const double c1 = s1[2] * e1[0] - s1[0] * e1[2];
  const double c2 = s1[0] * e1[1] - s1[1] * e1[0];
  const double nrm = std::sqrt(c0 * c0 + c1 * c1);
  const double ds = (l2.startPointX * c0 + l2.startPointY * c1 + 1.0 * c2) / nrm;
  const double de = (l2.endPointX * c0 + l2.endPointY * c1 + 1.0 * c2) / nrm;
  return std::sqrt(ds * ds + de * de);
}

static bool line_matching(const orbpl_keyline& k1, const orbpl_keyline& k2, const uint8_t* d1,
                          const uint8_t* d2, const double off[5]) {
  const double kPi = 3.14159265358979323846;
  if (popcnt_dist(d1, d2) > 45 + off[3]) return false;
  if (std::abs(k1.angle - k2.angle) > 15.0 * kPi / 180.0 + off[0] * kPi / 180.0) return false;
  if (std::min(k1.lineLength, k2.lineLength) / std::max(k1.lineLength, k2.lineLength) < 0.45 + off[1])
    return false;
  if (!line_overlap(k1, k2, 0.5 + off[2])) return false;
  if (reprojection_error(k1, k2) > 45) return false;
  return true;
}

}  // namespace line_track

using namespace line_track;

extern "C" {

// UndistortKeyLines + ComputeStereoFromRGBD for the lines of one frame.
int oracle_line_frame_prepare(const orbpl_camera* cam, const orbpl_keyline* kl, int nl,
                              const float* depth, orbpl_keyline* kl_un, float* dstart, float* dend,
                              float* ur_start, float* ur_end) {
  const int W = cam->width, H = cam->height;
  for (int i = 0; i < nl; i++) {
    orbpl_keyline k = kl[i];
    if (cam->k1 != 0.0f) {
      float x, y;
      oracle_undistort_point(cam, kl[i].startPointX, kl[i].startPointY, &x, &y);
      k.startPointX = x;
      k.startPointY = y;
      oracle_undistort_point(cam, kl[i].endPointX, kl[i].endPointY, &x, &y);
      k.endPointX = x;
      k.endPointY = y;
      k.sPointInOctaveX = k.startPointX;
      k.sPointInOctaveY = k.startPointY;
      k.ePointInOctaveX = k.endPointX;
      k.ePointInOctaveY = k.endPointY;
      refresh_keyline(k, W, H);
    }
    kl_un[i] = k;
    dstart[i] = dend[i] = ur_start[i] = ur_end[i] = -1;
    if (!depth) continue;
    auto at = [&](float v, float u) -> float {
      const long long idx = (long long)(int)v * W + (int)u;
      return (idx >= 0 && idx < (long long)W * H) ? depth[idx] : 0.f;
    };
    const float ds = at(kl[i].startPointY, kl[i].startPointX);
    const float de = at(kl[i].endPointY, kl[i].endPointX);
    if (ds > 0) {
      dstart[i] = ds;
      ur_start[i] = k.startPointX - cam->bf / ds;
    }
    if (de > 0) {
      dend[i] = de;
      ur_end[i] = k.endPointX - cam->bf / de;
    }
  }
  return 0;
}

}  // extern "C"

namespace line_track {
// The LineMatcher::SearchByProjection overloads share one body
// (LineMatcher.cpp:72-269 last frame, :527-721 reference keyframe, :755-952
// local map): map lines `valid` are projected with Tcw, clipped
// (LiangBarsky) and rebuilt (UpdateKeyLineData on a copy of base_kl[i], or on
// a default KeyLine when base_kl is NULL - every field LineMatching reads is
// rewritten); current lines whose map line has Observations() > 0 are skipped
// in the first pass; every passing pair counts, the last passing map line
// wins; if matches / ncur < 0.2 all assignments are wiped (*wiped = 1) and the
// relaxed pass runs.
static int line_search_core(const orbpl_camera* cam, const float* Tcw, int ncur,
                            const orbpl_keyline* cur_kl_un, const uint8_t* cur_desc,
                            const int32_t* cur_nobs, int nlast, const uint8_t* valid,
                            const orbpl_keyline* base_kl, const float* ml_xyz6,
                            const uint8_t* last_desc, int32_t* match, int* nmatches_out,
                            int* wiped) {
  const int W = cam->width, H = cam->height;
  double T[12];
  for (int r = 0; r < 3; r++)
    for (int c = 0; c < 4; c++) T[r * 4 + c] = Tcw[r * 4 + c];
  float b4[4];
  oracle_image_bounds(cam, b4);  // minX, maxX, minY, maxY
  const float bounds[4] = {b4[0], b4[2], b4[1], b4[3]};
  std::vector<orbpl_keyline> nk;
  std::vector<int> nidx;
  auto xform = [&](const double* X, double* o) {
    for (int r = 0; r < 3; r++) o[r] = (T[r * 4] * X[0] + T[r * 4 + 1] * X[1] + T[r * 4 + 2] * X[2]) + T[r * 4 + 3];
  };
  for (int i = 0; i < nlast; i++) {
    if (!valid[i]) continue;
    const double Xs[3] = {ml_xyz6[6 * i], ml_xyz6[6 * i + 1], ml_xyz6[6 * i + 2]};
    const double Xe[3] = {ml_xyz6[6 * i + 3], ml_xyz6[6 * i + 4], ml_xyz6[6 * i + 5]};
    double cs[3], ce[3];
    xform(Xs, cs);
    xform(Xe, ce);
    if (cs[2] < 0 && ce[2] < 0) continue;
    double lp[4];
    bool have = false;
    if (cs[2] < 0.0 || ce[2] < 0.0) {
      const double lambda = -1.0 * cs[2] / (cs[2] - ce[2]);
      const double xc = cs[0] + lambda * (cs[0] - ce[0]);
      const double yc = cs[1] + lambda * (cs[1] - ce[1]);
      if (cs[2] < 0.0) {
        const float u_end = cam->fx * ce[0] / ce[2] + cam->cx;
        const float v_end = cam->fy * ce[1] / ce[2] + cam->cy;
        lp[0] = xc; lp[1] = yc; lp[2] = u_end; lp[3] = v_end;
      } else {
        const float u_start = cam->fx * cs[0] / cs[2] + cam->cx;
        const float v_start = cam->fy * cs[1] / cs[2] + cam->cy;
        lp[0] = u_start; lp[1] = v_start; lp[2] = xc; lp[3] = yc;
      }
      have = true;
    }
    if (cs[2] > 0.0 && ce[2] > 0.0) {
      const float u_start = cam->fx * cs[0] / cs[2] + cam->cx;
      const float v_start = cam->fy * cs[1] / cs[2] + cam->cy;
      const float u_end = cam->fx * ce[0] / ce[2] + cam->cx;
      const float v_end = cam->fy * ce[1] / ce[2] + cam->cy;
      lp[0] = u_start; lp[1] = v_start; lp[2] = u_end; lp[3] = v_end;
      have = true;
    }
    if (!have) continue;
    double nl4[4];
    if (!liang_barsky(lp, nl4, bounds)) continue;
    orbpl_keyline k{};
    if (base_kl) k = base_kl[i];
    k.startPointX = (float)nl4[0];
    k.startPointY = (float)nl4[1];
    k.endPointX = (float)nl4[2];
    k.endPointY = (float)nl4[3];
    k.sPointInOctaveX = (float)nl4[0];
    k.sPointInOctaveY = (float)nl4[1];
    k.ePointInOctaveX = (float)nl4[2];
    k.ePointInOctaveY = (float)nl4[3];
    refresh_keyline(k, W, H);
    nk.push_back(k);
    nidx.push_back(i);
  }
  auto run = [&](const double off[5], bool skip) {
    int cnt = 0;
    for (int j = 0; j < ncur; j++) {
      match[j] = -1;
      if (skip && cur_nobs && cur_nobs[j] > 0) continue;
      for (size_t i = 0; i < nk.size(); i++)
        if (line_matching(nk[i], cur_kl_un[j], last_desc + 32 * nidx[i], cur_desc + 32 * j, off)) {
          match[j] = nidx[i];
          cnt++;
        }
    }
    return cnt;
  };
  const double off0[5] = {0, 0, 0, 0, 0};
  int n = run(off0, true);
  if (wiped) *wiped = 0;
  if (n * 1.0 / ncur < 0.2) {
    const double off1[5] = {10.0, -0.1, -0.1, 5, 10};
    n = run(off1, false);
    if (wiped) *wiped = 1;
  }
  *nmatches_out = n;
  return 0;
}
}  // namespace line_track

namespace line_track {
// The projection + clipping + KeyLine rebuild of line_search_core, alone
// (projected KeyLines in map-line order and their map-line index).
static void project_lines(const orbpl_camera* cam, const float* Tcw, int nml, const uint8_t* valid,
                          const orbpl_keyline* base_kl, const float* ml_xyz6,
                          std::vector<orbpl_keyline>& nk, std::vector<int>& nidx) {
  const int W = cam->width, H = cam->height;
  double T[12];
  for (int r = 0; r < 3; r++)
    for (int c = 0; c < 4; c++) T[r * 4 + c] = Tcw[r * 4 + c];
  float b4[4];
  oracle_image_bounds(cam, b4);
  const float bounds[4] = {b4[0], b4[2], b4[1], b4[3]};
  for (int i = 0; i < nml; i++) {
    if (!valid[i]) continue;
    double cs[3], ce[3];
    for (int r = 0; r < 3; r++) {
      cs[r] = (T[r * 4] * (double)ml_xyz6[6 * i] + T[r * 4 + 1] * (double)ml_xyz6[6 * i + 1] +
               T[r * 4 + 2] * (double)ml_xyz6[6 * i + 2]) + T[r * 4 + 3];
      ce[r] = (T[r * 4] * (double)ml_xyz6[6 * i + 3] + T[r * 4 + 1] * (double)ml_xyz6[6 * i + 4] +
               T[r * 4 + 2] * (double)ml_xyz6[6 * i + 5]) + T[r * 4 + 3];
    }
    if (cs[2] < 0 && ce[2] < 0) continue;
    double lp[4];
    bool have = false;
    if (cs[2] < 0.0 || ce[2] < 0.0) {
      const double lambda = -1.0 * cs[2] / (cs[2] - ce[2]);
      const double xc = cs[0] + lambda * (cs[0] - ce[0]);
      const double yc = cs[1] + lambda * (cs[1] - ce[1]);
      if (cs[2] < 0.0) {
        const float u_end = cam->fx * ce[0] / ce[2] + cam->cx;
        const float v_end = cam->fy * ce[1] / ce[2] + cam->cy;
        lp[0] = xc; lp[1] = yc; lp[2] = u_end; lp[3] = v_end;
      } else {
        const float u_start = cam->fx * cs[0] / cs[2] + cam->cx;
        const float v_start = cam->fy * cs[1] / cs[2] + cam->cy;
        lp[0] = u_start; lp[1] = v_start; lp[2] = xc; lp[3] = yc;
      }
      have = true;
    }
    if (cs[2] > 0.0 && ce[2] > 0.0) {
      const float u_start = cam->fx * cs[0] / cs[2] + cam->cx;
      const float v_start = cam->fy * cs[1] / cs[2] + cam->cy;
      const float u_end = cam->fx * ce[0] / ce[2] + cam->cx;
      const float v_end = cam->fy * ce[1] / ce[2] + cam->cy;
      lp[0] = u_start; lp[1] = v_start; lp[2] = u_end; lp[3] = v_end;
      have = true;
    }
    if (!have) continue;
    double nl4[4];
    if (!liang_barsky(lp, nl4, bounds)) continue;
    orbpl_keyline k{};
    if (base_kl) k = base_kl[i];
    k.startPointX = (float)nl4[0];
    k.startPointY = (float)nl4[1];
    k.endPointX = (float)nl4[2];
    k.endPointY = (float)nl4[3];
    k.sPointInOctaveX = (float)nl4[0];
    k.sPointInOctaveY = (float)nl4[1];
    k.ePointInOctaveX = (float)nl4[2];
    k.ePointInOctaveY = (float)nl4[3];
    refresh_keyline(k, W, H);
    nk.push_back(k);
    nidx.push_back(i);
  }
}
}  // namespace line_track

extern "C" {

// The reference's two defined harness overloads of SearchByProjection (the
// ones its Test/ demos call), which also return the projected KeyLines
// (new_kls, appended) and every passing (projected index, current index) pair
// (match_indices, cleared by the relaxed retry):
//   mode 0: (Frame&, const Frame&, new_kls, match_indices), LineMatcher.cpp:
//     272-487 (Test/LastFrameProjection.cpp:293): projected KeyLines are copies
//     of the last frame's (base_kl) rebuilt by UpdateKeyLineData; the
//     Observations() > 0 skip is tested per PAIR, on the map line the current
//     line holds at that moment (cur_nobs initially, then ml_nobs of the map
//     line a pass assigned); retry when matches * 1.0 / NL < 0.2;
//   mode 1: (Frame&, const vector<MapLine*>&, new_kls, match_indices), :954-
//     1170 (Test/LocalMapProjectionTest.cpp:334): fresh KeyLines (pinned to
//     zero-initialised fields before UpdateKeyLineData, base_kl ignored); the
//     skip is tested once per current line, before its pairs; retry when
//     matches <= 0.2 * NL.
// valid: mode 0 mvpMapLines[i] && !mvbLineOutlier[i] && !isBad(); mode 1
// mbTrackInView && !isBad(). match[j] = map line assigned to current line j
// by the final pass (-1: none; the caller keeps its line unless *wiped).
// Outputs: proj_kl / proj_src (nml capacity, *nproj written), pairs as
// (i, j) int pairs (pair_cap capacity, *npairs = the full count).
int oracle_line_search_pairs(const orbpl_camera* cam, const float* Tcw, int mode, int ncur,
                             const orbpl_keyline* cur_kl_un, const uint8_t* cur_desc,
                             const int32_t* cur_nobs, int nml, const uint8_t* valid,
                             const orbpl_keyline* base_kl, const float* ml_xyz6,
                             const uint8_t* ml_desc, const int32_t* ml_nobs,
                             orbpl_keyline* proj_kl, int32_t* proj_src, int* nproj,
                             int32_t* pairs, int pair_cap, int* npairs, int32_t* match,
                             int* nmatches_out, int* wiped) {
  using namespace line_track;
  std::vector<orbpl_keyline> nk;
  std::vector<int> nidx;
  project_lines(cam, Tcw, nml, valid, mode == 0 ? base_kl : nullptr, ml_xyz6, nk, nidx);
  *nproj = (int)nk.size();
  for (size_t i = 0; i < nk.size(); i++) {
    proj_kl[i] = nk[i];
    proj_src[i] = nidx[i];
  }
  std::vector<int> cnobs(ncur > 0 ? ncur : 1, 0);
  for (int j = 0; j < ncur; j++) cnobs[j] = cur_nobs ? cur_nobs[j] : 0;
  std::vector<int> pr;
  auto run = [&](const double off[5]) {
    int cnt = 0;
    pr.clear();
    for (int j = 0; j < ncur; j++) {
      match[j] = -1;
      if (mode == 1 && cnobs[j] > 0) continue;
      for (size_t i = 0; i < nk.size(); i++) {
        if (mode == 0 && cnobs[j] > 0) continue;
        if (line_matching(nk[i], cur_kl_un[j], ml_desc + 32 * nidx[i], cur_desc + 32 * j, off)) {
          match[j] = nidx[i];
          cnobs[j] = ml_nobs ? ml_nobs[nidx[i]] : 0;
          pr.push_back((int)i);
          pr.push_back(j);
          cnt++;
        }
      }
    }
    return cnt;
  };
  const double off0[5] = {0, 0, 0, 0, 0};
  int n = run(off0);
  *wiped = 0;
  const bool retry = mode == 0 ? (n * 1.0 / ncur < 0.2) : (n <= 0.2 * ncur);
  if (retry) {
    const double off1[5] = {10.0, -0.1, -0.1, 5, 10};
    std::fill(cnobs.begin(), cnobs.end(), 0);   // mvpMapLines wiped to NULL
    n = run(off1);
    *wiped = 1;
  }
  *nmatches_out = n;
  *npairs = (int)pr.size() / 2;
  for (int k = 0; k < std::min(*npairs, pair_cap); k++) {
    pairs[2 * k] = pr[2 * k];
    pairs[2 * k + 1] = pr[2 * k + 1];
  }
  return 0;
}

// LineMatcher::SearchByProjection(Frame&, KeyFrame*, vector<MapLine*>&)
// (LineMatcher.cpp:492-525): cv::BFMatcher(NORM_HAMMING).knnMatch(keyframe
// line descriptors, current line descriptors, k = 2); per query (keyframe
// line q, in order) with a best and a second match, best.distance /
// second.distance < 0.75 (float) assigns keyframe line q to the best train
// line (a later query overwrites) and counts. knnMatch keeps the two smallest
// distances in train order with ties to the lower train index (EXTERNAL:
// OpenCV batchDistance insertion, strict <). A query with fewer than two train
// descriptors has no second match (the reference reads past the end: pinned
// to no match). out[j] = keyframe line assigned to current line j, or -1.
int oracle_line_match_bf_knn(int nq, const uint8_t* qdesc, int nt, const uint8_t* tdesc,
                             int32_t* out, int* nmatches_out) {
  for (int j = 0; j < nt; j++) out[j] = -1;
  int n = 0;
  for (int q = 0; q < nq; q++) {
    int b = -1, s = -1, db = 0, ds = 0;
    for (int j = 0; j < nt; j++) {
      const int d = line_track::popcnt_dist(qdesc + 32 * q, tdesc + 32 * j);
      if (b < 0 || d < db) {
        s = b; ds = db;
        b = j; db = d;
      } else if (s < 0 || d < ds) {
        s = j; ds = d;
      }
    }
    if (s < 0) continue;
    const float ratio = (float)db / (float)ds;
    if (ratio < 0.75f) {
      out[b] = q;
      n++;
    }
  }
  *nmatches_out = n;
  return 0;
}

// LineMatcher(0.9, true).SearchByProjection(CurrentFrame, LastFrame)
// Tcw: current pose (16 floats). Last frame map lines: has_ml[i], outlier[i],
// xyz6[i] (start, end), desc[i]. match[j] = last-frame line index or -1.
int oracle_line_search_by_projection_last(const orbpl_camera* cam, const float* Tcw, int ncur,
                                          const orbpl_keyline* cur_kl_un, const uint8_t* cur_desc,
                                          int nlast, const orbpl_keyline* last_kl_un,
                                          const uint8_t* has_ml, const uint8_t* last_outlier,
                                          const float* ml_xyz6, const uint8_t* last_desc,
                                          int32_t* match, int* nmatches_out) {
  std::vector<uint8_t> valid(nlast);
  for (int i = 0; i < nlast; i++) valid[i] = has_ml[i] && !last_outlier[i];
  return line_track::line_search_core(cam, Tcw, ncur, cur_kl_un, cur_desc, nullptr, nlast,
                                      valid.data(), last_kl_un, ml_xyz6, last_desc, match,
                                      nmatches_out, nullptr);
}

// The local-map (valid = mbTrackInView) and reference-keyframe (valid =
// mvpMapLines[i] != NULL) overloads; cur_nobs = Observations() of the map
// line already at each current line (NULL: none).
int oracle_line_search_by_projection_list(const orbpl_camera* cam, const float* Tcw, int ncur,
                                          const orbpl_keyline* cur_kl_un, const uint8_t* cur_desc,
                                          const int32_t* cur_nobs, int nml, const uint8_t* valid,
                                          const float* ml_xyz6, const uint8_t* ml_desc,
                                          int32_t* match, int* nmatches_out, int* wiped) {
  return line_track::line_search_core(cam, Tcw, ncur, cur_kl_un, cur_desc, cur_nobs, nml, valid,
                                      nullptr, ml_xyz6, ml_desc, match, nmatches_out, wiped);
}

// Stereo line depths — a DEFINED mode: the reference's
// stereo Frame extracts no lines (Frame.cc:70-131) yet PoseOptimizationWithLines
// loops over NL (Optimizer.cc:2287-2303), so configs[3] "KITTI stereo
// points+lines" needs a definition. LineExtractor runs on both rectified
// images; left line i takes the right line j with the smallest LBD Hamming
// distance (first j on ties) among those that pass, in this order:
//   Hamming <= 45 (LineMatcher's TH), |angle_i - angle_j| <= 10 deg,
//   min/max length >= 0.45, both lines non-horizontal (|dy| >= 0.25 length),
//   row overlap >= 0.5 of the shorter row span, and both end-point
//   disparities d = x_i - x_j(y_i) in (0, maxD), maxD = mbf / mb
//   (ComputeStereoMatches' range, Frame.cc:897-899), where x_j(y) is the
//   right line's x on row y (double arithmetic).
// depth = mbf / (float)d for the start and end points (float division); no
// match leaves -1. kl = left KeyLines (rectified: distorted == undistorted).
int oracle_stereo_line_depths(const orbpl_camera* cam, const orbpl_keyline* kl,
                              const uint8_t* desc, int nl, const orbpl_keyline* kr,
                              const uint8_t* desc_r, int nr, float* dstart, float* dend) {
  const double kPi = 3.14159265358979323846;
  const float maxD = cam->bf / (cam->bf / cam->fx);
  for (int i = 0; i < nl; i++) {
    dstart[i] = -1.0f;
    dend[i] = -1.0f;
    const orbpl_keyline& a = kl[i];
    const double ady = (double)a.endPointY - a.startPointY;
    if (std::fabs(ady) < 0.25 * a.lineLength) continue;
    const double ay0 = std::min(a.startPointY, a.endPointY), ay1 = std::max(a.startPointY, a.endPointY);
    int best = 46;
    float bs = -1.0f, be = -1.0f;
    for (int j = 0; j < nr; j++) {
      const orbpl_keyline& b = kr[j];
      const int dist = popcnt_dist(desc + (size_t)i * 32, desc_r + (size_t)j * 32);
      if (dist > 45 || dist >= best) continue;
      if (std::fabs((double)a.angle - (double)b.angle) > 10.0 * kPi / 180.0) continue;
      if (std::min(a.lineLength, b.lineLength) / std::max(a.lineLength, b.lineLength) < 0.45f)
        continue;
      const double bdy = (double)b.endPointY - b.startPointY;
      if (std::fabs(bdy) < 0.25 * b.lineLength) continue;
      const double by0 = std::min(b.startPointY, b.endPointY), by1 = std::max(b.startPointY, b.endPointY);
      const double ov = std::min(ay1, by1) - std::max(ay0, by0);
      if (ov < 0.5 * std::min(ay1 - ay0, by1 - by0)) continue;
      const double slope = ((double)b.endPointX - b.startPointX) / bdy;
      const double xs = b.startPointX + ((double)a.startPointY - b.startPointY) * slope;
      const double xe = b.startPointX + ((double)a.endPointY - b.startPointY) * slope;
      const float ds = (float)((double)a.startPointX - xs);
      const float de = (float)((double)a.endPointX - xe);
      if (!(ds > 0.0f && ds < maxD && de > 0.0f && de < maxD)) continue;
      best = dist;
      bs = cam->bf / ds;
      be = cam->bf / de;
    }
    if (best <= 45) {
      dstart[i] = bs;
      dend[i] = be;
    }
  }
  return 0;
}

// Frame::IsInFrustum(MapLine*) (Frame.cc:403-430): in view unless both end
// points are behind the camera (Rcw X + tcw in float, P6).
int oracle_line_is_in_frustum(const float* Tcw, int n, const float* xyz6, uint8_t* in_view) {
  for (int i = 0; i < n; i++) {
    float zs = 0, ze = 0;
    for (int e = 0; e < 2; e++) {
      const float* X = xyz6 + 6 * i + 3 * e;
      double s = (double)Tcw[8] * X[0];
      s += (double)Tcw[9] * X[1];
      s += (double)Tcw[10] * X[2];
      const float z = (float)(s + (double)Tcw[11]);
      (e ? ze : zs) = z;
    }
    in_view[i] = !(zs < 0.0f && ze < 0.0f);
  }
  return 0;
}


}  // extern "C"

// ---------------------------------------------------------------------------
// Points + lines VO step (Tracking::TrackWithMotionModel, Tracking.cc:1212-
// 1330, with ORB and LSD/LBD extraction as Frame(RGB-D) runs them, and every
// frame acting as the next keyframe: map points and map lines are created
// StereoInitialization-style, Tracking.cc:627-690). Mirrors orbpl_tracker
// with lines enabled.
// ---------------------------------------------------------------------------
namespace line_track {

static void gemm44(const float* A, const float* B, float* Cm) {
  for (int r = 0; r < 4; r++)
    for (int c = 0; c < 4; c++) {
      double s = (double)A[r * 4] * B[c];
      s += (double)A[r * 4 + 1] * B[4 + c];
      s += (double)A[r * 4 + 2] * B[8 + c];
      s += (double)A[r * 4 + 3] * B[12 + c];
      Cm[r * 4 + c] = (float)s;
    }
}
static void neg_Rt_t(const float* T, float* o) {
  for (int r = 0; r < 3; r++) {
    double s = (double)T[0 * 4 + r] * T[3];
    s += (double)T[1 * 4 + r] * T[7];
    s += (double)T[2 * 4 + r] * T[11];
    o[r] = (float)(s * -1.0);
  }
}
static void pose_inv(const float* T, float* Ti) {
  float ow[3];
  neg_Rt_t(T, ow);
  for (int r = 0; r < 3; r++) {
    for (int c = 0; c < 3; c++) Ti[r * 4 + c] = T[c * 4 + r];
    Ti[r * 4 + 3] = ow[r];
  }
  Ti[12] = 0; Ti[13] = 0; Ti[14] = 0; Ti[15] = 1;
}
// Frame::UnprojectStereo*: Rwc * (x, y, z) + Ow, double-accumulated (P6)
static void unproject(const orbpl_camera& c, const float* T, const float* Ow, float u, float v,
                      float z, float* w) {
  const float invfx = 1.0f / c.fx, invfy = 1.0f / c.fy;
  const float x3[3] = {(u - c.cx) * z * invfx, (v - c.cy) * z * invfy, z};
  for (int r = 0; r < 3; r++) {
    double s = (double)T[0 * 4 + r] * x3[0];
    s += (double)T[1 * 4 + r] * x3[1];
    s += (double)T[2 * 4 + r] * x3[2];
    w[r] = (float)(s + (double)Ow[r]);
  }
}

// One keyframe's map in the local map (ORBPL_TRACK_LOCAL_MAP): every tracked
// frame is a keyframe whose map points are its keypoints with depth, with
// MapPoint::UpdateNormalAndDepth's normal and scale-invariance distances
// (MapPoint.cc:329-372, one observation; pinned P18).
struct KFMap {
  int n = 0, nl = 0;
  std::vector<float> xyz, normal, dmin, dmax;  // dmin / dmax: Get{Min,Max}DistanceInvariance
  std::vector<uint8_t> has, desc;
  std::vector<float> lxyz;
  std::vector<uint8_t> lhas, ldesc;
};
constexpr int kLocalKFs = 4;   // the local keyframes: the last 4 frames (P18)

struct LStream {
  bool has_last = false, has_velocity = false;
  int frame_id = 0;            // Frame::mnId
  std::vector<KFMap> local;    // most recent first, at most kLocalKFs
  int lm[4] = {0, 0, 0, 0};    // last step: local point matches, point inliers,
                               // local line matches, line inliers
  float Tcw[16], Tlast[16], Tlast2[16];
  std::vector<orbpl_keypoint> kps_un;
  std::vector<uint8_t> desc, has_mp, outlier;
  std::vector<float> xyz;
  std::vector<int32_t> nobs;
  std::vector<orbpl_keyline> kl_un;
  std::vector<uint8_t> ldesc, has_ml, loutlier;
  std::vector<float> lxyz;
  std::vector<int32_t> fnode;  // FeatureVector (KeyFrame::ComputeBoW): node per keypoint
  std::vector<float> kangle;   // keypoint angles (mvKeys / mvKeysUn)
  int trk = 0;                 // the last step ran TrackReferenceKeyFrame
};

// oracle_lvo_create_ex flags: the tracker's ORBPL_TRACK_* bits plus
constexpr int kTwoThreads = 1 << 16;  // ORB || LineExtractor on two host threads per
                                      // frame (Frame.cc:152-155), CPU baseline mode

struct LVO {
  orbpl_orb_params orb;
  orbpl_camera cam;
  int use_lines;
  int flags;
  void* voc = nullptr;          // oracle vocabulary (ORBPL_TRACK_REFKF / ComputeBoW)
  std::vector<LStream> st;
  std::vector<float> scale, inv_sigma2;
};

}  // namespace line_track

extern "C" {

void* oracle_lvo_create_ex(const orbpl_orb_params* orb, const orbpl_camera* cam, int n_streams,
                           int flags) {
  LVO* v = new LVO();
  v->orb = *orb;
  v->cam = *cam;
  v->flags = flags;
  v->use_lines = (flags & ORBPL_TRACK_LINES) ? 1 : 0;
  v->st.resize(n_streams);
  v->scale.resize(orb->nlevels);
  std::vector<float> isc(orb->nlevels);
  oracle_orb_level_sizes(orb, cam->width, cam->height, nullptr, nullptr, nullptr, v->scale.data(),
                         isc.data());
  v->inv_sigma2.resize(orb->nlevels);
  for (int l = 0; l < orb->nlevels; l++) v->inv_sigma2[l] = 1.0f / (v->scale[l] * v->scale[l]);
  return v;
}

void* oracle_lvo_create(const orbpl_orb_params* orb, const orbpl_camera* cam, int n_streams,
                        int use_lines) {
  return oracle_lvo_create_ex(orb, cam, n_streams, use_lines ? ORBPL_TRACK_LINES : 0);
}

void oracle_lvo_destroy(void* h) { delete static_cast<LVO*>(h); }

int oracle_lvo_reset(void* h, const float* Tcw0) {
  LVO* v = static_cast<LVO*>(h);
  for (size_t s = 0; s < v->st.size(); s++) {
    LStream z{};
    for (int k = 0; k < 16; k++) z.Tcw[k] = Tcw0 ? Tcw0[s * 16 + k] : ((k % 5 == 0) ? 1.f : 0.f);
    v->st[s] = z;
  }
  return 0;
}

}  // extern "C"

namespace line_track {

// Pose problem of the current frame from per-keypoint / per-line world
// positions (has* = an edge) and PoseOptimizationWithLines on it.
static int optimize_pose(LVO* v, LStream& S, int n, const std::vector<orbpl_keypoint>& ku,
                         const std::vector<float>& ur, const std::vector<uint8_t>& has,
                         const std::vector<float>& xyz, int nl,
                         const std::vector<orbpl_keyline>& klu, const std::vector<uint8_t>& hasl,
                         const std::vector<float>& lxyz, std::vector<uint8_t>& outl,
                         std::vector<uint8_t>& loutl) {
  std::vector<float> lobs((size_t)nl * 4, 0.f);
  std::vector<int32_t> loct(nl, 0);
  for (int j = 0; j < nl; j++) {
    loct[j] = klu[j].octave;
    lobs[4 * j] = klu[j].startPointX;
    lobs[4 * j + 1] = klu[j].startPointY;
    lobs[4 * j + 2] = klu[j].endPointX;
    lobs[4 * j + 3] = klu[j].endPointY;
  }
  orbpl_pose_problem P{};
  P.n = n;
  P.kps_un = ku.data();
  P.uright = ur.data();
  P.has_mp = has.data();
  P.mp_xyz = xyz.data();
  P.nl = nl;
  P.kl_obs = lobs.data();
  P.kl_octave = loct.data();
  P.has_ml = hasl.data();
  P.ml_xyz = lxyz.data();
  P.inv_sigma2 = v->inv_sigma2.data();
  P.nlevels = (int)v->inv_sigma2.size();
  int ninl = 0;
  oracle_pose_optimization_ex(&v->cam, &P,
                              (v->flags & ORBPL_TRACK_FIXED_LINE_JAC) ? ORBPL_POSE_FIXED_LINE_JAC : 0,
                              S.Tcw, outl.data(), loutl.data(), &ninl);
  return ninl;
}

// Tracking::TrackLocalMap (Tracking.cc:1332-1420) with the defined local map
// P18: the local keyframes are the last kLocalKFs frames (most recent
// first), the local map points / lines their map points / lines in index
// order, minus those the current frame already holds or that the motion
// model rejected as outliers (mnLastFrameSeen, Tracking.cc:1285-1292,
// 1750-1768). SearchLocalPoints (:1746-1813): IsInFrustum(pMP, 0.5) at the
// optimised pose, ORBmatcher(0.8).SearchByProjection with th = 3 (RGB-D) /
// 1 (stereo), 5 while mnId < mnLastRelocFrameId + 2; SearchLocalLines
// (:1816-1865): IsInFrustum(pML, 0.5), LineMatcher(0.8).SearchByProjection(F,
// local lines) with its relaxed retry (which wipes every current line
// assignment first). Then PoseOptimizationWithLines over all matches and the
// inlier decision (:1396-1419; mnLastRelocFrameId = 0, mMaxFrames = 30).
static bool track_local_map(LVO* v, LStream& S, bool stereo, int n,
                            const std::vector<orbpl_keypoint>& ku, const std::vector<uint8_t>& desc,
                            const std::vector<float>& ur, const std::vector<int32_t>& match,
                            const std::vector<int32_t>& match_pre, int nl,
                            const std::vector<orbpl_keyline>& klu,
                            const std::vector<uint8_t>& ldesc, const std::vector<int32_t>& lmatch,
                            const std::vector<int32_t>& lmatch_pre) {
  const orbpl_camera& cam = v->cam;
  const int K = (int)S.local.size();
  const int nlev = (int)v->scale.size();
  // ---- SearchLocalPoints ----
  std::vector<uint8_t> seen0(K ? S.local[0].n : 0, 0);
  for (int i = 0; i < n; i++)
    if (match_pre[i] >= 0) seen0[match_pre[i]] = 1;
  std::vector<int32_t> cur_nobs(n);
  for (int i = 0; i < n; i++) cur_nobs[i] = match[i] >= 0 ? 1 : 0;
  std::vector<float> Lx, Ln, Lmin, Lmax;
  std::vector<uint8_t> Ld;
  for (int k = 0; k < K; k++) {
    const KFMap& m = S.local[k];
    for (int j = 0; j < m.n; j++) {
      if (!m.has[j] || (k == 0 && seen0[j])) continue;
      Lx.insert(Lx.end(), &m.xyz[3 * j], &m.xyz[3 * j] + 3);
      Ln.insert(Ln.end(), &m.normal[3 * j], &m.normal[3 * j] + 3);
      Lmin.push_back(m.dmin[j]);
      Lmax.push_back(m.dmax[j]);
      Ld.insert(Ld.end(), &m.desc[32 * j], &m.desc[32 * j] + 32);
    }
  }
  const int nloc = (int)Lmin.size();
  std::vector<uint8_t> inview(nloc);
  std::vector<float> px(nloc), py(nloc), pxr(nloc), vcos(nloc);
  std::vector<int32_t> lev(nloc), mp_nobs(nloc, 1), lm(n, -1);
  const float log_scale = (float)pmath::log_((double)v->orb.scale_factor);   // P15
  oracle_frame_is_in_frustum(&cam, log_scale, nlev, S.Tcw, nloc, Lx.data(), Ln.data(), Lmin.data(),
                             Lmax.data(), 0.5f, inview.data(), px.data(), py.data(), pxr.data(),
                             lev.data(), vcos.data());
  int nto = 0;
  for (int i = 0; i < nloc; i++) nto += inview[i];
  int nlocal = 0;
  if (nto > 0) {
    const float th = S.frame_id < 2 ? 5.0f : (stereo ? 1.0f : 3.0f);
    orbpl_match_current cur{n, S.Tcw, ku.data(), desc.data(), ur.data()};
    oracle_search_by_projection_local(&cam, v->scale.data(), nlev, &cur, nloc, inview.data(),
                                      px.data(), py.data(), pxr.data(), lev.data(), vcos.data(),
                                      Ld.data(), mp_nobs.data(), cur_nobs.data(), th, 0.8f,
                                      lm.data(), &nlocal);
  }
  // ---- SearchLocalLines ----
  std::vector<float> LLx;
  std::vector<uint8_t> LLd;
  std::vector<int32_t> llm(nl, -1);
  int nllocal = 0, wiped = 0;
  if (v->use_lines) {
    std::vector<uint8_t> seen0l(K ? S.local[0].nl : 0, 0);
    for (int j = 0; j < nl; j++)
      if (lmatch_pre[j] >= 0) seen0l[lmatch_pre[j]] = 1;
    std::vector<int32_t> cur_nobs_l(nl);
    for (int j = 0; j < nl; j++) cur_nobs_l[j] = lmatch[j] >= 0 ? 1 : 0;
    for (int k = 0; k < K; k++) {
      const KFMap& m = S.local[k];
      for (int j = 0; j < m.nl; j++) {
        if (!m.lhas[j] || (k == 0 && seen0l[j])) continue;
        LLx.insert(LLx.end(), &m.lxyz[6 * j], &m.lxyz[6 * j] + 6);
        LLd.insert(LLd.end(), &m.ldesc[32 * j], &m.ldesc[32 * j] + 32);
      }
    }
    const int nll = (int)LLd.size() / 32;
    std::vector<uint8_t> lvalid(nll);
    oracle_line_is_in_frustum(S.Tcw, nll, LLx.data(), lvalid.data());
    int ntol = 0;
    for (int i = 0; i < nll; i++) ntol += lvalid[i];
    if (ntol > 0)
      oracle_line_search_by_projection_list(&cam, S.Tcw, nl, klu.data(), ldesc.data(),
                                            cur_nobs_l.data(), nll, lvalid.data(), LLx.data(),
                                            LLd.data(), llm.data(), &nllocal, &wiped);
  }
  // ---- PoseOptimizationWithLines over every match ----
  std::vector<uint8_t> has(n, 0), hasl(nl, 0), outl(n, 0), loutl(nl, 0);
  std::vector<float> xyz((size_t)n * 3, 0.f), lxyz((size_t)nl * 6, 0.f);
  for (int i = 0; i < n; i++) {
    const float* src = match[i] >= 0 ? &S.xyz[3 * match[i]] : lm[i] >= 0 ? &Lx[3 * lm[i]] : nullptr;
    if (!src) continue;
    has[i] = 1;
    for (int k = 0; k < 3; k++) xyz[3 * i + k] = src[k];
  }
  for (int j = 0; j < nl; j++) {
    const float* src = (!wiped && lmatch[j] >= 0) ? &S.lxyz[6 * lmatch[j]]
                       : llm[j] >= 0             ? &LLx[6 * llm[j]]
                                                 : nullptr;
    if (!src) continue;
    hasl[j] = 1;
    for (int k = 0; k < 6; k++) lxyz[6 * j + k] = src[k];
  }
  optimize_pose(v, S, n, ku, ur, has, xyz, nl, klu, hasl, lxyz, outl, loutl);
  int inl = 0, linl = 0;
  for (int i = 0; i < n; i++) inl += has[i] && !outl[i];
  for (int j = 0; j < nl; j++) linl += hasl[j] && !loutl[j];
  S.lm[0] = nlocal;
  S.lm[1] = inl;
  S.lm[2] = nllocal;
  S.lm[3] = linl;
  if (S.frame_id < 30 && inl + linl < 60) return false;
  return !(inl < 30 && linl < 20);
}

// The current frame joins the local map as its newest keyframe (its map
// points / lines were just created from depth in S.xyz / S.lxyz).
static void push_local_kf(LVO* v, LStream& S, const float* Ow,
                          const std::vector<orbpl_keypoint>& ku, const std::vector<uint8_t>& desc,
                          const std::vector<uint8_t>& ldesc) {
  KFMap m;
  m.n = (int)ku.size();
  m.xyz = S.xyz;
  m.has = S.has_mp;
  m.desc = desc;
  m.normal.assign((size_t)m.n * 3, 0.f);
  m.dmin.assign(m.n, 0.f);
  m.dmax.assign(m.n, 0.f);
  const int nlev = (int)v->scale.size();
  for (int i = 0; i < m.n; i++) {
    if (!m.has[i]) continue;
    const float PO[3] = {m.xyz[3 * i] - Ow[0], m.xyz[3 * i + 1] - Ow[1], m.xyz[3 * i + 2] - Ow[2]};
    const double nd = std::sqrt((double)PO[0] * PO[0] + (double)PO[1] * PO[1] + (double)PO[2] * PO[2]);
    const float inv = (float)(1.0 / nd);
    for (int k = 0; k < 3; k++) m.normal[3 * i + k] = PO[k] * inv;
    const float dist = (float)nd;
    const float maxd = dist * v->scale[ku[i].octave];
    const float mind = maxd / v->scale[nlev - 1];
    m.dmax[i] = maxd;   // mfMaxDistance / mfMinDistance (the in-frustum test
    m.dmin[i] = mind;   // applies GetMax/MinDistanceInvariance's 1.2f / 0.8f)
  }
  m.nl = (int)S.has_ml.size();
  m.lxyz = S.lxyz;
  m.lhas = S.has_ml;
  m.ldesc = ldesc;
  S.local.insert(S.local.begin(), std::move(m));
  if ((int)S.local.size() > kLocalKFs) S.local.pop_back();
}

// One TrackWithMotionModel step. RGB-D (right == NULL): Frame(imGray, imDepth)
// (Frame.cc:135-205). Stereo (right != NULL): Frame(imLeft, imRight)
// (Frame.cc:70-131): ORB on both images, UndistortKeyPoints, then
// ComputeStereoMatches on the two extractors' pyramids; the stereo Frame
// extracts no lines, and SearchByProjection uses th = 7 (Tracking.cc:1238-1241).
static int lvo_step(LVO* v, int stream, const uint8_t* gray, const float* depth,
                    const uint8_t* right, float* Tcw_out, int* out8) {
  LStream& S = v->st[stream];
  const orbpl_camera& cam = v->cam;
  const int cap = v->orb.nfeatures * 2 + 64;
  // lines: LineExtractor + UndistortKeyLines + line depths (Frame.cc:152-166);
  // with kTwoThreads on a second host thread concurrently with ORB, as the
  // reference's Frame(RGB-D) runs them (Frame.cc:152-155)
  int nl = 0, lrc = 0;
  std::vector<orbpl_keyline> kl(80), klu;
  std::vector<uint8_t> ldesc(80 * 32);
  std::vector<float> lds, lde, lurs, lure;
  auto extract_lines = [&]() {
    std::vector<double> coef(80 * 3);
    int nd = 0;
    lrc = oracle_line_extract(gray, cam.width, cam.height, kl.data(), ldesc.data(), coef.data(), 80,
                              &nl, &nd);
    if (lrc) return;
    kl.resize(nl);
    ldesc.resize((size_t)nl * 32);
    klu.resize(nl);
    lds.resize(nl); lde.resize(nl); lurs.resize(nl); lure.resize(nl);
    oracle_line_frame_prepare(&cam, kl.data(), nl, right ? nullptr : depth, klu.data(),
                              lds.data(), lde.data(), lurs.data(), lure.data());
    if (right) {
      // stereo: LineExtractor on the right image, end-point depths by the
      // defined stereo line matching (P17)
      std::vector<orbpl_keyline> klr(80);
      std::vector<uint8_t> ldr(80 * 32);
      int nr = 0, ndr = 0;
      lrc = oracle_line_extract(right, cam.width, cam.height, klr.data(), ldr.data(), coef.data(),
                                80, &nr, &ndr);
      if (lrc) return;
      oracle_stereo_line_depths(&cam, klu.data(), ldesc.data(), nl, klr.data(), ldr.data(), nr,
                                lds.data(), lde.data());
    }
  };
  const bool do_lines = v->use_lines != 0;
  std::thread lthread;
  if (do_lines && (v->flags & kTwoThreads)) lthread = std::thread(extract_lines);
  std::vector<orbpl_keypoint> kps(cap);
  std::vector<uint8_t> desc((size_t)cap * 32);
  int n = 0;
  int rc = oracle_orb_extract(&v->orb, gray, cam.width, cam.height, cam.width, kps.data(),
                              desc.data(), cap, &n, nullptr);
  if (lthread.joinable()) lthread.join();
  else if (do_lines) extract_lines();
  if (rc) return rc;
  if (lrc) return lrc;
  kps.resize(n);
  desc.resize((size_t)n * 32);
  std::vector<orbpl_keypoint> ku(n);
  std::vector<float> dep(n), ur(n);
  std::vector<int32_t> gc(n);
  oracle_frame_prepare(&cam, kps.data(), n, right ? nullptr : depth, ku.data(), dep.data(),
                       ur.data(), gc.data(), nullptr);
  if (right) {
    std::vector<orbpl_keypoint> kr(cap);
    std::vector<uint8_t> dr((size_t)cap * 32);
    int nr = 0;
    rc = oracle_orb_extract(&v->orb, right, cam.width, cam.height, cam.width, kr.data(), dr.data(),
                            cap, &nr, nullptr);
    if (rc) return rc;
    const int L = v->orb.nlevels;
    std::vector<int32_t> lw(L), lh(L);
    std::vector<float> sc(L), isc(L);
    oracle_orb_level_sizes(&v->orb, cam.width, cam.height, lw.data(), lh.data(), nullptr,
                           sc.data(), isc.data());
    size_t tot = 0;
    for (int l = 0; l < L; l++) tot += (size_t)(lw[l] + 38) * (lh[l] + 38);
    std::vector<uint8_t> pl(tot), pr(tot);
    oracle_orb_pyramid(&v->orb, gray, cam.width, cam.height, cam.width, pl.data(), 0);
    oracle_orb_pyramid(&v->orb, right, cam.width, cam.height, cam.width, pr.data(), 0);
    oracle_stereo_matches(&cam, sc.data(), isc.data(), L, lw.data(), lh.data(), pl.data(),
                          pr.data(), kps.data(), desc.data(), n, kr.data(), dr.data(), nr,
                          ur.data(), dep.data());
  }
  const float th = right ? 7.0f : 15.0f;
  std::vector<int32_t> match(n, -1), lmatch(nl, -1), match_pre, lmatch_pre;
  std::vector<uint8_t> outl(n, 0), loutl(nl, 0);
  int nmatches = 0, ninl = 0, nmap = 0, nlm = 0, lnmap = 0;
  bool tracked = false, motion_ok = false, local_ok = true;
  S.lm[0] = S.lm[1] = S.lm[2] = S.lm[3] = 0;
  // KeyFrame::ComputeBoW of the frame (every frame is a keyframe, P18)
  std::vector<int32_t> fnode(n, -1);
  if (v->voc) {
    std::vector<uint32_t> bw(n + 1);
    std::vector<double> bv(n + 1), fwt(n + 1);
    std::vector<int32_t> fw(n + 1);
    int bn = 0;
    oracle_voc_transform(v->voc, desc.data(), n, 4, bw.data(), bv.data(), &bn, fnode.data(),
                         fw.data(), fwt.data());
  }
  const bool refkf = (v->flags & ORBPL_TRACK_REFKF) && v->voc;
  S.trk = 0;
  if (S.has_last && !(refkf && !S.has_velocity)) {
    if (S.has_velocity) {
      float Twl[16], V[16];
      pose_inv(S.Tlast2, Twl);
      gemm44(S.Tlast, Twl, V);
      gemm44(V, S.Tlast, S.Tcw);
    } else {
      memcpy(S.Tcw, S.Tlast, 64);
    }
    orbpl_match_current cur{n, S.Tcw, ku.data(), desc.data(), ur.data()};
    orbpl_match_last last{(int)S.kps_un.size(), S.Tlast, S.kps_un.data(), S.has_mp.data(),
                          S.outlier.data(), S.xyz.data(), S.desc.data(), S.nobs.data()};
    oracle_search_by_projection_last(&cam, v->scale.data(), (int)v->scale.size(), &cur, &last, th,
                                     0, 1, match.data(), &nmatches);
    if (v->use_lines)
      oracle_line_search_by_projection_last(&cam, S.Tcw, nl, klu.data(), ldesc.data(),
                                            (int)S.kl_un.size(), S.kl_un.data(), S.has_ml.data(),
                                            S.loutlier.data(), S.lxyz.data(), S.ldesc.data(),
                                            lmatch.data(), &nlm);
    if (nmatches < 20) {
      std::fill(match.begin(), match.end(), -1);
      oracle_search_by_projection_last(&cam, v->scale.data(), (int)v->scale.size(), &cur, &last,
                                       2.0f * th, 0, 1, match.data(), &nmatches);
    }
    tracked = nmatches >= 20 && (!v->use_lines || nlm >= 15);
    if (tracked) {
      std::vector<uint8_t> has(n, 0), hasl(nl, 0);
      std::vector<float> xyz((size_t)n * 3, 0.f), lobs((size_t)nl * 4, 0.f), lxyz((size_t)nl * 6, 0.f);
      std::vector<int32_t> loct(nl, 0);
      for (int i = 0; i < n; i++)
        if (match[i] >= 0) {
          has[i] = 1;
          for (int k = 0; k < 3; k++) xyz[3 * i + k] = S.xyz[3 * match[i] + k];
        }
      for (int j = 0; j < nl; j++) {
        loct[j] = klu[j].octave;
        lobs[4 * j] = klu[j].startPointX;
        lobs[4 * j + 1] = klu[j].startPointY;
        lobs[4 * j + 2] = klu[j].endPointX;
        lobs[4 * j + 3] = klu[j].endPointY;
        if (lmatch[j] >= 0) {
          hasl[j] = 1;
          for (int k = 0; k < 6; k++) lxyz[6 * j + k] = S.lxyz[6 * lmatch[j] + k];
        }
      }
      orbpl_pose_problem P{};
      P.n = n;
      P.kps_un = ku.data();
      P.uright = ur.data();
      P.has_mp = has.data();
      P.mp_xyz = xyz.data();
      P.nl = nl;
      P.kl_obs = lobs.data();
      P.kl_octave = loct.data();
      P.has_ml = hasl.data();
      P.ml_xyz = lxyz.data();
      P.inv_sigma2 = v->inv_sigma2.data();
      P.nlevels = (int)v->inv_sigma2.size();
      oracle_pose_optimization_ex(&cam, &P,
                                  (v->flags & ORBPL_TRACK_FIXED_LINE_JAC) ? ORBPL_POSE_FIXED_LINE_JAC : 0,
                                  S.Tcw, outl.data(), loutl.data(), &ninl);
    }
    match_pre = match;
    lmatch_pre = lmatch;
    // outlier discard (Tracking.cc:1273-1314); without an optimisation every
    // flag is clear and the counts report the raw matches
    for (int i = 0; i < n; i++)
      if (match[i] >= 0) {
        if (outl[i]) match[i] = -1;
        else nmap++;
      }
    for (int j = 0; j < nl; j++)
      if (lmatch[j] >= 0) {
        if (loutl[j]) {
          lmatch[j] = -1;
          lnmap--;  // the reference decrements here (Tracking.cc:1306)
        } else {
          lnmap++;
        }
      }
    motion_ok = tracked && (v->use_lines ? (nmap >= 10 || lnmap >= 15) : nmap >= 10);
  }
  if (match_pre.empty() && lmatch_pre.empty()) {
    match_pre = match;
    lmatch_pre = lmatch;
  }
  if (S.has_last && refkf && !motion_ok) {
    // ---- TrackReferenceKeyFrame (Tracking.cc:942-1032), reference keyframe =
    // the last frame (P18, P22) ----
    S.trk = 1;
    memcpy(S.Tcw, S.Tlast, 64);   // SetPose(mLastFrame.mTcw)
    std::vector<float> fang(n);
    for (int i = 0; i < n; i++) fang[i] = ku[i].angle;
    const int nkf = (int)S.kps_un.size();
    std::vector<int32_t> bm(n, -1);
    nmatches = 0;
    oracle_search_by_bow(nkf, S.fnode.data(), S.has_mp.data(), S.desc.data(), S.kangle.data(), n,
                         fnode.data(), desc.data(), fang.data(), 0.7f, 1, bm.data(), &nmatches);
    // lines: the reference-keyframe overload over the frame's current line
    // assignments (the motion model's, after its outlier discard; none when
    // it did not run), LineMatcher.cpp:527-754
    std::vector<int32_t> lcur(nl, -1), tl(nl, -1), cur_nobs_l(nl, 0);
    if (S.has_velocity)
      for (int j = 0; j < nl; j++) lcur[j] = lmatch[j];
    for (int j = 0; j < nl; j++) cur_nobs_l[j] = lcur[j] >= 0 ? 1 : 0;
    int ntl = 0, wiped = 0;
    if (v->use_lines)
      oracle_line_search_by_projection_list(&cam, S.Tcw, nl, klu.data(), ldesc.data(),
                                            cur_nobs_l.data(), (int)S.kl_un.size(),
                                            S.has_ml.data(), S.lxyz.data(), S.ldesc.data(),
                                            tl.data(), &ntl, &wiped);
    for (int j = 0; j < nl; j++) lmatch[j] = (!wiped && lcur[j] >= 0) ? lcur[j] : tl[j];
    nlm = ntl;
    match = bm;
    std::fill(outl.begin(), outl.end(), 0);
    std::fill(loutl.begin(), loutl.end(), 0);
    ninl = 0;
    const bool go = nmatches >= 15 && (!v->use_lines || ntl >= 10);
    if (go) {
      std::vector<uint8_t> has(n, 0), hasl(nl, 0);
      std::vector<float> xyz((size_t)n * 3, 0.f), lxyz((size_t)nl * 6, 0.f);
      for (int i = 0; i < n; i++)
        if (match[i] >= 0) {
          has[i] = 1;
          for (int k = 0; k < 3; k++) xyz[3 * i + k] = S.xyz[3 * match[i] + k];
        }
      for (int j = 0; j < nl; j++)
        if (lmatch[j] >= 0) {
          hasl[j] = 1;
          for (int k = 0; k < 6; k++) lxyz[6 * j + k] = S.lxyz[6 * lmatch[j] + k];
        }
      ninl = optimize_pose(v, S, n, ku, ur, has, xyz, nl, klu, hasl, lxyz, outl, loutl);
    }
    match_pre = match;
    lmatch_pre = lmatch;
    nmap = 0;
    lnmap = 0;
    for (int i = 0; i < n; i++)
      if (match[i] >= 0) {
        if (outl[i]) match[i] = -1;
        else nmap++;
      }
    for (int j = 0; j < nl; j++)
      if (lmatch[j] >= 0) {
        if (loutl[j]) {
          lmatch[j] = -1;
          lnmap--;
        } else {
          lnmap++;
        }
      }
    motion_ok = go && nmap >= 10 && (!v->use_lines || lnmap >= 10);
  }
  if (S.has_last && (v->flags & ORBPL_TRACK_LOCAL_MAP) && motion_ok)
    local_ok = track_local_map(v, S, right != nullptr, n, ku, desc, ur, match, match_pre, nl, klu,
                               ldesc, lmatch, lmatch_pre);
  // this frame becomes the keyframe of the next one
  float Ow[3];
  neg_Rt_t(S.Tcw, Ow);
  S.kps_un = ku;
  S.desc = desc;
  S.has_mp.assign(n, 0);
  S.outlier.assign(n, 0);
  S.xyz.assign((size_t)n * 3, 0.f);
  S.nobs.assign(n, 0);
  for (int i = 0; i < n; i++)
    if (dep[i] > 0) {
      unproject(cam, S.Tcw, Ow, ku[i].x, ku[i].y, dep[i], &S.xyz[3 * i]);
      S.has_mp[i] = 1;
      S.nobs[i] = 1;
    }
  S.fnode = fnode;
  S.kangle.resize(n);
  for (int i = 0; i < n; i++) S.kangle[i] = ku[i].angle;
  S.kl_un = klu;
  S.ldesc = ldesc;
  S.has_ml.assign(nl, 0);
  S.loutlier.assign(nl, 0);
  S.lxyz.assign((size_t)nl * 6, 0.f);
  for (int j = 0; j < nl; j++)
    if (lds[j] > 0 && lde[j] > 0) {
      // UnprojectStereoLineEnd uses mvDepthLineStart (Frame.cc:1192)
      unproject(cam, S.Tcw, Ow, klu[j].startPointX, klu[j].startPointY, lds[j], &S.lxyz[6 * j]);
      unproject(cam, S.Tcw, Ow, klu[j].endPointX, klu[j].endPointY, lds[j], &S.lxyz[6 * j + 3]);
      S.has_ml[j] = 1;
    }
  if (v->flags & ORBPL_TRACK_LOCAL_MAP) push_local_kf(v, S, Ow, ku, desc, ldesc);
  bool ok = true;
  if (S.has_last) ok = motion_ok && local_ok;
  S.frame_id++;
  memcpy(S.Tlast2, S.Tlast, 64);
  memcpy(S.Tlast, S.Tcw, 64);
  S.has_velocity = S.has_last;
  S.has_last = true;
  if (Tcw_out) memcpy(Tcw_out, S.Tcw, 64);
  if (out8) {
    out8[0] = n; out8[1] = nmatches; out8[2] = ninl; out8[3] = nmap; out8[4] = ok;
    out8[5] = nl; out8[6] = nlm; out8[7] = lnmap;
  }
  return 0;
}

}  // namespace line_track

extern "C" {

// out8: nkeypoints, nmatches, ninliers, nmatches_map, ok, nlines, line_matches,
// line_nmatches_map
int oracle_lvo_step(void* h, int stream, const uint8_t* gray, const float* depth, float* Tcw_out,
                    int* out8) {
  return line_track::lvo_step(static_cast<line_track::LVO*>(h), stream, gray, depth, nullptr,
                              Tcw_out, out8);
}

// TrackLocalMap counts of the stream's last step (ORBPL_TRACK_LOCAL_MAP):
// local point matches, point inliers (mnMatchesInliers), local line matches,
// line inliers (mnLineMatchesInliers); zeros when it did not run.
// the vocabulary (oracle_voc_load_text handle) of KeyFrame::ComputeBoW and
// ORBPL_TRACK_REFKF; not owned
int oracle_lvo_set_vocabulary(void* h, void* voc) {
  static_cast<line_track::LVO*>(h)->voc = voc;
  return 0;
}

// 1 when the stream's last step ran TrackReferenceKeyFrame
int oracle_lvo_trk(void* h, int stream) { return static_cast<line_track::LVO*>(h)->st[stream].trk; }

int oracle_lvo_local_stats(void* h, int stream, int* out4) {
  const line_track::LStream& S = static_cast<line_track::LVO*>(h)->st[stream];
  for (int k = 0; k < 4; k++) out4[k] = S.lm[k];
  return 0;
}

// Stereo TrackWithMotionModel step (see lvo_step).
int oracle_lvo_step_stereo(void* h, int stream, const uint8_t* left, const uint8_t* right,
                           float* Tcw_out, int* out8) {
  return line_track::lvo_step(static_cast<line_track::LVO*>(h), stream, left, nullptr, right,
                              Tcw_out, out8);
}

}  // extern "C"
