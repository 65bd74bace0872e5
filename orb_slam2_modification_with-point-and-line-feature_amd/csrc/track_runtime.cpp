// Host runtime + C-ABI of the tracking half of the hot path:
// orbpl_frame_prepare / orbm_search_by_projection_last / orbpl_pose_optimization
// (single-frame host-pointer forms, drop-in for Frame / ORBmatcher / Optimizer
// calls) and the batched device-resident orbpl_tracker.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstddef>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/orbpl.h"
#include "orb_kernels.h"
#include "orbpl_runtime.h"
#include "track_kernels.h"
#include "lsd_kernels.h"
#include "lsd_math.h"
#include "map_kernels.h"

using namespace orbpl;

#define HIP_CHECK(expr)                                                \
  do {                                                                 \
    hipError_t _e = (expr);                                            \
    if (_e != hipSuccess) return orbpl::hip_fail(_e, #expr, __LINE__); \
  } while (0)

namespace {

// streams from which the RGB-D lines tracker splits its LSD batch in two
// offset halves (ORBPL_LSD_SPLIT overrides)
constexpr int kLsdSplitMin = 1024;
// likewise the ORB extraction batch (ORBPL_ORB_SPLIT=1 turns it on): the
// second half's pyramid beside the first half's FAST, and so on down the
// chain. Off by default: at 16 queues points +1.8 % and rig +3.5 % (within
// the run-to-run spread), lines -2 %
constexpr int kOrbSplitMin = 1 << 30;

// the HIP runtime runs with >= 8 hardware queues (recorded at library load,
// orbpl_runtime.cpp): with the default 4, extra streams share queues and
// serialise
bool enough_hw_queues() { return hw_queues() >= 8; }
// a split switch: env "0" off, "1" on, else on from `min_streams` when the
// runtime has the queues for it
bool split_on(const char* env, int n_streams, int min_streams) {
  if (n_streams < 2) return false;   // two halves need a frame each, even when forced
  const char* e = getenv(env);
  return e ? e[0] == '1' : n_streams >= min_streams && enough_hw_queues();
}

// RAII device buffer for the synchronous host-pointer entry points.
struct DBuf {
  void* p = nullptr;
  size_t n = 0;
  hipError_t alloc(size_t bytes) {
    n = bytes;
    return hipMalloc(&p, bytes ? bytes : 1);
  }
  ~DBuf() {
    if (p) (void)hipFree(p);
  }
  template <class T>
  T* as() const { return reinterpret_cast<T*>(p); }
};

// Frame constants (Frame.cc:180-203) from the camera and the extractor's
// scale tables; ComputeImageBounds uses the same undistortion code as the
// device kernel (host-compiled, same IEEE double sequence).
int make_consts(const orbpl_camera* cam, const float* scale, const float* inv_sigma2, int nlevels,
                TrackConsts* out) {
  if (!cam) return arg_fail("NULL camera");
  if (nlevels < 1 || nlevels > kMaxLevelsT) return arg_fail("nlevels out of range");
  TrackConsts c{};
  c.fx = cam->fx; c.fy = cam->fy; c.cx = cam->cx; c.cy = cam->cy;
  c.k1 = cam->k1; c.k2 = cam->k2; c.p1 = cam->p1; c.p2 = cam->p2; c.k3 = cam->k3;
  c.bf = cam->bf;
  c.mb = cam->bf / cam->fx;
  c.th_depth = cam->th_depth;
  c.invfx = 1.0f / cam->fx;
  c.invfy = 1.0f / cam->fy;
  c.width = cam->width;
  c.height = cam->height;
  if (cam->k1 != 0.0f) {
    float ux[4], uy[4];
    const float px[4] = {0.0f, (float)cam->width, 0.0f, (float)cam->width};
    const float py[4] = {0.0f, 0.0f, (float)cam->height, (float)cam->height};
    for (int i = 0; i < 4; i++) undistort_point_d(c, px[i], py[i], &ux[i], &uy[i]);
    c.minX = std::min(ux[0], ux[2]);
    c.maxX = std::max(ux[1], ux[3]);
    c.minY = std::min(uy[0], uy[1]);
    c.maxY = std::max(uy[2], uy[3]);
  } else {
    c.minX = 0.0f; c.maxX = (float)cam->width; c.minY = 0.0f; c.maxY = (float)cam->height;
  }
  c.gridInvW = static_cast<float>(kGridCols) / static_cast<float>(c.maxX - c.minX);
  c.gridInvH = static_cast<float>(kGridRows) / static_cast<float>(c.maxY - c.minY);
  c.nlevels = nlevels;
  for (int l = 0; l < nlevels; l++) {
    c.scale[l] = scale ? scale[l] : 1.0f;
    c.inv_sigma2[l] = inv_sigma2 ? inv_sigma2[l] : 1.0f;
  }
  *out = c;
  return ORBPL_OK;
}

hipStream_t scratch_stream() { return nullptr; }  // host-pointer APIs use the null stream

}  // namespace

bool orbpl::lsd_split_decision(int n_streams) {
  return split_on("ORBPL_LSD_SPLIT", n_streams, kLsdSplitMin);
}

extern "C" {

int orbpl_frame_prepare(const orbpl_camera* cam, const orbpl_keypoint* kps, int n,
                        const float* depth, orbpl_keypoint* kps_un, float* depth_out,
                        float* uright_out, int32_t* grid_cell, float* bounds) {
  if (!cam || n < 0 || (n > 0 && (!kps || !kps_un || !depth_out || !uright_out || !grid_cell)))
    return arg_fail("bad argument");
  TrackConsts c;
  int rc = make_consts(cam, nullptr, nullptr, 1, &c);
  if (rc) return rc;
  if (bounds) { bounds[0] = c.minX; bounds[1] = c.maxX; bounds[2] = c.minY; bounds[3] = c.maxY; }
  if (n == 0) return ORBPL_OK;
  DBuf dk, dn, dd, dku, ddo, dur, dgc;
  const size_t imgb = depth ? (size_t)cam->width * cam->height * 4 : 0;
  HIP_CHECK(dk.alloc((size_t)n * sizeof(KeyPointD)));
  HIP_CHECK(dn.alloc(4));
  if (depth) HIP_CHECK(dd.alloc(imgb));
  HIP_CHECK(dku.alloc((size_t)n * sizeof(KeyPointD)));
  HIP_CHECK(ddo.alloc((size_t)n * 4));
  HIP_CHECK(dur.alloc((size_t)n * 4));
  HIP_CHECK(dgc.alloc((size_t)n * 4));
  HIP_CHECK(hipMemcpy(dk.p, kps, (size_t)n * sizeof(KeyPointD), hipMemcpyHostToDevice));
  HIP_CHECK(hipMemcpy(dn.p, &n, 4, hipMemcpyHostToDevice));
  if (depth) HIP_CHECK(hipMemcpy(dd.p, depth, imgb, hipMemcpyHostToDevice));
  launch_frame_prepare(c, dk.as<KeyPointD>(), dn.as<int>(), n, depth ? dd.as<float>() : nullptr, 0,
                       dku.as<KeyPointD>(), ddo.as<float>(), dur.as<float>(), dgc.as<int>(), 1,
                       scratch_stream());
  HIP_CHECK(hipGetLastError());
  HIP_CHECK(hipMemcpy(kps_un, dku.p, (size_t)n * sizeof(KeyPointD), hipMemcpyDeviceToHost));
  HIP_CHECK(hipMemcpy(depth_out, ddo.p, (size_t)n * 4, hipMemcpyDeviceToHost));
  HIP_CHECK(hipMemcpy(uright_out, dur.p, (size_t)n * 4, hipMemcpyDeviceToHost));
  HIP_CHECK(hipMemcpy(grid_cell, dgc.p, (size_t)n * 4, hipMemcpyDeviceToHost));
  return ORBPL_OK;
}

int orbm_search_by_projection_last(const orbpl_camera* cam, const float* scale_factors, int nlevels,
                                   const orbpl_match_current* cur, const orbpl_match_last* last,
                                   float th, int mono, int check_orientation, int32_t* match,
                                   int* nmatches) {
  if (!cam || !scale_factors || !cur || !last || !match || !nmatches) return arg_fail("NULL argument");
  const int n = cur->n, nl = last->n;
  if (n < 0 || nl < 0 || n > kMatchMaxKp || nl > kMatchMaxKp)
    return arg_fail("keypoint count exceeds the matcher capacity (2048)");
  TrackConsts c;
  int rc = make_consts(cam, scale_factors, nullptr, nlevels, &c);
  if (rc) return rc;
  const int P = std::max(1, std::max(n, nl));
  DBuf d_cku, d_cdesc, d_cur, d_cg, d_cn, d_lku, d_lhas, d_lout, d_lxyz, d_ldesc, d_lnobs, d_ln, d_T,
      d_match, d_nm;
  HIP_CHECK(d_cku.alloc((size_t)P * sizeof(KeyPointD)));
  HIP_CHECK(d_cdesc.alloc((size_t)P * 32));
  HIP_CHECK(d_cur.alloc((size_t)P * 4));
  HIP_CHECK(d_cg.alloc((size_t)P * 4));
  HIP_CHECK(d_cn.alloc(4));
  HIP_CHECK(d_lku.alloc((size_t)P * sizeof(KeyPointD)));
  HIP_CHECK(d_lhas.alloc((size_t)P));
  HIP_CHECK(d_lout.alloc((size_t)P));
  HIP_CHECK(d_lxyz.alloc((size_t)P * 12));
  HIP_CHECK(d_ldesc.alloc((size_t)P * 32));
  HIP_CHECK(d_lnobs.alloc((size_t)P * 4));
  HIP_CHECK(d_ln.alloc(4));
  HIP_CHECK(d_T.alloc(32 * 4));
  HIP_CHECK(d_match.alloc((size_t)P * 4));
  HIP_CHECK(d_nm.alloc(4));
  if (n) {
    HIP_CHECK(hipMemcpy(d_cku.p, cur->kps_un, (size_t)n * sizeof(KeyPointD), hipMemcpyHostToDevice));
    HIP_CHECK(hipMemcpy(d_cdesc.p, cur->desc, (size_t)n * 32, hipMemcpyHostToDevice));
    HIP_CHECK(hipMemcpy(d_cur.p, cur->uright, (size_t)n * 4, hipMemcpyHostToDevice));
  }
  HIP_CHECK(hipMemcpy(d_cn.p, &n, 4, hipMemcpyHostToDevice));
  if (nl) {
    HIP_CHECK(hipMemcpy(d_lku.p, last->kps_un, (size_t)nl * sizeof(KeyPointD), hipMemcpyHostToDevice));
    HIP_CHECK(hipMemcpy(d_lhas.p, last->has_mp, (size_t)nl, hipMemcpyHostToDevice));
    HIP_CHECK(hipMemcpy(d_lout.p, last->outlier, (size_t)nl, hipMemcpyHostToDevice));
    HIP_CHECK(hipMemcpy(d_lxyz.p, last->mp_xyz, (size_t)nl * 12, hipMemcpyHostToDevice));
    HIP_CHECK(hipMemcpy(d_ldesc.p, last->mp_desc, (size_t)nl * 32, hipMemcpyHostToDevice));
    HIP_CHECK(hipMemcpy(d_lnobs.p, last->mp_nobs, (size_t)nl * 4, hipMemcpyHostToDevice));
  }
  HIP_CHECK(hipMemcpy(d_ln.p, &nl, 4, hipMemcpyHostToDevice));
  HIP_CHECK(hipMemcpy(d_T.as<float>(), cur->Tcw, 64, hipMemcpyHostToDevice));
  HIP_CHECK(hipMemcpy(d_T.as<float>() + 16, last->Tcw, 64, hipMemcpyHostToDevice));
  MatchLaunch m{};
  m.cur_kps_un = d_cku.as<KeyPointD>();
  m.cur_desc = d_cdesc.as<uint8_t>();
  m.cur_uright = d_cur.as<float>();
  m.cur_gcell = nullptr;  // computed on device from kps_un (PosInGrid)
  m.cur_n = d_cn.as<int>();
  m.last_kps_un = d_lku.as<KeyPointD>();
  m.last_has_mp = d_lhas.as<uint8_t>();
  m.last_outlier = d_lout.as<uint8_t>();
  m.last_xyz = d_lxyz.as<float>();
  m.last_desc = d_ldesc.as<uint8_t>();
  m.last_nobs = d_lnobs.as<int>();
  m.last_n = d_ln.as<int>();
  m.kp_pitch = P;
  m.Tcw = d_T.as<float>();
  m.Tlw = d_T.as<float>() + 16;
  m.pose_stride = 32;
  m.match = d_match.as<int>();
  m.nmatches = d_nm.as<int>();
  m.nm_stride = 1;
  m.th = th;
  m.mono = mono;
  m.check_ori = check_orientation;
  m.retry = 0;
  m.active = nullptr;
  launch_match_last(c, m, 1, scratch_stream());
  HIP_CHECK(hipGetLastError());
  if (n) HIP_CHECK(hipMemcpy(match, d_match.p, (size_t)n * 4, hipMemcpyDeviceToHost));
  HIP_CHECK(hipMemcpy(nmatches, d_nm.p, 4, hipMemcpyDeviceToHost));
  return ORBPL_OK;
}

int orbpl_pose_optimization(const orbpl_camera* cam, const orbpl_pose_problem* P, float* Tcw,
                            uint8_t* outlier, uint8_t* line_outlier, int* n_inliers) {
  return orbpl_pose_optimization_ex(cam, P, 0, Tcw, outlier, line_outlier, n_inliers);
}

int orbpl_pose_optimization_ex(const orbpl_camera* cam, const orbpl_pose_problem* P, int flags,
                               float* Tcw, uint8_t* outlier, uint8_t* line_outlier,
                               int* n_inliers) {
  if (!cam || !P || !Tcw || !n_inliers) return arg_fail("NULL argument");
  if (flags & ~ORBPL_POSE_FIXED_LINE_JAC) return arg_fail("unknown pose flag");
  const int n = P->n, nl = P->nl;
  if (n < 0 || nl < 0 || n + nl > kPoseMaxEdges) return arg_fail("too many edges (max 2304)");
  if (n > 0 && (!P->kps_un || !P->uright || !P->has_mp || !P->mp_xyz || !outlier))
    return arg_fail("NULL point arrays");
  if (nl > 0 && (!P->kl_obs || !P->kl_octave || !P->has_ml || !P->ml_xyz || !line_outlier))
    return arg_fail("NULL line arrays");
  TrackConsts c;
  int rc = make_consts(cam, nullptr, P->inv_sigma2, P->nlevels, &c);
  if (rc) return rc;
  const int Pn = std::max(1, n), Pl = std::max(1, nl);
  DBuf d_ku, d_ur, d_has, d_xyz, d_n, d_klo, d_klv, d_hml, d_mlx, d_T, d_out, d_lout, d_nin, d_edges;
  HIP_CHECK(d_ku.alloc((size_t)Pn * sizeof(KeyPointD)));
  HIP_CHECK(d_ur.alloc((size_t)Pn * 4));
  HIP_CHECK(d_has.alloc((size_t)Pn));
  HIP_CHECK(d_xyz.alloc((size_t)Pn * 12));
  HIP_CHECK(d_n.alloc(4));
  HIP_CHECK(d_klo.alloc((size_t)Pl * 16));
  HIP_CHECK(d_klv.alloc((size_t)Pl * 4));
  HIP_CHECK(d_hml.alloc((size_t)Pl));
  HIP_CHECK(d_mlx.alloc((size_t)Pl * 24));
  HIP_CHECK(d_T.alloc(64));
  HIP_CHECK(d_out.alloc((size_t)Pn));
  HIP_CHECK(d_lout.alloc((size_t)Pl));
  HIP_CHECK(d_nin.alloc(4));
  HIP_CHECK(d_edges.alloc((size_t)kPoseMaxEdges * pose_edge_bytes()));
  if (n) {
    HIP_CHECK(hipMemcpy(d_ku.p, P->kps_un, (size_t)n * sizeof(KeyPointD), hipMemcpyHostToDevice));
    HIP_CHECK(hipMemcpy(d_ur.p, P->uright, (size_t)n * 4, hipMemcpyHostToDevice));
    HIP_CHECK(hipMemcpy(d_has.p, P->has_mp, (size_t)n, hipMemcpyHostToDevice));
    HIP_CHECK(hipMemcpy(d_xyz.p, P->mp_xyz, (size_t)n * 12, hipMemcpyHostToDevice));
    HIP_CHECK(hipMemcpy(d_out.p, outlier, (size_t)n, hipMemcpyHostToDevice));
  }
  if (nl) {
    HIP_CHECK(hipMemcpy(d_klo.p, P->kl_obs, (size_t)nl * 16, hipMemcpyHostToDevice));
    HIP_CHECK(hipMemcpy(d_klv.p, P->kl_octave, (size_t)nl * 4, hipMemcpyHostToDevice));
    HIP_CHECK(hipMemcpy(d_hml.p, P->has_ml, (size_t)nl, hipMemcpyHostToDevice));
    HIP_CHECK(hipMemcpy(d_mlx.p, P->ml_xyz, (size_t)nl * 24, hipMemcpyHostToDevice));
    HIP_CHECK(hipMemcpy(d_lout.p, line_outlier, (size_t)nl, hipMemcpyHostToDevice));
  }
  HIP_CHECK(hipMemcpy(d_n.p, &n, 4, hipMemcpyHostToDevice));
  HIP_CHECK(hipMemcpy(d_T.p, Tcw, 64, hipMemcpyHostToDevice));
  PoseLaunch p{};
  p.kps_un = d_ku.as<KeyPointD>();
  p.uright = d_ur.as<float>();
  p.match = nullptr;
  p.has_mp = d_has.as<uint8_t>();
  p.mp_xyz = d_xyz.as<float>();
  p.n = d_n.as<int>();
  p.kp_pitch = Pn;
  p.kl_obs = d_klo.as<float>();
  p.kl_octave = d_klv.as<int>();
  p.has_ml = d_hml.as<uint8_t>();
  p.ml_xyz = d_mlx.as<float>();
  p.nl = nl;
  p.Tcw = d_T.as<float>();
  p.pose_stride = 16;
  p.outlier = d_out.as<uint8_t>();
  p.line_outlier = d_lout.as<uint8_t>();
  p.ninliers = d_nin.as<int>();
  p.nm_stride = 1;
  p.active = nullptr;
  p.edges = reinterpret_cast<PoseEdge*>(d_edges.p);
  p.fixed_line_jac = (flags & ORBPL_POSE_FIXED_LINE_JAC) ? 1 : 0;
  launch_pose(c, p, 1, scratch_stream());
  HIP_CHECK(hipGetLastError());
  HIP_CHECK(hipMemcpy(Tcw, d_T.p, 64, hipMemcpyDeviceToHost));
  if (n) HIP_CHECK(hipMemcpy(outlier, d_out.p, (size_t)n, hipMemcpyDeviceToHost));
  if (nl) HIP_CHECK(hipMemcpy(line_outlier, d_lout.p, (size_t)nl, hipMemcpyDeviceToHost));
  HIP_CHECK(hipMemcpy(n_inliers, d_nin.p, 4, hipMemcpyDeviceToHost));
  return ORBPL_OK;
}

int orbpl_frame_is_in_frustum(const orbpl_camera* cam, float scale_factor, int nlevels,
                              const float* Tcw, int n, const float* xyz, const float* normal,
                              const float* min_dist, const float* max_dist, float view_cos_limit,
                              uint8_t* in_view, float* proj_x, float* proj_y, float* proj_xr,
                              int32_t* level, float* view_cos) {
  if (!cam || !Tcw || n < 0 || nlevels < 1 || nlevels > kMaxLevelsT) return arg_fail("bad argument");
  if (n > 0 && (!xyz || !normal || !min_dist || !max_dist || !in_view || !proj_x || !proj_y ||
                !proj_xr || !level || !view_cos))
    return arg_fail("NULL map point arrays");
  TrackConsts c;
  int rc = make_consts(cam, nullptr, nullptr, nlevels, &c);
  if (rc) return rc;
  if (n == 0) return ORBPL_OK;
  // Frame::mfLogScaleFactor = log(mfScaleFactor) on a float (P15)
  const float log_scale = (float)lsdm::log_((double)scale_factor);
  DBuf dT, dx, dn, dmi, dma, div, dpx, dpy, dpr, dl, dvc;
  HIP_CHECK(dT.alloc(64));
  HIP_CHECK(dx.alloc((size_t)n * 12));
  HIP_CHECK(dn.alloc((size_t)n * 12));
  HIP_CHECK(dmi.alloc((size_t)n * 4));
  HIP_CHECK(dma.alloc((size_t)n * 4));
  HIP_CHECK(div.alloc(n));
  HIP_CHECK(dpx.alloc((size_t)n * 4));
  HIP_CHECK(dpy.alloc((size_t)n * 4));
  HIP_CHECK(dpr.alloc((size_t)n * 4));
  HIP_CHECK(dl.alloc((size_t)n * 4));
  HIP_CHECK(dvc.alloc((size_t)n * 4));
  HIP_CHECK(hipMemcpy(dT.p, Tcw, 64, hipMemcpyHostToDevice));
  HIP_CHECK(hipMemcpy(dx.p, xyz, (size_t)n * 12, hipMemcpyHostToDevice));
  HIP_CHECK(hipMemcpy(dn.p, normal, (size_t)n * 12, hipMemcpyHostToDevice));
  HIP_CHECK(hipMemcpy(dmi.p, min_dist, (size_t)n * 4, hipMemcpyHostToDevice));
  HIP_CHECK(hipMemcpy(dma.p, max_dist, (size_t)n * 4, hipMemcpyHostToDevice));
  InFrustumArgs a{n, dT.as<float>(), dx.as<float>(), dn.as<float>(), dmi.as<float>(),
                  dma.as<float>(), view_cos_limit, div.as<uint8_t>(), dpx.as<float>(),
                  dpy.as<float>(), dpr.as<float>(), dl.as<int>(), dvc.as<float>()};
  launch_in_frustum(c, log_scale, a, scratch_stream());
  HIP_CHECK(hipGetLastError());
  HIP_CHECK(hipMemcpy(in_view, div.p, n, hipMemcpyDeviceToHost));
  HIP_CHECK(hipMemcpy(proj_x, dpx.p, (size_t)n * 4, hipMemcpyDeviceToHost));
  HIP_CHECK(hipMemcpy(proj_y, dpy.p, (size_t)n * 4, hipMemcpyDeviceToHost));
  HIP_CHECK(hipMemcpy(proj_xr, dpr.p, (size_t)n * 4, hipMemcpyDeviceToHost));
  HIP_CHECK(hipMemcpy(level, dl.p, (size_t)n * 4, hipMemcpyDeviceToHost));
  HIP_CHECK(hipMemcpy(view_cos, dvc.p, (size_t)n * 4, hipMemcpyDeviceToHost));
  return ORBPL_OK;
}

int orbm_search_by_projection_local(const orbpl_camera* cam, const float* scale_factors,
                                    int nlevels, const orbpl_match_current* cur, int nmp,
                                    const uint8_t* in_view, const float* proj_x,
                                    const float* proj_y, const float* proj_xr,
                                    const int32_t* level, const float* view_cos,
                                    const uint8_t* mp_desc, const int32_t* mp_nobs,
                                    const int32_t* cur_nobs, float th, float nnratio,
                                    int32_t* match, int* nmatches) {
  if (!cam || !scale_factors || !cur || !nmatches || nmp < 0) return arg_fail("bad argument");
  const int n = cur->n;
  if (n < 0 || n > kMatchMaxKp) return arg_fail("keypoint count exceeds the matcher capacity (2048)");
  if (n > 0 && (!cur->kps_un || !cur->desc || !cur->uright || !match)) return arg_fail("NULL frame arrays");
  if (nmp > 0 && (!in_view || !proj_x || !proj_y || !proj_xr || !level || !view_cos || !mp_desc ||
                  !mp_nobs))
    return arg_fail("NULL map point arrays");
  for (int i = 0; i < nmp; i++)
    if (in_view[i] && (level[i] < 0 || level[i] >= nlevels)) return arg_fail("level out of range");
  TrackConsts c;
  int rc = make_consts(cam, scale_factors, nullptr, nlevels, &c);
  if (rc) return rc;
  const int P = std::max(1, n), M = std::max(1, nmp);
  DBuf dku, dde, dur, dcn, div, dpx, dpy, dpr, dl, dvc, dmd, dmn, dm, dnm, dsc;
  HIP_CHECK(dku.alloc((size_t)P * sizeof(KeyPointD)));
  HIP_CHECK(dde.alloc((size_t)P * 32));
  HIP_CHECK(dur.alloc((size_t)P * 4));
  HIP_CHECK(dcn.alloc((size_t)P * 4));
  HIP_CHECK(div.alloc(M));
  HIP_CHECK(dpx.alloc((size_t)M * 4));
  HIP_CHECK(dpy.alloc((size_t)M * 4));
  HIP_CHECK(dpr.alloc((size_t)M * 4));
  HIP_CHECK(dl.alloc((size_t)M * 4));
  HIP_CHECK(dvc.alloc((size_t)M * 4));
  HIP_CHECK(dmd.alloc((size_t)M * 32));
  HIP_CHECK(dmn.alloc((size_t)M * 4));
  HIP_CHECK(dm.alloc((size_t)P * 4));
  HIP_CHECK(dnm.alloc(4));
  HIP_CHECK(dsc.alloc((size_t)M * sizeof(int4)));
  if (n) {
    HIP_CHECK(hipMemcpy(dku.p, cur->kps_un, (size_t)n * sizeof(KeyPointD), hipMemcpyHostToDevice));
    HIP_CHECK(hipMemcpy(dde.p, cur->desc, (size_t)n * 32, hipMemcpyHostToDevice));
    HIP_CHECK(hipMemcpy(dur.p, cur->uright, (size_t)n * 4, hipMemcpyHostToDevice));
    if (cur_nobs) HIP_CHECK(hipMemcpy(dcn.p, cur_nobs, (size_t)n * 4, hipMemcpyHostToDevice));
  }
  if (nmp) {
    HIP_CHECK(hipMemcpy(div.p, in_view, nmp, hipMemcpyHostToDevice));
    HIP_CHECK(hipMemcpy(dpx.p, proj_x, (size_t)nmp * 4, hipMemcpyHostToDevice));
    HIP_CHECK(hipMemcpy(dpy.p, proj_y, (size_t)nmp * 4, hipMemcpyHostToDevice));
    HIP_CHECK(hipMemcpy(dpr.p, proj_xr, (size_t)nmp * 4, hipMemcpyHostToDevice));
    HIP_CHECK(hipMemcpy(dl.p, level, (size_t)nmp * 4, hipMemcpyHostToDevice));
    HIP_CHECK(hipMemcpy(dvc.p, view_cos, (size_t)nmp * 4, hipMemcpyHostToDevice));
    HIP_CHECK(hipMemcpy(dmd.p, mp_desc, (size_t)nmp * 32, hipMemcpyHostToDevice));
    HIP_CHECK(hipMemcpy(dmn.p, mp_nobs, (size_t)nmp * 4, hipMemcpyHostToDevice));
  }
  LocalArgs a{};
  a.kps_un = dku.as<KeyPointD>();
  a.desc = dde.as<uint8_t>();
  a.uright = dur.as<float>();
  a.n = n;
  a.cur_nobs = cur_nobs ? dcn.as<int>() : nullptr;
  a.nmp = nmp;
  a.in_view = div.as<uint8_t>();
  a.proj_x = dpx.as<float>();
  a.proj_y = dpy.as<float>();
  a.proj_xr = dpr.as<float>();
  a.level = dl.as<int>();
  a.view_cos = dvc.as<float>();
  a.mp_desc = dmd.as<uint8_t>();
  a.mp_nobs = dmn.as<int>();
  a.th = th;
  a.nnratio = nnratio;
  a.match = dm.as<int>();
  a.nmatches = dnm.as<int>();
  a.scratch = dsc.as<int4>();
  launch_match_local(c, a, scratch_stream());
  HIP_CHECK(hipGetLastError());
  if (n) HIP_CHECK(hipMemcpy(match, dm.p, (size_t)n * 4, hipMemcpyDeviceToHost));
  HIP_CHECK(hipMemcpy(nmatches, dnm.p, 4, hipMemcpyDeviceToHost));
  return ORBPL_OK;
}

int orbpl_line_frame_prepare(const orbpl_camera* cam, const orbpl_keyline* kl, int n,
                             const float* depth, orbpl_keyline* kl_un, float* dstart, float* dend,
                             float* ur_start, float* ur_end) {
  if (!cam || n < 0 || (n > 0 && (!kl || !kl_un || !dstart || !dend || !ur_start || !ur_end)))
    return arg_fail("bad argument");
  if (n > kLineKeep) return arg_fail("more key lines than LineExtractor keeps (80)");
  TrackConsts c;
  int rc = make_consts(cam, nullptr, nullptr, 1, &c);
  if (rc) return rc;
  if (n == 0) return ORBPL_OK;
  DBuf dn, dkl, dku, dd, dds, dde, dus, due;
  const size_t imgb = depth ? (size_t)cam->width * cam->height * 4 : 0;
  HIP_CHECK(dn.alloc(4));
  HIP_CHECK(dkl.alloc((size_t)kLineKeep * sizeof(orbpl_keyline)));
  HIP_CHECK(dku.alloc((size_t)kLineKeep * sizeof(orbpl_keyline)));
  if (depth) HIP_CHECK(dd.alloc(imgb));
  HIP_CHECK(dds.alloc(kLineKeep * 4));
  HIP_CHECK(dde.alloc(kLineKeep * 4));
  HIP_CHECK(dus.alloc(kLineKeep * 4));
  HIP_CHECK(due.alloc(kLineKeep * 4));
  DBuf dlm, dlo;
  HIP_CHECK(dlm.alloc(kLineKeep * 4));
  HIP_CHECK(dlo.alloc(kLineKeep));
  HIP_CHECK(hipMemcpy(dn.p, &n, 4, hipMemcpyHostToDevice));
  HIP_CHECK(hipMemcpy(dkl.p, kl, (size_t)n * sizeof(orbpl_keyline), hipMemcpyHostToDevice));
  if (depth) HIP_CHECK(hipMemcpy(dd.p, depth, imgb, hipMemcpyHostToDevice));
  LineTrackArgs a{};
  a.nl = dn.as<int>();
  a.kl = dkl.as<orbpl_keyline>();
  a.kl_un = dku.as<orbpl_keyline>();
  a.depth = depth ? dd.as<float>() : nullptr;
  a.depth_pitch = 0;
  a.dstart = dds.as<float>();
  a.dend = dde.as<float>();
  a.ur_start = dus.as<float>();
  a.ur_end = due.as<float>();
  a.lmatch = dlm.as<int>();
  a.loutlier = dlo.as<uint8_t>();
  launch_line_prepare(c, a, 1, scratch_stream());
  HIP_CHECK(hipGetLastError());
  HIP_CHECK(hipMemcpy(kl_un, dku.p, (size_t)n * sizeof(orbpl_keyline), hipMemcpyDeviceToHost));
  HIP_CHECK(hipMemcpy(dstart, dds.p, (size_t)n * 4, hipMemcpyDeviceToHost));
  HIP_CHECK(hipMemcpy(dend, dde.p, (size_t)n * 4, hipMemcpyDeviceToHost));
  HIP_CHECK(hipMemcpy(ur_start, dus.p, (size_t)n * 4, hipMemcpyDeviceToHost));
  HIP_CHECK(hipMemcpy(ur_end, due.p, (size_t)n * 4, hipMemcpyDeviceToHost));
  return ORBPL_OK;
}

int orbl_search_by_projection_last(const orbpl_camera* cam, const float* Tcw, int ncur,
                                   const orbpl_keyline* cur_kl_un, const uint8_t* cur_desc,
                                   int nlast, const orbpl_keyline* last_kl_un,
                                   const uint8_t* has_ml, const uint8_t* last_outlier,
                                   const float* ml_xyz6, const uint8_t* last_desc, int32_t* match,
                                   int* nmatches) {
  if (!cam || !Tcw || !nmatches || ncur < 0 || nlast < 0) return arg_fail("bad argument");
  if (ncur > kLineKeep || nlast > kLineKeep)
    return arg_fail("more key lines than LineExtractor keeps (80)");
  if ((ncur > 0 && (!cur_kl_un || !cur_desc || !match)) ||
      (nlast > 0 && (!last_kl_un || !has_ml || !last_outlier || !ml_xyz6 || !last_desc)))
    return arg_fail("NULL line arrays");
  TrackConsts c;
  int rc = make_consts(cam, nullptr, nullptr, 1, &c);
  if (rc) return rc;
  const size_t L = kLineKeep;
  DBuf dn, dln, dku, dde, dlk, dhm, dlo, dxyz, dld, dm, dst;
  HIP_CHECK(dn.alloc(4));
  HIP_CHECK(dln.alloc(4));
  HIP_CHECK(dku.alloc(L * sizeof(orbpl_keyline)));
  HIP_CHECK(dde.alloc(L * 32));
  HIP_CHECK(dlk.alloc(L * sizeof(orbpl_keyline)));
  HIP_CHECK(dhm.alloc(L));
  HIP_CHECK(dlo.alloc(L));
  HIP_CHECK(dxyz.alloc(L * 24));
  HIP_CHECK(dld.alloc(L * 32));
  HIP_CHECK(dm.alloc(L * 4));
  HIP_CHECK(dst.alloc(sizeof(StreamState)));
  StreamState st{};
  memcpy(st.Tcw, Tcw, 64);
  st.has_last = 1;
  HIP_CHECK(hipMemcpy(dst.p, &st, sizeof(st), hipMemcpyHostToDevice));
  HIP_CHECK(hipMemcpy(dn.p, &ncur, 4, hipMemcpyHostToDevice));
  HIP_CHECK(hipMemcpy(dln.p, &nlast, 4, hipMemcpyHostToDevice));
  if (ncur) {
    HIP_CHECK(hipMemcpy(dku.p, cur_kl_un, ncur * sizeof(orbpl_keyline), hipMemcpyHostToDevice));
    HIP_CHECK(hipMemcpy(dde.p, cur_desc, (size_t)ncur * 32, hipMemcpyHostToDevice));
  }
  if (nlast) {
    HIP_CHECK(hipMemcpy(dlk.p, last_kl_un, nlast * sizeof(orbpl_keyline), hipMemcpyHostToDevice));
    HIP_CHECK(hipMemcpy(dhm.p, has_ml, nlast, hipMemcpyHostToDevice));
    HIP_CHECK(hipMemcpy(dlo.p, last_outlier, nlast, hipMemcpyHostToDevice));
    HIP_CHECK(hipMemcpy(dxyz.p, ml_xyz6, (size_t)nlast * 24, hipMemcpyHostToDevice));
    HIP_CHECK(hipMemcpy(dld.p, last_desc, (size_t)nlast * 32, hipMemcpyHostToDevice));
  }
  LineTrackArgs a{};
  a.nl = dn.as<int>();
  a.kl_un = dku.as<orbpl_keyline>();
  a.desc = dde.as<uint8_t>();
  a.lmatch = dm.as<int>();
  a.last_nl = dln.as<int>();
  a.last_kl_un = dlk.as<orbpl_keyline>();
  a.last_has_ml = dhm.as<uint8_t>();
  a.last_loutlier = dlo.as<uint8_t>();
  a.last_ml_xyz = dxyz.as<float>();
  a.last_desc = dld.as<uint8_t>();
  launch_line_match(c, a, dst.as<StreamState>(), 1, scratch_stream());
  HIP_CHECK(hipGetLastError());
  if (ncur) HIP_CHECK(hipMemcpy(match, dm.p, (size_t)ncur * 4, hipMemcpyDeviceToHost));
  HIP_CHECK(hipMemcpy(&st, dst.p, sizeof(st), hipMemcpyDeviceToHost));
  *nmatches = st.nlmatches;
  return ORBPL_OK;
}

int orbm_search_by_bow(int nkf, const int32_t* kf_node, const uint8_t* kf_valid,
                       const uint8_t* kf_desc, const float* kf_angle, int nf, const int32_t* f_node,
                       const uint8_t* f_desc, const float* f_angle, float nnratio, int check_ori,
                       int32_t* match, int* nmatches) {
  if (nkf < 0 || nf < 0 || !nmatches) return arg_fail("bad argument");
  if (nkf > 2048 || nf > 2048) return arg_fail("more than 2048 features");
  if ((nkf > 0 && (!kf_node || !kf_valid || !kf_desc || !kf_angle)) ||
      (nf > 0 && (!f_node || !f_desc || !f_angle || !match)))
    return arg_fail("NULL feature arrays");
  for (int i = 0; i < nkf; i++)
    if (kf_node[i] >= (1 << 21) - 1) return arg_fail("vocabulary node id >= 2^21 - 1");
  for (int i = 0; i < nf; i++)
    if (f_node[i] >= (1 << 21) - 1) return arg_fail("vocabulary node id >= 2^21 - 1");
  const size_t K = std::max(1, nkf), F = std::max(1, nf);
  DBuf dkn, dkv, dkd, dka, dfn, dfd, dfa, dm, dnm;
  HIP_CHECK(dkn.alloc(K * 4));
  HIP_CHECK(dkv.alloc(K));
  HIP_CHECK(dkd.alloc(K * 32));
  HIP_CHECK(dka.alloc(K * 4));
  HIP_CHECK(dfn.alloc(F * 4));
  HIP_CHECK(dfd.alloc(F * 32));
  HIP_CHECK(dfa.alloc(F * 4));
  HIP_CHECK(dm.alloc(F * 4));
  HIP_CHECK(dnm.alloc(4));
  if (nkf) {
    HIP_CHECK(hipMemcpy(dkn.p, kf_node, K * 4, hipMemcpyHostToDevice));
    HIP_CHECK(hipMemcpy(dkv.p, kf_valid, K, hipMemcpyHostToDevice));
    HIP_CHECK(hipMemcpy(dkd.p, kf_desc, K * 32, hipMemcpyHostToDevice));
    HIP_CHECK(hipMemcpy(dka.p, kf_angle, K * 4, hipMemcpyHostToDevice));
  }
  if (nf) {
    HIP_CHECK(hipMemcpy(dfn.p, f_node, F * 4, hipMemcpyHostToDevice));
    HIP_CHECK(hipMemcpy(dfd.p, f_desc, F * 32, hipMemcpyHostToDevice));
    HIP_CHECK(hipMemcpy(dfa.p, f_angle, F * 4, hipMemcpyHostToDevice));
  }
  BowArgs a{nkf, dkn.as<int>(), dkv.as<uint8_t>(), dkd.as<uint8_t>(), dka.as<float>(), nf,
            dfn.as<int>(), dfd.as<uint8_t>(), dfa.as<float>(), nnratio, check_ori,
            dm.as<int>(), dnm.as<int>()};
  launch_match_bow(a, scratch_stream());
  HIP_CHECK(hipGetLastError());
  if (nf) HIP_CHECK(hipMemcpy(match, dm.p, F * 4, hipMemcpyDeviceToHost));
  HIP_CHECK(hipMemcpy(nmatches, dnm.p, 4, hipMemcpyDeviceToHost));
  return ORBPL_OK;
}

int orbpl_stereo_matches(const orbpl_camera* cam, orbx_ctx* left, orbx_ctx* right, int frame,
                         const orbpl_keypoint* kl, const uint8_t* dl, int n,
                         const orbpl_keypoint* kr, const uint8_t* dr, int nr, float* uright,
                         float* depth) {
  if (!cam || !left || !right || n < 0 || nr < 0) return arg_fail("bad argument");
  if (n > 4096 || nr > 4096) return arg_fail("more than 4096 keypoints");
  if ((n > 0 && (!kl || !dl || !uright || !depth)) || (nr > 0 && (!kr || !dr)))
    return arg_fail("NULL keypoint arrays");
  const uint8_t *pl = nullptr, *pr = nullptr;
  const OrbGeom *gl = nullptr, *gr = nullptr;
  hipStream_t sl, sr;
  int rc = orbx_device_pyramid(left, frame, &pl, &gl, &sl);
  if (rc) return rc;
  rc = orbx_device_pyramid(right, frame, &pr, &gr, &sr);
  if (rc) return rc;
  if (gl->nlevels != gr->nlevels || gl->W != gr->W || gl->H != gr->H || gl->nlevels > 8)
    return arg_fail("left and right extractors differ");
  if (gl->H > 1024) return arg_fail("image taller than 1024 rows");
  if (n == 0) return ORBPL_OK;
  HIP_CHECK(hipStreamSynchronize(sl));
  HIP_CHECK(hipStreamSynchronize(sr));
  const int cap = std::max(1, nr) * 20;
  DBuf dkl, ddl, dkr, ddr, dur, ddp, dsad, dent, derr;
  HIP_CHECK(dkl.alloc((size_t)n * sizeof(KeyPointD)));
  HIP_CHECK(ddl.alloc((size_t)n * 32));
  HIP_CHECK(dkr.alloc((size_t)std::max(1, nr) * sizeof(KeyPointD)));
  HIP_CHECK(ddr.alloc((size_t)std::max(1, nr) * 32));
  HIP_CHECK(dur.alloc((size_t)n * 4));
  HIP_CHECK(ddp.alloc((size_t)n * 4));
  HIP_CHECK(dsad.alloc((size_t)n * 4));
  HIP_CHECK(dent.alloc((size_t)cap * 2));
  HIP_CHECK(derr.alloc(4));
  HIP_CHECK(hipMemset(derr.p, 0, 4));
  HIP_CHECK(hipMemcpy(dkl.p, kl, (size_t)n * sizeof(KeyPointD), hipMemcpyHostToDevice));
  HIP_CHECK(hipMemcpy(ddl.p, dl, (size_t)n * 32, hipMemcpyHostToDevice));
  if (nr) {
    HIP_CHECK(hipMemcpy(dkr.p, kr, (size_t)nr * sizeof(KeyPointD), hipMemcpyHostToDevice));
    HIP_CHECK(hipMemcpy(ddr.p, dr, (size_t)nr * 32, hipMemcpyHostToDevice));
  }
  StereoArgs a{};
  a.n = n;
  a.kl = dkl.as<KeyPointD>();
  a.dl = ddl.as<uint8_t>();
  a.nr = nr;
  a.kr = dkr.as<KeyPointD>();
  a.dr = ddr.as<uint8_t>();
  a.pyrL = pl;
  a.pyrR = pr;
  for (int l = 0; l < gl->nlevels; l++) {
    a.lv[l] = gl->lv[l];
    a.scale[l] = gl->lv[l].scale;
    a.inv_scale[l] = 1.0f / gl->lv[l].scale;
  }
  a.nrows = gl->H;
  a.mb = cam->bf / cam->fx;
  a.mbf = cam->bf;
  a.uright = dur.as<float>();
  a.depth = ddp.as<float>();
  a.sad = dsad.as<int>();
  a.entries = dent.as<uint16_t>();
  a.entry_cap = cap;
  a.err = derr.as<int>();
  launch_stereo(a, 1, scratch_stream());
  HIP_CHECK(hipGetLastError());
  int err = 0;
  HIP_CHECK(hipMemcpy(&err, derr.p, 4, hipMemcpyDeviceToHost));
  if (err) return (arg_fail("stereo row band capacity exceeded"), ORBPL_ERR_OVERFLOW);
  HIP_CHECK(hipMemcpy(uright, dur.p, (size_t)n * 4, hipMemcpyDeviceToHost));
  HIP_CHECK(hipMemcpy(depth, ddp.p, (size_t)n * 4, hipMemcpyDeviceToHost));
  return ORBPL_OK;
}

int orbl_frame_is_in_frustum(const float* Tcw, int n, const float* xyz6, uint8_t* in_view) {
  if (!Tcw || n < 0 || (n > 0 && (!xyz6 || !in_view))) return arg_fail("bad argument");
  if (n == 0) return ORBPL_OK;
  DBuf dT, dx, dv;
  HIP_CHECK(dT.alloc(64));
  HIP_CHECK(dx.alloc((size_t)n * 24));
  HIP_CHECK(dv.alloc(n));
  HIP_CHECK(hipMemcpy(dT.p, Tcw, 64, hipMemcpyHostToDevice));
  HIP_CHECK(hipMemcpy(dx.p, xyz6, (size_t)n * 24, hipMemcpyHostToDevice));
  launch_line_in_frustum(dT.as<float>(), n, dx.as<float>(), dv.as<uint8_t>(), scratch_stream());
  HIP_CHECK(hipGetLastError());
  HIP_CHECK(hipMemcpy(in_view, dv.p, n, hipMemcpyDeviceToHost));
  return ORBPL_OK;
}

int orbl_search_by_projection_list(const orbpl_camera* cam, const float* Tcw, int ncur,
                                   const orbpl_keyline* cur_kl_un, const uint8_t* cur_desc,
                                   const int32_t* cur_nobs, int nml, const uint8_t* valid,
                                   const float* ml_xyz6, const uint8_t* ml_desc, int32_t* match,
                                   int* nmatches, int* wiped) {
  if (!cam || !Tcw || !nmatches || ncur < 0 || nml < 0) return arg_fail("bad argument");
  if (ncur > kLineKeep) return arg_fail("more key lines than LineExtractor keeps (80)");
  if ((ncur > 0 && (!cur_kl_un || !cur_desc || !match)) ||
      (nml > 0 && (!valid || !ml_xyz6 || !ml_desc)))
    return arg_fail("NULL line arrays");
  TrackConsts c;
  int rc = make_consts(cam, nullptr, nullptr, 1, &c);
  if (rc) return rc;
  const size_t L = kLineKeep, M = std::max(1, nml);
  DBuf dT, dku, dde, dcn, dv, dx, dmd, dpk, dps, dm, dnm, dw;
  HIP_CHECK(dT.alloc(64));
  HIP_CHECK(dku.alloc(L * sizeof(orbpl_keyline)));
  HIP_CHECK(dde.alloc(L * 32));
  HIP_CHECK(dcn.alloc(L * 4));
  HIP_CHECK(dv.alloc(M));
  HIP_CHECK(dx.alloc(M * 24));
  HIP_CHECK(dmd.alloc(M * 32));
  HIP_CHECK(dpk.alloc(M * sizeof(orbpl_keyline)));
  HIP_CHECK(dps.alloc(M * 4));
  HIP_CHECK(dm.alloc(L * 4));
  HIP_CHECK(dnm.alloc(4));
  HIP_CHECK(dw.alloc(4));
  HIP_CHECK(hipMemcpy(dT.p, Tcw, 64, hipMemcpyHostToDevice));
  if (ncur) {
    HIP_CHECK(hipMemcpy(dku.p, cur_kl_un, ncur * sizeof(orbpl_keyline), hipMemcpyHostToDevice));
    HIP_CHECK(hipMemcpy(dde.p, cur_desc, (size_t)ncur * 32, hipMemcpyHostToDevice));
    if (cur_nobs) HIP_CHECK(hipMemcpy(dcn.p, cur_nobs, (size_t)ncur * 4, hipMemcpyHostToDevice));
  }
  if (nml) {
    HIP_CHECK(hipMemcpy(dv.p, valid, nml, hipMemcpyHostToDevice));
    HIP_CHECK(hipMemcpy(dx.p, ml_xyz6, (size_t)nml * 24, hipMemcpyHostToDevice));
    HIP_CHECK(hipMemcpy(dmd.p, ml_desc, (size_t)nml * 32, hipMemcpyHostToDevice));
  }
  LineListArgs a{};
  a.Tcw = dT.as<float>();
  a.ncur = ncur;
  a.cur_kl_un = dku.as<orbpl_keyline>();
  a.cur_desc = dde.as<uint8_t>();
  a.cur_nobs = cur_nobs ? dcn.as<int>() : nullptr;
  a.nml = nml;
  a.valid = dv.as<uint8_t>();
  a.ml_xyz6 = dx.as<float>();
  a.ml_desc = dmd.as<uint8_t>();
  a.proj_kl = dpk.as<orbpl_keyline>();
  a.proj_src = dps.as<int>();
  a.match = dm.as<int>();
  a.nmatches = dnm.as<int>();
  a.wiped = dw.as<int>();
  launch_line_match_list(c, a, scratch_stream());
  HIP_CHECK(hipGetLastError());
  if (ncur) HIP_CHECK(hipMemcpy(match, dm.p, (size_t)ncur * 4, hipMemcpyDeviceToHost));
  HIP_CHECK(hipMemcpy(nmatches, dnm.p, 4, hipMemcpyDeviceToHost));
  if (wiped) HIP_CHECK(hipMemcpy(wiped, dw.p, 4, hipMemcpyDeviceToHost));
  return ORBPL_OK;
}

int orbl_search_by_projection_pairs(const orbpl_camera* cam, const float* Tcw, int mode, int ncur,
                                    const orbpl_keyline* cur_kl_un, const uint8_t* cur_desc,
                                    const int32_t* cur_nobs, int nml, const uint8_t* valid,
                                    const orbpl_keyline* base_kl, const float* ml_xyz6,
                                    const uint8_t* ml_desc, const int32_t* ml_nobs,
                                    orbpl_keyline* proj_kl, int32_t* proj_src, int* nproj,
                                    int32_t* pairs, int pair_cap, int* npairs, int32_t* match,
                                    int* nmatches, int* wiped) {
  if (!cam || !Tcw || !nmatches || !nproj || !npairs || !wiped || ncur < 0 || nml < 0 ||
      pair_cap < 0 || (mode != 0 && mode != 1))
    return arg_fail("bad argument");
  if (ncur > kLineKeep) return arg_fail("more key lines than LineExtractor keeps (80)");
  if ((ncur > 0 && (!cur_kl_un || !cur_desc || !match)) ||
      (nml > 0 && (!valid || !ml_xyz6 || !ml_desc || !proj_kl || !proj_src)) ||
      (pair_cap > 0 && !pairs))
    return arg_fail("NULL line arrays");
  TrackConsts c;
  int rc = make_consts(cam, nullptr, nullptr, 1, &c);
  if (rc) return rc;
  const size_t L = kLineKeep, M = std::max(1, nml), words = (size_t)(nml + 31) / 32;
  DBuf dT, dku, dde, dcn, dv, dbk, dx, dmd, dmn, dpk, dps, dnp, dok, dpr, dnpr, dm, dnm, dw;
  HIP_CHECK(dT.alloc(64));
  HIP_CHECK(dku.alloc(L * sizeof(orbpl_keyline)));
  HIP_CHECK(dde.alloc(L * 32));
  HIP_CHECK(dcn.alloc(L * 4));
  HIP_CHECK(dv.alloc(M));
  HIP_CHECK(dbk.alloc(M * sizeof(orbpl_keyline)));
  HIP_CHECK(dx.alloc(M * 24));
  HIP_CHECK(dmd.alloc(M * 32));
  HIP_CHECK(dmn.alloc(M * 4));
  HIP_CHECK(dpk.alloc(M * sizeof(orbpl_keyline)));
  HIP_CHECK(dps.alloc(M * 4));
  HIP_CHECK(dnp.alloc(4));
  HIP_CHECK(dok.alloc(std::max<size_t>(1, L * words) * 4));
  HIP_CHECK(dpr.alloc(std::max<size_t>(1, (size_t)pair_cap) * 8));
  HIP_CHECK(dnpr.alloc(4));
  HIP_CHECK(dm.alloc(L * 4));
  HIP_CHECK(dnm.alloc(4));
  HIP_CHECK(dw.alloc(4));
  HIP_CHECK(hipMemcpy(dT.p, Tcw, 64, hipMemcpyHostToDevice));
  if (ncur) {
    HIP_CHECK(hipMemcpy(dku.p, cur_kl_un, ncur * sizeof(orbpl_keyline), hipMemcpyHostToDevice));
    HIP_CHECK(hipMemcpy(dde.p, cur_desc, (size_t)ncur * 32, hipMemcpyHostToDevice));
    if (cur_nobs) HIP_CHECK(hipMemcpy(dcn.p, cur_nobs, (size_t)ncur * 4, hipMemcpyHostToDevice));
  }
  if (nml) {
    HIP_CHECK(hipMemcpy(dv.p, valid, nml, hipMemcpyHostToDevice));
    HIP_CHECK(hipMemcpy(dx.p, ml_xyz6, (size_t)nml * 24, hipMemcpyHostToDevice));
    HIP_CHECK(hipMemcpy(dmd.p, ml_desc, (size_t)nml * 32, hipMemcpyHostToDevice));
    if (base_kl)
      HIP_CHECK(hipMemcpy(dbk.p, base_kl, (size_t)nml * sizeof(orbpl_keyline), hipMemcpyHostToDevice));
    if (ml_nobs) HIP_CHECK(hipMemcpy(dmn.p, ml_nobs, (size_t)nml * 4, hipMemcpyHostToDevice));
  }
  LinePairArgs a{};
  a.Tcw = dT.as<float>();
  a.mode = mode;
  a.ncur = ncur;
  a.cur_kl_un = dku.as<orbpl_keyline>();
  a.cur_desc = dde.as<uint8_t>();
  a.cur_nobs = cur_nobs ? dcn.as<int>() : nullptr;
  a.nml = nml;
  a.valid = dv.as<uint8_t>();
  a.base_kl = base_kl ? dbk.as<orbpl_keyline>() : nullptr;
  a.ml_xyz6 = dx.as<float>();
  a.ml_desc = dmd.as<uint8_t>();
  a.ml_nobs = ml_nobs ? dmn.as<int>() : nullptr;
  a.proj_kl = dpk.as<orbpl_keyline>();
  a.proj_src = dps.as<int>();
  a.nproj = dnp.as<int>();
  a.okbits = dok.as<unsigned>();
  a.pairs = dpr.as<int>();
  a.pair_cap = pair_cap;
  a.npairs = dnpr.as<int>();
  a.match = dm.as<int>();
  a.nmatches = dnm.as<int>();
  a.wiped = dw.as<int>();
  launch_line_pairs(c, a, scratch_stream());
  HIP_CHECK(hipGetLastError());
  int np = 0, npr = 0;
  HIP_CHECK(hipMemcpy(&np, dnp.p, 4, hipMemcpyDeviceToHost));
  HIP_CHECK(hipMemcpy(&npr, dnpr.p, 4, hipMemcpyDeviceToHost));
  if (np) {
    HIP_CHECK(hipMemcpy(proj_kl, dpk.p, (size_t)np * sizeof(orbpl_keyline), hipMemcpyDeviceToHost));
    HIP_CHECK(hipMemcpy(proj_src, dps.p, (size_t)np * 4, hipMemcpyDeviceToHost));
  }
  if (std::min(npr, pair_cap) > 0)
    HIP_CHECK(hipMemcpy(pairs, dpr.p, (size_t)std::min(npr, pair_cap) * 8, hipMemcpyDeviceToHost));
  if (ncur) HIP_CHECK(hipMemcpy(match, dm.p, (size_t)ncur * 4, hipMemcpyDeviceToHost));
  HIP_CHECK(hipMemcpy(nmatches, dnm.p, 4, hipMemcpyDeviceToHost));
  HIP_CHECK(hipMemcpy(wiped, dw.p, 4, hipMemcpyDeviceToHost));
  *nproj = np;
  *npairs = npr;
  return ORBPL_OK;
}

int orbl_match_bf_knn(int nq, const uint8_t* qdesc, int nt, const uint8_t* tdesc, int32_t* out,
                      int* nmatches) {
  if (nq < 0 || nt < 0 || !nmatches) return arg_fail("bad argument");
  if (nq > 256) return arg_fail("more than 256 query descriptors");
  if ((nq > 0 && !qdesc) || (nt > 0 && (!tdesc || !out))) return arg_fail("NULL descriptor arrays");
  DBuf dq, dt, dout, dn;
  HIP_CHECK(dq.alloc(std::max(1, nq) * 32));
  HIP_CHECK(dt.alloc(std::max(1, nt) * 32));
  HIP_CHECK(dout.alloc(std::max(1, nt) * 4));
  HIP_CHECK(dn.alloc(4));
  if (nq) HIP_CHECK(hipMemcpy(dq.p, qdesc, (size_t)nq * 32, hipMemcpyHostToDevice));
  if (nt) HIP_CHECK(hipMemcpy(dt.p, tdesc, (size_t)nt * 32, hipMemcpyHostToDevice));
  launch_line_bf_knn(nq, dq.as<uint8_t>(), nt, dt.as<uint8_t>(), dout.as<int>(), dn.as<int>(),
                     scratch_stream());
  HIP_CHECK(hipGetLastError());
  if (nt) HIP_CHECK(hipMemcpy(out, dout.p, (size_t)nt * 4, hipMemcpyDeviceToHost));
  HIP_CHECK(hipMemcpy(nmatches, dn.p, 4, hipMemcpyDeviceToHost));
  return ORBPL_OK;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// Batched tracker
// ---------------------------------------------------------------------------
struct FrameBufs {
  KeyPointD* kps = nullptr;
  uint8_t* desc = nullptr;
  int* n = nullptr;
  KeyPointD* kps_un = nullptr;
  float* depth = nullptr;
  float* uright = nullptr;
  int* gcell = nullptr;
  int* match = nullptr;
  uint8_t* outlier = nullptr;
  uint8_t* has_mp = nullptr;
  float* mp_xyz = nullptr;
  int* nobs = nullptr;
  // lines (kLineKeep per stream)
  orbpl_keyline* kl = nullptr;
  orbpl_keyline* kl_un = nullptr;
  uint8_t* ldesc = nullptr;
  double* lcoef = nullptr;
  int* nl = nullptr;
  float* dstart = nullptr;
  float* dend = nullptr;
  int* lmatch = nullptr;
  uint8_t* loutlier = nullptr;
  uint8_t* has_ml = nullptr;
  float* ml_xyz = nullptr;
  // map model (ORBPL_TRACK_MAP): the frame's map elements (pool id, -1, or a
  // temporal element -2 - slot) and, as the last frame, the map point / line
  // descriptors the matchers read
  int* mpid = nullptr;
  uint8_t* mp_desc = nullptr;
  int* mlid = nullptr;
  uint8_t* ml_desc = nullptr;
  // DBoW2 (orbpl_tracker_set_vocabulary): KeyFrame::ComputeBoW of the frame
  int32_t* feat_node = nullptr;   // FeatureVector: node per keypoint, -1 = stopped
  int32_t* feat_word = nullptr;
  double* feat_weight = nullptr;
  uint32_t* bow_words = nullptr;  // BowVector (word order)
  double* bow_vals = nullptr;
  int* bow_n = nullptr;
};

// map-mode scratch of the matchers (local lists, reference-keyframe lines)
struct MapExtra {
  uint8_t* l_inview;
  float *l_px, *l_py, *l_pxr, *l_vcos;
  int* l_level;
  int4* l_scratch;
  uint8_t* ll_valid;
  orbpl_keyline* ll_proj;
  int* ll_src;
  orbpl_keyline* trk_proj;
  int* trk_src;
};

struct orbpl_tracker {
  orbx_ctx* ex = nullptr;
  int device = 0;
  int S = 0;
  int W = 0, H = 0;
  int kp_cap = 0;
  // Two HIP streams: extraction (+ frame glue) of step t+1 runs on `stream`
  // while matching / pose / finish of step t run on `tstream`. Three frame
  // buffers: step t extracts into fb[t%3] and tracks against fb[(t-1)%3].
  hipStream_t stream = nullptr;    // owned by the extractor context
  hipStream_t tstream = nullptr;   // tracking stream
  TrackConsts consts{};
  FrameBufs fb[3];
  hipEvent_t ev_free[3] = {};      // fb[b] no longer read as "last frame"
  bool free_pending[3] = {};
  int pipelined = 0;               // 0: every stage on `stream`
  // line features (ORBPL_TRACK_LINES): LSD + LBD + UndistortKeyLines run on
  // their own stream, concurrently with the ORB extraction of the same step
  int lines = 0;
  lsdx_ctx* lx = nullptr;
  hipStream_t lstream = nullptr;
  hipEvent_t ev_in = nullptr;      // step start on `stream`
  // split LSD (ORBPL_LSD_SPLIT, lines at >= kLsdSplitMin streams): the
  // first lsplit frames on lstream_a (context lx), the rest on lstream_b
  // (lx2) started once the first half's pseudo-ordering sort is done, so the
  // halves' chains run offset: one half's latency-bound sort and validation
  // beside the other's VALU-bound seed loop. The line glue then runs on
  // lstream after both.
  int lsplit = 0;
  // split ORB extraction (points / RGB-D lines at >= kOrbSplitMin streams):
  // the first osplit frames on `stream` (context ex), the rest on stream2
  // (ex2) once the first half's pyramid is done
  int osplit = 0;
  orbx_ctx* ex2 = nullptr;
  hipStream_t stream2 = nullptr;   // owned by ex2
  hipEvent_t ev_ob_done = nullptr;
  lsdx_ctx* lx2 = nullptr;
  hipStream_t lstream_a = nullptr, lstream_b = nullptr;
  hipEvent_t ev_la_sort = nullptr, ev_la_done = nullptr, ev_lb_done = nullptr;
  // stereo (ORBPL_TRACK_STEREO): the right image's ORB extraction runs on the
  // right extractor's stream, concurrently with the left one; the batched
  // ComputeStereoMatches then fills depth / uRight on the extraction stream
  int stereo = 0;
  int fixed_line_jac = 0;          // ORBPL_TRACK_FIXED_LINE_JAC
  orbx_ctx* exr = nullptr;
  hipStream_t rstream = nullptr;   // owned by exr
  hipEvent_t ev_rin = nullptr;     // step start on `stream`
  KeyPointD* r_kps = nullptr;      // right keypoints (S x kp_cap), one buffer
  uint8_t* r_desc = nullptr;
  int* r_n = nullptr;
  int* st_sad = nullptr;           // stereo scratch: SAD per left keypoint
  uint16_t* st_entries = nullptr;  // stereo scratch: row-band entries
  int st_entry_cap = 0;            // entries per frame
  int* d_err = nullptr;            // stereo capacity flag
  // stereo + lines (P17): LineExtractor on the right images on its own
  // stream, then k_stereo_lines on the line stream
  lsdx_ctx* lxr = nullptr;
  hipStream_t rlstream = nullptr;
  hipEvent_t ev_rlin = nullptr;    // step start on `stream`
  hipEvent_t ev_sl_done = nullptr; // k_stereo_lines finished reading the right lines
  orbpl_keyline* r_kl = nullptr;   // right KeyLines (S x kLineKeep), one buffer
  uint8_t* r_ldesc = nullptr;
  double* r_lcoef = nullptr;
  int* r_nl = nullptr;
  StreamState* d_state = nullptr;
  PoseEdge* d_edges = nullptr;
  static constexpr int kRing = 64;   // steps kept in the timing ring
  static constexpr int kEvGlue = 36 + kKernelBrackets;   // glue start (frame_prepare)
  static constexpr int kEvXdone = kEvGlue + 1;            // extraction done (glue on ts)
  static constexpr int kEv = kEvXdone + 1;   // events per step (28..35: kernel brackets,
                                             // 36..: extraction launch brackets)
  std::vector<hipEvent_t> ring;      // kRing * kEv events
  int ring_pos = 0, ring_count = 0;
  // TrackLocalMap (ORBPL_TRACK_LOCAL_MAP): ring of the last kLmK keyframes'
  // maps, the gathered local lists and the second pose's buffers
  static constexpr int kLmK = 4;
  int local_map = 0;
  int refkf = 0;                   // ORBPL_TRACK_REFKF (needs a vocabulary)
  int glue_on_ts = 0;              // pipelined RGB-D: glue + BoW on the tracking stream
  int *trk_lcur = nullptr, *trk_nobs = nullptr, *trk_lm = nullptr, *trk_nml = nullptr;
  orbpl_keyline* trk_proj = nullptr;
  int* trk_src = nullptr;
  int lm_step = 0;                 // frames since reset (Frame::mnId)
  // host-buffer ingress (orbpl_tracker_step_host): 3 device slots of gray,
  // u16 depth and converted f32 depth, filled on a copy stream
  static constexpr int kIn = 3;
  hipStream_t cstream = nullptr;
  uint8_t* in_gray[kIn] = {};
  uint16_t* in_d16[kIn] = {};
  float* in_depth[kIn] = {};
  hipEvent_t in_copied[kIn] = {}, in_done_s[kIn] = {}, in_done_l[kIn] = {};
  bool in_used[kIn] = {};
  int in_pos = 0;
  orbv_vocab* voc = nullptr;       // orbpl_tracker_set_vocabulary (not owned)
  int voc_levelsup = 4;
  int* d_bow_err = nullptr;
  float scale_factor = 1.2f;
  long long lp = 0, llp = 0;
  float *kr_xyz = nullptr, *kr_nrm = nullptr, *kr_dmin = nullptr, *kr_dmax = nullptr;
  uint8_t *kr_has = nullptr, *kr_desc = nullptr;
  int* kr_n = nullptr;
  float* rl_xyz = nullptr;
  uint8_t *rl_has = nullptr, *rl_desc = nullptr;
  int* rl_n = nullptr;
  float *l_xyz = nullptr, *l_nrm = nullptr, *l_dmin = nullptr, *l_dmax = nullptr;
  uint8_t* l_desc = nullptr;
  int* l_n = nullptr;
  uint8_t* l_inview = nullptr;
  float *l_px = nullptr, *l_py = nullptr, *l_pxr = nullptr, *l_vcos = nullptr;
  int* l_level = nullptr;
  int4* l_scratch = nullptr;
  float* ll_xyz = nullptr;
  uint8_t *ll_desc = nullptr, *ll_valid = nullptr;
  int* ll_n = nullptr;
  orbpl_keyline* ll_proj = nullptr;
  int* ll_src = nullptr;
  int *cur_nobs = nullptr, *cur_nobs_l = nullptr, *lm_match = nullptr, *llm_match = nullptr;
  int *match2 = nullptr, *lmatch2 = nullptr;
  float *xyz2 = nullptr, *lxyz2 = nullptr;
  uint8_t *outlier2 = nullptr, *loutlier2 = nullptr;
  // per-step history (orbpl_tracker_set_history): StreamState and keypoint /
  // line counts of every stream after each step, device-side D2D copies on
  // the tracking stream (no host synchronisation inside a step)
  int hist_cap = 0, hist_count = 0;
  StreamState* d_hist_state = nullptr;
  int* d_hist_n = nullptr;
  int* d_hist_nl = nullptr;
  // map model (ORBPL_TRACK_MAP, map_kernels.hip): keyframe table and point /
  // line pools per stream, the reference keyframe staged as a frame, the
  // pose inputs in current-frame index space
  int map = 0;
  int map_kfc = 0;
  MapArgs ma{};
  MapExtra mx{};
  std::vector<void*> map_allocs;
  std::vector<void*> allocs;
};

namespace orbpl {
hipStream_t orbx_stream(orbx_ctx* c);
}

static int tr_alloc(orbpl_tracker* t, void** p, size_t bytes) {
  hipError_t e = hipMalloc(p, bytes ? bytes : 1);
  if (e != hipSuccess) return hip_fail(e, "hipMalloc", __LINE__);
  t->allocs.push_back(*p);
  return hipMemset(*p, 0, bytes ? bytes : 1) == hipSuccess ? ORBPL_OK : ORBPL_ERR_HIP;
}

// Map-model buffers for `kfc` keyframes per stream (pools of kfc x keypoint
// capacity points and kfc x 80 lines, the local lists of the same sizes);
// replaces earlier ones. Per-stream state is reset by the caller.

static int map_alloc(orbpl_tracker* t, int kfc) {
  MapExtra* x = &t->mx;
  for (void* p : t->map_allocs) (void)hipFree(p);
  t->map_allocs.clear();
  const size_t S = t->S, K = t->kp_cap, L = kLineKeep, F = (size_t)kfc;
  const size_t MPC = F * K, MLC = F * L;
  auto A = [&](void** p, size_t bytes) -> int {
    hipError_t e = hipMalloc(p, bytes ? bytes : 1);
    if (e != hipSuccess) return hip_fail(e, "hipMalloc (map model)", __LINE__);
    t->map_allocs.push_back(*p);
    return ORBPL_OK;
  };
#define MA(ptr, bytes)                                  \
  do {                                                  \
    int _r = A((void**)&(ptr), (bytes));                \
    if (_r) return _r;                                  \
  } while (0)
  MapArgs& m = t->ma;
  m.kfc = kfc;
  m.kp_pitch = (int)K;
  m.mpc = (long long)MPC;
  m.mlc = (long long)MLC;
  m.lines = t->lines;
  m.stereo = t->stereo;
  m.max_frames = 30;   // Camera.fps 30 (TUM); orbpl_tracker_set_fps
  m.lp = (long long)MPC;
  m.llp = (long long)MLC;
  MA(m.ms, S * sizeof(MapState));
  MA(m.kf_T, S * F * 16 * 4);
  MA(m.kf_Ow, S * F * 4 * 4);
  MA(m.kf_N, S * F * 4);
  MA(m.kf_NL, S * F * 4);
  MA(m.kf_frame, S * F * 4);
  MA(m.kf_mp, S * F * K * 4);
  MA(m.kf_kp, S * F * K * sizeof(KeyPointD));
  MA(m.kf_ur, S * F * K * 4);
  MA(m.kf_desc, S * F * K * 32);
  MA(m.kf_node, S * F * K * 4);
  MA(m.kf_ml, S * F * L * 4);
  MA(m.kf_ldesc, S * F * L * 32);
  MA(m.kf_ds, S * F * L * 4);
  MA(m.kf_de, S * F * L * 4);
  MA(m.kf_w, S * F * F * 4);
  MA(m.kf_ord, S * F * F);
  MA(m.kf_nord, S * F * 4);
  MA(m.kf_parent, S * F * 4);
  MA(m.kf_first, S * F * 4);
  MA(m.kf_child, S * F * 8);
  MA(m.mp_pos, S * MPC * 16);
  MA(m.mp_nrm, S * MPC * 16);
  MA(m.mp_dist, S * MPC * 8);
  MA(m.mp_desc, S * MPC * 32);
  MA(m.mp_nobs, S * MPC * 4);
  MA(m.mp_nob, S * MPC * 4);
  MA(m.mp_obs, S * MPC * F * 4);
  MA(m.mp_seen, S * MPC * 4);
  MA(m.mp_tref, S * MPC * 4);
  MA(m.ml_pos, S * MLC * 24);
  MA(m.ml_desc, S * MLC * 32);
  MA(m.ml_nobs, S * MLC * 4);
  MA(m.ml_seen, S * MLC * 4);
  MA(m.ml_tref, S * MLC * 4);
  MA(m.r_n, S * 4);
  MA(m.r_kps_un, S * K * sizeof(KeyPointD));
  MA(m.r_desc, S * K * 32);
  MA(m.r_has_mp, S * K);
  MA(m.r_mp_xyz, S * K * 12);
  MA(m.r_node, S * K * 4);
  MA(m.r_mpid, S * K * 4);
  MA(m.r_nl, S * 4);
  MA(m.r_has_ml, S * L);
  MA(m.r_ml_xyz, S * L * 24);
  MA(m.r_ml_desc, S * L * 32);
  MA(m.r_mlid, S * L * 4);
  MA(m.trk_cur_nobs, S * L * 4);
  MA(m.trk_lm, S * L * 4);
  MA(m.trk_nml, S * 4);
  MA(m.trk_list, S * 4);
  MA(m.trk_count, 4);
  MA(m.m2, S * K * 4);
  MA(m.pxyz, S * K * 12);
  MA(m.lm2, S * L * 4);
  MA(m.lpxyz, S * L * 24);
  MA(m.l_xyz, S * MPC * 12);
  MA(m.l_nrm, S * MPC * 12);
  MA(m.l_dmin, S * MPC * 4);
  MA(m.l_dmax, S * MPC * 4);
  MA(m.l_ldesc_pts, S * MPC * 32);
  MA(m.l_count, S * 4);
  MA(m.l_id, S * MPC * 4);
  MA(m.ll_xyz, S * MLC * 24);
  MA(m.ll_desc, S * MLC * 32);
  MA(m.ll_count, S * 4);
  MA(m.ll_id, S * MLC * 4);
  MA(m.cur_nobs, S * K * 4);
  MA(m.cur_nobs_l, S * L * 4);
  MA(x->l_inview, S * MPC);
  MA(x->l_px, S * MPC * 4);
  MA(x->l_py, S * MPC * 4);
  MA(x->l_pxr, S * MPC * 4);
  MA(x->l_vcos, S * MPC * 4);
  MA(x->l_level, S * MPC * 4);
  MA(x->l_scratch, S * MPC * sizeof(int4));
  MA(x->ll_valid, S * MLC);
  MA(x->ll_proj, S * MLC * sizeof(orbpl_keyline));
  MA(x->ll_src, S * MLC * 4);
  MA(x->trk_proj, S * L * sizeof(orbpl_keyline));
  MA(x->trk_src, S * L * 4);
  int* lm_match = nullptr;
  int* llm_match = nullptr;
  MA(lm_match, S * K * 4);
  MA(llm_match, S * L * 4);
  m.lm_match = lm_match;
  m.llm_match = llm_match;
#undef MA
  if (hipMemset(m.kf_w, 0, S * F * F * 4) != hipSuccess) return hip_fail(hipErrorUnknown, "hipMemset", __LINE__);
  t->map_kfc = kfc;
  return ORBPL_OK;
}

extern "C" {

int orbpl_tracker_destroy(orbpl_tracker* t) {
  if (!t) return ORBPL_OK;
  (void)hipSetDevice(t->device);
  for (void* p : t->allocs) (void)hipFree(p);
  for (void* p : t->map_allocs) (void)hipFree(p);
  if (t->tstream) (void)hipStreamSynchronize(t->tstream);
  for (auto& e : t->ring)
    if (e) (void)hipEventDestroy(e);
  for (auto& e : t->ev_free)
    if (e) (void)hipEventDestroy(e);
  if (t->lstream) (void)hipStreamSynchronize(t->lstream);
  if (t->rstream) (void)hipStreamSynchronize(t->rstream);
  if (t->rlstream) (void)hipStreamSynchronize(t->rlstream);
  if (t->ev_rlin) (void)hipEventDestroy(t->ev_rlin);
  if (t->ev_sl_done) (void)hipEventDestroy(t->ev_sl_done);
  if (t->rlstream) (void)hipStreamDestroy(t->rlstream);
  if (t->lxr) lsdx_destroy(t->lxr);
  if (t->ev_in) (void)hipEventDestroy(t->ev_in);
  if (t->ev_rin) (void)hipEventDestroy(t->ev_rin);
  if (t->exr) orbx_destroy(t->exr);
  if (t->cstream) {
    (void)hipStreamSynchronize(t->cstream);
    (void)hipStreamDestroy(t->cstream);
  }
  for (int k = 0; k < orbpl_tracker::kIn; k++) {
    if (t->in_copied[k]) (void)hipEventDestroy(t->in_copied[k]);
    if (t->in_done_s[k]) (void)hipEventDestroy(t->in_done_s[k]);
    if (t->in_done_l[k]) (void)hipEventDestroy(t->in_done_l[k]);
  }
  if (t->tstream) (void)hipStreamDestroy(t->tstream);
  if (t->lstream_a) (void)hipStreamSynchronize(t->lstream_a);
  if (t->lstream_b) (void)hipStreamSynchronize(t->lstream_b);
  if (t->lstream) (void)hipStreamDestroy(t->lstream);
  if (t->lstream_a) (void)hipStreamDestroy(t->lstream_a);
  if (t->lstream_b) (void)hipStreamDestroy(t->lstream_b);
  for (hipEvent_t e : {t->ev_la_sort, t->ev_la_done, t->ev_lb_done})
    if (e) (void)hipEventDestroy(e);
  if (t->lx) lsdx_destroy(t->lx);
  if (t->lx2) lsdx_destroy(t->lx2);
  if (t->ex) orbx_destroy(t->ex);
  if (t->ex2) orbx_destroy(t->ex2);
  if (t->ev_ob_done) (void)hipEventDestroy(t->ev_ob_done);
  delete t;
  return ORBPL_OK;
}

int orbpl_tracker_create(const orbpl_orb_params* orb, const orbpl_camera* cam, int n_streams,
                         int device, orbpl_tracker** out) {
  return orbpl_tracker_create_ex(orb, cam, n_streams, device, 0, out);
}

int orbpl_tracker_create_ex(const orbpl_orb_params* orb, const orbpl_camera* cam, int n_streams,
                            int device, int flags, orbpl_tracker** out) {
  if (!orb || !cam || !out || n_streams <= 0) return arg_fail("bad argument");
  if (flags & ~(ORBPL_TRACK_LINES | ORBPL_TRACK_STEREO | ORBPL_TRACK_LOCAL_MAP |
                ORBPL_TRACK_FIXED_LINE_JAC | ORBPL_TRACK_REFKF | ORBPL_TRACK_MAP))
    return arg_fail("unknown tracker flag");
  // ORBPL_TRACK_LINES | ORBPL_TRACK_STEREO: the defined stereo line mode (P17;
  // the reference's stereo Frame extracts no lines, Frame.cc:70-131)
  if ((flags & ORBPL_TRACK_STEREO) && cam->height > 1024)
    return arg_fail("stereo tracking supports images up to 1024 rows");
  *out = nullptr;
  orbpl_tracker* t = new orbpl_tracker();
  t->device = device;
  t->lines = (flags & ORBPL_TRACK_LINES) ? 1 : 0;
  t->stereo = (flags & ORBPL_TRACK_STEREO) ? 1 : 0;
  t->fixed_line_jac = (flags & ORBPL_TRACK_FIXED_LINE_JAC) ? 1 : 0;
  t->local_map = (flags & ORBPL_TRACK_LOCAL_MAP) ? 1 : 0;
  t->refkf = (flags & ORBPL_TRACK_REFKF) ? 1 : 0;
  t->map = (flags & ORBPL_TRACK_MAP) ? 1 : 0;
  if (t->map) t->local_map = 0;   // the map model has its own TrackLocalMap
  t->scale_factor = orb->scale_factor;
  t->S = n_streams;
  t->W = cam->width;
  t->H = cam->height;
  const bool osplit = !(flags & ORBPL_TRACK_STEREO) && split_on("ORBPL_ORB_SPLIT", n_streams, kOrbSplitMin);
  t->osplit = osplit ? (n_streams + 1) / 2 : 0;
  int rc = orbx_create(orb, cam->width, cam->height, osplit ? t->osplit : n_streams, device, &t->ex);
  if (rc) {
    delete t;
    return rc;
  }
  if (osplit) {
    rc = orbx_create(orb, cam->width, cam->height, n_streams - t->osplit, device, &t->ex2);
    if (!rc && hipEventCreateWithFlags(&t->ev_ob_done, hipEventDisableTiming) != hipSuccess)
      rc = hip_fail(hipErrorUnknown, "hipEventCreate", __LINE__);
    if (rc) {
      orbpl_tracker_destroy(t);
      return rc;
    }
    t->stream2 = orbpl::orbx_stream(t->ex2);
  }
  t->kp_cap = orbx_max_keypoints(t->ex);
  if (t->kp_cap > kMatchMaxKp) {
    orbpl_tracker_destroy(t);
    return arg_fail("nfeatures too large for the tracker (max 2048 keypoints per frame)");
  }
  float scale[16], inv_sigma2[16];
  int nlev = 0;
  orbx_get_scale_info(t->ex, &nlev, scale, nullptr, nullptr, inv_sigma2);
  rc = make_consts(cam, scale, inv_sigma2, nlev, &t->consts);
  if (rc) {
    orbpl_tracker_destroy(t);
    return rc;
  }
  t->stream = orbpl::orbx_stream(t->ex);
  const size_t S = n_streams, K = t->kp_cap;
#define TA(ptr, bytes)                                        \
  do {                                                        \
    int _r = tr_alloc(t, (void**)&(ptr), (bytes));            \
    if (_r) { orbpl_tracker_destroy(t); return _r; }          \
  } while (0)
  for (int b = 0; b < 3; b++) {
    FrameBufs& f = t->fb[b];
    TA(f.kps, S * K * sizeof(KeyPointD));
    TA(f.desc, S * K * 32);
    TA(f.n, S * 4);
    TA(f.kps_un, S * K * sizeof(KeyPointD));
    TA(f.depth, S * K * 4);
    TA(f.uright, S * K * 4);
    TA(f.gcell, S * K * 4);
    TA(f.match, S * K * 4);
    TA(f.outlier, S * K);
    TA(f.has_mp, S * K);
    TA(f.mp_xyz, S * K * 12);
    TA(f.nobs, S * K * 4);
    if (t->map) {
      TA(f.mpid, S * K * 4);
      TA(f.mp_desc, S * K * 32);
      TA(f.mlid, S * kLineKeep * 4);
      TA(f.ml_desc, S * kLineKeep * 32);
    }
    if (t->lines) {
      const size_t L = S * kLineKeep;
      TA(f.kl, L * sizeof(orbpl_keyline));
      TA(f.kl_un, L * sizeof(orbpl_keyline));
      TA(f.ldesc, L * 32);
      TA(f.lcoef, L * 3 * sizeof(double));
      TA(f.nl, S * 4);
      TA(f.dstart, L * 4);
      TA(f.dend, L * 4);
      TA(f.lmatch, L * 4);
      TA(f.loutlier, L);
      TA(f.has_ml, L);
      TA(f.ml_xyz, L * 6 * 4);
    }
  }
  TA(t->d_state, S * sizeof(StreamState));
  if (t->local_map) {
    const size_t R = S * orbpl_tracker::kLmK * K, RL = S * orbpl_tracker::kLmK * kLineKeep;
    t->lp = (long long)orbpl_tracker::kLmK * K;
    t->llp = (long long)orbpl_tracker::kLmK * kLineKeep;
    const size_t LP = S * (size_t)t->lp, LLP = S * (size_t)t->llp;
    TA(t->kr_xyz, R * 12);
    TA(t->kr_nrm, R * 12);
    TA(t->kr_dmin, R * 4);
    TA(t->kr_dmax, R * 4);
    TA(t->kr_has, R);
    TA(t->kr_desc, R * 32);
    TA(t->kr_n, S * orbpl_tracker::kLmK * 4);
    TA(t->l_xyz, LP * 12);
    TA(t->l_nrm, LP * 12);
    TA(t->l_dmin, LP * 4);
    TA(t->l_dmax, LP * 4);
    TA(t->l_desc, LP * 32);
    TA(t->l_n, S * 4);
    TA(t->l_inview, LP);
    TA(t->l_px, LP * 4);
    TA(t->l_py, LP * 4);
    TA(t->l_pxr, LP * 4);
    TA(t->l_vcos, LP * 4);
    TA(t->l_level, LP * 4);
    TA(t->l_scratch, LP * sizeof(int4));
    TA(t->cur_nobs, S * K * 4);
    TA(t->lm_match, S * K * 4);
    TA(t->match2, S * K * 4);
    TA(t->xyz2, S * K * 12);
    TA(t->outlier2, S * K);
    if (t->lines) {
      TA(t->rl_xyz, RL * 24);
      TA(t->rl_has, RL);
      TA(t->rl_desc, RL * 32);
      TA(t->rl_n, S * orbpl_tracker::kLmK * 4);
      TA(t->ll_xyz, LLP * 24);
      TA(t->ll_desc, LLP * 32);
      TA(t->ll_valid, LLP);
      TA(t->ll_n, S * 4);
      TA(t->ll_proj, LLP * sizeof(orbpl_keyline));
      TA(t->ll_src, LLP * 4);
      TA(t->cur_nobs_l, S * kLineKeep * 4);
      TA(t->llm_match, S * kLineKeep * 4);
      TA(t->lmatch2, S * kLineKeep * 4);
      TA(t->lxyz2, S * kLineKeep * 24);
      TA(t->loutlier2, S * kLineKeep);
    }
  }
  TA(t->d_edges, S * kPoseMaxEdges * pose_edge_bytes());
  if (t->refkf) {
    const size_t L = S * kLineKeep;
    TA(t->trk_lcur, L * 4);
    TA(t->trk_nobs, L * 4);
    TA(t->trk_lm, L * 4);
    TA(t->trk_nml, S * 4);
    TA(t->trk_proj, L * sizeof(orbpl_keyline));
    TA(t->trk_src, L * 4);
  }
  if (t->stereo) {
    // a right keypoint spans at most 4 * scale + 2 <= 18 rows (8 levels of 1.2)
    t->st_entry_cap = (int)K * 20;
    // test hook: a smaller row-band capacity forces the overflow path
    if (const char* e = getenv("ORBPL_STEREO_ENTRY_CAP")) {
      const int v = atoi(e);
      if (v > 0 && v < t->st_entry_cap) t->st_entry_cap = v;
    }
    TA(t->r_kps, S * K * sizeof(KeyPointD));
    TA(t->r_desc, S * K * 32);
    TA(t->r_n, S * 4);
    TA(t->st_sad, S * K * 4);
    TA(t->st_entries, S * (size_t)t->st_entry_cap * 2);
    TA(t->d_err, 4);
    if (t->lines) {
      const size_t L = S * kLineKeep;
      TA(t->r_kl, L * sizeof(orbpl_keyline));
      TA(t->r_ldesc, L * 32);
      TA(t->r_lcoef, L * 3 * sizeof(double));
      TA(t->r_nl, S * 4);
    }
  }
#undef TA
  if (const char* e = getenv("ORBPL_GLUE_ON_TRACK")) t->glue_on_ts = e[0] != '0';
  if (t->map) {
    int kfc = 32;
    if (const char* e = getenv("ORBPL_MAP_KF")) kfc = atoi(e);
    if (kfc < 2 || kfc > kMapMaxKF) {
      orbpl_tracker_destroy(t);
      return arg_fail("ORBPL_MAP_KF out of [2, 64]");
    }
    rc = map_alloc(t, kfc);
    if (rc) {
      orbpl_tracker_destroy(t);
      return rc;
    }
  }
  t->ring.assign(orbpl_tracker::kRing * orbpl_tracker::kEv, nullptr);
  for (auto& e : t->ring)
    if (hipEventCreate(&e) != hipSuccess) {
      orbpl_tracker_destroy(t);
      return hip_fail(hipErrorUnknown, "hipEventCreate", __LINE__);
    }
  for (auto& e : t->ev_free)
    if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) {
      orbpl_tracker_destroy(t);
      return hip_fail(hipErrorUnknown, "hipEventCreate", __LINE__);
    }
  if (hipStreamCreateWithFlags(&t->tstream, hipStreamNonBlocking) != hipSuccess) {
    orbpl_tracker_destroy(t);
    return hip_fail(hipErrorUnknown, "hipStreamCreate", __LINE__);
  }
  if (t->lines) {
    // "0" off, "1" on, else by size when the HIP runtime has the hardware
    // queues for the extra streams (with the default 4, streams share queues
    // and the halves serialise with the ORB stream: measured no gain)
    // (stereo: the left image's batch; the right one has its own stream and
    // context. KITTI leg, 1024 pairs: 4.9k -> 5.2k frames/s)
    const bool split = split_on("ORBPL_LSD_SPLIT", n_streams, kLsdSplitMin);
    t->lsplit = split ? (n_streams + 1) / 2 : 0;
    rc = lsdx_create(cam->width, cam->height, split ? t->lsplit : n_streams, device, &t->lx);
    if (!rc && split) rc = lsdx_create(cam->width, cam->height, n_streams - t->lsplit, device, &t->lx2);
    if (rc) {
      orbpl_tracker_destroy(t);
      return rc;
    }
    if (hipStreamCreateWithFlags(&t->lstream, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&t->ev_in, hipEventDisableTiming) != hipSuccess) {
      orbpl_tracker_destroy(t);
      return hip_fail(hipErrorUnknown, "hipStreamCreate", __LINE__);
    }
    if (split && (hipStreamCreateWithFlags(&t->lstream_a, hipStreamNonBlocking) != hipSuccess ||
                  hipStreamCreateWithFlags(&t->lstream_b, hipStreamNonBlocking) != hipSuccess ||
                  hipEventCreateWithFlags(&t->ev_la_sort, hipEventDisableTiming) != hipSuccess ||
                  hipEventCreateWithFlags(&t->ev_la_done, hipEventDisableTiming) != hipSuccess ||
                  hipEventCreateWithFlags(&t->ev_lb_done, hipEventDisableTiming) != hipSuccess)) {
      orbpl_tracker_destroy(t);
      return hip_fail(hipErrorUnknown, "hipStreamCreate", __LINE__);
    }
  }
  if (t->stereo) {
    rc = orbx_create(orb, cam->width, cam->height, n_streams, device, &t->exr);
    if (rc) {
      orbpl_tracker_destroy(t);
      return rc;
    }
    t->rstream = orbpl::orbx_stream(t->exr);
    if (hipEventCreateWithFlags(&t->ev_rin, hipEventDisableTiming) != hipSuccess) {
      orbpl_tracker_destroy(t);
      return hip_fail(hipErrorUnknown, "hipEventCreate", __LINE__);
    }
    if (t->lines) {
      rc = lsdx_create(cam->width, cam->height, n_streams, device, &t->lxr);
      if (rc) {
        orbpl_tracker_destroy(t);
        return rc;
      }
      if (hipStreamCreateWithFlags(&t->rlstream, hipStreamNonBlocking) != hipSuccess ||
          hipEventCreateWithFlags(&t->ev_rlin, hipEventDisableTiming) != hipSuccess ||
          hipEventCreateWithFlags(&t->ev_sl_done, hipEventDisableTiming) != hipSuccess) {
        orbpl_tracker_destroy(t);
        return hip_fail(hipErrorUnknown, "hipStreamCreate", __LINE__);
      }
    }
  }
  rc = orbpl_tracker_reset(t, nullptr);
  if (rc) {
    orbpl_tracker_destroy(t);
    return rc;
  }
  *out = t;
  return ORBPL_OK;
}

int orbpl_tracker_reset(orbpl_tracker* t, const float* Tcw0) {
  if (!t) return arg_fail("NULL tracker");
  HIP_CHECK(hipSetDevice(t->device));
  std::vector<StreamState> st(t->S);
  for (int s = 0; s < t->S; s++) {
    StreamState z{};
    for (int k = 0; k < 16; k++) z.Tcw[k] = Tcw0 ? Tcw0[s * 16 + k] : (k % 5 == 0 ? 1.f : 0.f);
    st[s] = z;
  }
  if (t->cstream) HIP_CHECK(hipStreamSynchronize(t->cstream));
  HIP_CHECK(hipStreamSynchronize(t->stream));
  if (t->tstream) HIP_CHECK(hipStreamSynchronize(t->tstream));
  if (t->lstream) HIP_CHECK(hipStreamSynchronize(t->lstream));
  if (t->rstream) HIP_CHECK(hipStreamSynchronize(t->rstream));
  if (t->rlstream) HIP_CHECK(hipStreamSynchronize(t->rlstream));
  HIP_CHECK(hipMemcpy(t->d_state, st.data(), sizeof(StreamState) * t->S, hipMemcpyHostToDevice));
  if (t->d_err) HIP_CHECK(hipMemset(t->d_err, 0, 4));
  if (t->map) {
    // every stream starts uninitialised; the first frame takes its Tcw0
    float* dT0 = nullptr;
    if (Tcw0) {
      HIP_CHECK(hipMalloc(&dT0, (size_t)t->S * 64));
      HIP_CHECK(hipMemcpy(dT0, Tcw0, (size_t)t->S * 64, hipMemcpyHostToDevice));
    }
    launch_map_reset(t->ma, dT0, t->S, nullptr);
    HIP_CHECK(hipGetLastError());
    HIP_CHECK(hipDeviceSynchronize());
    if (dT0) HIP_CHECK(hipFree(dT0));
  }
  t->hist_count = 0;
  t->lm_step = 0;
  return ORBPL_OK;
}

int orbpl_tracker_set_fps(orbpl_tracker* t, float fps) {
  if (!t) return arg_fail("NULL tracker");
  if (!t->map) return arg_fail("tracker created without ORBPL_TRACK_MAP");
  if (!(fps >= 0.0f) || fps > 1e6f) return arg_fail("orbpl_tracker_set_fps: fps out of range");
  // Tracking::Tracking: if(fps==0) fps=30; mMaxFrames = fps (Tracking.cc:81-87)
  t->ma.max_frames = (int)(fps == 0.0f ? 30.0f : fps);
  return ORBPL_OK;
}

int orbpl_tracker_clear_velocity(orbpl_tracker* t, const uint8_t* mask) {
  if (!t || !mask) return arg_fail("orbpl_tracker_clear_velocity: NULL argument");
  HIP_CHECK(hipSetDevice(t->device));
  if (t->cstream) HIP_CHECK(hipStreamSynchronize(t->cstream));
  HIP_CHECK(hipStreamSynchronize(t->stream));
  if (t->tstream) HIP_CHECK(hipStreamSynchronize(t->tstream));
  DBuf d;
  HIP_CHECK(d.alloc((size_t)t->S));
  HIP_CHECK(hipMemcpy(d.p, mask, (size_t)t->S, hipMemcpyHostToDevice));
  launch_clear_velocity(t->map ? t->ma.ms : nullptr, t->d_state, d.as<uint8_t>(), t->S, nullptr);
  HIP_CHECK(hipGetLastError());
  HIP_CHECK(hipDeviceSynchronize());
  return ORBPL_OK;
}

}  // extern "C"

// Tracking::Track with the map model (ORBPL_TRACK_MAP) on the tracking stream:
// the map kernels (map_kernels.hip) around the batched matchers and k_pose.
// ev: the step's events (brackets as in the P18 path).
static int map_track(orbpl_tracker* t, FrameBufs& C, FrameBufs& L, const LineTrackArgs& la0,
                      hipEvent_t* ev, hipStream_t ts) {
  const int S = t->S, K = t->kp_cap;
  const int pstride = (int)(sizeof(StreamState) / sizeof(float));
  char* stb = reinterpret_cast<char*>(t->d_state);
  float* dTcw = reinterpret_cast<float*>(stb + offsetof(StreamState, Tcw));
  float* dTlast = reinterpret_cast<float*>(stb + offsetof(StreamState, Tlast));
  auto field = [&](size_t off) { return reinterpret_cast<int*>(stb + off); };
  MapArgs a = t->ma;
  a.st = t->d_state;
  a.lines = t->lines;
  a.refkf = t->refkf;
  a.vocab = t->voc ? 1 : 0;
  a.n = C.n; a.kps_un = C.kps_un; a.depth = C.depth; a.uright = C.uright; a.desc = C.desc;
  a.feat_node = C.feat_node; a.match = C.match; a.outlier = C.outlier; a.mpid = C.mpid;
  a.nl = C.nl; a.kl_un = C.kl_un; a.dstart = C.dstart; a.dend = C.dend; a.ldesc = C.ldesc;
  a.lmatch = C.lmatch; a.loutlier = C.loutlier; a.mlid = C.mlid;
  a.l_n = L.n; a.l_kps_un = L.kps_un; a.l_depth = L.depth; a.l_desc = L.desc; a.l_mpid = L.mpid;
  a.l_has_mp = L.has_mp; a.l_mp_xyz = L.mp_xyz; a.l_mp_desc = L.mp_desc; a.l_nobs = L.nobs;
  a.l_nl = L.nl; a.l_kl_un = L.kl_un; a.l_dstart = L.dstart; a.l_dend = L.dend; a.l_ldesc = L.ldesc;
  a.l_mlid = L.mlid; a.l_has_ml = L.has_ml; a.l_ml_xyz = L.ml_xyz; a.l_ml_desc = L.ml_desc;
  const MapExtra& x = t->mx;
  // ---- frame id, path, UpdateLastFrame, the constant-velocity prediction ----
  launch_map_begin(t->consts, a, S, ts);
  // ---- TrackWithMotionModel (Tracking.cc:1212-1330) ----
  MatchLaunch m{};
  m.cur_kps_un = C.kps_un;
  m.cur_desc = C.desc;
  m.cur_uright = C.uright;
  m.cur_gcell = C.gcell;
  m.cur_n = C.n;
  m.last_kps_un = L.kps_un;
  m.last_has_mp = L.has_mp;
  m.last_outlier = L.outlier;
  m.last_xyz = L.mp_xyz;
  m.last_desc = L.mp_desc;     // pMP->GetDescriptor()
  m.last_nobs = L.nobs;
  m.last_n = L.n;
  m.kp_pitch = K;
  m.Tcw = dTcw;
  m.Tlw = dTlast;
  m.pose_stride = pstride;
  m.match = C.match;
  m.nmatches = field(offsetof(StreamState, nmatches));
  m.nm_stride = pstride;
  m.th = t->stereo ? 7.0f : 15.0f;   // Tracking.cc:1238-1241
  m.mono = 0;
  m.check_ori = 1;
  m.retry = 1;
  m.active = t->d_state;
  launch_match_last(t->consts, m, S, ts);
  HIP_CHECK(hipEventRecord(ev[8], ts));
  if (t->lines) {
    LineTrackArgs la = la0;
    la.last_desc = L.ml_desc;  // the map lines' descriptors
    launch_line_match(t->consts, la, t->d_state, S, ts);
  }
  HIP_CHECK(hipEventRecord(ev[14], ts));
  PoseLaunch p{};
  p.kps_un = C.kps_un;
  p.uright = C.uright;
  p.match = C.match;
  p.mp_xyz = L.mp_xyz;
  p.n = C.n;
  p.kp_pitch = K;
  p.Tcw = dTcw;
  p.pose_stride = pstride;
  p.outlier = C.outlier;
  p.ninliers = field(offsetof(StreamState, ninliers));
  p.nm_stride = pstride;
  p.active = t->d_state;
  p.edges = t->d_edges;
  if (t->lines) {
    p.t_kl_un = C.kl_un;
    p.t_lmatch = C.lmatch;
    p.t_ml_xyz = L.ml_xyz;
    p.t_nl = C.nl;
    p.t_loutlier = C.loutlier;
    p.lpitch = kLineKeep;
  }
  p.fixed_line_jac = t->fixed_line_jac;
  HIP_CHECK(hipEventRecord(ev[28], ts));
  launch_pose(t->consts, p, S, ts);
  HIP_CHECK(hipEventRecord(ev[29], ts));
  launch_map_resolve_motion(a, S, ts);
  // the later poses read the frame's map elements in its own index space
  PoseLaunch pm = p;
  pm.match = a.m2;
  pm.mp_xyz = a.pxyz;
  if (t->lines) {
    pm.t_lmatch = a.lm2;
    pm.t_ml_xyz = a.lpxyz;
  }
  HIP_CHECK(hipEventRecord(ev[30], ts));
  if (t->refkf) {
    // ---- TrackReferenceKeyFrame (Tracking.cc:942-1032) ----
    TrkArgs ta{};
    ta.st = t->d_state;
    ta.kp_pitch = K;
    ta.lines = t->lines;
    ta.n = C.n;
    ta.match = C.match;
    ta.kps_un = C.kps_un;
    ta.desc = C.desc;
    ta.feat_node = C.feat_node;
    ta.last_n = a.r_n;
    ta.last_kps_un = a.r_kps_un;
    ta.last_desc = a.r_desc;
    ta.last_has_mp = a.r_has_mp;
    ta.last_feat_node = a.r_node;
    ta.list = a.trk_list;      // only the streams k_map_resolve_motion listed
    ta.list_n = a.trk_count;
    launch_trk_bow(ta, S, ts);
    if (t->lines) {
      LineListArgs lr{};
      lr.Tcw = dTcw;
      lr.cur_kl_un = C.kl_un;
      lr.cur_desc = C.ldesc;
      lr.cur_nobs = a.trk_cur_nobs;
      lr.valid = a.r_has_ml;
      lr.ml_xyz6 = a.r_ml_xyz;
      lr.ml_desc = a.r_ml_desc;
      lr.proj_kl = x.trk_proj;
      lr.proj_src = x.trk_src;
      lr.match = a.trk_lm;
      lr.nmatches = field(offsetof(StreamState, trk_nlm));
      lr.wiped = field(offsetof(StreamState, trk_wiped));
      lr.refkf = 1;
      lr.ncur_arr = C.nl;
      lr.nml_arr = a.trk_nml;
      lr.cur_pitch = kLineKeep;
      lr.ml_pitch = kLineKeep;
      lr.pose_stride = pstride;
      lr.nm_stride = pstride;
      lr.list = a.trk_list;
      lr.list_n = a.trk_count;
      launch_line_match_list(t->consts, lr, ts, S);
    }
    launch_map_trk_merge(a, S, ts);
    PoseLaunch pt = pm;
    pt.gate_lm = 2;
    pt.list = a.trk_list;
    pt.list_n = a.trk_count;
    launch_pose(t->consts, pt, S, ts);
  }
  HIP_CHECK(hipEventRecord(ev[31], ts));
  launch_map_resolve_trk(a, S, ts);
  HIP_CHECK(hipEventRecord(ev[9], ts));
  // ---- TrackLocalMap (Tracking.cc:1332-1420) ----
  launch_map_local(a, S, ts);
  InFrustumArgs fa{};
  fa.Tcw = dTcw;
  fa.xyz = a.l_xyz;
  fa.normal = a.l_nrm;
  fa.min_dist = a.l_dmin;
  fa.max_dist = a.l_dmax;
  fa.view_cos_limit = 0.5f;
  fa.in_view = x.l_inview;
  fa.proj_x = x.l_px;
  fa.proj_y = x.l_py;
  fa.proj_xr = x.l_pxr;
  fa.level = x.l_level;
  fa.view_cos = x.l_vcos;
  fa.n_arr = a.l_count;
  fa.pitch = a.lp;
  fa.pose_stride = pstride;
  const float log_scale = (float)lsdm::log_((double)t->scale_factor);   // P15
  launch_in_frustum(t->consts, log_scale, fa, ts, S);
  LocalArgs ml{};
  ml.kps_un = C.kps_un;
  ml.desc = C.desc;
  ml.uright = C.uright;
  ml.cur_nobs = a.cur_nobs;
  ml.in_view = x.l_inview;
  ml.proj_x = x.l_px;
  ml.proj_y = x.l_py;
  ml.proj_xr = x.l_pxr;
  ml.level = x.l_level;
  ml.view_cos = x.l_vcos;
  ml.mp_desc = a.l_ldesc_pts;
  ml.mp_nobs = nullptr;        // every local map point is observed
  // RGB-D 3, stereo 1; 5 within mnLastRelocFrameId + 2 (Tracking.cc:1801-1809)
  ml.th = t->lm_step < 2 ? 5.0f : (t->stereo ? 1.0f : 3.0f);
  ml.nnratio = 0.8f;
  ml.match = const_cast<int*>(a.lm_match);
  ml.nmatches = field(offsetof(StreamState, lm_nlocal));
  ml.scratch = x.l_scratch;
  ml.n_arr = C.n;
  ml.nmp_arr = a.l_count;
  ml.kp_pitch = K;
  ml.mp_pitch = a.lp;
  ml.nm_stride = pstride;
  HIP_CHECK(hipEventRecord(ev[32], ts));
  launch_match_local(t->consts, ml, ts, S);
  HIP_CHECK(hipEventRecord(ev[33], ts));
  if (t->lines) {
    launch_line_in_frustum_batched(dTcw, pstride, a.ll_count, a.llp, a.ll_xyz, x.ll_valid, S, ts);
    LineListArgs l3{};
    l3.Tcw = dTcw;
    l3.cur_kl_un = C.kl_un;
    l3.cur_desc = C.ldesc;
    l3.cur_nobs = a.cur_nobs_l;
    l3.valid = x.ll_valid;
    l3.ml_xyz6 = a.ll_xyz;
    l3.ml_desc = a.ll_desc;
    l3.proj_kl = x.ll_proj;
    l3.proj_src = x.ll_src;
    l3.match = const_cast<int*>(a.llm_match);
    l3.nmatches = field(offsetof(StreamState, lm_nllocal));
    l3.wiped = field(offsetof(StreamState, lm_wiped));
    l3.ncur_arr = C.nl;
    l3.nml_arr = a.ll_count;
    l3.cur_pitch = kLineKeep;
    l3.ml_pitch = a.llp;
    l3.pose_stride = pstride;
    l3.nm_stride = pstride;
    launch_line_match_list(t->consts, l3, ts, S);
  }
  launch_map_assemble(a, S, ts);
  PoseLaunch p2 = pm;
  p2.ninliers = field(offsetof(StreamState, lm_ninl));
  p2.gate_lm = 1;
  HIP_CHECK(hipEventRecord(ev[34], ts));
  launch_pose(t->consts, p2, S, ts);
  HIP_CHECK(hipEventRecord(ev[35], ts));
  HIP_CHECK(hipEventRecord(ev[26], ts));
  // ---- decision, keyframe insertion, ProcessNewKeyFrame, relative pose ----
  launch_map_finish(t->consts, a, S, ts);
  t->lm_step++;
  return ORBPL_OK;
}

// One TrackWithMotionModel step for every stream: RGB-D (d_depth) or stereo
// (d_right, ORBPL_TRACK_STEREO trackers).
static int tracker_step(orbpl_tracker* t, const uint8_t* d_gray, const float* d_depth,
                        const uint8_t* d_right) {
  if (t->refkf && !t->voc)
    return arg_fail("ORBPL_TRACK_REFKF tracker: orbpl_tracker_set_vocabulary first");
  HIP_CHECK(hipSetDevice(t->device));
  const int ci = t->ring_pos % 3, li = (t->ring_pos + 2) % 3;
  FrameBufs& C = t->fb[ci];
  FrameBufs& L = t->fb[li];
  const int S = t->S, K = t->kp_cap;
  hipStream_t s = t->stream, ts = t->pipelined ? t->tstream : t->stream;
  const int pstride = (int)(sizeof(StreamState) / sizeof(float));
  char* st0 = reinterpret_cast<char*>(t->d_state);
  float* dTcw = reinterpret_cast<float*>(st0 + offsetof(StreamState, Tcw));
  float* dTlast = reinterpret_cast<float*>(st0 + offsetof(StreamState, Tlast));
  int* dNm = reinterpret_cast<int*>(st0 + offsetof(StreamState, nmatches));
  int* dNin = reinterpret_cast<int*>(st0 + offsetof(StreamState, ninliers));
  hipEvent_t* ev = &t->ring[(size_t)(t->ring_pos % orbpl_tracker::kRing) * orbpl_tracker::kEv];
  // ---- extraction stream: wait until tracking of step t-1 released fb[ci]
  if (t->free_pending[ci]) HIP_CHECK(hipStreamWaitEvent(s, t->ev_free[ci], 0));
  if (t->stereo) {
    // ---- right stream: ORB on the right images (Frame.cc:88-91). Ordered
    // after the previous step's stereo matching, which read r_kps and the
    // right pyramid on `s`.
    HIP_CHECK(hipEventRecord(t->ev_rin, s));
    HIP_CHECK(hipStreamWaitEvent(t->rstream, t->ev_rin, 0));
    HIP_CHECK(hipEventRecord(ev[15], t->rstream));
    int rrc = orbx_run(t->exr, d_right, S, t->W, (long long)t->W * t->H,
                       reinterpret_cast<orbpl_keypoint_dev*>(t->r_kps), t->r_desc, K, t->r_n);
    if (rrc) return rrc;
    HIP_CHECK(hipEventRecord(ev[16], t->rstream));
  }
  if (t->lines && t->stereo) {
    // ---- right line stream: LineExtractor on the right images (P17), after
    // the previous step's k_stereo_lines has read the right KeyLines
    HIP_CHECK(hipEventRecord(t->ev_rlin, s));
    HIP_CHECK(hipStreamWaitEvent(t->rlstream, t->ev_rlin, 0));
    HIP_CHECK(hipStreamWaitEvent(t->rlstream, t->ev_sl_done, 0));
    HIP_CHECK(hipEventRecord(ev[23], t->rlstream));
    LineOut ro{};
    ro.kl = t->r_kl;
    ro.desc = t->r_ldesc;
    ro.coef = t->r_lcoef;
    ro.n = t->r_nl;
    int lrc = lsdx_run(t->lxr, d_right, S, t->W, (int64_t)t->W * t->H, &ro, t->rlstream, nullptr);
    if (lrc) return lrc;
    HIP_CHECK(hipEventRecord(ev[24], t->rlstream));
  }
  LineTrackArgs la{};
  if (t->lines) {
    // ---- line stream: LineExtractor + UndistortKeyLines + line depths
    HIP_CHECK(hipEventRecord(t->ev_in, s));
    LineOut lo{};
    lo.kl = C.kl;
    lo.desc = C.ldesc;
    lo.coef = C.lcoef;
    lo.n = C.nl;
    if (t->lsplit) {
      // first half on lstream_a (its stage events are the step's LSD
      // timings), the second on lstream_b once the first half is sorted
      const int S1 = t->lsplit, S2 = S - S1;
      const int64_t fp = (int64_t)t->W * t->H;
      HIP_CHECK(hipStreamWaitEvent(t->lstream_a, t->ev_in, 0));
      HIP_CHECK(hipEventRecord(ev[11], t->lstream_a));
      int lrc = lsdx_run(t->lx, d_gray, S1, t->W, fp, &lo, t->lstream_a, ev[12], &ev[18]);
      if (lrc) return lrc;
      HIP_CHECK(hipEventRecord(t->ev_la_done, t->lstream_a));
      // the second half starts once the first half is sorted (ev_stage[1]);
      // ORBPL_LSD_STAGGER=0 / 2: at the step start / after its seed loop (A/B)
      static const char* stg = getenv("ORBPL_LSD_STAGGER");
      const int stagger = stg ? atoi(stg) : 1;
      HIP_CHECK(hipStreamWaitEvent(t->lstream_b, stagger == 0 ? t->ev_in : ev[stagger == 2 ? 20 : 19], 0));
      LineOut lo2 = lo;
      lo2.kl = C.kl + (size_t)S1 * kLineKeep;
      lo2.desc = C.ldesc + (size_t)S1 * kLineKeep * 32;
      lo2.coef = C.lcoef + (size_t)S1 * kLineKeep * 3;
      lo2.n = C.nl + S1;
      lrc = lsdx_run(t->lx2, d_gray + (size_t)S1 * fp, S2, t->W, fp, &lo2, t->lstream_b, nullptr);
      if (lrc) return lrc;
      HIP_CHECK(hipEventRecord(t->ev_lb_done, t->lstream_b));
      HIP_CHECK(hipStreamWaitEvent(t->lstream, t->ev_la_done, 0));
      HIP_CHECK(hipStreamWaitEvent(t->lstream, t->ev_lb_done, 0));
    } else {
      HIP_CHECK(hipStreamWaitEvent(t->lstream, t->ev_in, 0));
      HIP_CHECK(hipEventRecord(ev[11], t->lstream));
      int lrc = lsdx_run(t->lx, d_gray, S, t->W, (int64_t)t->W * t->H, &lo, t->lstream, ev[12],
                         &ev[18]);
      if (lrc) return lrc;
    }
    la.nl = C.nl;
    la.kl = C.kl;
    la.kl_un = C.kl_un;
    la.depth = d_depth;
    la.depth_pitch = (long long)t->W * t->H;
    la.dstart = C.dstart;
    la.dend = C.dend;
    la.lmatch = C.lmatch;
    la.loutlier = C.loutlier;
    la.desc = C.ldesc;
    la.last_nl = L.nl;
    la.last_kl_un = L.kl_un;
    la.last_has_ml = L.has_ml;
    la.last_loutlier = L.loutlier;
    la.last_ml_xyz = L.ml_xyz;
    la.last_desc = L.ldesc;
    launch_line_prepare(t->consts, la, S, t->lstream);
    if (t->stereo) {
      // end-point depths from the right image's lines (P17)
      HIP_CHECK(hipStreamWaitEvent(t->lstream, ev[24], 0));
      HIP_CHECK(hipEventRecord(ev[25], t->lstream));
      StereoLineArgs sa{C.nl, C.kl_un, C.ldesc, t->r_nl, t->r_kl, t->r_ldesc, C.dstart, C.dend};
      launch_stereo_lines(t->consts, sa, S, t->lstream);
      HIP_CHECK(hipEventRecord(t->ev_sl_done, t->lstream));
    }
    HIP_CHECK(hipEventRecord(ev[13], t->lstream));
  }
  int rc;
  if (t->osplit) {
    // first half on `s` (its stage events are the step's extraction
    // timings), the second on stream2 after the first half's pyramid
    const int S1 = t->osplit, S2 = S - S1;
    const long long fp = (long long)t->W * t->H;
    rc = orbx_run(t->ex, d_gray, S1, t->W, fp, reinterpret_cast<orbpl_keypoint_dev*>(C.kps),
                  C.desc, K, C.n, ev, ev + 36);
    if (rc) return rc;
    HIP_CHECK(hipStreamWaitEvent(t->stream2, ev[1], 0));
    rc = orbx_run(t->ex2, d_gray + (size_t)S1 * fp, S2, t->W, fp,
                  reinterpret_cast<orbpl_keypoint_dev*>(C.kps + (size_t)S1 * K),
                  C.desc + (size_t)S1 * K * 32, K, C.n + S1, nullptr);
    if (rc) return rc;
    HIP_CHECK(hipEventRecord(t->ev_ob_done, t->stream2));
    HIP_CHECK(hipStreamWaitEvent(s, t->ev_ob_done, 0));
  } else {
    rc = orbx_run(t->ex, d_gray, S, t->W, (long long)t->W * t->H,
                  reinterpret_cast<orbpl_keypoint_dev*>(C.kps), C.desc, K, C.n, ev, ev + 36);
    if (rc) return rc;
  }
  // The frame glue and KeyFrame::ComputeBoW read only this step's frame
  // buffers (and the depth input), so a pipelined RGB-D tracker can run them
  // at the head of the tracking stream (ORBPL_GLUE_ON_TRACK=1): the next
  // step's extraction on `s` then follows this step's orientation launch
  // directly. Measured 1-3 % slower at 2048 streams (the tracking chain
  // becomes the longer one; profiles/r06/ab/glue_on_track_ab.txt), so off by
  // default. Stereo keeps them on `s` regardless: ComputeStereoMatches reads
  // the extractors' device pyramids, which the next extraction overwrites.
  hipStream_t gs = s;
  if (t->glue_on_ts && ts != s && !t->stereo) {
    gs = ts;
    HIP_CHECK(hipEventRecord(ev[orbpl_tracker::kEvXdone], s));
    HIP_CHECK(hipStreamWaitEvent(ts, ev[orbpl_tracker::kEvXdone], 0));
  }
  HIP_CHECK(hipEventRecord(ev[orbpl_tracker::kEvGlue], gs));
  launch_frame_prepare(t->consts, C.kps, C.n, K, t->stereo ? nullptr : d_depth,
                       (long long)t->W * t->H, C.kps_un, C.depth, C.uright, C.gcell, S, gs);
  if (t->stereo) {
    // ComputeStereoMatches (Frame.cc:886-1063) for the whole batch
    HIP_CHECK(hipStreamWaitEvent(s, ev[16], 0));
    HIP_CHECK(hipEventRecord(ev[17], s));
    const uint8_t *pl = nullptr, *pr = nullptr;
    const OrbGeom *gl = nullptr, *gr = nullptr;
    hipStream_t sl, sr;
    int prc = orbx_device_pyramid(t->ex, 0, &pl, &gl, &sl);
    if (!prc) prc = orbx_device_pyramid(t->exr, 0, &pr, &gr, &sr);
    if (prc) return prc;
    StereoArgs a{};
    a.n_arr = C.n;
    a.nr_arr = t->r_n;
    a.kp_pitch = K;
    a.pyr_pitch = (long long)gl->pyr_bytes;
    a.kl = C.kps;
    a.dl = C.desc;
    a.kr = t->r_kps;
    a.dr = t->r_desc;
    a.pyrL = pl;
    a.pyrR = pr;
    for (int l = 0; l < gl->nlevels; l++) {
      a.lv[l] = gl->lv[l];
      a.scale[l] = gl->lv[l].scale;
      a.inv_scale[l] = 1.0f / gl->lv[l].scale;
    }
    a.nrows = gl->H;
    a.mb = t->consts.mb;
    a.mbf = t->consts.bf;
    a.uright = C.uright;
    a.depth = C.depth;
    a.sad = t->st_sad;
    a.entries = t->st_entries;
    a.entry_cap = t->st_entry_cap;
    a.err = t->d_err;
    launch_stereo(a, S, s);
  }
  HIP_CHECK(hipEventRecord(ev[27], gs));
  if (t->voc) {
    // every tracked frame is a keyframe (P18): KeyFrame::ComputeBoW
    // (KeyFrame.cc:67, Frame.cc:730) after the glue
    rc = orbv_transform_batch_device(t->voc, C.desc, K, C.n, S, K, t->voc_levelsup, C.feat_node,
                                     C.feat_word, C.feat_weight, C.bow_words, C.bow_vals, C.bow_n,
                                     K, t->d_bow_err, (void*)gs);
    if (rc) return rc;
  }
  HIP_CHECK(hipEventRecord(ev[6], gs));
  // ---- tracking stream
  HIP_CHECK(hipStreamWaitEvent(ts, ev[6], 0));
  if (t->lines) HIP_CHECK(hipStreamWaitEvent(ts, ev[13], 0));
  HIP_CHECK(hipEventRecord(ev[7], ts));
  if (t->map) {
    const int mrc = map_track(t, C, L, la, ev, ts);
    if (mrc) return mrc;
  } else {
  launch_predict(t->d_state, S, ts);
  MatchLaunch m{};
  m.cur_kps_un = C.kps_un;
  m.cur_desc = C.desc;
  m.cur_uright = C.uright;
  m.cur_gcell = C.gcell;
  m.cur_n = C.n;
  m.last_kps_un = L.kps_un;
  m.last_has_mp = L.has_mp;
  m.last_outlier = L.outlier;
  m.last_xyz = L.mp_xyz;
  m.last_desc = L.desc;
  m.last_nobs = L.nobs;
  m.last_n = L.n;
  m.kp_pitch = K;
  m.Tcw = dTcw;
  m.Tlw = dTlast;
  m.pose_stride = pstride;
  m.match = C.match;
  m.nmatches = dNm;
  m.nm_stride = pstride;
  m.th = t->stereo ? 7.0f : 15.0f;   // Tracking.cc:1238-1241
  m.mono = 0;
  m.check_ori = 1;       // ORBmatcher(0.9, true) (Tracking.cc:1216)
  m.retry = 1;
  m.active = t->d_state;
  launch_match_last(t->consts, m, S, ts);
  HIP_CHECK(hipEventRecord(ev[8], ts));
  if (t->lines) launch_line_match(t->consts, la, t->d_state, S, ts);
  HIP_CHECK(hipEventRecord(ev[14], ts));
  PoseLaunch p{};
  p.kps_un = C.kps_un;
  p.uright = C.uright;
  p.match = C.match;
  p.has_mp = nullptr;
  p.mp_xyz = L.mp_xyz;
  p.n = C.n;
  p.kp_pitch = K;
  p.nl = 0;
  p.Tcw = dTcw;
  p.pose_stride = pstride;
  p.outlier = C.outlier;
  p.line_outlier = nullptr;
  p.ninliers = dNin;
  p.nm_stride = pstride;
  p.active = t->d_state;
  p.edges = t->d_edges;
  if (t->lines) {
    p.t_kl_un = C.kl_un;
    p.t_lmatch = C.lmatch;
    p.t_ml_xyz = L.ml_xyz;
    p.t_nl = C.nl;
    p.t_loutlier = C.loutlier;
    p.lpitch = kLineKeep;
  }
  p.fixed_line_jac = t->fixed_line_jac;
  HIP_CHECK(hipEventRecord(ev[28], ts));
  launch_pose(t->consts, p, S, ts);
  HIP_CHECK(hipEventRecord(ev[29], ts));
  HIP_CHECK(hipEventRecord(ev[30], ts));   // k_pose of TrackReferenceKeyFrame (0 without)
  bool refkf_pose = false;
  if (t->refkf) {
    // ---- TrackReferenceKeyFrame where the motion model did not run or
    // failed (Tracking.cc:324-338, 942-1032; P22) ----
    TrkArgs ta{};
    ta.st = t->d_state;
    ta.kp_pitch = K;
    ta.lines = t->lines;
    ta.n = C.n;
    ta.match = C.match;
    ta.outlier = C.outlier;
    ta.nl = C.nl;
    ta.lmatch = C.lmatch;
    ta.loutlier = C.loutlier;
    ta.kps_un = C.kps_un;
    ta.desc = C.desc;
    ta.feat_node = C.feat_node;
    ta.last_n = L.n;
    ta.last_nl = L.nl;
    ta.last_kps_un = L.kps_un;
    ta.last_desc = L.desc;
    ta.last_has_mp = L.has_mp;
    ta.last_feat_node = L.feat_node;
    ta.lcur = t->trk_lcur;
    ta.cur_nobs_l = t->trk_nobs;
    ta.tlm = t->trk_lm;
    ta.nml = t->trk_nml;
    launch_trk_prep(ta, S, ts);
    launch_trk_bow(ta, S, ts);
    if (t->lines) {
      // LineMatcher(0.7, true).SearchByProjection(mCurrentFrame, mpReferenceKF)
      char* stb = reinterpret_cast<char*>(t->d_state);
      LineListArgs lr{};
      lr.Tcw = dTcw;
      lr.cur_kl_un = C.kl_un;
      lr.cur_desc = C.ldesc;
      lr.cur_nobs = t->trk_nobs;
      lr.valid = L.has_ml;      // mvpMapLines[i] != NULL
      lr.ml_xyz6 = L.ml_xyz;
      lr.ml_desc = L.ldesc;
      lr.proj_kl = t->trk_proj;
      lr.proj_src = t->trk_src;
      lr.match = t->trk_lm;
      lr.nmatches = reinterpret_cast<int*>(stb + offsetof(StreamState, trk_nlm));
      lr.wiped = reinterpret_cast<int*>(stb + offsetof(StreamState, trk_wiped));
      lr.refkf = 1;
      lr.ncur_arr = C.nl;
      lr.nml_arr = t->trk_nml;
      lr.cur_pitch = kLineKeep;
      lr.ml_pitch = kLineKeep;
      lr.pose_stride = pstride;
      lr.nm_stride = pstride;
      launch_line_match_list(t->consts, lr, ts, S);
    }
    launch_trk_merge(ta, S, ts);
    PoseLaunch pt = p;
    pt.gate_lm = 2;
    HIP_CHECK(hipEventRecord(ev[30], ts));
    launch_pose(t->consts, pt, S, ts);
    HIP_CHECK(hipEventRecord(ev[31], ts));
    refkf_pose = true;
  }
  if (!refkf_pose) HIP_CHECK(hipEventRecord(ev[31], ts));
  HIP_CHECK(hipEventRecord(ev[9], ts));
  // TrackLocalMap's k_match_local / k_pose brackets (0 without it)
  HIP_CHECK(hipEventRecord(ev[32], ts));
  HIP_CHECK(hipEventRecord(ev[34], ts));
  LocalMapArgs lm{};
  if (t->local_map) {
    // ---- TrackLocalMap (Tracking.cc:1332-1420), defined local map P18 ----
    const int K4 = orbpl_tracker::kLmK, fid = t->lm_step;
    lm.st = t->d_state;
    lm.kp_pitch = K;
    lm.lines = t->lines;
    lm.n = C.n;
    lm.match = C.match;
    lm.outlier = C.outlier;
    lm.nl = C.nl;
    lm.lmatch = C.lmatch;
    lm.loutlier = C.loutlier;
    lm.kps_un = C.kps_un;
    lm.desc = C.desc;
    lm.ldesc = C.ldesc;
    lm.has_mp = C.has_mp;
    lm.mp_xyz = C.mp_xyz;
    lm.has_ml = C.has_ml;
    lm.ml_xyz = C.ml_xyz;
    lm.last_xyz = L.mp_xyz;
    lm.last_lxyz = L.ml_xyz;
    lm.K = K4;
    lm.nslots = std::min(fid, K4);
    lm.head = ((fid - 1) % K4 + K4) % K4;
    lm.push_slot = fid % K4;
    lm.r_xyz = t->kr_xyz; lm.r_nrm = t->kr_nrm; lm.r_dmin = t->kr_dmin; lm.r_dmax = t->kr_dmax;
    lm.r_has = t->kr_has; lm.r_desc = t->kr_desc; lm.r_n = t->kr_n;
    lm.rl_xyz = t->rl_xyz; lm.rl_has = t->rl_has; lm.rl_desc = t->rl_desc; lm.rl_n = t->rl_n;
    lm.lp = t->lp;
    lm.llp = t->llp;
    lm.l_xyz = t->l_xyz; lm.l_nrm = t->l_nrm; lm.l_dmin = t->l_dmin; lm.l_dmax = t->l_dmax;
    lm.l_desc = t->l_desc; lm.l_n = t->l_n;
    lm.ll_xyz = t->ll_xyz; lm.ll_desc = t->ll_desc; lm.ll_n = t->ll_n;
    lm.cur_nobs = t->cur_nobs;
    lm.cur_nobs_l = t->cur_nobs_l;
    lm.lm_match = t->lm_match;
    lm.llm_match = t->llm_match;
    lm.match2 = t->match2; lm.xyz2 = t->xyz2; lm.lmatch2 = t->lmatch2; lm.lxyz2 = t->lxyz2;
    lm.outlier2 = t->outlier2; lm.loutlier2 = t->loutlier2;
    launch_lm_gather(lm, S, ts);
    // SearchLocalPoints: IsInFrustum(pMP, 0.5), ORBmatcher(0.8).SearchByProjection
    InFrustumArgs fa{};
    fa.Tcw = dTcw;
    fa.xyz = t->l_xyz;
    fa.normal = t->l_nrm;
    fa.min_dist = t->l_dmin;
    fa.max_dist = t->l_dmax;
    fa.view_cos_limit = 0.5f;
    fa.in_view = t->l_inview;
    fa.proj_x = t->l_px;
    fa.proj_y = t->l_py;
    fa.proj_xr = t->l_pxr;
    fa.level = t->l_level;
    fa.view_cos = t->l_vcos;
    fa.n_arr = t->l_n;
    fa.pitch = t->lp;
    fa.pose_stride = pstride;
    const float log_scale = (float)lsdm::log_((double)t->scale_factor);   // P15
    launch_in_frustum(t->consts, log_scale, fa, ts, S);
    char* stb = reinterpret_cast<char*>(t->d_state);
    LocalArgs ma{};
    ma.kps_un = C.kps_un;
    ma.desc = C.desc;
    ma.uright = C.uright;
    ma.cur_nobs = t->cur_nobs;
    ma.in_view = t->l_inview;
    ma.proj_x = t->l_px;
    ma.proj_y = t->l_py;
    ma.proj_xr = t->l_pxr;
    ma.level = t->l_level;
    ma.view_cos = t->l_vcos;
    ma.mp_desc = t->l_desc;
    ma.mp_nobs = nullptr;
    ma.th = fid < 2 ? 5.0f : (t->stereo ? 1.0f : 3.0f);
    ma.nnratio = 0.8f;
    ma.match = t->lm_match;
    ma.nmatches = reinterpret_cast<int*>(stb + offsetof(StreamState, lm_nlocal));
    ma.scratch = t->l_scratch;
    ma.n_arr = C.n;
    ma.nmp_arr = t->l_n;
    ma.kp_pitch = K;
    ma.mp_pitch = t->lp;
    ma.nm_stride = pstride;
    HIP_CHECK(hipEventRecord(ev[32], ts));
    launch_match_local(t->consts, ma, ts, S);
    HIP_CHECK(hipEventRecord(ev[33], ts));
    if (t->lines) {
      // SearchLocalLines: IsInFrustum(pML, 0.5), LineMatcher(0.8) local-map overload
      launch_line_in_frustum_batched(dTcw, pstride, t->ll_n, t->llp, t->ll_xyz, t->ll_valid, S, ts);
      LineListArgs la3{};
      la3.Tcw = dTcw;
      la3.cur_kl_un = C.kl_un;
      la3.cur_desc = C.ldesc;
      la3.cur_nobs = t->cur_nobs_l;
      la3.valid = t->ll_valid;
      la3.ml_xyz6 = t->ll_xyz;
      la3.ml_desc = t->ll_desc;
      la3.proj_kl = t->ll_proj;
      la3.proj_src = t->ll_src;
      la3.match = t->llm_match;
      la3.nmatches = reinterpret_cast<int*>(stb + offsetof(StreamState, lm_nllocal));
      la3.wiped = reinterpret_cast<int*>(stb + offsetof(StreamState, lm_wiped));
      la3.ncur_arr = C.nl;
      la3.nml_arr = t->ll_n;
      la3.cur_pitch = kLineKeep;
      la3.ml_pitch = t->llp;
      la3.pose_stride = pstride;
      la3.nm_stride = pstride;
      launch_line_match_list(t->consts, la3, ts, S);
    }
    launch_lm_assemble(lm, S, ts);
    // PoseOptimizationWithLines over every match of the frame
    PoseLaunch p2 = p;
    p2.match = t->match2;
    p2.mp_xyz = t->xyz2;
    p2.outlier = t->outlier2;
    p2.ninliers = reinterpret_cast<int*>(stb + offsetof(StreamState, lm_ninl));
    if (t->lines) {
      p2.t_lmatch = t->lmatch2;
      p2.t_ml_xyz = t->lxyz2;
      p2.t_loutlier = t->loutlier2;
    }
    p2.gate_lm = 1;
    HIP_CHECK(hipEventRecord(ev[34], ts));
    launch_pose(t->consts, p2, S, ts);
    HIP_CHECK(hipEventRecord(ev[35], ts));
    launch_lm_count(lm, fid, S, ts);
  }
  if (!t->local_map) {
    HIP_CHECK(hipEventRecord(ev[33], ts));
    HIP_CHECK(hipEventRecord(ev[35], ts));
  }
  HIP_CHECK(hipEventRecord(ev[26], ts));
  LineFinish lf{};
  if (t->lines) {
    lf.nl = C.nl;
    lf.lmatch = C.lmatch;
    lf.loutlier = C.loutlier;
    lf.dstart = C.dstart;
    lf.dend = C.dend;
    lf.kl_un = C.kl_un;
    lf.has_ml = C.has_ml;
    lf.ml_xyz = C.ml_xyz;
  }
  launch_finish(t->consts, t->d_state, C.n, K, C.kps_un, C.depth, C.match, C.outlier, C.has_mp,
                C.mp_xyz, C.nobs, lf, S, ts, t->local_map);
  if (t->local_map) {
    launch_lm_push(t->consts, lm, S, ts);   // the frame joins the local map
    t->lm_step++;
  }
  }   // !t->map
  HIP_CHECK(hipEventRecord(ev[10], ts));
  if (t->hist_count < t->hist_cap) {
    const size_t k = (size_t)t->hist_count++ * S;
    HIP_CHECK(hipMemcpyAsync(t->d_hist_state + k, t->d_state, sizeof(StreamState) * S,
                             hipMemcpyDeviceToDevice, ts));
    HIP_CHECK(hipMemcpyAsync(t->d_hist_n + k, C.n, 4 * (size_t)S, hipMemcpyDeviceToDevice, ts));
    if (t->lines)
      HIP_CHECK(hipMemcpyAsync(t->d_hist_nl + k, C.nl, 4 * (size_t)S, hipMemcpyDeviceToDevice, ts));
  }
  HIP_CHECK(hipEventRecord(t->ev_free[li], ts));
  t->free_pending[li] = true;
  HIP_CHECK(hipGetLastError());
  t->ring_pos++;
  t->ring_count = std::min(t->ring_count + 1, (int)orbpl_tracker::kRing);
  return ORBPL_OK;
}

extern "C" {

int orbpl_tracker_step(orbpl_tracker* t, const uint8_t* d_gray, const float* d_depth) {
  if (!t || !d_gray || !d_depth) return arg_fail("NULL argument");
  if (t->stereo) return arg_fail("stereo tracker: use orbpl_tracker_step_stereo");
  return tracker_step(t, d_gray, d_depth, nullptr);
}

int orbpl_tracker_step_host(orbpl_tracker* t, const uint8_t* h_gray, const uint16_t* h_depth,
                            float depth_map_factor) {
  if (!t || !h_gray || !h_depth) return arg_fail("NULL argument");
  if (t->stereo) return arg_fail("stereo tracker: orbpl_tracker_step_host takes RGB-D frames");
  if (!(depth_map_factor > 0.f)) return arg_fail("depth_map_factor must be > 0");
  HIP_CHECK(hipSetDevice(t->device));
  const size_t npx = (size_t)t->S * t->W * t->H;
  if (!t->cstream) {
    // everything into locals first: a failed allocation leaves the tracker
    // as it was (no half-initialised slots behind a non-null copy stream)
    std::vector<void*> got;
    auto fail = [&](hipError_t e, int line) {
      for (void* p : got) (void)hipFree(p);
      return hip_fail(e, "ingress slot allocation", line);
    };
    uint8_t* g[orbpl_tracker::kIn];
    uint16_t* d16[orbpl_tracker::kIn];
    float* df[orbpl_tracker::kIn];
    for (int k = 0; k < orbpl_tracker::kIn; k++) {
      void* p = nullptr;
      hipError_t e = hipMalloc(&p, npx);
      if (e != hipSuccess) return fail(e, __LINE__);
      got.push_back(p);
      g[k] = (uint8_t*)p;
      if ((e = hipMalloc(&p, npx * 2)) != hipSuccess) return fail(e, __LINE__);
      got.push_back(p);
      d16[k] = (uint16_t*)p;
      if ((e = hipMalloc(&p, npx * 4)) != hipSuccess) return fail(e, __LINE__);
      got.push_back(p);
      df[k] = (float*)p;
    }
    hipEvent_t evs[3 * orbpl_tracker::kIn] = {};
    hipStream_t cs = nullptr;
    hipError_t e = hipSuccess;
    for (int i = 0; i < 3 * orbpl_tracker::kIn && e == hipSuccess; i++)
      e = hipEventCreateWithFlags(&evs[i], hipEventDisableTiming);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&cs, hipStreamNonBlocking);
    if (e != hipSuccess) {
      for (hipEvent_t x : evs)
        if (x) (void)hipEventDestroy(x);
      return fail(e, __LINE__);
    }
    for (int k = 0; k < orbpl_tracker::kIn; k++) {
      t->in_gray[k] = g[k];
      t->in_d16[k] = d16[k];
      t->in_depth[k] = df[k];
      t->in_copied[k] = evs[3 * k];
      t->in_done_s[k] = evs[3 * k + 1];
      t->in_done_l[k] = evs[3 * k + 2];
    }
    t->allocs.insert(t->allocs.end(), got.begin(), got.end());
    t->cstream = cs;
  }
  const int k = t->in_pos % orbpl_tracker::kIn;
  // the slot's previous frames must have been read (extraction + line stream)
  if (t->in_used[k]) {
    HIP_CHECK(hipStreamWaitEvent(t->cstream, t->in_done_s[k], 0));
    if (t->lines) HIP_CHECK(hipStreamWaitEvent(t->cstream, t->in_done_l[k], 0));
  }
  HIP_CHECK(hipMemcpyAsync(t->in_gray[k], h_gray, npx, hipMemcpyHostToDevice, t->cstream));
  HIP_CHECK(hipMemcpyAsync(t->in_d16[k], h_depth, npx * 2, hipMemcpyHostToDevice, t->cstream));
  HIP_CHECK(hipEventRecord(t->in_copied[k], t->cstream));
  HIP_CHECK(hipStreamWaitEvent(t->stream, t->in_copied[k], 0));
  // mDepthMapFactor = 1.0f / DepthMapFactor (Tracking.cc:142-146)
  launch_depth_u16(t->in_d16[k], t->in_depth[k], (long long)npx, 1.0f / depth_map_factor,
                   t->stream);
  const int rc = tracker_step(t, t->in_gray[k], t->in_depth[k], nullptr);
  if (rc) return rc;
  // the depth slot is read by the frame glue, on the tracking stream when the
  // glue runs there (which follows the extraction stream's reads of the slot)
  HIP_CHECK(hipEventRecord(t->in_done_s[k], t->glue_on_ts && t->pipelined ? t->tstream : t->stream));
  if (t->lines) HIP_CHECK(hipEventRecord(t->in_done_l[k], t->lstream));
  t->in_used[k] = true;
  t->in_pos++;
  return ORBPL_OK;
}

int orbpl_tracker_step_stereo(orbpl_tracker* t, const uint8_t* d_left, const uint8_t* d_right) {
  if (!t || !d_left || !d_right) return arg_fail("NULL argument");
  if (!t->stereo) return arg_fail("tracker created without ORBPL_TRACK_STEREO");
  return tracker_step(t, d_left, nullptr, d_right);
}

int orbpl_tracker_launch_frames(const orbpl_tracker* t, int* orb_frames, int* lsd_frames) {
  if (!t) return arg_fail("NULL tracker");
  if (orb_frames) *orb_frames = t->osplit ? t->osplit : t->S;
  if (lsd_frames) *lsd_frames = !t->lines ? 0 : (t->lsplit ? t->lsplit : t->S);
  return ORBPL_OK;
}

int orbpl_tracker_set_pipelined(orbpl_tracker* t, int on) {
  if (!t) return arg_fail("NULL tracker");
  HIP_CHECK(hipSetDevice(t->device));
  HIP_CHECK(hipStreamSynchronize(t->stream));
  HIP_CHECK(hipStreamSynchronize(t->tstream));
  t->pipelined = on ? 1 : 0;
  return ORBPL_OK;
}

int orbpl_tracker_synchronize(orbpl_tracker* t) {
  if (!t) return arg_fail("NULL tracker");
  HIP_CHECK(hipSetDevice(t->device));
  if (t->cstream) HIP_CHECK(hipStreamSynchronize(t->cstream));
  HIP_CHECK(hipStreamSynchronize(t->tstream));
  if (t->lines) {
    HIP_CHECK(hipStreamSynchronize(t->lstream));
    int rc = t->lsplit ? lsdx_check(t->lx, t->lsplit) : lsdx_check(t->lx, t->S);
    if (!rc && t->lsplit) rc = lsdx_check(t->lx2, t->S - t->lsplit);
    if (rc) return rc;
  }
  if (t->stereo) {
    int rc = orbx_synchronize(t->exr);
    if (rc) return rc;
    if (t->lxr) {
      HIP_CHECK(hipStreamSynchronize(t->rlstream));
      rc = lsdx_check(t->lxr, t->S);
      if (rc) return rc;
    }
    HIP_CHECK(hipStreamSynchronize(t->stream));
    int err = 0;
    HIP_CHECK(hipMemcpy(&err, t->d_err, 4, hipMemcpyDeviceToHost));
    if (err) {
      // reported once: clear the flag so that later steps start clean
      HIP_CHECK(hipMemset(t->d_err, 0, 4));
      return (arg_fail("stereo row band capacity exceeded"), ORBPL_ERR_OVERFLOW);
    }
  }
  if (t->ex2) {
    const int rc = orbx_synchronize(t->ex2);
    if (rc) return rc;
  }
  return orbx_synchronize(t->ex);
}

int orbpl_tracker_get_state(orbpl_tracker* t, float* Tcw, int* nkps, int* nmatches, int* ninliers,
                            int* nmatches_map) {
  if (!t) return arg_fail("NULL tracker");
  HIP_CHECK(hipSetDevice(t->device));
  HIP_CHECK(hipStreamSynchronize(t->stream));
  HIP_CHECK(hipStreamSynchronize(t->tstream));
  if (t->lines) HIP_CHECK(hipStreamSynchronize(t->lstream));
  std::vector<StreamState> st(t->S);
  HIP_CHECK(hipMemcpy(st.data(), t->d_state, sizeof(StreamState) * t->S, hipMemcpyDeviceToHost));
  std::vector<int> n(t->S);
  // the frame just tracked
  HIP_CHECK(hipMemcpy(n.data(), t->fb[(t->ring_pos + 2) % 3].n, 4 * t->S, hipMemcpyDeviceToHost));
  for (int s = 0; s < t->S; s++) {
    if (Tcw) memcpy(Tcw + 16 * s, st[s].Tlast, 64);
    if (nkps) nkps[s] = n[s];
    if (nmatches) nmatches[s] = st[s].nmatches;
    if (ninliers) ninliers[s] = st[s].ninliers;
    if (nmatches_map) nmatches_map[s] = st[s].nmatches_map;
  }
  return ORBPL_OK;
}

int orbpl_tracker_timing_counts(int* counts5) {
  if (!counts5) return arg_fail("NULL argument");
  counts5[0] = kTimingStages;
  counts5[1] = kLineTimingStages;
  counts5[2] = kLsdTimingStages;
  counts5[3] = kStereoTimingStages;
  counts5[4] = kKernelTimingStages;
  return ORBPL_OK;
}

int orbpl_tracker_kernel_timings(orbpl_tracker* t, int max_steps, float* ms, int* n_steps) {
  if (!t || !ms || !n_steps) return arg_fail("NULL argument");
  HIP_CHECK(hipSetDevice(t->device));
  HIP_CHECK(hipStreamSynchronize(t->stream));
  HIP_CHECK(hipStreamSynchronize(t->tstream));
  // every k_pose launch of the step (TrackWithMotionModel, TrackReferenceKeyFrame,
  // TrackLocalMap) and TrackLocalMap's k_match_local, each bracketed alone
  static const int kPair[kKernelTimingStages][2] = {{28, 29}, {30, 31}, {34, 35}, {32, 33}};
  const int n = std::min(max_steps, t->ring_count);
  for (int k = 0; k < n; k++) {
    const int step = t->ring_pos - n + k;
    hipEvent_t* ev = &t->ring[(size_t)(step % orbpl_tracker::kRing) * orbpl_tracker::kEv];
    for (int i = 0; i < kKernelTimingStages; i++)
      HIP_CHECK(hipEventElapsedTime(&ms[k * kKernelTimingStages + i], ev[kPair[i][0]], ev[kPair[i][1]]));
  }
  *n_steps = n;
  return ORBPL_OK;
}

int orbpl_tracker_timings(orbpl_tracker* t, int max_steps, float* ms, int* n_steps) {
  if (!t || !ms || !n_steps) return arg_fail("NULL argument");
  HIP_CHECK(hipSetDevice(t->device));
  HIP_CHECK(hipStreamSynchronize(t->stream));
  HIP_CHECK(hipStreamSynchronize(t->tstream));
  // stage intervals: 5 extraction stages, glue (extraction stream), then
  // match (incl. prediction), pose, finish (tracking stream)
  // (+ TrackLocalMap: gather, frustum, local matching, second pose, count)
  // (+ KeyFrame::ComputeBoW with a vocabulary; 0 without)
  // (FAST, octree, orientation + descriptors, stages 2-4: the summed kernel
  // time of their level-group launches on the extractor's FAST stream, which
  // overlap the pyramid's later levels under the level pipeline)
  static const int kPair[kTimingStages][2] = {{0, 1}, {1, 2}, {36, 37}, {3, 4}, {4, 5},
                                              {orbpl_tracker::kEvGlue, 27},
                                              {7, 8}, {14, 9}, {26, 10}, {9, 26}, {27, 6}};
  const int n = std::min(max_steps, t->ring_count);
  for (int k = 0; k < n; k++) {
    const int step = t->ring_pos - n + k;
    hipEvent_t* ev = &t->ring[(size_t)(step % orbpl_tracker::kRing) * orbpl_tracker::kEv];
    for (int i = 0; i < kTimingStages; i++)
      HIP_CHECK(hipEventElapsedTime(&ms[k * kTimingStages + i], ev[kPair[i][0]], ev[kPair[i][1]]));
    // FAST (2), octree (3), orientation + descriptors (4): summed launch brackets
    for (int kind = 0; kind < 3; kind++) {
      float sum = 0.f;
      for (int gi = 0; gi < kFastGroups; gi++) {
        float m = 0.f;
        const int e = 36 + 2 * (kind * kFastGroups + gi);
        HIP_CHECK(hipEventElapsedTime(&m, ev[e], ev[e + 1]));
        sum += m;
      }
      ms[k * kTimingStages + 2 + kind] = sum;
    }
  }
  *n_steps = n;
  return ORBPL_OK;
}

int orbpl_tracker_line_timings(orbpl_tracker* t, int max_steps, float* ms, int* n_steps) {
  if (!t || !ms || !n_steps) return arg_fail("NULL argument");
  if (!t->lines) return arg_fail("tracker created without ORBPL_TRACK_LINES");
  HIP_CHECK(hipSetDevice(t->device));
  HIP_CHECK(hipStreamSynchronize(t->stream));
  HIP_CHECK(hipStreamSynchronize(t->tstream));
  HIP_CHECK(hipStreamSynchronize(t->lstream));
  // LSD (line stream), KeyLines + LBD + UndistortKeyLines (line stream),
  // LineMatcher::SearchByProjection (tracking stream)
  static const int kPair[kLineTimingStages][2] = {{11, 12}, {12, 13}, {8, 14}};
  const int n = std::min(max_steps, t->ring_count);
  for (int k = 0; k < n; k++) {
    const int step = t->ring_pos - n + k;
    hipEvent_t* ev = &t->ring[(size_t)(step % orbpl_tracker::kRing) * orbpl_tracker::kEv];
    for (int i = 0; i < kLineTimingStages; i++)
      HIP_CHECK(hipEventElapsedTime(&ms[k * kLineTimingStages + i], ev[kPair[i][0]], ev[kPair[i][1]]));
  }
  *n_steps = n;
  return ORBPL_OK;
}

int orbpl_tracker_set_history(orbpl_tracker* t, int max_steps) {
  if (!t || max_steps < 0) return arg_fail("bad argument");
  HIP_CHECK(hipSetDevice(t->device));
  HIP_CHECK(hipStreamSynchronize(t->stream));
  HIP_CHECK(hipStreamSynchronize(t->tstream));
  for (void* p : {(void*)t->d_hist_state, (void*)t->d_hist_n, (void*)t->d_hist_nl})
    if (p) {
      t->allocs.erase(std::remove(t->allocs.begin(), t->allocs.end(), p), t->allocs.end());
      HIP_CHECK(hipFree(p));
    }
  t->d_hist_state = nullptr;
  t->d_hist_n = t->d_hist_nl = nullptr;
  t->hist_cap = t->hist_count = 0;
  if (max_steps == 0) return ORBPL_OK;
  const size_t n = (size_t)max_steps * t->S;
  int rc = tr_alloc(t, (void**)&t->d_hist_state, n * sizeof(StreamState));
  if (!rc) rc = tr_alloc(t, (void**)&t->d_hist_n, n * 4);
  if (!rc) rc = tr_alloc(t, (void**)&t->d_hist_nl, n * 4);
  if (rc) return rc;
  t->hist_cap = max_steps;
  return ORBPL_OK;
}

int orbpl_tracker_get_history(orbpl_tracker* t, int stream, int max_steps, float* Tcw,
                              int* counts12, int* n_steps) {
  if (!t || !n_steps || stream < 0 || stream >= t->S || max_steps < 0) return arg_fail("bad argument");
  HIP_CHECK(hipSetDevice(t->device));
  HIP_CHECK(hipStreamSynchronize(t->tstream));
  const int n = std::min(max_steps, t->hist_count);
  *n_steps = n;
  for (int k = 0; k < n; k++) {
    const size_t o = (size_t)k * t->S + stream;
    StreamState st;
    int nk = 0, nl = 0;
    HIP_CHECK(hipMemcpy(&st, t->d_hist_state + o, sizeof(st), hipMemcpyDeviceToHost));
    HIP_CHECK(hipMemcpy(&nk, t->d_hist_n + o, 4, hipMemcpyDeviceToHost));
    if (t->lines) HIP_CHECK(hipMemcpy(&nl, t->d_hist_nl + o, 4, hipMemcpyDeviceToHost));
    if (Tcw) memcpy(Tcw + 16 * k, st.Tlast, 64);
    if (counts12) {
      int* c = counts12 + 12 * k;
      c[0] = nk; c[1] = st.nmatches; c[2] = st.ninliers; c[3] = st.nmatches_map; c[4] = st.ok;
      c[5] = nl; c[6] = t->lines ? st.nlmatches : 0; c[7] = t->lines ? st.nlmatches_map : 0;
      const bool lm = (t->local_map || t->map) && st.lm_active;
      c[8] = lm ? st.lm_nlocal : 0; c[9] = lm ? st.lm_inl : 0;
      c[10] = lm && t->lines ? st.lm_nllocal : 0; c[11] = lm && t->lines ? st.lm_linl : 0;
    }
  }
  return ORBPL_OK;
}

int orbpl_tracker_get_map_history(orbpl_tracker* t, int stream, int max_steps, int* counts24,
                                  int* n_steps) {
  if (!t || !n_steps || !counts24 || stream < 0 || stream >= t->S || max_steps < 0)
    return arg_fail("bad argument");
  if (!t->map) return arg_fail("tracker created without ORBPL_TRACK_MAP");
  std::vector<int> c12((size_t)std::max(max_steps, 1) * 12);
  int rc = orbpl_tracker_get_history(t, stream, max_steps, nullptr, c12.data(), n_steps);
  if (rc) return rc;
  for (int k = 0; k < *n_steps; k++) {
    StreamState st;
    HIP_CHECK(hipMemcpy(&st, t->d_hist_state + (size_t)k * t->S + stream, sizeof(st),
                        hipMemcpyDeviceToHost));
    int* c = counts24 + 24 * k;
    for (int q = 0; q < 12; q++) c[q] = c12[(size_t)k * 12 + q];
    for (int q = 0; q < kMapOut; q++) c[12 + q] = st.map_out[q];
  }
  return ORBPL_OK;
}

// one stream's map (host copies; tests and inspection): keyframes with their
// parent and covisibility order, map points, map lines
static int map_stream_state(orbpl_tracker* t, int stream, MapState* ms) {
  if (!t || stream < 0 || stream >= t->S) return arg_fail("bad argument");
  if (!t->map) return arg_fail("tracker created without ORBPL_TRACK_MAP");
  HIP_CHECK(hipSetDevice(t->device));
  HIP_CHECK(hipStreamSynchronize(t->tstream));
  HIP_CHECK(hipStreamSynchronize(t->stream));
  HIP_CHECK(hipMemcpy(ms, t->ma.ms + stream, sizeof(MapState), hipMemcpyDeviceToHost));
  return ORBPL_OK;
}

int orbpl_tracker_get_map_keyframes(orbpl_tracker* t, int stream, int* parent, int* ord, int cap,
                                    int* nord, int* n_kf) {
  MapState ms;
  int rc = map_stream_state(t, stream, &ms);
  if (rc) return rc;
  if (!n_kf || cap < 0) return arg_fail("bad argument");
  const int n = ms.n_kf, F = t->map_kfc;
  *n_kf = n;
  const size_t kb = (size_t)stream * F;
  std::vector<int> par(F), no(F);
  std::vector<uint8_t> o((size_t)F * F);
  HIP_CHECK(hipMemcpy(par.data(), t->ma.kf_parent + kb, 4 * (size_t)F, hipMemcpyDeviceToHost));
  HIP_CHECK(hipMemcpy(no.data(), t->ma.kf_nord + kb, 4 * (size_t)F, hipMemcpyDeviceToHost));
  HIP_CHECK(hipMemcpy(o.data(), t->ma.kf_ord + kb * F, (size_t)F * F, hipMemcpyDeviceToHost));
  for (int k = 0; k < n; k++) {
    if (parent) parent[k] = par[k];
    if (nord) nord[k] = no[k];
    if (ord)
      for (int j = 0; j < cap; j++) ord[(size_t)k * cap + j] = j < no[k] && j < F ? o[(size_t)k * F + j] : -1;
  }
  return ORBPL_OK;
}

int orbpl_tracker_get_map_points(orbpl_tracker* t, int stream, int cap, int* nobs, uint8_t* desc,
                                 float* xyz, float* normal, float* dist2, int* n_mp) {
  MapState ms;
  int rc = map_stream_state(t, stream, &ms);
  if (rc) return rc;
  if (!n_mp || cap < 0) return arg_fail("bad argument");
  *n_mp = ms.n_mp;
  const int n = std::min(ms.n_mp, cap);
  const size_t g = (size_t)stream * t->ma.mpc;
  std::vector<float> f4((size_t)n * 4 + 1);
  if (nobs && n) HIP_CHECK(hipMemcpy(nobs, t->ma.mp_nobs + g, 4 * (size_t)n, hipMemcpyDeviceToHost));
  if (desc && n) HIP_CHECK(hipMemcpy(desc, t->ma.mp_desc + g * 32, 32 * (size_t)n, hipMemcpyDeviceToHost));
  if (xyz && n) {
    HIP_CHECK(hipMemcpy(f4.data(), t->ma.mp_pos + g, 16 * (size_t)n, hipMemcpyDeviceToHost));
    for (int p = 0; p < n; p++)
      for (int q = 0; q < 3; q++) xyz[3 * p + q] = f4[4 * p + q];
  }
  if (normal && n) {
    HIP_CHECK(hipMemcpy(f4.data(), t->ma.mp_nrm + g, 16 * (size_t)n, hipMemcpyDeviceToHost));
    for (int p = 0; p < n; p++)
      for (int q = 0; q < 3; q++) normal[3 * p + q] = f4[4 * p + q];
  }
  if (dist2 && n) HIP_CHECK(hipMemcpy(dist2, t->ma.mp_dist + g, 8 * (size_t)n, hipMemcpyDeviceToHost));
  return ORBPL_OK;
}

int orbpl_tracker_get_map_lines(orbpl_tracker* t, int stream, int cap, int* nobs, uint8_t* desc,
                                float* pos6, int* n_ml) {
  MapState ms;
  int rc = map_stream_state(t, stream, &ms);
  if (rc) return rc;
  if (!n_ml || cap < 0) return arg_fail("bad argument");
  *n_ml = ms.n_ml;
  const int n = std::min(ms.n_ml, cap);
  const size_t g = (size_t)stream * t->ma.mlc;
  if (nobs && n) HIP_CHECK(hipMemcpy(nobs, t->ma.ml_nobs + g, 4 * (size_t)n, hipMemcpyDeviceToHost));
  if (desc && n) HIP_CHECK(hipMemcpy(desc, t->ma.ml_desc + g * 32, 32 * (size_t)n, hipMemcpyDeviceToHost));
  if (pos6 && n) HIP_CHECK(hipMemcpy(pos6, t->ma.ml_pos + g * 6, 24 * (size_t)n, hipMemcpyDeviceToHost));
  return ORBPL_OK;
}

int orbpl_tracker_get_map_errors(orbpl_tracker* t, int* err) {
  if (!t || !err) return arg_fail("NULL argument");
  if (!t->map) return arg_fail("tracker created without ORBPL_TRACK_MAP");
  HIP_CHECK(hipSetDevice(t->device));
  HIP_CHECK(hipStreamSynchronize(t->tstream));
  HIP_CHECK(hipStreamSynchronize(t->stream));
  std::vector<MapState> ms(t->S);
  HIP_CHECK(hipMemcpy(ms.data(), t->ma.ms, sizeof(MapState) * t->S, hipMemcpyDeviceToHost));
  for (int s = 0; s < t->S; s++) err[s] = ms[s].err;
  return ORBPL_OK;
}

int orbpl_tracker_lsd_timings(orbpl_tracker* t, int max_steps, float* ms, int* n_steps) {
  if (!t || !ms || !n_steps) return arg_fail("NULL argument");
  if (!t->lines) return arg_fail("tracker created without ORBPL_TRACK_LINES");
  HIP_CHECK(hipSetDevice(t->device));
  HIP_CHECK(hipStreamSynchronize(t->lstream));
  // line stream: blur+resize+grad, sort, seed loop, validate, KeyLines,
  // blur5+Sobel+LBD, UndistortKeyLines + line depths
  static const int kPair[kLsdTimingStages][2] = {{11, 18}, {18, 19}, {19, 20}, {20, 12},
                                                 {12, 21}, {21, 22}, {22, 13}};
  const int n = std::min(max_steps, t->ring_count);
  for (int k = 0; k < n; k++) {
    const int step = t->ring_pos - n + k;
    hipEvent_t* ev = &t->ring[(size_t)(step % orbpl_tracker::kRing) * orbpl_tracker::kEv];
    for (int i = 0; i < kLsdTimingStages; i++)
      HIP_CHECK(hipEventElapsedTime(&ms[k * kLsdTimingStages + i], ev[kPair[i][0]], ev[kPair[i][1]]));
  }
  *n_steps = n;
  return ORBPL_OK;
}

int orbpl_tracker_stereo_timings(orbpl_tracker* t, int max_steps, float* ms, int* n_steps) {
  if (!t || !ms || !n_steps) return arg_fail("NULL argument");
  if (!t->stereo) return arg_fail("tracker created without ORBPL_TRACK_STEREO");
  HIP_CHECK(hipSetDevice(t->device));
  HIP_CHECK(hipStreamSynchronize(t->stream));
  HIP_CHECK(hipStreamSynchronize(t->tstream));
  HIP_CHECK(hipStreamSynchronize(t->rstream));
  // right ORB extraction (right stream), ComputeStereoMatches (extraction
  // stream); with lines: right LineExtractor (right line stream),
  // k_stereo_lines (line stream); 0 without lines
  static const int kPair[kStereoTimingStages][2] = {{15, 16}, {17, 27}, {23, 24}, {25, 13}};
  if (t->rlstream) HIP_CHECK(hipStreamSynchronize(t->rlstream));
  if (t->lstream) HIP_CHECK(hipStreamSynchronize(t->lstream));
  const int n = std::min(max_steps, t->ring_count);
  for (int k = 0; k < n; k++) {
    const int step = t->ring_pos - n + k;
    hipEvent_t* ev = &t->ring[(size_t)(step % orbpl_tracker::kRing) * orbpl_tracker::kEv];
    for (int i = 0; i < kStereoTimingStages; i++) {
      float* o = &ms[k * kStereoTimingStages + i];
      *o = 0.0f;
      if (i < 2 || t->lines) HIP_CHECK(hipEventElapsedTime(o, ev[kPair[i][0]], ev[kPair[i][1]]));
    }
  }
  *n_steps = n;
  return ORBPL_OK;
}

// Debug (ORBPL_POSE_PROFILE): stream 0's PoseOptimization phase times of the
// last step, ns: edges, linearize+reduce, solve+exp, trial errors+reduce,
// classify; then LM iterations and trials (counts).
int orbpl_tracker_debug_pose_profile(orbpl_tracker* t, long long* out7) {  // 8 values
  if (!t || !out7) return arg_fail("NULL argument");
  HIP_CHECK(hipSetDevice(t->device));
  HIP_CHECK(hipDeviceSynchronize());
  long long p[8];
  if (read_pose_profile(p)) return arg_fail("pose profile unavailable");
  for (int k = 0; k < 5; k++) out7[k] = p[k] * 10;
  out7[5] = p[5];
  out7[6] = p[6];
  out7[7] = p[7] * 10;
  return ORBPL_OK;
}

// Debug (ORBPL_MATCH_PROFILE): stream 0's SearchByProjection(last frame)
// phase times of the last step, ns: grid, candidates, ordered claims,
// rotation check, output.
int orbpl_tracker_debug_match_profile(orbpl_tracker* t, long long* out5) {
  if (!t || !out5) return arg_fail("NULL argument");
  HIP_CHECK(hipSetDevice(t->device));
  HIP_CHECK(hipDeviceSynchronize());
  long long p[8];
  if (read_match_profile(p)) return arg_fail("match profile unavailable");
  for (int k = 0; k < 5; k++) out5[k] = p[k] * 10;
  return ORBPL_OK;
}

int orbpl_tracker_timings_reset(orbpl_tracker* t) {
  if (!t) return arg_fail("NULL tracker");
  t->ring_count = 0;
  return ORBPL_OK;
}

int orbpl_tracker_stage_ms(orbpl_tracker* t, float* ms5) {
  if (!t || !ms5) return arg_fail("NULL argument");
  if (t->ring_count == 0) return arg_fail("no step recorded yet");
  float m[kTimingStages];
  int n = 0;
  int rc = orbpl_tracker_timings(t, 1, m, &n);
  if (rc) return rc;
  ms5[0] = m[0] + m[1] + m[2] + m[3] + m[4];
  for (int i = 0; i < 4; i++) ms5[1 + i] = m[5 + i];
  ms5[1] += m[10];  // glue: + KeyFrame::ComputeBoW
  ms5[3] += m[9];   // pose: both PoseOptimizations (+ the local map search)
  return ORBPL_OK;
}

int orbpl_tracker_kp_capacity(const orbpl_tracker* t) { return t ? t->kp_cap : 0; }

int orbpl_tracker_get_frame(orbpl_tracker* t, int stream, orbpl_keypoint* kps_un, uint8_t* desc,
                            int32_t* match, uint8_t* outlier, int* n) {
  if (!t || stream < 0 || stream >= t->S) return arg_fail("bad argument");
  HIP_CHECK(hipSetDevice(t->device));
  HIP_CHECK(hipStreamSynchronize(t->stream));
  HIP_CHECK(hipStreamSynchronize(t->tstream));
  const FrameBufs& F = t->fb[(t->ring_pos + 2) % 3];
  const size_t K = t->kp_cap, o = (size_t)stream * K;
  int cnt = 0;
  HIP_CHECK(hipMemcpy(&cnt, F.n + stream, 4, hipMemcpyDeviceToHost));
  if (n) *n = cnt;
  if (kps_un) HIP_CHECK(hipMemcpy(kps_un, F.kps_un + o, K * sizeof(KeyPointD), hipMemcpyDeviceToHost));
  if (desc) HIP_CHECK(hipMemcpy(desc, F.desc + o * 32, K * 32, hipMemcpyDeviceToHost));
  if (match) HIP_CHECK(hipMemcpy(match, F.match + o, K * 4, hipMemcpyDeviceToHost));
  if (outlier) HIP_CHECK(hipMemcpy(outlier, F.outlier + o, K, hipMemcpyDeviceToHost));
  return ORBPL_OK;
}

int orbpl_tracker_get_status(orbpl_tracker* t, int* ok, int* nlines, int* line_matches,
                             int* line_nmatches_map) {
  if (!t) return arg_fail("NULL tracker");
  HIP_CHECK(hipSetDevice(t->device));
  HIP_CHECK(hipStreamSynchronize(t->stream));
  HIP_CHECK(hipStreamSynchronize(t->tstream));
  if (t->lines) HIP_CHECK(hipStreamSynchronize(t->lstream));
  std::vector<StreamState> st(t->S);
  HIP_CHECK(hipMemcpy(st.data(), t->d_state, sizeof(StreamState) * t->S, hipMemcpyDeviceToHost));
  std::vector<int> nl(t->S, 0);
  if (t->lines)
    HIP_CHECK(hipMemcpy(nl.data(), t->fb[(t->ring_pos + 2) % 3].nl, 4 * t->S, hipMemcpyDeviceToHost));
  for (int s = 0; s < t->S; s++) {
    if (ok) ok[s] = st[s].ok;
    if (nlines) nlines[s] = nl[s];
    if (line_matches) line_matches[s] = t->lines ? st[s].nlmatches : 0;
    if (line_nmatches_map) line_nmatches_map[s] = t->lines ? st[s].nlmatches_map : 0;
  }
  return ORBPL_OK;
}

int orbpl_tracker_set_vocabulary(orbpl_tracker* t, orbv_vocab* voc, int levelsup) {
  if (!t) return arg_fail("NULL tracker");
  HIP_CHECK(hipSetDevice(t->device));
  HIP_CHECK(hipStreamSynchronize(t->stream));
  HIP_CHECK(hipStreamSynchronize(t->tstream));
  if (!voc) {
    t->voc = nullptr;
    return ORBPL_OK;
  }
  if (t->kp_cap > 4096) return arg_fail("orbpl_tracker_set_vocabulary: > 4096 keypoints per frame");
  const int rc = orbv_upload(voc, t->device);
  if (rc) return rc;
  if (!t->d_bow_err) {
    const size_t SK = (size_t)t->S * t->kp_cap;
    auto alloc = [&](void** p, size_t bytes) -> int {
      HIP_CHECK(hipMalloc(p, bytes));
      t->allocs.push_back(*p);
      return ORBPL_OK;
    };
    for (FrameBufs& f : t->fb) {
      if (alloc((void**)&f.feat_node, SK * 4) || alloc((void**)&f.feat_word, SK * 4) ||
          alloc((void**)&f.feat_weight, SK * 8) || alloc((void**)&f.bow_words, SK * 4) ||
          alloc((void**)&f.bow_vals, SK * 8) || alloc((void**)&f.bow_n, (size_t)t->S * 4))
        return ORBPL_ERR_HIP;
      HIP_CHECK(hipMemset(f.bow_n, 0, (size_t)t->S * 4));
    }
    if (alloc((void**)&t->d_bow_err, 4)) return ORBPL_ERR_HIP;
    HIP_CHECK(hipMemset(t->d_bow_err, 0, 4));
  }
  t->voc = voc;
  t->voc_levelsup = levelsup;
  return ORBPL_OK;
}

int orbpl_tracker_get_bow(orbpl_tracker* t, int stream, uint32_t* bow_words, double* bow_vals,
                          int* bow_n, int32_t* feat_node, int* n) {
  if (!t || stream < 0 || stream >= t->S) return arg_fail("bad argument");
  if (!t->d_bow_err) return arg_fail("orbpl_tracker_get_bow: no vocabulary set");
  HIP_CHECK(hipSetDevice(t->device));
  HIP_CHECK(hipStreamSynchronize(t->stream));
  HIP_CHECK(hipStreamSynchronize(t->tstream));
  const FrameBufs& F = t->fb[(t->ring_pos + 2) % 3];
  const size_t K = t->kp_cap, o = (size_t)stream * K;
  int cnt = 0, bn = 0, err = 0;
  HIP_CHECK(hipMemcpy(&cnt, F.n + stream, 4, hipMemcpyDeviceToHost));
  HIP_CHECK(hipMemcpy(&bn, F.bow_n + stream, 4, hipMemcpyDeviceToHost));
  HIP_CHECK(hipMemcpy(&err, t->d_bow_err, 4, hipMemcpyDeviceToHost));
  if (err) {
    HIP_CHECK(hipMemset(t->d_bow_err, 0, 4));
    return arg_fail("BoW transform: feature capacity exceeded");
  }
  if (n) *n = cnt;
  if (bow_n) *bow_n = bn;
  if (bow_words && bn) HIP_CHECK(hipMemcpy(bow_words, F.bow_words + o, 4 * (size_t)bn, hipMemcpyDeviceToHost));
  if (bow_vals && bn) HIP_CHECK(hipMemcpy(bow_vals, F.bow_vals + o, 8 * (size_t)bn, hipMemcpyDeviceToHost));
  if (feat_node && cnt) HIP_CHECK(hipMemcpy(feat_node, F.feat_node + o, 4 * (size_t)cnt, hipMemcpyDeviceToHost));
  return ORBPL_OK;
}

int orbpl_tracker_get_trk(orbpl_tracker* t, int* trk) {
  if (!t || !trk) return arg_fail("NULL argument");
  HIP_CHECK(hipSetDevice(t->device));
  HIP_CHECK(hipStreamSynchronize(t->stream));
  HIP_CHECK(hipStreamSynchronize(t->tstream));
  std::vector<StreamState> st(t->S);
  HIP_CHECK(hipMemcpy(st.data(), t->d_state, sizeof(StreamState) * t->S, hipMemcpyDeviceToHost));
  for (int s = 0; s < t->S; s++) trk[s] = t->refkf ? st[s].trk : 0;
  return ORBPL_OK;
}

int orbpl_tracker_get_local_stats(orbpl_tracker* t, int* local_matches, int* local_inliers,
                                  int* local_line_matches, int* local_line_inliers) {
  if (!t) return arg_fail("NULL tracker");
  HIP_CHECK(hipSetDevice(t->device));
  HIP_CHECK(hipStreamSynchronize(t->tstream));
  HIP_CHECK(hipStreamSynchronize(t->stream));
  std::vector<StreamState> st(t->S);
  HIP_CHECK(hipMemcpy(st.data(), t->d_state, sizeof(StreamState) * t->S, hipMemcpyDeviceToHost));
  for (int s = 0; s < t->S; s++) {
    const bool lm = (t->local_map || t->map) && st[s].lm_active;
    if (local_matches) local_matches[s] = lm ? st[s].lm_nlocal : 0;
    if (local_inliers) local_inliers[s] = lm ? st[s].lm_inl : 0;
    if (local_line_matches) local_line_matches[s] = lm && t->lines ? st[s].lm_nllocal : 0;
    if (local_line_inliers) local_line_inliers[s] = lm && t->lines ? st[s].lm_linl : 0;
  }
  return ORBPL_OK;
}

int orbpl_tracker_get_lines(orbpl_tracker* t, int stream, orbpl_keyline* kl_un, uint8_t* desc,
                            int32_t* lmatch, uint8_t* loutlier, int* n) {
  if (!t || stream < 0 || stream >= t->S) return arg_fail("bad argument");
  if (!t->lines) return arg_fail("tracker created without ORBPL_TRACK_LINES");
  HIP_CHECK(hipSetDevice(t->device));
  HIP_CHECK(hipStreamSynchronize(t->stream));
  HIP_CHECK(hipStreamSynchronize(t->tstream));
  HIP_CHECK(hipStreamSynchronize(t->lstream));
  const FrameBufs& F = t->fb[(t->ring_pos + 2) % 3];
  const size_t K = kLineKeep, o = (size_t)stream * K;
  int cnt = 0;
  HIP_CHECK(hipMemcpy(&cnt, F.nl + stream, 4, hipMemcpyDeviceToHost));
  if (n) *n = cnt;
  if (kl_un) HIP_CHECK(hipMemcpy(kl_un, F.kl_un + o, K * sizeof(orbpl_keyline), hipMemcpyDeviceToHost));
  if (desc) HIP_CHECK(hipMemcpy(desc, F.ldesc + o * 32, K * 32, hipMemcpyDeviceToHost));
  if (lmatch) HIP_CHECK(hipMemcpy(lmatch, F.lmatch + o, K * 4, hipMemcpyDeviceToHost));
  if (loutlier) HIP_CHECK(hipMemcpy(loutlier, F.loutlier + o, K, hipMemcpyDeviceToHost));
  return ORBPL_OK;
}

}  // extern "C"
