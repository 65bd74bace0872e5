// Exercises the drop-in classes the way Tracking uses them on three RGB-D
// frames and writes every output for tests/test_gpu_dropin.py to check
// against the oracle:
//   frame 0: StereoInitialization-style map (Tracking.cc:608-690): a map
//            point per keypoint with depth, a map line per line with both
//            end-point depths; the initial keyframe KF0 with its BoW;
//   frame 1: TrackWithMotionModel's matching and pose with zero velocity
//            (Tracking.cc:1228-1271);
//   frame 2: TrackReferenceKeyFrame against KF0 (Tracking.cc:942-1032:
//            ComputeBoW, ORBmatcher(0.7).SearchByBoW, the last frame's pose,
//            LineMatcher(0.7).SearchByProjection(F, KF), the pose, the outlier
//            discard), then TrackLocalMap with KF0 as the local map
//            (Tracking.cc:1332-1420, 1746-1865: IsInFrustum,
//            ORBmatcher(0.8).SearchByProjection(F, points, 3),
//            LineMatcher(0.8).SearchByProjection(F, lines), the second pose).
//   dropin_driver <in.bin> <out.bin>
//   dropin_driver --time <in.bin> <K>: K Frame constructions of frame 0 (ORB ||
//   LineExtractor on two host threads + the frame glue, one frame at a time as
//   the reference's Tracking builds them), median / mean latency in ms
//   dropin_driver --stereo <in.bin> <out.bin>: two rectified stereo pairs
//   through the stereo Frame (Frame.cc:71-132: ORB left || right,
//   ComputeStereoMatches), GetFeaturesInArea queries on frame 0, frame 0's
//   map from the stereo depths and frame 1's TrackWithMotionModel with zero
//   velocity and th = 7 (Tracking.cc:1228-1271, points only: the stereo Frame
//   has no lines); formats at stereo_mode()
//   dropin_driver --harness <in.bin> <out.bin>: the reference's Test/ demos'
//   calls (Test/LastFrameProjection.cpp:262-293, LocalMapProjectionTest.cpp:
//   334): frame 0's map lines from both end-point depths (Observations() = 1
//   for every third line, 0 otherwise: the fork's harness MapLines have none),
//   LineMatcher::SearchByProjection(F1, F0, new_kls, match_indices) at frame
//   0's pose, SearchByProjection(F2, frame 0's map lines with IsInFrustum,
//   new_kls, match_indices) and SearchByProjection(F2, KF0, vpMapLineMatches);
//   formats at harness_mode()
//   dropin_driver --fail: a Frame from an 8x8 image, which the library's
//   extractors reject: the error must reach the caller as an exception (the
//   line thread joined first), printed as "caught: <message>", exit 0
// in.bin : int32 W, H; float fx fy cx cy k1 k2 p1 p2 k3 bf thdepth;
//          int32 nfeatures; float scale; int32 nlevels, iniTh, minTh;
//          float Tcw0[16]; 3 x (gray W*H u8, depth W*H f32);
//          int32 len; vocabulary path (len bytes, DBoW2 text format)
// out.bin: per frame: N, kps (N x 28 B), desc (N x 32), NL, keylines (NL x
//          68 B), line desc (NL x 32), coef (NL x 3 f64), keysUn (N x 28 B),
//          depth (N f32); frame 0's pyramid: nlevels x (w, h, w*h bytes);
//          frame 1: nmatches, line matches, inliers, Tcw1[16], match[N1]
//          (frame-0 index or -1), outlier[N1] u8, line match[NL1], line
//          outlier[NL1] u8;
//          the map of frame 0: per keypoint has_mp u8, xyz f32x3, normal
//          f32x3, min / max distance invariance f32x2; per line has_ml u8,
//          xyz6 f32x6; the FeatureVector node of every frame-0 and frame-2
//          feature (int32, -1 none);
//          frame 2, TrackReferenceKeyFrame: nmatches, bow match[N2], line
//          nmatches, line match[NL2], go, inliers, Tcw[16], outlier[N2] u8,
//          line outlier[NL2] u8, nmatchesMap, line_nmatchesMap;
//          TrackLocalMap: seen[N0] u8 (skipped: matched by frame 2), in_view
//          [N0] u8, local nmatches, match[N2] after the search, line seen
//          [NL0], line in_view[NL0], local line nmatches, line match[NL2],
//          inliers, Tcw[16]
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "Frame.h"
#include "KeyFrame.h"
#include "LineMatcher.h"
#include "ORBmatcher.h"
#include "Optimizer.h"

using namespace ORB_SLAM2;

template <class T>
static void rd(FILE* f, T* p, size_t n) {
  if (n && fread(p, sizeof(T), n, f) != n) throw std::runtime_error("short input");
}
template <class T>
static void wr(FILE* f, const T* p, size_t n) {
  if (n && fwrite(p, sizeof(T), n, f) != n) throw std::runtime_error("short write");
}
template <class T>
static void wr1(FILE* f, T v) {
  wr(f, &v, 1);
}

static void write_frame(FILE* o, const Frame& F) {
  wr(o, &F.N, 1);
  wr(o, F.mvKeys.data(), F.N);
  wr(o, F.mDescriptors.data, (size_t)F.N * 32);
  wr(o, &F.NL, 1);
  wr(o, F.mvKeyLines.data(), F.NL);
  wr(o, F.mLineDescriptors.data, (size_t)F.NL * 32);
  for (int i = 0; i < F.NL; i++) wr(o, F.mvKeyLineCoefficient[i].v, 3);
  wr(o, F.mvKeysUn.data(), F.N);
  wr(o, F.mvDepth.data(), F.N);
}

// index of a frame-0 map element in the frame-0 feature indexing (-1: NULL)
template <class P>
static void write_index(FILE* o, const std::vector<P*>& v, std::map<const P*, int>& idx) {
  for (P* p : v) wr1<int32_t>(o, p ? idx.at(p) : -1);
}

static std::vector<int32_t> node_of(const DBoW2::FeatureVector& fv, int n) {
  std::vector<int32_t> node(n, -1);
  for (const auto& kv : fv)
    for (unsigned i : kv.second) node[i] = (int32_t)kv.first;
  return node;
}

// Tracking::StereoInitialization's map (Tracking.cc:633-660): a map point per
// keypoint with depth, its normal and scale-invariance distances as
// MapPoint::UpdateNormalAndDepth sets them with the one observation
static void map_points_from_depth(Frame& F0, std::vector<std::unique_ptr<MapPoint>>& mps,
                                  std::map<const MapPoint*, int>& mp_index) {
  const cv::Mat Ow = F0.GetCameraCenter();
  for (int i = 0; i < F0.N; i++) {
    if (!(F0.mvDepth[i] > 0)) continue;
    cv::Mat X = F0.UnprojectStereo(i);
    mps.emplace_back(new MapPoint(X.ptr<float>(), F0.mDescriptors.ptr<uint8_t>(i)));
    float nrm[3];
    double dd = 0;
    for (int k = 0; k < 3; k++) {
      nrm[k] = X.at<float>(k, 0) - Ow.at<float>(k, 0);
      dd += (double)nrm[k] * nrm[k];
    }
    const float dn = (float)std::sqrt(dd);
    for (int k = 0; k < 3; k++) nrm[k] = nrm[k] * (1.0f / dn);
    const float maxd = dn * F0.mvScaleFactors[F0.mvKeysUn[i].octave];
    mps.back()->SetNormalAndDistances(nrm, maxd / F0.mvScaleFactors[F0.mnScaleLevels - 1], maxd);
    F0.mvpMapPoints[i] = mps.back().get();
    mp_index[mps.back().get()] = i;
  }
}

// in.bin : int32 W, H; float fx fy cx cy k1 k2 p1 p2 k3 bf thdepth;
//          int32 nfeatures; float scale; int32 nlevels, iniTh, minTh;
//          float Tcw0[16]; 2 x (left W*H u8, right W*H u8);
//          int32 Q; Q x (float x, y, r; int32 minLevel, maxLevel)
// out.bin: per frame: N, kps (N x 28 B), desc (N x 32), Nr, right kps (Nr x
//          28 B), keysUn (N x 28 B), uRight (N f32), depth (N f32);
//          frame 0: per query the count and the indices (int32);
//          frame 1: nmatches, inliers, Tcw1[16], match[N1] (frame-0 index or
//          -1), outlier[N1] u8
static int stereo_mode(const char* inp, const char* outp) {
  FILE* in = fopen(inp, "rb");
  if (!in) throw std::runtime_error("cannot open input");
  int32_t wh[2];
  float camv[11], Tcw0[16];
  int32_t nf, nl, ini, mn;
  float sf;
  rd(in, wh, 2);
  rd(in, camv, 11);
  rd(in, &nf, 1);
  rd(in, &sf, 1);
  rd(in, &nl, 1);
  rd(in, &ini, 1);
  rd(in, &mn, 1);
  rd(in, Tcw0, 16);
  const int W = wh[0], H = wh[1];
  std::vector<cv::Mat> L(2), R(2);
  for (int k = 0; k < 2; k++) {
    L[k] = cv::Mat(H, W, cv::CV_8U);
    R[k] = cv::Mat(H, W, cv::CV_8U);
    rd(in, L[k].data, (size_t)W * H);
    rd(in, R[k].data, (size_t)W * H);
  }
  int32_t nq = 0;
  rd(in, &nq, 1);
  std::vector<float> qf(3 * (size_t)nq);
  std::vector<int32_t> qi(2 * (size_t)nq);
  for (int q = 0; q < nq; q++) {
    rd(in, &qf[3 * q], 3);
    rd(in, &qi[2 * q], 2);
  }
  fclose(in);
  cv::Mat K = cv::Mat::eye(3, 3, cv::CV_32F);
  K.at<float>(0, 0) = camv[0];
  K.at<float>(1, 1) = camv[1];
  K.at<float>(0, 2) = camv[2];
  K.at<float>(1, 2) = camv[3];
  cv::Mat dist(5, 1, cv::CV_32F);
  for (int k = 0; k < 5; k++) dist.at<float>(k, 0) = camv[4 + k];
  const float bf = camv[9], thDepth = camv[10];
  // Tracking::Tracking: mpORBextractorLeft / Right (Tracking.cc:115-120)
  ORBextractor exL(nf, sf, nl, ini, mn), exR(nf, sf, nl, ini, mn);
  Frame F0(L[0], R[0], 0.0, &exL, &exR, nullptr, K, dist, bf, thDepth);
  Frame F1(L[1], R[1], 1.0, &exL, &exR, nullptr, K, dist, bf, thDepth);
  FILE* o = fopen(outp, "wb");
  if (!o) throw std::runtime_error("cannot open output");
  for (const Frame* F : {&F0, &F1}) {
    wr(o, &F->N, 1);
    wr(o, F->mvKeys.data(), F->N);
    wr(o, F->mDescriptors.data, (size_t)F->N * 32);
    const int32_t nr = (int32_t)F->mvKeysRight.size();
    wr(o, &nr, 1);
    wr(o, F->mvKeysRight.data(), nr);
    wr(o, F->mvKeysUn.data(), F->N);
    wr(o, F->mvuRight.data(), F->N);
    wr(o, F->mvDepth.data(), F->N);
  }
  for (int q = 0; q < nq; q++) {
    const std::vector<size_t> v =
        F0.GetFeaturesInArea(qf[3 * q], qf[3 * q + 1], qf[3 * q + 2], qi[2 * q], qi[2 * q + 1]);
    wr1<int32_t>(o, (int32_t)v.size());
    for (size_t j : v) wr1<int32_t>(o, (int32_t)j);
  }
  // frame 0: pose Tcw0, its map; frame 1: TrackWithMotionModel, zero velocity
  cv::Mat T0(4, 4, cv::CV_32F);
  std::memcpy(T0.data, Tcw0, 64);
  F0.SetPose(T0);
  std::vector<std::unique_ptr<MapPoint>> mps;
  std::map<const MapPoint*, int> mp_index;
  map_points_from_depth(F0, mps, mp_index);
  F1.SetPose(F0.mTcw);
  ORBmatcher matcher(0.9f, true);
  const int th = 7;   // STEREO (Tracking.cc:1238-1241)
  int nmatches = matcher.SearchByProjection(F1, F0, th, false);
  if (nmatches < 20) {
    std::fill(F1.mvpMapPoints.begin(), F1.mvpMapPoints.end(), nullptr);
    nmatches = matcher.SearchByProjection(F1, F0, 2 * th, false);
  }
  int ninl = 0;
  if (nmatches >= 20) ninl = Optimizer::PoseOptimizationWithLines(&F1);   // NL = 0: points
  wr(o, &nmatches, 1);
  wr(o, &ninl, 1);
  wr(o, F1.mTcw.ptr<float>(), 16);
  write_index(o, F1.mvpMapPoints, mp_index);
  for (int i = 0; i < F1.N; i++) wr1<uint8_t>(o, F1.mvbOutlier[i]);
  fclose(o);
  return 0;
}

// out.bin: per frame 0..2: NL, kl_un (NL x 68 B), line desc (NL x 32);
// frame 0's map lines: per line has u8, xyz6 f32x6, nobs i32; then
// A (last frame): Tcw1[16], n, nnew, new_kls (nnew x 68 B), npairs, pairs
//   (npairs x 2 i32), F1 line match[NL1] (frame-0 index or -1);
// B (local map): Tcw2[16], in_view[NL0] u8, n, nnew, new_kls, npairs, pairs,
//   F2 line match[NL2];
// C (BFMatcher vs KF0): n, vpMapLineMatches[NL2] (frame-0 index or -1).
static int harness_mode(const char* inp, const char* outp) {
  FILE* in = fopen(inp, "rb");
  if (!in) throw std::runtime_error("cannot open input");
  int32_t wh[2];
  float camv[11], Tcw0[16];
  int32_t nf, nl, ini, mn;
  float sf;
  rd(in, wh, 2);
  rd(in, camv, 11);
  rd(in, &nf, 1);
  rd(in, &sf, 1);
  rd(in, &nl, 1);
  rd(in, &ini, 1);
  rd(in, &mn, 1);
  rd(in, Tcw0, 16);
  const int W = wh[0], H = wh[1];
  std::vector<cv::Mat> g(3), d(3);
  for (int k = 0; k < 3; k++) {
    g[k] = cv::Mat(H, W, cv::CV_8U);
    d[k] = cv::Mat(H, W, cv::CV_32F);
    rd(in, g[k].data, (size_t)W * H);
    rd(in, d[k].ptr<float>(), (size_t)W * H);
  }
  fclose(in);
  cv::Mat K = cv::Mat::eye(3, 3, cv::CV_32F);
  K.at<float>(0, 0) = camv[0];
  K.at<float>(1, 1) = camv[1];
  K.at<float>(0, 2) = camv[2];
  K.at<float>(1, 2) = camv[3];
  cv::Mat dist(5, 1, cv::CV_32F);
  for (int k = 0; k < 5; k++) dist.at<float>(k, 0) = camv[4 + k];
  ORBextractor ex(nf, sf, nl, ini, mn);
  std::vector<std::unique_ptr<Frame>> F;
  for (int k = 0; k < 3; k++)
    F.emplace_back(new Frame(g[k], d[k], (double)k, &ex, nullptr, K, dist, camv[9], camv[10]));
  cv::Mat T0(4, 4, cv::CV_32F);
  std::memcpy(T0.data, Tcw0, 64);
  for (auto& f : F) f->SetPose(T0);
  FILE* o = fopen(outp, "wb");
  if (!o) throw std::runtime_error("cannot open output");
  for (auto& f : F) {
    wr(o, &f->NL, 1);
    wr(o, f->mvKeyLinesUn.data(), f->NL);
    wr(o, f->mLineDescriptors.data, (size_t)f->NL * 32);
  }
  // Test/LastFrameProjection.cpp:262-284
  Frame& F0 = *F[0];
  std::vector<std::unique_ptr<MapLine>> mls;
  std::map<const MapLine*, int> ml_index;
  for (int j = 0; j < F0.NL; j++) {
    float v[6] = {0, 0, 0, 0, 0, 0};
    int32_t nobs = j % 3 == 0 ? 1 : 0;
    const bool has = F0.mvDepthLineStart[j] > 0 && F0.mvDepthLineEnd[j] > 0;
    if (has) {
      cv::Mat s = F0.UnprojectStereoLineStart(j), e = F0.UnprojectStereoLineEnd(j);
      for (int k = 0; k < 3; k++) {
        v[k] = s.at<float>(k, 0);
        v[3 + k] = e.at<float>(k, 0);
      }
      mls.emplace_back(new MapLine(v, F0.mLineDescriptors.ptr<uint8_t>(j), nobs));
      F0.mvpMapLines[j] = mls.back().get();
      ml_index[mls.back().get()] = j;
    }
    wr1<uint8_t>(o, has);
    wr(o, v, 6);
    wr1<int32_t>(o, has ? nobs : 0);
  }
  auto write_kls = [&](const std::vector<KeyLine>& kls,
                       const std::vector<std::pair<int, int>>& mi) {
    const int32_t nn = (int32_t)kls.size(), np = (int32_t)mi.size();
    wr(o, &nn, 1);
    wr(o, kls.data(), kls.size());
    wr(o, &np, 1);
    for (const auto& p : mi) {
      wr1<int32_t>(o, p.first);
      wr1<int32_t>(o, p.second);
    }
  };
  // A: Test/LastFrameProjection.cpp:290-293
  LineMatcher line_matcher(0.9f, true);
  Frame& F1 = *F[1];
  std::fill(F1.mvpMapLines.begin(), F1.mvpMapLines.end(), nullptr);
  std::vector<KeyLine> new_kls;
  std::vector<std::pair<int, int>> match_indices;
  const int32_t nA = line_matcher.SearchByProjection(F1, F0, new_kls, match_indices);
  wr(o, F1.mTcw.ptr<float>(), 16);
  wr(o, &nA, 1);
  write_kls(new_kls, match_indices);
  write_index(o, F1.mvpMapLines, ml_index);
  // B: Test/LocalMapProjectionTest.cpp:322-334 (local map = frame 0's lines)
  Frame& F2 = *F[2];
  std::vector<MapLine*> local;
  for (int j = 0; j < F0.NL; j++)
    if (F0.mvpMapLines[j]) local.push_back(F0.mvpMapLines[j]);
  wr(o, F2.mTcw.ptr<float>(), 16);
  std::vector<uint8_t> seen(F0.NL, 0);
  for (int j = 0; j < F0.NL; j++)
    if (F0.mvpMapLines[j]) seen[j] = F2.IsInFrustum(F0.mvpMapLines[j], 0.5f);
  wr(o, seen.data(), seen.size());
  std::fill(F2.mvpMapLines.begin(), F2.mvpMapLines.end(), nullptr);
  std::vector<KeyLine> new_kls2;
  std::vector<std::pair<int, int>> mi2;
  const int32_t nB = line_matcher.SearchByProjection(F2, local, new_kls2, mi2);
  wr(o, &nB, 1);
  write_kls(new_kls2, mi2);
  write_index(o, F2.mvpMapLines, ml_index);
  // C: LineMatcher.cpp:492-525 against the keyframe of frame 0
  KeyFrame KF0(F0);
  std::vector<MapLine*> vpMapLineMatches;
  const int32_t nC = line_matcher.SearchByProjection(F2, &KF0, vpMapLineMatches);
  wr(o, &nC, 1);
  write_index(o, vpMapLineMatches, ml_index);
  fclose(o);
  return 0;
}

static int fail_mode() {
  ORBextractor ex(1000, 1.2f, 8, 20, 7);
  cv::Mat K = cv::Mat::eye(3, 3, cv::CV_32F);
  K.at<float>(0, 0) = K.at<float>(1, 1) = 500.f;
  K.at<float>(0, 2) = K.at<float>(1, 2) = 4.f;
  cv::Mat dist(5, 1, cv::CV_32F);
  for (int k = 0; k < 5; k++) dist.at<float>(k, 0) = 0.f;
  cv::Mat g(8, 8, cv::CV_8U), d(8, 8, cv::CV_32F);
  for (int i = 0; i < 64; i++) {
    g.data[i] = (uint8_t)(i * 37);
    d.ptr<float>()[i] = 1.f;
  }
  try {
    Frame F(g, d, 0.0, &ex, nullptr, K, dist, 40.f, 40.f);
  } catch (const std::exception& e) {
    printf("caught: %s\n", e.what());
    return 0;
  }
  printf("no error\n");
  return 1;
}

int main(int argc, char** argv) {
  if (argc == 2 && std::string(argv[1]) == "--fail") return fail_mode();
  if (argc == 4 && std::string(argv[1]) == "--harness") {
    try {
      return harness_mode(argv[2], argv[3]);
    } catch (const std::exception& e) {
      fprintf(stderr, "dropin_driver: %s\n", e.what());
      return 1;
    }
  }
  if (argc == 4 && std::string(argv[1]) == "--stereo") {
    try {
      return stereo_mode(argv[2], argv[3]);
    } catch (const std::exception& e) {
      fprintf(stderr, "dropin_driver: %s\n", e.what());
      return 1;
    }
  }
  const bool timing = argc == 4 && std::string(argv[1]) == "--time";
  if (argc != 3 && !timing) {
    fprintf(stderr, "usage: dropin_driver in.bin out.bin | dropin_driver --time in.bin K\n");
    return 2;
  }
  try {
    FILE* in = fopen(argv[timing ? 2 : 1], "rb");
    if (!in) throw std::runtime_error("cannot open input");
    int32_t wh[2];
    float camv[11], Tcw0[16];
    int32_t nf, nl, ini, mn;
    float sf;
    rd(in, wh, 2);
    rd(in, camv, 11);
    rd(in, &nf, 1);
    rd(in, &sf, 1);
    rd(in, &nl, 1);
    rd(in, &ini, 1);
    rd(in, &mn, 1);
    rd(in, Tcw0, 16);
    const int W = wh[0], H = wh[1];
    std::vector<cv::Mat> g(3), d(3);
    for (int k = 0; k < 3; k++) {
      g[k] = cv::Mat(H, W, cv::CV_8U);
      d[k] = cv::Mat(H, W, cv::CV_32F);
      rd(in, g[k].data, (size_t)W * H);
      rd(in, d[k].ptr<float>(), (size_t)W * H);
    }
    int32_t plen = 0;
    rd(in, &plen, 1);
    std::string vpath(plen, '\0');
    rd(in, &vpath[0], plen);
    fclose(in);

    // Tracking::Tracking: K, DistCoef, mbf, mThDepth = bf * ThDepth / fx
    // (Tracking.cc:54-138)
    cv::Mat K = cv::Mat::eye(3, 3, cv::CV_32F);
    K.at<float>(0, 0) = camv[0];
    K.at<float>(1, 1) = camv[1];
    K.at<float>(0, 2) = camv[2];
    K.at<float>(1, 2) = camv[3];
    cv::Mat dist(5, 1, cv::CV_32F);
    for (int k = 0; k < 5; k++) dist.at<float>(k, 0) = camv[4 + k];
    const float bf = camv[9], thDepth = camv[10];
    ORBextractor ex(nf, sf, nl, ini, mn);
    if (timing) {
      const int reps = std::max(1, atoi(argv[3]));
      std::vector<double> ms;
      for (int r = 0; r < reps + 3; r++) {   // 3 warm-up constructions
        const auto t0 = std::chrono::steady_clock::now();
        // the timed constructor reads no vocabulary (ComputeBoW is not part of it)
        Frame Ft(g[r % 3], d[r % 3], r, &ex, nullptr, K, dist, bf, thDepth);
        const auto t1 = std::chrono::steady_clock::now();
        if (r >= 3) ms.push_back(std::chrono::duration<double, std::milli>(t1 - t0).count());
      }
      std::sort(ms.begin(), ms.end());
      double mean = 0;
      for (double v : ms) mean += v / ms.size();
      printf("time: median %.3f ms mean %.3f ms frames %d\n", ms[ms.size() / 2], mean, reps);
      return 0;
    }
    ORBVocabulary voc;
    if (!voc.loadFromTextFile(vpath)) throw std::runtime_error("cannot load the vocabulary");
    Frame F0(g[0], d[0], 0.0, &ex, &voc, K, dist, bf, thDepth);
    std::vector<cv::Mat> pyr = ex.FetchPyramid();   // lazy: only this check reads it
    Frame F1(g[1], d[1], 1.0, &ex, &voc, K, dist, bf, thDepth);

    // ---- frame 0: pose Tcw0, map points / lines from depth (Tracking.cc:633-692)
    cv::Mat T0(4, 4, cv::CV_32F);
    std::memcpy(T0.data, Tcw0, 64);
    F0.SetPose(T0);
    std::vector<std::unique_ptr<MapPoint>> mps;
    std::vector<std::unique_ptr<MapLine>> mls;
    std::map<const MapPoint*, int> mp_index;
    std::map<const MapLine*, int> ml_index;
    map_points_from_depth(F0, mps, mp_index);
    for (int j = 0; j < F0.NL; j++) {
      if (!(F0.mvDepthLineStart[j] > 0 && F0.mvDepthLineEnd[j] > 0)) continue;
      cv::Mat s = F0.UnprojectStereoLineStart(j), e = F0.UnprojectStereoLineEnd(j);
      const float xyz6[6] = {s.at<float>(0, 0), s.at<float>(1, 0), s.at<float>(2, 0),
                             e.at<float>(0, 0), e.at<float>(1, 0), e.at<float>(2, 0)};
      mls.emplace_back(new MapLine(xyz6, F0.mLineDescriptors.ptr<uint8_t>(j)));
      F0.mvpMapLines[j] = mls.back().get();
      ml_index[mls.back().get()] = j;
    }
    // the initial keyframe (Tracking.cc:637-640: KeyFrame + ComputeBoW)
    KeyFrame KF0(F0);
    KF0.ComputeBoW();

    // ---- frame 1: TrackWithMotionModel with zero velocity (Tracking.cc:1228-1271)
    F1.SetPose(F0.mTcw);
    ORBmatcher matcher(0.9f, true);
    LineMatcher line_matcher(0.9f, true);
    int nmatches = matcher.SearchByProjection(F1, F0, 15, false);
    const int line_nmatches = line_matcher.SearchByProjection(F1, F0);
    if (nmatches < 20) {
      std::fill(F1.mvpMapPoints.begin(), F1.mvpMapPoints.end(), nullptr);
      nmatches = matcher.SearchByProjection(F1, F0, 30, false);
    }
    int ninl = 0;
    if (nmatches >= 20 && line_nmatches >= 15) ninl = Optimizer::PoseOptimizationWithLines(&F1);

    FILE* o = fopen(argv[2], "wb");
    if (!o) throw std::runtime_error("cannot open output");
    write_frame(o, F0);
    write_frame(o, F1);
    const int nlev = (int)pyr.size();
    wr(o, &nlev, 1);
    for (const cv::Mat& m : pyr) {
      wr(o, &m.cols, 1);
      wr(o, &m.rows, 1);
      wr(o, m.data, (size_t)m.cols * m.rows);
    }
    wr(o, &nmatches, 1);
    wr(o, &line_nmatches, 1);
    wr(o, &ninl, 1);
    wr(o, F1.mTcw.ptr<float>(), 16);
    write_index(o, F1.mvpMapPoints, mp_index);
    for (int i = 0; i < F1.N; i++) wr1<uint8_t>(o, F1.mvbOutlier[i]);
    write_index(o, F1.mvpMapLines, ml_index);
    for (int j = 0; j < F1.NL; j++) wr1<uint8_t>(o, F1.mvbLineOutlier[j]);

    // ---- the map of frame 0 and the FeatureVectors
    for (int i = 0; i < F0.N; i++) {
      const MapPoint* p = F0.mvpMapPoints[i];
      wr1<uint8_t>(o, p != nullptr);
      float v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      if (p) {
        const cv::Mat X = p->GetWorldPos(), Nv = p->GetNormal();
        for (int k = 0; k < 3; k++) {
          v[k] = X.at<float>(k, 0);
          v[3 + k] = Nv.at<float>(k, 0);
        }
        v[6] = p->GetMinDistance();   // raw mfMinDistance / mfMaxDistance
        v[7] = p->GetMaxDistance();
      }
      wr(o, v, 8);
    }
    for (int j = 0; j < F0.NL; j++) {
      const MapLine* l = F0.mvpMapLines[j];
      wr1<uint8_t>(o, l != nullptr);
      float v[6] = {0, 0, 0, 0, 0, 0};
      if (l)
        for (int k = 0; k < 3; k++) {
          v[k] = (float)l->mStart3d[k];
          v[3 + k] = (float)l->mEnd3d[k];
        }
      wr(o, v, 6);
    }

    // ---- frame 2: TrackReferenceKeyFrame against KF0 (Tracking.cc:942-1032)
    Frame F2(g[2], d[2], 2.0, &ex, &voc, K, dist, bf, thDepth);
    F2.ComputeBoW();
    const std::vector<int32_t> n0 = node_of(KF0.mFeatVec, KF0.N), n2 = node_of(F2.mFeatVec, F2.N);
    wr(o, n0.data(), n0.size());
    write_frame(o, F2);
    wr(o, n2.data(), n2.size());
    ORBmatcher matcher7(0.7f, true);
    LineMatcher line_matcher7(0.7f, true);
    std::vector<MapPoint*> vpMapPointMatches;
    int nm2 = matcher7.SearchByBoW(&KF0, F2, vpMapPointMatches);
    F2.SetPose(F1.mTcw);
    const int nlm2 = line_matcher7.SearchByProjection(F2, &KF0);
    wr(o, &nm2, 1);
    write_index(o, vpMapPointMatches, mp_index);
    wr(o, &nlm2, 1);
    write_index(o, F2.mvpMapLines, ml_index);
    const int go = nm2 >= 15 && nlm2 >= 10;
    int ninl2 = 0, nmatchesMap = 0, line_nmatchesMap = 0;
    if (go) {
      F2.mvpMapPoints = vpMapPointMatches;
      ninl2 = Optimizer::PoseOptimizationWithLines(&F2);
    }
    wr(o, &go, 1);
    wr(o, &ninl2, 1);
    wr(o, F2.mTcw.ptr<float>(), 16);
    for (int i = 0; i < F2.N; i++) wr1<uint8_t>(o, F2.mvbOutlier[i]);
    for (int j = 0; j < F2.NL; j++) wr1<uint8_t>(o, F2.mvbLineOutlier[j]);
    if (go) {
      // the discard (Tracking.cc:999-1029)
      for (int i = 0; i < F2.N; i++) {
        if (!F2.mvpMapPoints[i]) continue;
        if (F2.mvbOutlier[i]) {
          MapPoint* p = F2.mvpMapPoints[i];
          F2.mvpMapPoints[i] = nullptr;
          F2.mvbOutlier[i] = false;
          p->mbTrackInView = false;
          p->mnLastFrameSeen = F2.mnId;
        } else if (F2.mvpMapPoints[i]->Observations() > 0) {
          nmatchesMap++;
        }
      }
      for (int j = 0; j < F2.NL; j++) {
        if (!F2.mvpMapLines[j]) continue;
        if (F2.mvbLineOutlier[j]) {
          MapLine* l = F2.mvpMapLines[j];
          F2.mvpMapLines[j] = nullptr;
          F2.mvbLineOutlier[j] = false;
          l->mbTrackInView = false;
          l->mnLastFrameSeen = F2.mnId;
          line_nmatchesMap--;
        } else if (F2.mvpMapLines[j]->Observations() > 0) {
          line_nmatchesMap++;
        }
      }
    }
    wr(o, &nmatchesMap, 1);
    wr(o, &line_nmatchesMap, 1);

    // ---- TrackLocalMap with KF0 as the local map (Tracking.cc:1746-1865)
    std::vector<MapPoint*> local_points;   // UpdateLocalPoints: KF0's, index order
    for (MapPoint* p : KF0.GetMapPointMatches())
      if (p) local_points.push_back(p);
    std::vector<MapLine*> local_lines;
    for (MapLine* l : KF0.mvpMapLines)
      if (l) local_lines.push_back(l);
    // SearchLocalPoints
    for (MapPoint* p : F2.mvpMapPoints)
      if (p) {
        p->mnLastFrameSeen = F2.mnId;
        p->mbTrackInView = false;
      }
    std::vector<uint8_t> seen(F0.N, 0), inview(F0.N, 0);
    int nToMatch = 0;
    for (MapPoint* p : local_points) {
      const int i = mp_index.at(p);
      if (p->mnLastFrameSeen == F2.mnId) {
        seen[i] = 1;
        continue;
      }
      if (p->isBad()) continue;
      if (F2.IsInFrustum(p, 0.5f)) {
        inview[i] = 1;
        nToMatch++;
      }
    }
    int nlocal = 0;
    if (nToMatch > 0) nlocal = ORBmatcher(0.8f).SearchByProjection(F2, local_points, 3);
    wr(o, seen.data(), seen.size());
    wr(o, inview.data(), inview.size());
    wr(o, &nlocal, 1);
    write_index(o, F2.mvpMapPoints, mp_index);
    // SearchLocalLines
    for (MapLine* l : F2.mvpMapLines)
      if (l) {
        l->mnLastFrameSeen = F2.mnId;
        l->mbTrackInView = false;
      }
    std::vector<uint8_t> lseen(F0.NL, 0), linview(F0.NL, 0);
    int nlToMatch = 0;
    for (MapLine* l : local_lines) {
      const int j = ml_index.at(l);
      if (l->mnLastFrameSeen == F2.mnId) {
        lseen[j] = 1;
        continue;
      }
      if (l->isBad()) continue;
      if (F2.IsInFrustum(l, 0.5f)) {
        linview[j] = 1;
        nlToMatch++;
      }
    }
    int nllocal = 0;
    if (nlToMatch > 0) nllocal = LineMatcher(0.8f).SearchByProjection(F2, local_lines);
    wr(o, lseen.data(), lseen.size());
    wr(o, linview.data(), linview.size());
    wr(o, &nllocal, 1);
    write_index(o, F2.mvpMapLines, ml_index);
    const int ninl3 = Optimizer::PoseOptimizationWithLines(&F2);
    wr(o, &ninl3, 1);
    wr(o, F2.mTcw.ptr<float>(), 16);
    fclose(o);
    printf("dropin: N0 %d NL0 %d N1 %d NL1 %d matches %d line matches %d inliers %d | "
           "TRK bow %d lines %d inliers %d | local %d lines %d inliers %d\n",
           F0.N, F0.NL, F1.N, F1.NL, nmatches, line_nmatches, ninl, nm2, nlm2, ninl2, nlocal,
           nllocal, ninl3);
  } catch (const std::exception& e) {
    fprintf(stderr, "dropin_driver: %s\n", e.what());
    return 1;
  }
  return 0;
}
