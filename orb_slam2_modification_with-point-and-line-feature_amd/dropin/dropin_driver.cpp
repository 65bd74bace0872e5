// Exercises the drop-in classes the way Tracking uses them for the first two
// RGB-D frames (StereoInitialization-style map from frame 0, then
// TrackWithMotionModel's matching and pose for frame 1, Tracking.cc:608-690,
// 1212-1271), and writes every output for tests/test_gpu_dropin.py to check
// against the oracle.
//   dropin_driver <in.bin> <out.bin>
// in.bin : int32 W, H; float fx fy cx cy k1 k2 p1 p2 k3 bf thdepth;
//          int32 nfeatures; float scale; int32 nlevels, iniTh, minTh;
//          float Tcw0[16]; gray0 (W*H u8), depth0 (W*H f32), gray1, depth1
// out.bin: per frame: N, kps (N x 28 B), desc (N x 32), NL, keylines (NL x
//          68 B), line desc (NL x 32), coef (NL x 3 f64), keysUn (N x 28 B),
//          depth (N f32); frame 0's pyramid: nlevels x (w, h, w*h bytes);
//          then nmatches, line matches, inliers, Tcw1[16], match[N1] (frame-0
//          index or -1), outlier[N1] u8, line match[NL1], line outlier[NL1] u8
#include <cstdio>
#include <map>
#include <memory>
#include <vector>

#include "Frame.h"
#include "LineMatcher.h"
#include "ORBmatcher.h"
#include "Optimizer.h"

using namespace ORB_SLAM2;

template <class T>
static void rd(FILE* f, T* p, size_t n) {
  if (fread(p, sizeof(T), n, f) != n) throw std::runtime_error("short input");
}
template <class T>
static void wr(FILE* f, const T* p, size_t n) {
  if (n && fwrite(p, sizeof(T), n, f) != n) throw std::runtime_error("short write");
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

int main(int argc, char** argv) {
  if (argc != 3) {
    fprintf(stderr, "usage: dropin_driver in.bin out.bin\n");
    return 2;
  }
  try {
    FILE* in = fopen(argv[1], "rb");
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
    cv::Mat g0(H, W, cv::CV_8U), d0(H, W, cv::CV_32F), g1(H, W, cv::CV_8U), d1(H, W, cv::CV_32F);
    rd(in, g0.data, (size_t)W * H);
    rd(in, d0.ptr<float>(), (size_t)W * H);
    rd(in, g1.data, (size_t)W * H);
    rd(in, d1.ptr<float>(), (size_t)W * H);
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
    Frame F0(g0, d0, 0.0, &ex, nullptr, K, dist, bf, thDepth);
    std::vector<cv::Mat> pyr = ex.mvImagePyramid;
    Frame F1(g1, d1, 1.0, &ex, nullptr, K, dist, bf, thDepth);

    // frame 0: pose Tcw0, map points / lines from depth (Tracking.cc:633-692)
    cv::Mat T0(4, 4, cv::CV_32F);
    std::memcpy(T0.data, Tcw0, 64);
    F0.SetPose(T0);
    std::vector<std::unique_ptr<MapPoint>> mps;
    std::vector<std::unique_ptr<MapLine>> mls;
    std::map<const MapPoint*, int> mp_index;
    std::map<const MapLine*, int> ml_index;
    for (int i = 0; i < F0.N; i++) {
      if (!(F0.mvDepth[i] > 0)) continue;
      cv::Mat X = F0.UnprojectStereo(i);
      mps.emplace_back(new MapPoint(X.ptr<float>(), F0.mDescriptors.ptr<uint8_t>(i)));
      F0.mvpMapPoints[i] = mps.back().get();
      mp_index[mps.back().get()] = i;
    }
    for (int j = 0; j < F0.NL; j++) {
      if (!(F0.mvDepthLineStart[j] > 0 && F0.mvDepthLineEnd[j] > 0)) continue;
      cv::Mat s = F0.UnprojectStereoLineStart(j), e = F0.UnprojectStereoLineEnd(j);
      const float xyz6[6] = {s.at<float>(0, 0), s.at<float>(1, 0), s.at<float>(2, 0),
                             e.at<float>(0, 0), e.at<float>(1, 0), e.at<float>(2, 0)};
      mls.emplace_back(new MapLine(xyz6, F0.mLineDescriptors.ptr<uint8_t>(j)));
      F0.mvpMapLines[j] = mls.back().get();
      ml_index[mls.back().get()] = j;
    }

    // frame 1: TrackWithMotionModel with zero velocity (Tracking.cc:1228-1271)
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
    for (int i = 0; i < F1.N; i++) {
      const int m = F1.mvpMapPoints[i] ? mp_index[F1.mvpMapPoints[i]] : -1;
      wr(o, &m, 1);
    }
    for (int i = 0; i < F1.N; i++) {
      const uint8_t b = F1.mvbOutlier[i];
      wr(o, &b, 1);
    }
    for (int j = 0; j < F1.NL; j++) {
      const int m = F1.mvpMapLines[j] ? ml_index[F1.mvpMapLines[j]] : -1;
      wr(o, &m, 1);
    }
    for (int j = 0; j < F1.NL; j++) {
      const uint8_t b = F1.mvbLineOutlier[j];
      wr(o, &b, 1);
    }
    fclose(o);
    printf("dropin: N0 %d NL0 %d N1 %d NL1 %d matches %d line matches %d inliers %d\n", F0.N,
           F0.NL, F1.N, F1.NL, nmatches, line_nmatches, ninl);
  } catch (const std::exception& e) {
    fprintf(stderr, "dropin_driver: %s\n", e.what());
    return 1;
  }
  return 0;
}
