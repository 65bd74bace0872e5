// Drop-in ORB_SLAM2::ORBmatcher, per-frame overloads (include/ORBmatcher.h:49-90,
// src/ORBmatcher.cc:72-183, 1710-1879, 2083-2103) over orbm_*.
#pragma once
#include <vector>

#include "Frame.h"

namespace ORB_SLAM2 {

class ORBmatcher {
 public:
  ORBmatcher(float nnratio = 0.6, bool checkOri = true)
      : mfNNratio(nnratio), mbCheckOrientation(checkOri) {}

  static int DescriptorDistance(const cv::Mat& a, const cv::Mat& b);

  // Tracking::TrackWithMotionModel (Tracking.cc:1244, 1258)
  int SearchByProjection(Frame& CurrentFrame, const Frame& LastFrame, const float th,
                         const bool bMono);

  // Tracking::SearchLocalPoints (Tracking.cc:1812): the map points'
  // IsInFrustum outputs are computed here from their world positions, normals
  // and distance invariances (given per point by the caller's map)
  struct LocalPoint {
    MapPoint* mp;
    float normal[3];
    float min_dist, max_dist;   // GetMinDistanceInvariance / GetMaxDistanceInvariance
  };
  int SearchByProjection(Frame& F, const std::vector<LocalPoint>& vpMapPoints, const float th = 3);

  float mfNNratio;
  bool mbCheckOrientation;
};

}  // namespace ORB_SLAM2
