// The parts of ORB_SLAM2::MapPoint / MapLine the per-frame hot path reads
// (world position, descriptor, observation count; MapPoint.h, MapLine.h).
// The map itself (observations per keyframe, normals, culling) belongs to the
// caller's Tracking / LocalMapping and is outside the drop-in.
#pragma once
#include "cvmini.h"

namespace ORB_SLAM2 {

class MapPoint {
 public:
  MapPoint(const float xyz[3], const uint8_t desc32[32], int nobs = 1) : mnObs(nobs) {
    mWorldPos.create(3, 1, cv::CV_32F);
    for (int k = 0; k < 3; k++) mWorldPos.at<float>(k, 0) = xyz[k];
    mDescriptor.create(1, 32, cv::CV_8U);
    std::memcpy(mDescriptor.data, desc32, 32);
  }
  cv::Mat GetWorldPos() const { return mWorldPos.clone(); }
  cv::Mat GetDescriptor() const { return mDescriptor.clone(); }
  int Observations() const { return mnObs; }

  bool mbTrackInView = false;
  long unsigned int mnLastFrameSeen = 0;

 private:
  cv::Mat mWorldPos, mDescriptor;
  int mnObs;
};

class MapLine {
 public:
  MapLine(const float xyz6[6], const uint8_t desc32[32], int nobs = 1) : mnObs(nobs) {
    for (int k = 0; k < 3; k++) {
      mStart[k] = xyz6[k];
      mEnd[k] = xyz6[3 + k];
    }
    mDescriptor.create(1, 32, cv::CV_8U);
    std::memcpy(mDescriptor.data, desc32, 32);
  }
  Eigen::Vector3d GetWorldStartPos() const { return mStart; }
  Eigen::Vector3d GetWorldEndPos() const { return mEnd; }
  cv::Mat GetDescriptor() const { return mDescriptor.clone(); }
  int Observations() const { return mnObs; }

  bool mbTrackInView = false;
  long unsigned int mnLastFrameSeen = 0;

 private:
  Eigen::Vector3d mStart, mEnd;
  cv::Mat mDescriptor;
  int mnObs;
};

}  // namespace ORB_SLAM2
