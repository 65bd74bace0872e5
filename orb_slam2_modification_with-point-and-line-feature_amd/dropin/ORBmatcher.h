// Drop-in ORB_SLAM2::ORBmatcher, the tracking overloads (include/ORBmatcher.h:
// 49-140, src/ORBmatcher.cc:72-183, 247-410, 1710-1879, 2083-2103) over orbm_*.
#pragma once
#include <vector>

#include "Frame.h"
#include "KeyFrame.h"

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
  // mbTrackInView / mTrackProj* / mnTrackScaleLevel / mTrackViewCos, as
  // Frame::IsInFrustum left them (ORBmatcher.h:74, ORBmatcher.cc:72-183)
  int SearchByProjection(Frame& F, const std::vector<MapPoint*>& vpMapPoints, const float th = 3);

  // Tracking::TrackReferenceKeyFrame (Tracking.cc:958): the keyframe's and the
  // frame's FeatureVectors (ComputeBoW first), ORBmatcher.h:140,
  // ORBmatcher.cc:247-410
  int SearchByBoW(KeyFrame* pKF, Frame& F, std::vector<MapPoint*>& vpMapPointMatches);

  float mfNNratio;
  bool mbCheckOrientation;
};

}  // namespace ORB_SLAM2
