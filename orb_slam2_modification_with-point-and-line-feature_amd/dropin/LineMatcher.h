// Drop-in ORB_SLAM2::LineMatcher, the tracking overloads (include/LineMatcher.h:
// 36-64): last frame (LineMatcher.cpp:72-269, orbl_search_by_projection_last),
// reference keyframe (:527-721) and local map lines (:755-952), both over
// orbl_search_by_projection_list.
#pragma once
#include "Frame.h"
#include "KeyFrame.h"

namespace ORB_SLAM2 {

class LineMatcher {
 public:
  LineMatcher(float nnratio = 0.6, bool checkOri = true)
      : mfNNratio(nnratio), mbCheckOrientation(checkOri) {}
  static int DescriptorDistance(const cv::Mat& a, const cv::Mat& b);
  int SearchByProjection(Frame& CurrentFrame, const Frame& LastFrame);
  // Tracking::TrackReferenceKeyFrame (Tracking.cc:966): RefFrame->mvpMapLines
  int SearchByProjection(Frame& CurrentFrame, KeyFrame* RefFrame);
  // Tracking::SearchLocalLines (Tracking.cc:1863): lines with mbTrackInView
  int SearchByProjection(Frame& F, const std::vector<MapLine*>& vpMapLines);

  float mfNNratio;
  bool mbCheckOrientation;
};

}  // namespace ORB_SLAM2
