// Drop-in ORB_SLAM2::LineMatcher, last-frame overload (include/LineMatcher.h:36-52,
// src/LineMatcher.cpp:72-269) over orbl_search_by_projection_last.
#pragma once
#include "Frame.h"

namespace ORB_SLAM2 {

class LineMatcher {
 public:
  LineMatcher(float nnratio = 0.6, bool checkOri = true)
      : mfNNratio(nnratio), mbCheckOrientation(checkOri) {}
  static int DescriptorDistance(const cv::Mat& a, const cv::Mat& b);
  int SearchByProjection(Frame& CurrentFrame, const Frame& LastFrame);

  float mfNNratio;
  bool mbCheckOrientation;
};

}  // namespace ORB_SLAM2
