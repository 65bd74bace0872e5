// Drop-in ORB_SLAM2::LineMatcher (include/LineMatcher.h:36-66): the tracking
// overloads - last frame (LineMatcher.cpp:72-269, orbl_search_by_projection_last),
// reference keyframe (:527-721) and local map lines (:755-952), both over
// orbl_search_by_projection_list - and the harness overloads the reference's
// Test/ demos call: the new_kls / match_indices variants of the last-frame
// (:272-487) and local-map (:954-1170) searches (orbl_search_by_projection_pairs)
// and the BFMatcher reference-keyframe variant (:492-525, orbl_match_bf_knn).
#pragma once
#include <utility>
#include <vector>

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

  // harness overloads (LineMatcher.h:51, 56, 66): new_kls gets the projected,
  // clipped KeyLines appended; match_indices every passing (new_kls index,
  // current line index) pair of the final pass
  int SearchByProjection(Frame& CurrentFrame, const Frame& LastFrame, std::vector<KeyLine>& new_kls,
                         std::vector<std::pair<int, int>>& match_indices);
  int SearchByProjection(Frame& CurrentFrame, KeyFrame* RefFrame,
                         std::vector<MapLine*>& vpMapLineMatches);
  int SearchByProjection(Frame& F, const std::vector<MapLine*>& vpMapLines,
                         std::vector<KeyLine>& new_kls,
                         std::vector<std::pair<int, int>>& match_indices);
  // (LineMatcher.h:59 declares SearchByProjection(Frame&, KeyFrame*, new_kls,
  // match_indices), which the reference never defines: not provided)

  float mfNNratio;
  bool mbCheckOrientation;
};

}  // namespace ORB_SLAM2
