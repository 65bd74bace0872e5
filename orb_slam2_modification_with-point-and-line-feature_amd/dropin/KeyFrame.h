// Minimal ORB_SLAM2::KeyFrame stand-in (include/KeyFrame.h, src/KeyFrame.cc:
// 36-80): the members TrackReferenceKeyFrame's matchers read from the
// reference keyframe - its undistorted keypoints, descriptors, map point
// matches and FeatureVector (ORBmatcher::SearchByBoW, ORBmatcher.cc:247-410),
// its key lines, line descriptors and map lines (LineMatcher::
// SearchByProjection(Frame&, KeyFrame*), LineMatcher.cpp:527-721) - copied
// from the Frame it is made of, as KeyFrame::KeyFrame(Frame&, ...) does. The
// covisibility graph, spanning tree and map bookkeeping stay the caller's.
#pragma once
#include <stdexcept>
#include <vector>

#include "Frame.h"

namespace ORB_SLAM2 {

class KeyFrame {
 public:
  explicit KeyFrame(const Frame& F)
      : mnFrameId(F.mnId), N(F.N), NL(F.NL), mvKeys(F.mvKeys), mvKeysUn(F.mvKeysUn),
        mvuRight(F.mvuRight), mvDepth(F.mvDepth), mDescriptors(F.mDescriptors.clone()),
        mBowVec(F.mBowVec), mFeatVec(F.mFeatVec), mvKeyLines(F.mvKeyLines),
        mvKeyLinesUn(F.mvKeyLinesUn), mLineDescriptors(F.mLineDescriptors.clone()),
        mvpMapLines(F.mvpMapLines), mvScaleFactors(F.mvScaleFactors),
        mpORBvocabulary(F.mpORBvocabulary), mvpMapPoints(F.mvpMapPoints),
        Tcw(F.mTcw.clone()) {
    mnId = nNextId++;
  }

  // KeyFrame::ComputeBoW (KeyFrame.cc:67-80)
  void ComputeBoW() {
    if (!mpORBvocabulary) throw std::runtime_error("KeyFrame::ComputeBoW: no vocabulary");
    if (mBowVec.empty() || mFeatVec.empty())
      mpORBvocabulary->transform(toDescriptorVector(mDescriptors), mBowVec, mFeatVec, 4);
  }
  std::vector<MapPoint*> GetMapPointMatches() const { return mvpMapPoints; }
  std::vector<MapLine*> GetMapLineMatches() const { return mvpMapLines; }
  MapPoint* GetMapPoint(const size_t& idx) const { return mvpMapPoints[idx]; }
  cv::Mat GetPose() const { return Tcw.clone(); }

  static long unsigned int nNextId;
  long unsigned int mnId = 0;
  const long unsigned int mnFrameId;
  const int N, NL;
  const std::vector<cv::KeyPoint> mvKeys, mvKeysUn;
  const std::vector<float> mvuRight, mvDepth;
  const cv::Mat mDescriptors;
  DBoW2::BowVector mBowVec;
  DBoW2::FeatureVector mFeatVec;
  const std::vector<KeyLine> mvKeyLines, mvKeyLinesUn;
  const cv::Mat mLineDescriptors;
  std::vector<MapLine*> mvpMapLines;   // public in the fork (LineMatcher.cpp:561)
  const std::vector<float> mvScaleFactors;
  ORBVocabulary* mpORBvocabulary;

 private:
  std::vector<MapPoint*> mvpMapPoints;
  cv::Mat Tcw;
};

}  // namespace ORB_SLAM2
