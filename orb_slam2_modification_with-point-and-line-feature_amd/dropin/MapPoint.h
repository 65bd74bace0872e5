// The parts of ORB_SLAM2::MapPoint / MapLine the per-frame hot path reads and
// writes (MapPoint.h:96-167, MapLine.h:87-212): world position, descriptor,
// observation count, the viewing normal and scale-invariance distances
// Frame::IsInFrustum reads, and the mTrack* fields IsInFrustum writes and
// ORBmatcher / LineMatcher::SearchByProjection read. The map itself
// (observations per keyframe, UpdateNormalAndDepth, culling) belongs to the
// caller's Tracking / LocalMapping and is outside the drop-in: the caller sets
// the normal and distances (SetNormalAndDistances) and the observation count.
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
    mNormalVector.create(3, 1, cv::CV_32F);
  }
  cv::Mat GetWorldPos() const { return mWorldPos.clone(); }
  cv::Mat GetDescriptor() const { return mDescriptor.clone(); }
  cv::Mat GetNormal() const { return mNormalVector.clone(); }
  int Observations() const { return mnObs; }
  bool isBad() const { return mbBad; }
  void SetBadFlag() { mbBad = true; }
  void SetObservations(int n) { mnObs = n; }
  // MapPoint::UpdateNormalAndDepth's results (MapPoint.cc:360-411)
  void SetNormalAndDistances(const float normal[3], float minDistance, float maxDistance) {
    for (int k = 0; k < 3; k++) mNormalVector.at<float>(k, 0) = normal[k];
    mfMinDistance = minDistance;
    mfMaxDistance = maxDistance;
  }
  // MapPoint.cc:413-423
  float GetMinDistanceInvariance() const { return 0.8f * mfMinDistance; }
  float GetMaxDistanceInvariance() const { return 1.2f * mfMaxDistance; }
  // the raw distances: Frame::IsInFrustum hands these to the library, which
  // applies the 0.8f / 1.2f above and PredictScale's mfMaxDistance / dist
  float GetMinDistance() const { return mfMinDistance; }
  float GetMaxDistance() const { return mfMaxDistance; }

  // Tracking variables (MapPoint.h:155-175), written by Frame::IsInFrustum
  float mTrackProjX = 0, mTrackProjY = 0, mTrackProjXR = 0;
  bool mbTrackInView = false;
  int mnTrackScaleLevel = 0;
  float mTrackViewCos = 0;
  long unsigned int mnTrackReferenceForFrame = 0;
  long unsigned int mnLastFrameSeen = 0;

 private:
  cv::Mat mWorldPos, mDescriptor, mNormalVector;
  float mfMinDistance = 0, mfMaxDistance = 0;
  int mnObs;
  bool mbBad = false;
};

class MapLine {
 public:
  MapLine(const float xyz6[6], const uint8_t desc32[32], int nobs = 1) : mnObs(nobs) {
    for (int k = 0; k < 3; k++) {
      mStart3d[k] = xyz6[k];
      mEnd3d[k] = xyz6[3 + k];
    }
    mLineDescriptor.create(1, 32, cv::CV_8U);
    std::memcpy(mLineDescriptor.data, desc32, 32);
  }
  Eigen::Vector3d GetWorldStartPos() const { return mStart3d; }
  Eigen::Vector3d GetWorldEndPos() const { return mEnd3d; }
  cv::Mat GetDescriptor() const { return mLineDescriptor.clone(); }
  int Observations() const { return mnObs; }
  bool isBad() const { return mbBad; }
  void SetBadFlag() { mbBad = true; }
  void SetObservations(int n) { mnObs = n; }

  // MapLine.h:164-172: written by Frame::IsInFrustum(MapLine*) / Tracking
  bool mbTrackInView = false;
  long unsigned int mnLastFrameSeen = 0;
  // the reference's LineMatcher reads these members directly
  // (LineMatcher.cpp:566-567, 607)
  Eigen::Vector3d mStart3d, mEnd3d;
  cv::Mat mLineDescriptor;

 private:
  int mnObs;
  bool mbBad = false;
};

}  // namespace ORB_SLAM2
