// Drop-in ORB_SLAM2::Frame, RGB-D constructor (include/Frame.h,
// src/Frame.cc:135-205): ORB and LineExtractor on two host threads
// (Frame.cc:152-155), then the frame glue (undistortion, RGB-D depths, grid)
// on the MI355X through orbpl_frame_prepare / orbpl_line_frame_prepare.
#pragma once
#include <cstddef>
#include <vector>

#include "LineExtractor.h"
#include "MapPoint.h"
#include "ORBVocabulary.h"
#include "ORBextractor.h"

namespace ORB_SLAM2 {

#define FRAME_GRID_ROWS 48
#define FRAME_GRID_COLS 64

class Frame {
 public:
  Frame() = default;
  Frame(const Frame&) = default;
  // RGB-D (Frame.cc:135-205); voc is kept for ComputeBoW (may be NULL when
  // the caller never computes a BoW)
  Frame(const cv::Mat& imGray, const cv::Mat& imDepth, const double& timeStamp,
        ORBextractor* extractor, ORBVocabulary* voc, cv::Mat& K, cv::Mat& distCoef,
        const float& bf, const float& thDepth, LineExtractor* lineExtractor = nullptr);

  // Frame::ComputeBoW (Frame.cc:721-735): mBowVec / mFeatVec at levelsup 4
  void ComputeBoW();
  // Frame::IsInFrustum (Frame.cc:345-401, 403-430): the map point's / line's
  // mbTrackInView and (points) mTrackProjX / Y / XR, mnTrackScaleLevel,
  // mTrackViewCos, through orbpl_frame_is_in_frustum / orbl_frame_is_in_frustum
  bool IsInFrustum(MapPoint* pMP, float viewingCosLimit);
  bool IsInFrustum(MapLine* pML, float viewingCosLimit);
  // Extension: the same for a whole local map in one call (Tracking::
  // SearchLocalPoints' loop, Tracking.cc:1780-1795, without a device round
  // trip per point); in_view[i] per point, returns the number in view
  int IsInFrustumBatch(const std::vector<MapPoint*>& vpMapPoints, float viewingCosLimit,
                       std::vector<uint8_t>* in_view = nullptr);

  void SetPose(cv::Mat Tcw);
  void UpdatePoseMatrices();
  cv::Mat GetCameraCenter() { return mOw.clone(); }
  cv::Mat GetRotationInverse() { return mRwc.clone(); }
  // Frame.cc:1119-1139, 1169-1199 (UnprojectStereoLineEnd uses the start
  // depth, Frame.cc:1192, replicated)
  cv::Mat UnprojectStereo(const int& i);
  cv::Mat UnprojectStereoLineStart(const int& i);
  cv::Mat UnprojectStereoLineEnd(const int& i);

  // the camera as the C ABI takes it
  orbpl_camera Camera() const;

  double mTimeStamp = 0;
  cv::Mat mK, mDistCoef;
  static float fx, fy, cx, cy, invfx, invfy;
  float mbf = 0, mb = 0, mThDepth = 0;
  int N = 0, NL = 0;
  int mnWidth = 0, mnHeight = 0;
  std::vector<cv::KeyPoint> mvKeys, mvKeysUn;
  std::vector<float> mvuRight, mvDepth;
  cv::Mat mDescriptors;
  ORBVocabulary* mpORBvocabulary = nullptr;
  DBoW2::BowVector mBowVec;
  DBoW2::FeatureVector mFeatVec;
  std::vector<MapPoint*> mvpMapPoints;
  std::vector<bool> mvbOutlier;
  std::vector<KeyLine> mvKeyLines, mvKeyLinesUn;
  std::vector<float> mvuRightLineStart, mvuRightLineEnd, mvDepthLineStart, mvDepthLineEnd;
  cv::Mat mLineDescriptors;
  std::vector<Eigen::Vector3d> mvKeyLineCoefficient;
  std::vector<MapLine*> mvpMapLines;
  std::vector<bool> mvbLineOutlier;
  std::vector<std::size_t> mGrid[FRAME_GRID_COLS][FRAME_GRID_ROWS];
  cv::Mat mTcw;
  static long unsigned int nNextId;
  long unsigned int mnId = 0;
  int mnScaleLevels = 0;
  float mfScaleFactor = 0;
  std::vector<float> mvScaleFactors, mvInvScaleFactors, mvLevelSigma2, mvInvLevelSigma2;
  static float mnMinX, mnMaxX, mnMinY, mnMaxY;
  cv::Mat mRcw, mtcw, mRwc, mOw;
};

}  // namespace ORB_SLAM2
