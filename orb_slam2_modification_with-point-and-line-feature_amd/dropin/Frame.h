// Drop-in ORB_SLAM2::Frame (include/Frame.h). RGB-D constructor
// (src/Frame.cc:135-205): ORB and LineExtractor on two host threads
// (Frame.cc:152-155), then the frame glue (undistortion, RGB-D depths, grid)
// on the MI355X through orbpl_frame_prepare / orbpl_line_frame_prepare.
// Stereo constructor (Frame.cc:71-132): ORB on the left and right images on
// two host threads (Frame.cc:88-91), the glue, ComputeStereoMatches on the two
// extractors' device pyramids (orbpl_stereo_matches, Frame.cc:888-1062).
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

  // Stereo (Frame.cc:71-132). The reference's stereo Frame extracts no lines
  // and leaves NL uninitialised: here NL = 0 and the
  // line containers are empty. Like the reference, a left image without
  // keypoints returns right after the extraction (N = 0, nothing else set).
  Frame(const cv::Mat& imLeft, const cv::Mat& imRight, const double& timeStamp,
        ORBextractor* extractorLeft, ORBextractor* extractorRight, ORBVocabulary* voc,
        cv::Mat& K, cv::Mat& distCoef, const float& bf, const float& thDepth);

  // Frame::ComputeStereoMatches (Frame.cc:888-1062): mvuRight / mvDepth of
  // every left keypoint from the right keypoints (row bands, Hamming, SAD
  // window refinement, parabola, median-distance cut), on the device
  // pyramids the last extraction of mpORBextractorLeft / Right left there
  void ComputeStereoMatches();
  // Frame::GetFeaturesInArea (Frame.cc:432-485): keypoint indices in the
  // square of half side r around (x, y), grid cells in column-major order,
  // octave window [minLevel, maxLevel] when either is set
  std::vector<size_t> GetFeaturesInArea(const float& x, const float& y, const float& r,
                                        const int minLevel = -1, const int maxLevel = -1) const;

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
  ORBextractor* mpORBextractorLeft = nullptr;
  ORBextractor* mpORBextractorRight = nullptr;   // stereo only
  std::vector<cv::KeyPoint> mvKeys, mvKeysUn, mvKeysRight;
  std::vector<float> mvuRight, mvDepth;
  cv::Mat mDescriptors, mDescriptorsRight;
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
  static float mfGridElementWidthInv, mfGridElementHeightInv;
  cv::Mat mRcw, mtcw, mRwc, mOw;

 private:
  void ScaleInfo(ORBextractor* ex);
  // UndistortKeyPoints + (RGB-D: imDepth, stereo: NULL) ComputeStereoFromRGBD +
  // ComputeImageBounds + AssignFeaturesToGrid through orbpl_frame_prepare
  void PrepareKeys(const float* depth);
};

}  // namespace ORB_SLAM2
