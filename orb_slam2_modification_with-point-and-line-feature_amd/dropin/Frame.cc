// Drop-in ORB_SLAM2::Frame (see Frame.h).
#include "Frame.h"

#include "KeyFrame.h"

#include <algorithm>
#include <cmath>
#include <stdexcept>
#include <thread>

namespace ORB_SLAM2 {

float Frame::fx, Frame::fy, Frame::cx, Frame::cy, Frame::invfx, Frame::invfy;
float Frame::mnMinX, Frame::mnMaxX, Frame::mnMinY, Frame::mnMaxY;
float Frame::mfGridElementWidthInv, Frame::mfGridElementHeightInv;
long unsigned int Frame::nNextId = 0;
long unsigned int KeyFrame::nNextId = 0;

static void check(int rc) {
  if (rc != ORBPL_OK) throw std::runtime_error(orbpl_last_error());
}

orbpl_camera Frame::Camera() const {
  const float* d = mDistCoef.ptr<float>();
  const int nd = mDistCoef.rows * mDistCoef.cols;
  return orbpl_camera{fx, fy, cx, cy, d[0], d[1], d[2], d[3], nd > 4 ? d[4] : 0.0f, mbf,
                      mThDepth, mnWidth, mnHeight};
}

// Frame.cc:78-85 / 141-148: the scale level info of the (left) extractor
void Frame::ScaleInfo(ORBextractor* ex) {
  mnScaleLevels = ex->GetLevels();
  mfScaleFactor = ex->GetScaleFactor();
  mvScaleFactors = ex->GetScaleFactors();
  mvInvScaleFactors = ex->GetInverseScaleFactors();
  mvLevelSigma2 = ex->GetScaleSigmaSquares();
  mvInvLevelSigma2 = ex->GetInverseScaleSigmaSquares();
}

// UndistortKeyPoints, ComputeStereoFromRGBD (depth != NULL; stereo: NULL, the
// stereo matcher fills mvuRight / mvDepth after), ComputeImageBounds and
// AssignFeaturesToGrid (Frame.cc:98-131, 160-204) in one library call
void Frame::PrepareKeys(const float* depth) {
  const orbpl_camera cam = Camera();
  mvKeysUn.resize(N);
  mvDepth.resize(N);
  mvuRight.resize(N);
  std::vector<int32_t> cell(N);
  float bounds[4];
  check(orbpl_frame_prepare(&cam, reinterpret_cast<const orbpl_keypoint*>(mvKeys.data()), N, depth,
                            reinterpret_cast<orbpl_keypoint*>(mvKeysUn.data()), mvDepth.data(),
                            mvuRight.data(), cell.data(), bounds));
  mnMinX = bounds[0];
  mnMaxX = bounds[1];
  mnMinY = bounds[2];
  mnMaxY = bounds[3];
  // Frame.cc:113-115
  mfGridElementWidthInv = static_cast<float>(FRAME_GRID_COLS) / (mnMaxX - mnMinX);
  mfGridElementHeightInv = static_cast<float>(FRAME_GRID_ROWS) / (mnMaxY - mnMinY);
  for (int i = 0; i < N; i++)
    if (cell[i] >= 0) mGrid[cell[i] % FRAME_GRID_COLS][cell[i] / FRAME_GRID_COLS].push_back(i);
  mvpMapPoints.assign(N, nullptr);
  mvbOutlier.assign(N, false);
}

Frame::Frame(const cv::Mat& imGray, const cv::Mat& imDepth, const double& timeStamp,
             ORBextractor* extractor, ORBVocabulary* voc, cv::Mat& K, cv::Mat& distCoef,
             const float& bf, const float& thDepth, LineExtractor* lineExtractor)
    : mTimeStamp(timeStamp), mK(K.clone()), mDistCoef(distCoef.clone()), mbf(bf),
      mThDepth(thDepth), mpORBextractorLeft(extractor), mpORBvocabulary(voc) {
  mnId = nNextId++;
  ScaleInfo(extractor);
  mnWidth = imGray.cols;
  mnHeight = imGray.rows;
  fx = K.at<float>(0, 0);
  fy = K.at<float>(1, 1);
  cx = K.at<float>(0, 2);
  cy = K.at<float>(1, 2);
  invfx = 1.0f / fx;
  invfy = 1.0f / fy;
  mb = mbf / fx;
  // ORB || LineExtractor (Frame.cc:152-155)
  thread_local LineExtractor own_lines;
  LineExtractor* lx = lineExtractor ? lineExtractor : &own_lines;
  std::exception_ptr lerr, oerr;
  std::thread tl([&]() {
    try {
      lx->ExtractLineSegment(imGray, mvKeyLines, mLineDescriptors, mvKeyLineCoefficient);
    } catch (...) {
      lerr = std::current_exception();
    }
  });
  // the ORB call may throw (library error): the line thread is joined on
  // every path before anything propagates
  try {
    (*extractor)(imGray, cv::Mat(), mvKeys, mDescriptors);
  } catch (...) {
    oerr = std::current_exception();
  }
  tl.join();
  if (oerr) std::rethrow_exception(oerr);
  if (lerr) std::rethrow_exception(lerr);
  N = (int)mvKeys.size();
  NL = (int)mvKeyLines.size();
  // UndistortKeyPoints + ComputeStereoFromRGBD + AssignFeaturesToGrid
  // (Frame.cc:160-204) in one call
  PrepareKeys(imDepth.ptr<float>());
  const orbpl_camera cam = Camera();
  // UndistortKeyLines + the line part of ComputeStereoFromRGBD
  mvKeyLinesUn.resize(NL);
  mvDepthLineStart.resize(NL);
  mvDepthLineEnd.resize(NL);
  mvuRightLineStart.resize(NL);
  mvuRightLineEnd.resize(NL);
  check(orbpl_line_frame_prepare(&cam, reinterpret_cast<const orbpl_keyline*>(mvKeyLines.data()),
                                 NL, imDepth.ptr<float>(),
                                 reinterpret_cast<orbpl_keyline*>(mvKeyLinesUn.data()),
                                 mvDepthLineStart.data(), mvDepthLineEnd.data(),
                                 mvuRightLineStart.data(), mvuRightLineEnd.data()));
  mvpMapLines.assign(NL, nullptr);
  mvbLineOutlier.assign(NL, false);
}

Frame::Frame(const cv::Mat& imLeft, const cv::Mat& imRight, const double& timeStamp,
             ORBextractor* extractorLeft, ORBextractor* extractorRight, ORBVocabulary* voc,
             cv::Mat& K, cv::Mat& distCoef, const float& bf, const float& thDepth)
    : mTimeStamp(timeStamp), mK(K.clone()), mDistCoef(distCoef.clone()), mbf(bf),
      mThDepth(thDepth), mpORBextractorLeft(extractorLeft), mpORBextractorRight(extractorRight),
      mpORBvocabulary(voc) {
  mnId = nNextId++;
  ScaleInfo(extractorLeft);
  mnWidth = imLeft.cols;
  mnHeight = imLeft.rows;
  // ORB extraction, left || right (Frame.cc:88-91); each extractor owns its
  // own device context, so the two host threads never share one
  std::exception_ptr rerr, lerr;
  std::thread tr([&]() {
    try {
      (*mpORBextractorRight)(imRight, cv::Mat(), mvKeysRight, mDescriptorsRight);
    } catch (...) {
      rerr = std::current_exception();
    }
  });
  try {
    (*mpORBextractorLeft)(imLeft, cv::Mat(), mvKeys, mDescriptors);
  } catch (...) {
    lerr = std::current_exception();
  }
  tr.join();
  if (lerr) std::rethrow_exception(lerr);
  if (rerr) std::rethrow_exception(rerr);
  N = (int)mvKeys.size();
  NL = 0;
  if (mvKeys.empty()) return;   // Frame.cc:95-96
  fx = K.at<float>(0, 0);
  fy = K.at<float>(1, 1);
  cx = K.at<float>(0, 2);
  cy = K.at<float>(1, 2);
  invfx = 1.0f / fx;
  invfy = 1.0f / fy;
  mb = mbf / fx;   // Frame.cc:128
  // UndistortKeyPoints, then ComputeStereoMatches, the map point slots,
  // ComputeImageBounds and the grid (Frame.cc:98-131): the glue runs first
  // here (no depth image: mvuRight / mvDepth = -1), the stereo matcher
  // then overwrites them - the same values in the reference's order
  PrepareKeys(nullptr);
  ComputeStereoMatches();
}

void Frame::ComputeStereoMatches() {
  if (!mpORBextractorLeft || !mpORBextractorRight || !mpORBextractorLeft->ctx() ||
      !mpORBextractorRight->ctx())
    throw std::runtime_error("Frame::ComputeStereoMatches: no stereo extractors");
  mvuRight.assign(N, -1.0f);
  mvDepth.assign(N, -1.0f);
  if (N == 0) return;
  const orbpl_camera cam = Camera();
  const int nr = (int)mvKeysRight.size();
  check(orbpl_stereo_matches(&cam, mpORBextractorLeft->ctx(), mpORBextractorRight->ctx(), 0,
                             reinterpret_cast<const orbpl_keypoint*>(mvKeys.data()),
                             mDescriptors.data, N,
                             reinterpret_cast<const orbpl_keypoint*>(mvKeysRight.data()),
                             nr ? mDescriptorsRight.data : nullptr, nr, mvuRight.data(),
                             mvDepth.data()));
}

std::vector<size_t> Frame::GetFeaturesInArea(const float& x, const float& y, const float& r,
                                              const int minLevel, const int maxLevel) const {
  std::vector<size_t> vIndices;
  vIndices.reserve(N);
  const int nMinCellX = std::max(0, (int)std::floor((x - mnMinX - r) * mfGridElementWidthInv));
  if (nMinCellX >= FRAME_GRID_COLS) return vIndices;
  const int nMaxCellX = std::min((int)FRAME_GRID_COLS - 1,
                                 (int)std::ceil((x - mnMinX + r) * mfGridElementWidthInv));
  if (nMaxCellX < 0) return vIndices;
  const int nMinCellY = std::max(0, (int)std::floor((y - mnMinY - r) * mfGridElementHeightInv));
  if (nMinCellY >= FRAME_GRID_ROWS) return vIndices;
  const int nMaxCellY = std::min((int)FRAME_GRID_ROWS - 1,
                                 (int)std::ceil((y - mnMinY + r) * mfGridElementHeightInv));
  if (nMaxCellY < 0) return vIndices;
  const bool bCheckLevels = (minLevel > 0) || (maxLevel >= 0);
  for (int ix = nMinCellX; ix <= nMaxCellX; ix++)
    for (int iy = nMinCellY; iy <= nMaxCellY; iy++) {
      for (size_t j : mGrid[ix][iy]) {
        const cv::KeyPoint& kpUn = mvKeysUn[j];
        if (bCheckLevels) {
          if (kpUn.octave < minLevel) continue;
          if (maxLevel >= 0 && kpUn.octave > maxLevel) continue;
        }
        const float distx = kpUn.pt.x - x;
        const float disty = kpUn.pt.y - y;
        if (std::fabs(distx) < r && std::fabs(disty) < r) vIndices.push_back(j);
      }
    }
  return vIndices;
}

void Frame::ComputeBoW() {
  if (!mBowVec.empty()) return;
  if (!mpORBvocabulary) throw std::runtime_error("Frame::ComputeBoW: no vocabulary");
  mpORBvocabulary->transform(toDescriptorVector(mDescriptors), mBowVec, mFeatVec, 4);
}

int Frame::IsInFrustumBatch(const std::vector<MapPoint*>& vp, float viewingCosLimit,
                            std::vector<uint8_t>* in_view) {
  const int M = (int)vp.size();
  std::vector<float> xyz(3 * (size_t)M), nrm(3 * (size_t)M), dmin(M), dmax(M);
  std::vector<float> px(M), py(M), pxr(M), vcos(M);
  std::vector<int32_t> level(M);
  std::vector<uint8_t> iv(M);
  for (int j = 0; j < M; j++) {
    const cv::Mat X = vp[j]->GetWorldPos(), Nv = vp[j]->GetNormal();
    for (int k = 0; k < 3; k++) {
      xyz[3 * j + k] = X.at<float>(k, 0);
      nrm[3 * j + k] = Nv.at<float>(k, 0);
    }
    dmin[j] = vp[j]->GetMinDistance();   // the library applies GetMin/MaxDistanceInvariance's
    dmax[j] = vp[j]->GetMaxDistance();   // 0.8f / 1.2f and PredictScale's mfMaxDistance / dist
  }
  const orbpl_camera cam = Camera();
  check(orbpl_frame_is_in_frustum(&cam, mfScaleFactor, mnScaleLevels, mTcw.ptr<float>(), M,
                                  xyz.data(), nrm.data(), dmin.data(), dmax.data(),
                                  viewingCosLimit, iv.data(), px.data(), py.data(), pxr.data(),
                                  level.data(), vcos.data()));
  int n = 0;
  for (int j = 0; j < M; j++) {
    MapPoint* p = vp[j];
    p->mbTrackInView = iv[j] != 0;
    if (!iv[j]) continue;   // the reference sets the projection only when in view
    p->mTrackProjX = px[j];
    p->mTrackProjY = py[j];
    p->mTrackProjXR = pxr[j];
    p->mnTrackScaleLevel = level[j];
    p->mTrackViewCos = vcos[j];
    n++;
  }
  if (in_view) in_view->assign(iv.begin(), iv.end());
  return n;
}

bool Frame::IsInFrustum(MapPoint* pMP, float viewingCosLimit) {
  return IsInFrustumBatch(std::vector<MapPoint*>{pMP}, viewingCosLimit) == 1;
}

bool Frame::IsInFrustum(MapLine* pML, float viewingCosLimit) {
  const Eigen::Vector3d s = pML->GetWorldStartPos(), e = pML->GetWorldEndPos();
  // the reference casts both end points to float (cv::Mat_<float>, Frame.cc:408-409)
  const float xyz6[6] = {(float)s[0], (float)s[1], (float)s[2], (float)e[0], (float)e[1], (float)e[2]};
  uint8_t iv = 0;
  check(orbl_frame_is_in_frustum(mTcw.ptr<float>(), 1, xyz6, &iv));
  pML->mbTrackInView = iv != 0;
  return iv != 0;
}

void Frame::SetPose(cv::Mat Tcw) {
  mTcw = Tcw.clone();
  UpdatePoseMatrices();
}

// Frame.cc:335-344: Rwc = Rcw^T, Ow = -Rcw^T tcw (float products summed in
// double, one rounding: pinned P6)
void Frame::UpdatePoseMatrices() {
  mRcw.create(3, 3, cv::CV_32F);
  mtcw.create(3, 1, cv::CV_32F);
  mRwc.create(3, 3, cv::CV_32F);
  mOw.create(3, 1, cv::CV_32F);
  for (int r = 0; r < 3; r++) {
    for (int c = 0; c < 3; c++) {
      mRcw.at<float>(r, c) = mTcw.at<float>(r, c);
      mRwc.at<float>(c, r) = mTcw.at<float>(r, c);
    }
    mtcw.at<float>(r, 0) = mTcw.at<float>(r, 3);
  }
  for (int r = 0; r < 3; r++) {
    double s = 0;
    for (int k = 0; k < 3; k++) s += (double)mRwc.at<float>(r, k) * mtcw.at<float>(k, 0);
    mOw.at<float>(r, 0) = (float)(-s);
  }
}

static cv::Mat unproject(const Frame& F, float u, float v, float z) {
  const float x = (u - Frame::cx) * z * Frame::invfx;
  const float y = (v - Frame::cy) * z * Frame::invfy;
  const float xc[3] = {x, y, z};
  cv::Mat w(3, 1, cv::CV_32F);
  for (int r = 0; r < 3; r++) {
    double s = 0;
    for (int k = 0; k < 3; k++) s += (double)F.mRwc.at<float>(r, k) * xc[k];
    w.at<float>(r, 0) = (float)(s + (double)F.mOw.at<float>(r, 0));
  }
  return w;
}

cv::Mat Frame::UnprojectStereo(const int& i) {
  const float z = mvDepth[i];
  if (z <= 0) return cv::Mat();
  return unproject(*this, mvKeysUn[i].pt.x, mvKeysUn[i].pt.y, z);
}

cv::Mat Frame::UnprojectStereoLineStart(const int& i) {
  const float z = mvDepthLineStart[i];
  if (z <= 0) return cv::Mat();
  return unproject(*this, mvKeyLinesUn[i].startPointX, mvKeyLinesUn[i].startPointY, z);
}

cv::Mat Frame::UnprojectStereoLineEnd(const int& i) {
  const float z = mvDepthLineStart[i];   // Frame.cc:1192 reads the start depth
  if (z <= 0) return cv::Mat();
  return unproject(*this, mvKeyLinesUn[i].endPointX, mvKeyLinesUn[i].endPointY, z);
}

}  // namespace ORB_SLAM2
