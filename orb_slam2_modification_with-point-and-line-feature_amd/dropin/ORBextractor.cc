// Drop-in ORB_SLAM2::ORBextractor over orbx_* (see ORBextractor.h).
#include "ORBextractor.h"

#include <cassert>
#include <stdexcept>

namespace ORB_SLAM2 {

static_assert(sizeof(cv::KeyPoint) == sizeof(orbpl_keypoint), "cv::KeyPoint layout");

static void check(int rc) {
  if (rc != ORBPL_OK) throw std::runtime_error(orbpl_last_error());
}

// ORBextractor.cc:410-470: the scale tables come from the library's own
// geometry (orbx_describe, no device needed), so the getters work before the
// first image, as in the reference
ORBextractor::ORBextractor(int _nfeatures, float _scaleFactor, int _nlevels, int _iniThFAST,
                           int _minThFAST)
    : nfeatures(_nfeatures), scaleFactor(_scaleFactor), nlevels(_nlevels),
      iniThFAST(_iniThFAST), minThFAST(_minThFAST),
      params_{_nfeatures, _scaleFactor, _nlevels, _iniThFAST, _minThFAST} {
  mvScaleFactor.assign(nlevels, 1.f);
  mnFeaturesPerLevel.assign(nlevels, 0);
  std::vector<int> lw(nlevels), lh(nlevels);
  int cap = 0;
  // a geometry whose every level passes the library's bounds (<= 1024 FAST
  // cells per level, coarse levels large enough); the scale tables and
  // budgets do not depend on it
  check(orbx_describe(&params_, 960, 960, lw.data(), lh.data(), mnFeaturesPerLevel.data(),
                      mvScaleFactor.data(), &cap));
  mvInvScaleFactor.resize(nlevels);
  mvLevelSigma2.resize(nlevels);
  mvInvLevelSigma2.resize(nlevels);
  for (int l = 0; l < nlevels; l++) {
    mvInvScaleFactor[l] = 1.0f / mvScaleFactor[l];
    mvLevelSigma2[l] = mvScaleFactor[l] * mvScaleFactor[l];
    mvInvLevelSigma2[l] = 1.0f / mvLevelSigma2[l];
  }
}

ORBextractor::~ORBextractor() {
  if (ctx_) orbx_destroy(ctx_);
}

void ORBextractor::operator()(cv::InputArray _image, cv::InputArray, std::vector<cv::KeyPoint>& kps,
                              cv::OutputArray _descriptors) {
  if (_image.empty()) return;                           // ORBextractor.cc:1046-1047
  cv::Mat image = _image.getMat();
  assert(image.type() == cv::CV_8UC1);                  // ORBextractor.cc:1049-1050
  if (!ctx_ || ctx_w_ != image.cols || ctx_h_ != image.rows) {
    if (ctx_) orbx_destroy(ctx_);
    ctx_ = nullptr;
    check(orbx_create(&params_, image.cols, image.rows, 1, device, &ctx_));
    ctx_w_ = image.cols;
    ctx_h_ = image.rows;
  }
  const int cap = orbx_max_keypoints(ctx_);
  kps.resize(cap);
  cv::Mat desc(cap, 32, cv::CV_8U);
  int n = 0;
  check(orbx_extract(ctx_, image.data, image.cols, image.rows, (int)image.step,
                     reinterpret_cast<orbpl_keypoint*>(kps.data()), desc.data, cap, &n));
  kps.resize(n);
  if (n == 0) {
    _descriptors.release();                             // ORBextractor.cc:1064-1065
  } else {
    _descriptors.create(n, 32, cv::CV_8U);
    std::memcpy(_descriptors.getMatRef().data, desc.data, (size_t)n * 32);
  }
  mvImagePyramid.clear();
  pyr_valid_ = true;
  if (mbKeepPyramid) FetchPyramid();
}

// the last call's level contents, device-to-host on request
const std::vector<cv::Mat>& ORBextractor::FetchPyramid() {
  if (!pyr_valid_ || (int)mvImagePyramid.size() == nlevels) return mvImagePyramid;
  mvImagePyramid.resize(nlevels);
  for (int l = 0; l < nlevels; l++) {
    int w = 0, h = 0;
    check(orbx_get_pyramid(ctx_, 0, l, 0, 0, nullptr, 0, &w, &h));
    mvImagePyramid[l].create(h, w, cv::CV_8U);
    check(orbx_get_pyramid(ctx_, 0, l, 0, 0, mvImagePyramid[l].data, w * h, &w, &h));
  }
  return mvImagePyramid;
}

}  // namespace ORB_SLAM2
