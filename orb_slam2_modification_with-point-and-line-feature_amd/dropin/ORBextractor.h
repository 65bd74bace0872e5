// Drop-in ORB_SLAM2::ORBextractor (include/ORBextractor.h:44-112): the
// reference's constructor, operator() and getters over the MI355X C ABI
// (orbx_*). One instance per host thread, as the reference uses one extractor
// per Frame thread (Frame.cc:152-155).
#pragma once
#include <vector>

#include "cvmini.h"
#include "orbpl.h"

namespace ORB_SLAM2 {

class ORBextractor {
 public:
  enum { HARRIS_SCORE = 0, FAST_SCORE = 1 };

  ORBextractor(int nfeatures, float scaleFactor, int nlevels, int iniThFAST, int minThFAST);
  ~ORBextractor();
  ORBextractor(const ORBextractor&) = delete;
  ORBextractor& operator=(const ORBextractor&) = delete;

  // ORBextractor.cc:1043-1105. The mask is ignored, as in the reference.
  void operator()(cv::InputArray image, cv::InputArray mask, std::vector<cv::KeyPoint>& keypoints,
                  cv::OutputArray descriptors);

  int GetLevels() { return nlevels; }
  float GetScaleFactor() { return (float)scaleFactor; }
  std::vector<float> GetScaleFactors() { return mvScaleFactor; }
  std::vector<float> GetInverseScaleFactors() { return mvInvScaleFactor; }
  std::vector<float> GetScaleSigmaSquares() { return mvLevelSigma2; }
  std::vector<float> GetInverseScaleSigmaSquares() { return mvInvLevelSigma2; }

  // the level images of the last call (content, w x h), as the public member
  // the reference's stereo matcher reads (Frame.cc:895-1002). The pyramid
  // stays on the device: the drop-in Frame's ComputeStereoMatches reads it
  // there (orbpl_stereo_matches), so an RGB-D frame copies nothing back.
  // FetchPyramid() fills mvImagePyramid from the last call on request (a host
  // that keeps the reference's own ComputeStereoMatches calls it, or sets
  // mbKeepPyramid to have every call fill it); otherwise it is left empty.
  std::vector<cv::Mat> mvImagePyramid;
  bool mbKeepPyramid = false;
  const std::vector<cv::Mat>& FetchPyramid();

  // the device context (orbpl_stereo_matches reads the pyramid on the device)
  orbx_ctx* ctx() { return ctx_; }
  int device = 0;

 protected:
  int nfeatures;
  double scaleFactor;
  int nlevels;
  int iniThFAST;
  int minThFAST;
  std::vector<int> mnFeaturesPerLevel;
  std::vector<float> mvScaleFactor, mvInvScaleFactor, mvLevelSigma2, mvInvLevelSigma2;

 private:
  orbpl_orb_params params_;
  orbx_ctx* ctx_ = nullptr;
  int ctx_w_ = 0, ctx_h_ = 0;
  bool pyr_valid_ = false;   // the device holds a pyramid of the last call
};

}  // namespace ORB_SLAM2
