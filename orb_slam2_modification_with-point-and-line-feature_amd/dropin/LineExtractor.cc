// Drop-in ORB_SLAM2::LineExtractor over lsdx_* (see LineExtractor.h).
#include "LineExtractor.h"

#include <stdexcept>

namespace ORB_SLAM2 {

static_assert(sizeof(KeyLine) == sizeof(orbpl_keyline), "KeyLine layout");

constexpr int kKeep = 80;   // nums_lineFeature (LineExtractor.cpp:87)

LineExtractor::~LineExtractor() {
  if (ctx_) lsdx_destroy(ctx_);
}

void LineExtractor::ExtractLineSegment(const cv::Mat& img, std::vector<KeyLine>& key_lines,
                                       cv::Mat& line_descriptor,
                                       std::vector<Eigen::Vector3d>& coef, int, int) {
  if (!ctx_ || ctx_w_ != img.cols || ctx_h_ != img.rows) {
    if (ctx_) lsdx_destroy(ctx_);
    ctx_ = nullptr;
    if (lsdx_create(img.cols, img.rows, 1, device, &ctx_) != ORBPL_OK)
      throw std::runtime_error(orbpl_last_error());
    ctx_w_ = img.cols;
    ctx_h_ = img.rows;
  }
  key_lines.resize(kKeep);
  cv::Mat desc(kKeep, 32, cv::CV_8U);
  std::vector<double> c(3 * kKeep);
  int n = 0;
  if (lsdx_extract(ctx_, img.data, img.cols, img.rows, (int)img.step,
                   reinterpret_cast<orbpl_keyline*>(key_lines.data()), desc.data, c.data(), kKeep,
                   &n) != ORBPL_OK)
    throw std::runtime_error(orbpl_last_error());
  key_lines.resize(n);
  line_descriptor = desc.rowRange(0, n).clone();
  coef.resize(n);
  for (int i = 0; i < n; i++) coef[i] = Eigen::Vector3d(c[3 * i], c[3 * i + 1], c[3 * i + 2]);
}

}  // namespace ORB_SLAM2
