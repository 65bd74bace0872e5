// Drop-in ORB_SLAM2::LineExtractor (include/LineExtractor.h:25-30) over
// lsdx_*: LSDDetector::detect + the 80 longest + BinaryDescriptor (LBD) +
// line coefficients on the MI355X (LineExtractor.cpp:76-134).
#pragma once
#include <vector>

#include "cvmini.h"
#include "orbpl.h"

namespace ORB_SLAM2 {

using cv::line_descriptor::KeyLine;

class LineExtractor {
 public:
  LineExtractor() = default;
  ~LineExtractor();
  LineExtractor(const LineExtractor&) = delete;
  LineExtractor& operator=(const LineExtractor&) = delete;

  // `scale` / `num_octaves` are accepted and ignored: the reference's
  // `int scale = 1.2` truncates to 1 and LSDDetector runs one octave
  // (LineExtractor.h:29, LineExtractor.cpp:85)
  void ExtractLineSegment(const cv::Mat& img, std::vector<KeyLine>& key_lines,
                          cv::Mat& line_descriptor,
                          std::vector<Eigen::Vector3d>& keyline_coefficients, int scale = 1.2,
                          int num_octaves = 1);
  int device = 0;

 private:
  lsdx_ctx* ctx_ = nullptr;
  int ctx_w_ = 0, ctx_h_ = 0;
};

}  // namespace ORB_SLAM2
