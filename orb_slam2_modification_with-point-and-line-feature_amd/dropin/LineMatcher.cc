// Drop-in ORB_SLAM2::LineMatcher (see LineMatcher.h).
#include "LineMatcher.h"

#include <stdexcept>

namespace ORB_SLAM2 {

int LineMatcher::DescriptorDistance(const cv::Mat& a, const cv::Mat& b) {
  return orbpl_descriptor_distance(a.ptr<uint8_t>(), b.ptr<uint8_t>());
}

int LineMatcher::SearchByProjection(Frame& Cur, const Frame& Last) {
  const int NL = Last.NL;
  std::vector<uint8_t> has(NL, 0), out(NL, 0);
  std::vector<float> xyz(6 * (size_t)NL, 0.f);
  cv::Mat lastDesc(NL > 0 ? NL : 1, 32, cv::CV_8U);
  for (int i = 0; i < NL; i++) {
    MapLine* l = Last.mvpMapLines[i];
    has[i] = l != nullptr;
    out[i] = Last.mvbLineOutlier[i];
    if (!l) continue;
    const Eigen::Vector3d s = l->GetWorldStartPos(), e = l->GetWorldEndPos();
    for (int k = 0; k < 3; k++) {
      xyz[6 * i + k] = (float)s[k];
      xyz[6 * i + 3 + k] = (float)e[k];
    }
    std::memcpy(lastDesc.ptr<uint8_t>(i), l->GetDescriptor().data, 32);
  }
  std::vector<int32_t> match(Cur.NL, -1);
  const orbpl_camera cam = Cur.Camera();
  int n = 0;
  if (orbl_search_by_projection_last(&cam, Cur.mTcw.ptr<float>(), Cur.NL,
                                     reinterpret_cast<const orbpl_keyline*>(Cur.mvKeyLinesUn.data()),
                                     Cur.mLineDescriptors.data, NL,
                                     reinterpret_cast<const orbpl_keyline*>(Last.mvKeyLinesUn.data()),
                                     has.data(), out.data(), xyz.data(), lastDesc.data, match.data(),
                                     &n) != ORBPL_OK)
    throw std::runtime_error(orbpl_last_error());
  for (int j = 0; j < Cur.NL; j++)
    Cur.mvpMapLines[j] = match[j] >= 0 ? Last.mvpMapLines[match[j]] : nullptr;
  return n;
}

}  // namespace ORB_SLAM2
