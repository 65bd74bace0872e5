// Drop-in ORB_SLAM2::Optimizer (see Optimizer.h).
#include "Optimizer.h"

#include <stdexcept>

namespace ORB_SLAM2 {

static int pose(Frame* F, bool lines) {
  const int N = F->N, NL = lines ? F->NL : 0;
  std::vector<uint8_t> has(N, 0), hasl(NL, 0), out(N), lout(NL);
  std::vector<float> xyz(3 * (size_t)N, 0.f), lobs(4 * (size_t)NL, 0.f), lxyz(6 * (size_t)NL, 0.f);
  std::vector<int32_t> loct(NL, 0);
  for (int i = 0; i < N; i++) {
    out[i] = F->mvbOutlier[i];
    if (MapPoint* p = F->mvpMapPoints[i]) {
      has[i] = 1;
      cv::Mat X = p->GetWorldPos();
      for (int k = 0; k < 3; k++) xyz[3 * i + k] = X.at<float>(k, 0);
    }
  }
  for (int j = 0; j < NL; j++) {
    lout[j] = F->mvbLineOutlier[j];
    const KeyLine& kl = F->mvKeyLinesUn[j];
    lobs[4 * j] = kl.startPointX;
    lobs[4 * j + 1] = kl.startPointY;
    lobs[4 * j + 2] = kl.endPointX;
    lobs[4 * j + 3] = kl.endPointY;
    loct[j] = kl.octave;
    if (MapLine* l = F->mvpMapLines[j]) {
      hasl[j] = 1;
      const Eigen::Vector3d s = l->GetWorldStartPos(), e = l->GetWorldEndPos();
      for (int k = 0; k < 3; k++) {
        lxyz[6 * j + k] = (float)s[k];
        lxyz[6 * j + 3 + k] = (float)e[k];
      }
    }
  }
  orbpl_pose_problem P{N,          reinterpret_cast<const orbpl_keypoint*>(F->mvKeysUn.data()),
                       F->mvuRight.data(), has.data(), xyz.data(), NL, lobs.data(), loct.data(),
                       hasl.data(), lxyz.data(), F->mvInvLevelSigma2.data(),
                       (int)F->mvInvLevelSigma2.size()};
  cv::Mat T = F->mTcw.clone();
  const orbpl_camera cam = F->Camera();
  int inliers = 0;
  if (orbpl_pose_optimization(&cam, &P, T.ptr<float>(), out.data(), lout.data(), &inliers) !=
      ORBPL_OK)
    throw std::runtime_error(orbpl_last_error());
  F->SetPose(T);
  for (int i = 0; i < N; i++) F->mvbOutlier[i] = out[i] != 0;
  for (int j = 0; j < NL; j++) F->mvbLineOutlier[j] = lout[j] != 0;
  return inliers;
}

int Optimizer::PoseOptimization(Frame* pFrame) { return pose(pFrame, false); }
int Optimizer::PoseOptimizationWithLines(Frame* pFrame) { return pose(pFrame, true); }

}  // namespace ORB_SLAM2
