// Drop-in ORB_SLAM2::ORBmatcher (see ORBmatcher.h).
#include "ORBmatcher.h"

#include <stdexcept>

namespace ORB_SLAM2 {

static void check(int rc) {
  if (rc != ORBPL_OK) throw std::runtime_error(orbpl_last_error());
}

int ORBmatcher::DescriptorDistance(const cv::Mat& a, const cv::Mat& b) {
  return orbpl_descriptor_distance(a.ptr<uint8_t>(), b.ptr<uint8_t>());
}

int ORBmatcher::SearchByProjection(Frame& Cur, const Frame& Last, const float th,
                                   const bool bMono) {
  const int N = Cur.N, NL = Last.N;
  std::vector<uint8_t> has(NL, 0), out(NL, 0);
  std::vector<float> xyz(3 * (size_t)NL, 0.f);
  std::vector<int32_t> nobs(NL, 0), match(N, -1);
  cv::Mat mpDesc(NL > 0 ? NL : 1, 32, cv::CV_8U);
  for (int i = 0; i < NL; i++) {
    MapPoint* p = Last.mvpMapPoints[i];
    has[i] = p != nullptr;
    out[i] = Last.mvbOutlier[i];
    if (!p) continue;
    cv::Mat X = p->GetWorldPos();
    for (int k = 0; k < 3; k++) xyz[3 * i + k] = X.at<float>(k, 0);
    std::memcpy(mpDesc.ptr<uint8_t>(i), p->GetDescriptor().data, 32);
    nobs[i] = p->Observations();
  }
  const orbpl_match_current c{N, Cur.mTcw.ptr<float>(),
                              reinterpret_cast<const orbpl_keypoint*>(Cur.mvKeysUn.data()),
                              Cur.mDescriptors.data, Cur.mvuRight.data()};
  const orbpl_match_last l{NL, Last.mTcw.ptr<float>(),
                           reinterpret_cast<const orbpl_keypoint*>(Last.mvKeysUn.data()),
                           has.data(), out.data(), xyz.data(), mpDesc.data, nobs.data()};
  const orbpl_camera cam = Cur.Camera();
  int nmatches = 0;
  check(orbm_search_by_projection_last(&cam, Cur.mvScaleFactors.data(), Cur.mnScaleLevels, &c, &l,
                                       th, bMono ? 1 : 0, mbCheckOrientation ? 1 : 0, match.data(),
                                       &nmatches));
  for (int i = 0; i < N; i++)
    if (match[i] >= 0) Cur.mvpMapPoints[i] = Last.mvpMapPoints[match[i]];
  return nmatches;
}

int ORBmatcher::SearchByProjection(Frame& F, const std::vector<MapPoint*>& vp, const float th) {
  const int M = (int)vp.size(), N = F.N;
  std::vector<float> px(M), py(M), pxr(M), vcos(M);
  std::vector<int32_t> level(M), nobs(M), curNobs(N, 0), match(N, -1);
  std::vector<uint8_t> inView(M);
  cv::Mat desc(M > 0 ? M : 1, 32, cv::CV_8U);
  for (int j = 0; j < M; j++) {
    const MapPoint* p = vp[j];
    // ORBmatcher.cc:91-98: only points IsInFrustum put in view, and not bad
    inView[j] = p->mbTrackInView && !p->isBad();
    px[j] = p->mTrackProjX;
    py[j] = p->mTrackProjY;
    pxr[j] = p->mTrackProjXR;
    level[j] = p->mnTrackScaleLevel;
    vcos[j] = p->mTrackViewCos;
    std::memcpy(desc.ptr<uint8_t>(j), p->GetDescriptor().data, 32);
    nobs[j] = p->Observations();
  }
  for (int i = 0; i < N; i++)
    if (F.mvpMapPoints[i]) curNobs[i] = F.mvpMapPoints[i]->Observations();
  const orbpl_camera cam = F.Camera();
  const orbpl_match_current c{N, F.mTcw.ptr<float>(),
                              reinterpret_cast<const orbpl_keypoint*>(F.mvKeysUn.data()),
                              F.mDescriptors.data, F.mvuRight.data()};
  int n = 0;
  check(orbm_search_by_projection_local(&cam, F.mvScaleFactors.data(), F.mnScaleLevels, &c, M,
                                        inView.data(), px.data(), py.data(), pxr.data(),
                                        level.data(), vcos.data(), desc.data, nobs.data(),
                                        curNobs.data(), th, mfNNratio, match.data(), &n));
  for (int i = 0; i < N; i++)
    if (match[i] >= 0) F.mvpMapPoints[i] = vp[match[i]];
  return n;
}

// the FeatureVector as one node id per feature (-1: none)
static std::vector<int32_t> nodes_of(const DBoW2::FeatureVector& fv, int n) {
  std::vector<int32_t> node(n > 0 ? n : 1, -1);
  for (const auto& kv : fv)
    for (unsigned i : kv.second)
      if ((int)i < n) node[i] = (int32_t)kv.first;
  return node;
}

int ORBmatcher::SearchByBoW(KeyFrame* pKF, Frame& F, std::vector<MapPoint*>& vpMapPointMatches) {
  const std::vector<MapPoint*> vpMapPointsKF = pKF->GetMapPointMatches();
  vpMapPointMatches.assign(F.N, nullptr);
  const int nkf = pKF->N, nf = F.N;
  const std::vector<int32_t> kf_node = nodes_of(pKF->mFeatVec, nkf), f_node = nodes_of(F.mFeatVec, nf);
  std::vector<uint8_t> kf_valid(nkf > 0 ? nkf : 1, 0);
  std::vector<float> kf_angle(nkf > 0 ? nkf : 1), f_angle(nf > 0 ? nf : 1);
  for (int i = 0; i < nkf; i++) {
    const MapPoint* p = vpMapPointsKF[i];
    kf_valid[i] = p && !p->isBad();   // ORBmatcher.cc:298-303
    kf_angle[i] = pKF->mvKeysUn[i].angle;
  }
  for (int j = 0; j < nf; j++) f_angle[j] = F.mvKeys[j].angle;
  std::vector<int32_t> match(nf > 0 ? nf : 1, -1);
  int n = 0;
  check(orbm_search_by_bow(nkf, kf_node.data(), kf_valid.data(), pKF->mDescriptors.data,
                           kf_angle.data(), nf, f_node.data(), F.mDescriptors.data, f_angle.data(),
                           mfNNratio, mbCheckOrientation ? 1 : 0, match.data(), &n));
  for (int j = 0; j < nf; j++)
    if (match[j] >= 0) vpMapPointMatches[j] = vpMapPointsKF[match[j]];
  return n;
}

}  // namespace ORB_SLAM2
