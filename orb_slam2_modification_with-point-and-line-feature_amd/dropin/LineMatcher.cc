// Drop-in ORB_SLAM2::LineMatcher (see LineMatcher.h).
#include "LineMatcher.h"

#include <algorithm>
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

// both list overloads: projection + Liang-Barsky of the valid map lines, all
// LineMatching pairs against the current lines whose map line has no
// observations, the relaxed retry (which first clears F.mvpMapLines)
static int search_list(Frame& F, const std::vector<MapLine*>& ml, const std::vector<uint8_t>& valid) {
  const int M = (int)ml.size(), NLc = F.NL;
  std::vector<float> xyz(6 * (size_t)(M > 0 ? M : 1), 0.f);
  cv::Mat desc(M > 0 ? M : 1, 32, cv::CV_8U);
  for (int i = 0; i < M; i++) {
    const MapLine* l = ml[i];
    if (!l) continue;
    for (int k = 0; k < 3; k++) {
      xyz[6 * i + k] = (float)l->mStart3d[k];
      xyz[6 * i + 3 + k] = (float)l->mEnd3d[k];
    }
    std::memcpy(desc.ptr<uint8_t>(i), l->mLineDescriptor.data, 32);
  }
  std::vector<int32_t> curNobs(NLc > 0 ? NLc : 1, 0), match(NLc > 0 ? NLc : 1, -1);
  for (int j = 0; j < NLc; j++)
    if (F.mvpMapLines[j]) curNobs[j] = F.mvpMapLines[j]->Observations();
  const orbpl_camera cam = F.Camera();
  int n = 0, wiped = 0;
  if (orbl_search_by_projection_list(&cam, F.mTcw.ptr<float>(), NLc,
                                     reinterpret_cast<const orbpl_keyline*>(F.mvKeyLinesUn.data()),
                                     F.mLineDescriptors.data, curNobs.data(), M, valid.data(),
                                     xyz.data(), desc.data, match.data(), &n, &wiped) != ORBPL_OK)
    throw std::runtime_error(orbpl_last_error());
  if (wiped) std::fill(F.mvpMapLines.begin(), F.mvpMapLines.end(), nullptr);
  for (int j = 0; j < NLc; j++)
    if (match[j] >= 0) F.mvpMapLines[j] = ml[match[j]];
  return n;
}

int LineMatcher::SearchByProjection(Frame& CurrentFrame, KeyFrame* RefFrame) {
  const std::vector<MapLine*>& ml = RefFrame->mvpMapLines;
  std::vector<uint8_t> valid(ml.size() > 0 ? ml.size() : 1, 0);
  for (size_t i = 0; i < ml.size(); i++) valid[i] = ml[i] != nullptr;   // LineMatcher.cpp:562-564
  return search_list(CurrentFrame, ml, valid);
}

int LineMatcher::SearchByProjection(Frame& F, const std::vector<MapLine*>& vpMapLines) {
  std::vector<uint8_t> valid(vpMapLines.size() > 0 ? vpMapLines.size() : 1, 0);
  for (size_t i = 0; i < vpMapLines.size(); i++)   // LineMatcher.cpp:788-793
    valid[i] = vpMapLines[i]->mbTrackInView && !vpMapLines[i]->isBad();
  return search_list(F, vpMapLines, valid);
}

// the harness searches over orbl_search_by_projection_pairs (mode 0 / 1)
static int search_pairs(Frame& F, int mode, const std::vector<MapLine*>& ml,
                        const std::vector<uint8_t>& valid, const std::vector<KeyLine>* base,
                        std::vector<KeyLine>& new_kls,
                        std::vector<std::pair<int, int>>& match_indices) {
  const int M = (int)ml.size(), NLc = F.NL;
  std::vector<float> xyz(6 * (size_t)(M > 0 ? M : 1), 0.f);
  std::vector<int32_t> mlNobs(M > 0 ? M : 1, 0);
  cv::Mat desc(M > 0 ? M : 1, 32, cv::CV_8U);
  for (int i = 0; i < M; i++) {
    const MapLine* l = ml[i];
    if (!l) continue;
    for (int k = 0; k < 3; k++) {
      xyz[6 * i + k] = (float)l->mStart3d[k];
      xyz[6 * i + 3 + k] = (float)l->mEnd3d[k];
    }
    std::memcpy(desc.ptr<uint8_t>(i), l->mLineDescriptor.data, 32);
    mlNobs[i] = l->Observations();
  }
  std::vector<int32_t> curNobs(NLc > 0 ? NLc : 1, 0), match(NLc > 0 ? NLc : 1, -1);
  for (int j = 0; j < NLc; j++)
    if (F.mvpMapLines[j]) curNobs[j] = F.mvpMapLines[j]->Observations();
  std::vector<KeyLine> proj(M > 0 ? M : 1);
  std::vector<int32_t> src(M > 0 ? M : 1, -1);
  const int cap = std::max(1, NLc * M);
  std::vector<int32_t> pairs(2 * (size_t)cap);
  const orbpl_camera cam = F.Camera();
  int n = 0, wiped = 0, nproj = 0, npairs = 0;
  if (orbl_search_by_projection_pairs(
          &cam, F.mTcw.ptr<float>(), mode, NLc,
          reinterpret_cast<const orbpl_keyline*>(F.mvKeyLinesUn.data()), F.mLineDescriptors.data,
          curNobs.data(), M, valid.data(),
          base ? reinterpret_cast<const orbpl_keyline*>(base->data()) : nullptr, xyz.data(),
          desc.data, mlNobs.data(), reinterpret_cast<orbpl_keyline*>(proj.data()), src.data(),
          &nproj, pairs.data(), cap, &npairs, match.data(), &n, &wiped) != ORBPL_OK)
    throw std::runtime_error(orbpl_last_error());
  new_kls.insert(new_kls.end(), proj.begin(), proj.begin() + nproj);
  if (wiped) match_indices.clear();   // the retry clears; the first pass appends
  for (int k = 0; k < std::min(npairs, cap); k++)
    match_indices.emplace_back(pairs[2 * k], pairs[2 * k + 1]);
  if (wiped) std::fill(F.mvpMapLines.begin(), F.mvpMapLines.end(), nullptr);
  for (int j = 0; j < NLc; j++)
    if (match[j] >= 0) F.mvpMapLines[j] = ml[match[j]];
  return n;
}

// LineMatcher.cpp:272-487 (Test/LastFrameProjection.cpp:293)
int LineMatcher::SearchByProjection(Frame& Cur, const Frame& Last, std::vector<KeyLine>& new_kls,
                                    std::vector<std::pair<int, int>>& match_indices) {
  const int NL = Last.NL;
  std::vector<uint8_t> valid(NL > 0 ? NL : 1, 0);
  for (int i = 0; i < NL; i++) {   // :303-311
    const MapLine* l = Last.mvpMapLines[i];
    valid[i] = l && !Last.mvbLineOutlier[i] && !l->isBad();
  }
  return search_pairs(Cur, 0, Last.mvpMapLines, valid, &Last.mvKeyLinesUn, new_kls,
                      match_indices);
}

// LineMatcher.cpp:954-1170 (Test/LocalMapProjectionTest.cpp:334)
int LineMatcher::SearchByProjection(Frame& F, const std::vector<MapLine*>& vpMapLines,
                                    std::vector<KeyLine>& new_kls,
                                    std::vector<std::pair<int, int>>& match_indices) {
  std::vector<uint8_t> valid(vpMapLines.size() > 0 ? vpMapLines.size() : 1, 0);
  for (size_t i = 0; i < vpMapLines.size(); i++)   // :991-997
    valid[i] = vpMapLines[i]->mbTrackInView && !vpMapLines[i]->isBad();
  return search_pairs(F, 1, vpMapLines, valid, nullptr, new_kls, match_indices);
}

// LineMatcher.cpp:492-525: knnMatch(RefFrame lines, current lines, 2), ratio
// 0.75; vpMapLineMatches (size NL) gets the keyframe's map line of each
// passing query at its best current line (NULL entries included, as there)
int LineMatcher::SearchByProjection(Frame& CurrentFrame, KeyFrame* RefFrame,
                                    std::vector<MapLine*>& vpMapLineMatches) {
  vpMapLineMatches.assign(CurrentFrame.NL, nullptr);
  const std::vector<MapLine*> vpMapLinesKF = RefFrame->GetMapLineMatches();
  const int nq = RefFrame->mLineDescriptors.rows, nt = CurrentFrame.mLineDescriptors.rows;
  std::vector<int32_t> out(nt > 0 ? nt : 1, -1);
  int n = 0;
  if (orbl_match_bf_knn(nq, RefFrame->mLineDescriptors.data, nt, CurrentFrame.mLineDescriptors.data,
                        out.data(), &n) != ORBPL_OK)
    throw std::runtime_error(orbpl_last_error());
  for (int j = 0; j < nt && j < CurrentFrame.NL; j++)
    if (out[j] >= 0) vpMapLineMatches[j] = vpMapLinesKF[out[j]];
  return n;
}

}  // namespace ORB_SLAM2
