// Drop-in ORB_SLAM2::ORBVocabulary (include/ORBVocabulary.h: the DBoW2
// TemplatedVocabulary over FORB) reduced to what the hot path calls:
// loadFromTextFile (TemplatedVocabulary.h:1338-1420) and transform(features,
// BowVector, FeatureVector, levelsup) (:1127-1262), over orbv_load_text /
// orbv_transform (the tree walk and the BowVector build run on the MI355X).
// DBoW2's BowVector / FeatureVector are the std::map types the reference
// declares (BowVector.h:20-56, FeatureVector.h:21).
#pragma once
#include <map>
#include <stdexcept>
#include <string>
#include <vector>

#include "orbpl.h"
#include "cvmini.h"

namespace DBoW2 {
typedef unsigned int WordId;
typedef double WordValue;
typedef unsigned int NodeId;
class BowVector : public std::map<WordId, WordValue> {};
class FeatureVector : public std::map<NodeId, std::vector<unsigned int>> {};
}  // namespace DBoW2

namespace ORB_SLAM2 {

class ORBVocabulary {
 public:
  explicit ORBVocabulary(int device = 0) : device_(device) {}
  ~ORBVocabulary() { orbv_destroy(v_); }
  ORBVocabulary(const ORBVocabulary&) = delete;
  ORBVocabulary& operator=(const ORBVocabulary&) = delete;

  // TemplatedVocabulary::loadFromTextFile: false when the file cannot be read
  bool loadFromTextFile(const std::string& filename) {
    orbv_vocab* v = nullptr;
    if (orbv_load_text(filename.c_str(), &v) != ORBPL_OK) return false;
    orbv_destroy(v_);
    v_ = v;
    return true;
  }
  bool empty() const { return v_ == nullptr; }

  // TemplatedVocabulary::transform(features, v, fv, levelsup): one 32-byte
  // row per feature; fv lists each feature under its node at level L -
  // levelsup, in feature order
  void transform(const std::vector<cv::Mat>& features, DBoW2::BowVector& v,
                 DBoW2::FeatureVector& fv, int levelsup) const {
    v.clear();
    fv.clear();
    if (!v_) return;   // empty(): nothing is added
    const int n = (int)features.size();
    std::vector<uint8_t> desc(32 * (size_t)(n > 0 ? n : 1));
    for (int i = 0; i < n; i++) std::memcpy(&desc[32 * (size_t)i], features[i].data, 32);
    std::vector<uint32_t> words(n > 0 ? n : 1);
    std::vector<double> vals(n > 0 ? n : 1);
    std::vector<int32_t> node(n > 0 ? n : 1);
    int nb = 0;
    if (orbv_transform(v_, device_, desc.data(), n, levelsup, words.data(), vals.data(), &nb,
                       node.data()) != ORBPL_OK)
      throw std::runtime_error(orbpl_last_error());
    for (int k = 0; k < nb; k++) v[words[k]] = vals[k];
    for (int i = 0; i < n; i++)
      if (node[i] >= 0) fv[(DBoW2::NodeId)node[i]].push_back((unsigned)i);
  }

  orbv_vocab* handle() const { return v_; }

 private:
  orbv_vocab* v_ = nullptr;
  int device_;
};

// Converter::toDescriptorVector (Converter.cc:29-37): one row per descriptor
inline std::vector<cv::Mat> toDescriptorVector(const cv::Mat& Descriptors) {
  std::vector<cv::Mat> v;
  v.reserve(Descriptors.rows);
  for (int j = 0; j < Descriptors.rows; j++) v.push_back(Descriptors.row(j));
  return v;
}

}  // namespace ORB_SLAM2
