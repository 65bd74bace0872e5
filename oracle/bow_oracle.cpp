// ORACLE — test infrastructure only (see orb_oracle.cpp header): never linked
// into liborbpl.so, loaded only by tests/ and bench.py's cpu_baseline.
//
// DBoW2's ORB vocabulary (ORBVocabulary = TemplatedVocabulary<FORB::TDescriptor,
// FORB>) restated with the reference's own stream semantics:
//   loadFromTextFile      Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1338-1420
//                         (getline until eof: a file that ends with '\n' yields
//                         one more, empty line, whose parent the reference
//                         reads from an indeterminate int; pinned P19: no node)
//   transform(features, BowVector, FeatureVector, levelsup)   :1127-1205
//   transform(feature, word_id, weight, nid, levelsup)         :1226-1262
//   FORB::distance        Thirdparty/DBoW2/DBoW2/FORB.cpp:81-101
//   BowVector::addWeight / addIfNotExist / normalize           BowVector.cpp
//   FeatureVector::addFeature                                  FeatureVector.cpp:31-45
// Frame::ComputeBoW calls transform(desc, mBowVec, mFeatVec, 4) (Frame.cc:730).
#include <cmath>
#include <cstdint>
#include <cstring>
#include <fstream>
#include <map>
#include <sstream>
#include <string>
#include <vector>

namespace bow_oracle {

struct Node {
  int parent = 0;
  std::vector<int> children;
  uint8_t desc[32] = {0};
  double weight = 0;
  int word_id = 0;          // Node(): word_id(0)
};

struct Voc {
  int k = 0, L = 0, scoring = 0, weighting = 0;
  std::vector<Node> nodes;
  int nwords = 0;
};

static int distance(const uint8_t* a, const uint8_t* b) {
  int d = 0;
  for (int i = 0; i < 8; i++) {
    uint32_t x, y;
    std::memcpy(&x, a + 4 * i, 4);
    std::memcpy(&y, b + 4 * i, 4);
    d += __builtin_popcount(x ^ y);
  }
  return d;
}

// enum ScoringType {L1_NORM, L2_NORM, CHI_SQUARE, KL, BHATTACHARYYA, DOT_PRODUCT}
// mustNormalize (ScoringObject.h): L1 for L1/CHI_SQUARE/KL/BHATTACHARYYA, L2
// for L2_NORM, none for DOT_PRODUCT. Returns 0 none, 1 L1, 2 L2.
static int norm_kind(int scoring) {
  switch (scoring) {
    case 0: case 2: case 3: case 4: return 1;
    case 1: return 2;
    default: return 0;
  }
}

// transform of one feature: propagate down the tree (strict <: the first
// child of minimal distance), the node at level L - levelsup
static void transform_one(const Voc& v, const uint8_t* f, int levelsup, int& word, double& w,
                          int& nid) {
  const int nid_level = v.L - levelsup;
  if (nid_level <= 0) nid = 0;
  int final_id = 0, level = 0;
  do {
    ++level;
    const std::vector<int>& ch = v.nodes[final_id].children;
    final_id = ch[0];
    int best = distance(f, v.nodes[final_id].desc);
    for (size_t q = 1; q < ch.size(); q++) {
      const int d = distance(f, v.nodes[ch[q]].desc);
      if (d < best) {
        best = d;
        final_id = ch[q];
      }
    }
    if (level == nid_level) nid = final_id;
  } while (!v.nodes[final_id].children.empty());
  // P20: a leaf above level L - levelsup leaves the reference's nid
  // unassigned; the restatement reports the leaf
  if (level < nid_level) nid = final_id;
  word = v.nodes[final_id].word_id;
  w = v.nodes[final_id].weight;
}

}  // namespace bow_oracle

using namespace bow_oracle;

extern "C" {

void* oracle_voc_load_text(const char* path) {
  std::ifstream f(path);
  if (!f.is_open() || f.eof()) return nullptr;
  Voc* v = new Voc();
  std::string s;
  std::getline(f, s);
  std::stringstream ss;
  ss << s;
  int n1 = -1, n2 = -1;
  ss >> v->k >> v->L >> n1 >> n2;
  if (v->k < 0 || v->k > 20 || v->L < 1 || v->L > 10 || n1 < 0 || n1 > 5 || n2 < 0 || n2 > 3) {
    delete v;
    return nullptr;
  }
  v->scoring = n1;
  v->weighting = n2;
  v->nodes.resize(1);
  while (!f.eof()) {
    std::string sn;
    std::getline(f, sn);
    std::stringstream sl;
    sl << sn;
    const int nid = (int)v->nodes.size();
    int pid = 0;
    // P19: a line without tokens (the one after a final '\n') leaves the
    // reference's pid indeterminate (the stream's sentry fails before the
    // extraction); it makes no node here
    if (!(sl >> pid)) continue;
    v->nodes.resize(v->nodes.size() + 1);
    if (pid < 0 || pid >= nid) {
      delete v;
      return nullptr;
    }
    v->nodes[nid].parent = pid;
    v->nodes[pid].children.push_back(nid);
    int leaf = 0;
    sl >> leaf;
    std::stringstream sd;
    for (int i = 0; i < 32; i++) {
      std::string e;
      sl >> e;
      sd << e << " ";
    }
    for (int i = 0; i < 32; i++) {   // FORB::fromString
      int x;
      sd >> x;
      if (!sd.fail()) v->nodes[nid].desc[i] = (uint8_t)x;
    }
    double w = 0;
    sl >> w;
    v->nodes[nid].weight = w;
    if (leaf > 0) v->nodes[nid].word_id = v->nwords++;
  }
  return v;
}

// the same tree from flat node arrays (node 0 = root, parent[i] < i; word
// ids follow the leaf flags in node order), e.g. the bench's shared vocabulary
void* oracle_voc_create(int k, int L, int scoring, int weighting, int n_nodes,
                        const int32_t* parent, const uint8_t* leaf, const uint8_t* desc,
                        const double* weight) {
  if (n_nodes < 1) return nullptr;
  Voc* v = new Voc();
  v->k = k;
  v->L = L;
  v->scoring = scoring;
  v->weighting = weighting;
  v->nodes.resize(n_nodes);
  for (int i = 1; i < n_nodes; i++) {
    if (parent[i] < 0 || parent[i] >= i) {
      delete v;
      return nullptr;
    }
    Node& nd = v->nodes[i];
    nd.parent = parent[i];
    v->nodes[parent[i]].children.push_back(i);
    std::memcpy(nd.desc, desc + 32 * (size_t)i, 32);
    nd.weight = weight[i];
    if (leaf[i]) nd.word_id = v->nwords++;
  }
  return v;
}

void oracle_voc_destroy(void* h) { delete static_cast<Voc*>(h); }

int oracle_voc_info(void* h, int* out6) {
  const Voc* v = static_cast<const Voc*>(h);
  out6[0] = v->k;
  out6[1] = v->L;
  out6[2] = v->scoring;
  out6[3] = v->weighting;
  out6[4] = (int)v->nodes.size();
  out6[5] = v->nwords;
  return 0;
}

// flat node arrays (node 0 = root): parent (-1 for the root), leaf flag
// (children empty), word id, weight, descriptor rows
int oracle_voc_nodes(void* h, int32_t* parent, uint8_t* leaf, int32_t* word, double* weight,
                     uint8_t* desc) {
  const Voc* v = static_cast<const Voc*>(h);
  for (size_t i = 0; i < v->nodes.size(); i++) {
    const Node& n = v->nodes[i];
    parent[i] = i ? n.parent : -1;
    leaf[i] = n.children.empty() ? 1 : 0;
    word[i] = n.word_id;
    weight[i] = n.weight;
    std::memcpy(desc + 32 * i, n.desc, 32);
  }
  return 0;
}

// TemplatedVocabulary::transform(features, BowVector, FeatureVector, levelsup):
// BowVector as (word, value) in word order; FeatureVector as the node of
// every feature (-1: stopped word, not in the FeatureVector); also the
// per-feature word and weight.
int oracle_voc_transform(void* h, const uint8_t* desc, int n, int levelsup, uint32_t* bow_words,
                         double* bow_vals, int* bow_n, int32_t* feat_node, int32_t* feat_word,
                         double* feat_weight) {
  const Voc* v = static_cast<const Voc*>(h);
  std::map<uint32_t, double> bv;   // BowVector : std::map<WordId, WordValue>
  *bow_n = 0;
  if (v->nodes.size() <= 1 || v->nodes[0].children.empty()) {
    for (int i = 0; i < n; i++) feat_node[i] = -1;
    return 0;
  }
  const int nk = norm_kind(v->scoring);
  const bool tf = v->weighting == 0 || v->weighting == 1;   // TF_IDF, TF
  for (int i = 0; i < n; i++) {
    int word = 0, nid = 0;
    double w = 0;
    transform_one(*v, desc + 32 * (size_t)i, levelsup, word, w, nid);
    feat_word[i] = word;
    feat_weight[i] = w;
    feat_node[i] = -1;
    if (w > 0) {
      auto it = bv.lower_bound((uint32_t)word);
      if (it != bv.end() && it->first == (uint32_t)word) {
        if (tf) it->second += w;             // addWeight
      } else {
        bv.insert(it, {(uint32_t)word, w});   // addWeight / addIfNotExist
      }
      feat_node[i] = nid;                     // fv.addFeature(nid, i)
    }
  }
  if (tf && !bv.empty() && nk == 0) {
    const double nd = (double)bv.size();
    for (auto& e : bv) e.second /= nd;
  }
  if (nk) {   // BowVector::normalize
    double norm = 0.0;
    if (nk == 1)
      for (auto& e : bv) norm += std::fabs(e.second);
    else {
      for (auto& e : bv) norm += e.second * e.second;
      norm = std::sqrt(norm);
    }
    if (norm > 0.0)
      for (auto& e : bv) e.second /= norm;
  }
  int k = 0;
  for (auto& e : bv) {
    bow_words[k] = e.first;
    bow_vals[k] = e.second;
    k++;
  }
  *bow_n = k;
  return 0;
}

}  // extern "C"
