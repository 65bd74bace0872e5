// DBoW2 ORB vocabulary on gfx950 (restated in oracle/bow_oracle.cpp):
//   host          TemplatedVocabulary::loadFromTextFile (Thirdparty/DBoW2/DBoW2/
//                 TemplatedVocabulary.h:1338-1420) as one pass over the file
//                 with the same line semantics (P19: a line without tokens
//                 makes no node); node arrays in CSR form for the device
//   k_bow_words   transform(feature, word_id, weight, nid, levelsup)
//                 (:1226-1262): one lane per feature walks the tree, the
//                 children of its node compared in order (strict <: the first
//                 child of minimal FORB::distance, FORB.cpp:81-101)
//   k_bow_vector  transform(features, BowVector, FeatureVector, levelsup)
//                 (:1127-1205) per frame: (word, feature) keys sorted in LDS;
//                 a word's weights summed in feature order (BowVector::
//                 addWeight) or its first kept (addIfNotExist); the L1 / L2
//                 norm (BowVector::normalize) summed by one lane in word order
// Frame::ComputeBoW is transform(desc, mBowVec, mFeatVec, 4) (Frame.cc:730).
// The FeatureVector is returned as the node of every feature (-1: stopped
// word), the form orbm_search_by_bow takes.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cerrno>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/orbpl.h"
#include "orbpl_runtime.h"

namespace orbpl {
namespace {

constexpr int kBowMaxFeat = 4096;   // features per frame (sort keys: index < 2^12)
constexpr uint32_t kNoKey = 0xFFFFFFFFu;

struct VocDev {
  const int32_t* child_start;   // [n_nodes + 1]
  const int32_t* child;         // children of every node, in id order
  const uint4* desc;            // [n_nodes][2]
  const int32_t* word;          // word id (0 for non-word nodes, Node())
  const double* weight;
  int L;
  int norm;                     // 0 none, 1 L1, 2 L2 (ScoringObject::mustNormalize)
  int tf;                       // TF / TF_IDF: addWeight, else addIfNotExist
};

struct BowBatch {
  const uint8_t* desc;          // frame f at desc + f * desc_pitch * 32
  long long desc_pitch;
  const int* n;                 // features per frame
  int levelsup;
  int32_t* feat_node;           // [f * out_pitch + i]
  int32_t* feat_word;
  double* feat_weight;
  uint32_t* bow_words;          // [f * out_pitch + r]
  double* bow_vals;
  int* bow_n;
  long long out_pitch;
  int* err;                     // bit 1: more than kBowMaxFeat (or cap) features
  int cap;                      // k_bow_vector's LDS keys: a power of two >= max_n
};

}  // namespace

// the descriptor of node c: a 32-bit byte offset from the (uniform) node
// descriptor base (n_nodes * 32 B < 2^32)
__device__ __forceinline__ const uint4* node_desc(const uint4* base, int c) {
  return reinterpret_cast<const uint4*>(reinterpret_cast<const char*>(base) + ((uint32_t)c << 5));
}

// Children compared per level: up to kBowBatch of them have their ids and
// descriptors loaded together before any distance is taken (the loads of a
// level are then one dependent round instead of one per child); the
// distances are compared in child order, so the first minimum wins as in
// the reference loop.
constexpr int kBowBatch = 10;   // the k of ORBvoc (and the bench vocabulary)

__global__ void __launch_bounds__(256) k_bow_words(VocDev v, BowBatch b) {
  const int f = blockIdx.y, i = blockIdx.x * 256 + threadIdx.x;
  const int n = b.n[f];
  if (i >= n) return;
  const uint4* d = reinterpret_cast<const uint4*>(b.desc + ((long long)f * b.desc_pitch + i) * 32);
  const uint4 a0 = d[0], a1 = d[1];
  const int nid_level = v.L - b.levelsup;
  int nid = 0, node = 0, level = 0;
  while (true) {
    const int cs = v.child_start[node], ce = v.child_start[node + 1];
    if (cs == ce) break;   // isLeaf(): children empty
    ++level;
    int best = -1, bd = 0x7fffffff;
    for (int q0 = cs; q0 < ce; q0 += kBowBatch) {
      const int m = min(kBowBatch, ce - q0);
      int c[kBowBatch];
#pragma unroll
      for (int k = 0; k < kBowBatch; k++) c[k] = k < m ? v.child[q0 + k] : 0;
      uint4 e0[kBowBatch], e1[kBowBatch];
#pragma unroll
      for (int k = 0; k < kBowBatch; k++) {
        if (k < m) {
          const uint4* p = node_desc(v.desc, c[k]);
          e0[k] = p[0];
          e1[k] = p[1];
        }
      }
#pragma unroll
      for (int k = 0; k < kBowBatch; k++) {
        if (k < m) {
          const int dd = __popc(a0.x ^ e0[k].x) + __popc(a0.y ^ e0[k].y) + __popc(a0.z ^ e0[k].z) +
                         __popc(a0.w ^ e0[k].w) + __popc(a1.x ^ e1[k].x) + __popc(a1.y ^ e1[k].y) +
                         __popc(a1.z ^ e1[k].z) + __popc(a1.w ^ e1[k].w);
          if (best < 0 || dd < bd) {
            bd = dd;
            best = c[k];
          }
        }
      }
    }
    node = best;
    if (level == nid_level) nid = node;
  }
  if (level < nid_level) nid = node;   // P20 (oracle transform_one)
  const double w = v.weight[node];
  const long long o = (long long)f * b.out_pitch + i;
  b.feat_word[o] = v.word[node];
  b.feat_weight[o] = w;
  b.feat_node[o] = w > 0 ? nid : -1;
}

// LDS sized by the batch's feature cap (b.cap: 12 KB at 1000 features
// instead of a static 48 KB, so more frames share a CU)
__global__ void __launch_bounds__(256) k_bow_vector(VocDev v, BowBatch b) {
  extern __shared__ double bow_dyn[];
  double* sval = bow_dyn;                                        // BowVector values in word order
  uint32_t* key = reinterpret_cast<uint32_t*>(bow_dyn + b.cap);  // sort keys
  __shared__ int wsum[4];
  __shared__ double s_norm;
  const int f = blockIdx.x, t = threadIdx.x, lane = t & 63, wave = t >> 6;
  int n = b.n[f];
  if (n > b.cap) {
    if (t == 0) atomicOr(b.err, 2);
    n = b.cap;
  }
  const long long o = (long long)f * b.out_pitch;
  int np = 1;
  while (np < n) np <<= 1;
  for (int i = t; i < np; i += 256) {
    uint32_t k = kNoKey;
    if (i < n && b.feat_weight[o + i] > 0) k = ((uint32_t)b.feat_word[o + i] << 12) | (uint32_t)i;
    key[i] = k;
  }
  __syncthreads();
  for (int kk = 2; kk <= np; kk <<= 1)
    for (int j = kk >> 1; j > 0; j >>= 1) {
      for (int i = t; i < np; i += 256) {
        const int l = i ^ j;
        if (l > i) {
          const uint32_t x = key[i], y = key[l];
          if (((i & kk) == 0) ? (x > y) : (x < y)) {
            key[i] = y;
            key[l] = x;
          }
        }
      }
      __syncthreads();
    }
  // runs of one word: thread t owns positions [t * per, (t + 1) * per)
  const int per = (np + 255) / 256;
  const int p0 = min(np, t * per), p1 = min(np, p0 + per);
  int starts = 0;
  for (int p = p0; p < p1; p++)
    starts += key[p] != kNoKey && (p == 0 || (key[p - 1] >> 12) != (key[p] >> 12));
  int incl = starts;
#pragma unroll
  for (int s = 1; s < 64; s <<= 1) {
    const int u = __shfl_up(incl, s, 64);
    if (lane >= s) incl += u;
  }
  if (lane == 63) wsum[wave] = incl;
  __syncthreads();
  int r = incl - starts;
  for (int w = 0; w < wave; w++) r += wsum[w];
  const int nruns = wsum[0] + wsum[1] + wsum[2] + wsum[3];
  for (int p = p0; p < p1; p++) {
    const uint32_t k = key[p];
    if (k == kNoKey || !(p == 0 || (key[p - 1] >> 12) != (k >> 12))) continue;
    double val = b.feat_weight[o + (k & 4095u)];
    if (v.tf)
      for (int q = p + 1; q < np && key[q] != kNoKey && (key[q] >> 12) == (k >> 12); q++)
        val += b.feat_weight[o + (key[q] & 4095u)];
    b.bow_words[o + r] = k >> 12;
    sval[r] = val;
    r++;
  }
  __syncthreads();
  double div = 1.0;
  if (v.norm == 0 && v.tf && nruns > 0) {
    div = (double)nruns;
  } else if (v.norm) {
    if (t == 0) {
      // one sequential sum in word order (BowVector::normalize), loads from
      // LDS eight ahead of the dependent adds
      double norm = 0.0;
      int q = 0;
      for (; q + 8 <= nruns; q += 8) {
        double x[8];
#pragma unroll
        for (int u = 0; u < 8; u++) x[u] = sval[q + u];
#pragma unroll
        for (int u = 0; u < 8; u++) norm += v.norm == 1 ? fabs(x[u]) : x[u] * x[u];
      }
      for (; q < nruns; q++) norm += v.norm == 1 ? fabs(sval[q]) : sval[q] * sval[q];
      if (v.norm == 2) norm = sqrt(norm);
      s_norm = norm;
    }
    __syncthreads();
    div = s_norm > 0.0 ? s_norm : 1.0;
  }
  const bool scale = (v.norm == 0 && v.tf) || (v.norm && s_norm > 0.0);
  for (int q = t; q < nruns; q += 256) b.bow_vals[o + q] = scale ? sval[q] / div : sval[q];
  if (t == 0) b.bow_n[f] = nruns;
}

namespace {

int norm_of(int scoring) {
  switch (scoring) {
    case 0: case 2: case 3: case 4: return 1;
    case 1: return 2;
    default: return 0;
  }
}

}  // namespace
}  // namespace orbpl

using namespace orbpl;

#define HIP_CHECK(expr)                                              \
  do {                                                               \
    hipError_t e_ = (expr);                                          \
    if (e_ != hipSuccess) return orbpl::hip_fail(e_, #expr, __LINE__); \
  } while (0)

// One device's copy of the tree (orbv_upload): trackers on different GPUs may
// share one vocabulary, so every device keeps its own buffers until
// orbv_destroy.
struct VocCopy {
  int device = -1;
  int32_t *d_child_start = nullptr, *d_child = nullptr, *d_word = nullptr;
  uint8_t* d_desc = nullptr;
  double* d_weight = nullptr;
  // host-API scratch (one frame)
  int host_cap = 0;
  uint8_t* h_desc = nullptr;
  int* h_n = nullptr;
  int32_t *h_node = nullptr, *h_word = nullptr;
  double *h_wt = nullptr, *h_vals = nullptr;
  uint32_t* h_words = nullptr;
  int *h_bn = nullptr, *h_err = nullptr;
  hipStream_t stream = nullptr;
};

struct orbv_vocab {
  int k = 0, L = 0, scoring = 0, weighting = 0;
  std::vector<int32_t> parent;   // -1 for the root
  std::vector<uint8_t> leaf_flag, desc;
  std::vector<double> weight;
  std::vector<int32_t> word;
  int n_words = 0;
  std::vector<int32_t> child_start, child;
  // one per device the tree was uploaded to; a deque keeps the handed-out
  // pointers valid while another thread uploads to a further device, `mu`
  // guards the list, `host_mu` the host-pointer transform's scratch
  std::deque<VocCopy> copies;
  std::mutex mu, host_mu;
  VocCopy* on(int device) {
    std::lock_guard<std::mutex> g(mu);
    for (auto& c : copies)
      if (c.device == device) return &c;
    return nullptr;
  }
};

namespace {

int build_csr(orbv_vocab* v) {
  const int nn = (int)v->parent.size();
  v->child_start.assign(nn + 1, 0);
  for (int i = 1; i < nn; i++) {
    const int p = v->parent[i];
    if (p < 0 || p >= i) return arg_fail("vocabulary: a node's parent must precede it");
    v->child_start[p + 1]++;
  }
  for (int i = 0; i < nn; i++) v->child_start[i + 1] += v->child_start[i];
  v->child.assign(nn > 0 ? nn - 1 : 0, 0);
  std::vector<int32_t> fill(v->child_start.begin(), v->child_start.end() - 1);
  for (int i = 1; i < nn; i++) v->child[fill[v->parent[i]]++] = i;   // id order
  v->word.assign(nn, 0);
  v->n_words = 0;
  for (int i = 0; i < nn; i++)
    if (v->leaf_flag[i]) v->word[i] = v->n_words++;
  if (v->n_words > (1 << 20)) return arg_fail("vocabulary: more than 2^20 words");
  if (nn >= (1 << 21) - 1) return arg_fail("vocabulary: more than 2^21 - 2 nodes");
  return ORBPL_OK;
}

void free_copy(VocCopy* c) {
  if (c->device < 0) return;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  (void)hipFree(c->d_child_start);
  (void)hipFree(c->d_child);
  (void)hipFree(c->d_word);
  (void)hipFree(c->d_desc);
  (void)hipFree(c->d_weight);
  (void)hipFree(c->h_desc);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  *c = VocCopy{};
}

// one whitespace-separated token of [p, e) (stringstream >> semantics)
bool next_token(const char*& p, const char* e, const char** tb, const char** te) {
  while (p < e && (*p == ' ' || *p == '\t' || *p == '\r' || *p == '\v' || *p == '\f')) p++;
  if (p >= e) return false;
  *tb = p;
  while (p < e && !(*p == ' ' || *p == '\t' || *p == '\r' || *p == '\v' || *p == '\f')) p++;
  *te = p;
  return true;
}

bool parse_int(const char* b, const char* e, long* out) {
  std::string s(b, e);
  char* end = nullptr;
  errno = 0;
  const long x = strtol(s.c_str(), &end, 10);
  if (end == s.c_str() || errno) return false;
  *out = x;
  return true;
}

}  // namespace

extern "C" {

int orbv_create(int k, int L, int scoring, int weighting, int n_nodes, const int32_t* parent,
                const uint8_t* leaf_flag, const uint8_t* desc, const double* weight,
                orbv_vocab** out) {
  if (!out || !parent || !leaf_flag || !desc || !weight || n_nodes < 1)
    return arg_fail("orbv_create: bad argument");
  if (k < 0 || k > 20 || L < 1 || L > 10 || scoring < 0 || scoring > 5 || weighting < 0 ||
      weighting > 3)
    return arg_fail("orbv_create: k / L / scoring / weighting out of range");
  orbv_vocab* v = new orbv_vocab();
  v->k = k;
  v->L = L;
  v->scoring = scoring;
  v->weighting = weighting;
  v->parent.assign(parent, parent + n_nodes);
  v->parent[0] = -1;
  v->leaf_flag.assign(leaf_flag, leaf_flag + n_nodes);
  v->leaf_flag[0] = 0;
  v->desc.assign(desc, desc + 32 * (size_t)n_nodes);
  v->weight.assign(weight, weight + n_nodes);
  const int rc = build_csr(v);
  if (rc) {
    delete v;
    return rc;
  }
  *out = v;
  return ORBPL_OK;
}

int orbv_load_text(const char* path, orbv_vocab** out) {
  if (!path || !out) return arg_fail("orbv_load_text: NULL argument");
  FILE* fp = fopen(path, "rb");
  if (!fp) return arg_fail("orbv_load_text: cannot open the file");
  std::string buf;
  char tmp[1 << 16];
  size_t r;
  while ((r = fread(tmp, 1, sizeof(tmp), fp)) > 0) buf.append(tmp, r);
  fclose(fp);
  if (buf.empty()) return arg_fail("orbv_load_text: empty file");
  const char* p = buf.data();
  const char* e = p + buf.size();
  const char* nl = (const char*)memchr(p, '\n', e - p);
  const char* he = nl ? nl : e;
  long hv[4] = {-1, -1, -1, -1};
  {
    const char* q = p;
    for (int i = 0; i < 4; i++) {
      const char *tb, *te;
      if (!next_token(q, he, &tb, &te) || !parse_int(tb, te, &hv[i])) break;
    }
  }
  std::vector<int32_t> parent(1, -1);
  std::vector<uint8_t> leaf(1, 0), desc(32, 0);
  std::vector<double> weight(1, 0.0);
  // node lines: what follows the header, split at '\n' (getline until eof)
  const char* q = nl ? nl + 1 : e;
  while (nl) {
    const char* le = (const char*)memchr(q, '\n', e - q);
    const char* lend = le ? le : e;
    const char* c = q;
    const char *tb, *te;
    long pid;
    if (next_token(c, lend, &tb, &te) && parse_int(tb, te, &pid)) {   // P19
      const int nid = (int)parent.size();
      if (pid < 0 || pid >= nid) return arg_fail("orbv_load_text: bad parent id");
      parent.push_back((int32_t)pid);
      long lf = 0;
      if (next_token(c, lend, &tb, &te)) parse_int(tb, te, &lf);
      uint8_t d[32] = {0};
      for (int i = 0; i < 32; i++) {   // FORB::fromString
        long x;
        if (!next_token(c, lend, &tb, &te)) break;
        if (parse_int(tb, te, &x)) d[i] = (uint8_t)x;
      }
      desc.insert(desc.end(), d, d + 32);
      double w = 0.0;
      if (next_token(c, lend, &tb, &te)) {
        std::string s(tb, te);
        char* end = nullptr;
        const double x = strtod(s.c_str(), &end);
        if (end != s.c_str()) w = x;
      }
      weight.push_back(w);
      leaf.push_back(lf > 0 ? 1 : 0);
    }
    if (!le) break;
    q = le + 1;
  }
  return orbv_create((int)hv[0], (int)hv[1], (int)hv[2], (int)hv[3], (int)parent.size(),
                     parent.data(), leaf.data(), desc.data(), weight.data(), out);
}

int orbv_destroy(orbv_vocab* v) {
  if (!v) return ORBPL_OK;
  for (auto& c : v->copies) free_copy(&c);
  delete v;
  return ORBPL_OK;
}

int orbv_info(const orbv_vocab* v, int* out6) {
  if (!v || !out6) return arg_fail("orbv_info: NULL argument");
  out6[0] = v->k;
  out6[1] = v->L;
  out6[2] = v->scoring;
  out6[3] = v->weighting;
  out6[4] = (int)v->parent.size();
  out6[5] = v->n_words;
  return ORBPL_OK;
}

int orbv_export(const orbv_vocab* v, int32_t* parent, uint8_t* leaf_flag, uint8_t* desc,
                double* weight) {
  if (!v || !parent || !leaf_flag || !desc || !weight) return arg_fail("orbv_export: NULL argument");
  memcpy(parent, v->parent.data(), 4 * v->parent.size());
  memcpy(leaf_flag, v->leaf_flag.data(), v->leaf_flag.size());
  memcpy(desc, v->desc.data(), v->desc.size());
  memcpy(weight, v->weight.data(), 8 * v->weight.size());
  return ORBPL_OK;
}

int orbv_upload(orbv_vocab* v, int device) {
  if (!v) return arg_fail("orbv_upload: NULL vocabulary");
  std::lock_guard<std::mutex> g(v->mu);
  for (auto& c : v->copies)
    if (c.device == device) return ORBPL_OK;
  HIP_CHECK(hipSetDevice(device));
  const size_t nn = v->parent.size();
  VocCopy c;
  c.device = device;
  hipError_t e = hipMalloc(&c.d_child_start, 4 * (nn + 1));
  if (e == hipSuccess) e = hipMalloc(&c.d_child, 4 * std::max<size_t>(1, v->child.size()));
  if (e == hipSuccess) e = hipMalloc(&c.d_word, 4 * nn);
  if (e == hipSuccess) e = hipMalloc(&c.d_desc, 32 * nn);
  if (e == hipSuccess) e = hipMalloc(&c.d_weight, 8 * nn);
  if (e == hipSuccess) e = hipMemcpy(c.d_child_start, v->child_start.data(), 4 * (nn + 1), hipMemcpyHostToDevice);
  if (e == hipSuccess && !v->child.empty())
    e = hipMemcpy(c.d_child, v->child.data(), 4 * v->child.size(), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(c.d_word, v->word.data(), 4 * nn, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(c.d_desc, v->desc.data(), 32 * nn, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(c.d_weight, v->weight.data(), 8 * nn, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&c.stream, hipStreamNonBlocking);
  if (e != hipSuccess) {
    free_copy(&c);
    return hip_fail(e, "orbv_upload", __LINE__);
  }
  v->copies.push_back(c);
  return ORBPL_OK;
}

int orbv_transform_batch_device(orbv_vocab* v, const uint8_t* d_desc, int64_t desc_pitch,
                                const int* d_n, int nframes, int max_n, int levelsup,
                                int32_t* d_feat_node, int32_t* d_feat_word, double* d_feat_weight,
                                uint32_t* d_bow_words, double* d_bow_vals, int* d_bow_n,
                                int64_t out_pitch, int* d_err, void* stream) {
  if (!v || !d_desc || !d_n || !d_feat_node || !d_feat_word || !d_feat_weight || !d_bow_words ||
      !d_bow_vals || !d_bow_n || !d_err)
    return arg_fail("orbv_transform_batch_device: NULL argument");
  // the copy of the calling thread's current device (the tracker sets it)
  int dev = -1;
  HIP_CHECK(hipGetDevice(&dev));
  VocCopy* c = v->on(dev);
  if (!c) return arg_fail("orbv_transform_batch_device: vocabulary not uploaded to this device");
  if (nframes <= 0 || max_n < 0) return ORBPL_OK;
  if (max_n > kBowMaxFeat || out_pitch < max_n || desc_pitch < max_n)
    return arg_fail("orbv_transform_batch_device: max_n > 4096 or pitch < max_n");
  hipStream_t s = stream ? (hipStream_t)stream : c->stream;
  VocDev vd{c->d_child_start, c->d_child, reinterpret_cast<const uint4*>(c->d_desc), c->d_word,
            c->d_weight, v->L, norm_of(v->scoring), (v->weighting == 0 || v->weighting == 1) ? 1 : 0};
  if (v->parent.size() <= 1) {   // empty(): nothing is added
    HIP_CHECK(hipMemsetAsync(d_bow_n, 0, 4 * (size_t)nframes, s));
    HIP_CHECK(hipMemsetAsync(d_feat_node, 0xFF, 4 * (size_t)(out_pitch * nframes), s));
    return ORBPL_OK;
  }
  int cap = 1;
  while (cap < max_n) cap <<= 1;
  BowBatch b{d_desc, desc_pitch, d_n, levelsup, d_feat_node, d_feat_word, d_feat_weight,
             d_bow_words, d_bow_vals, d_bow_n, out_pitch, d_err, cap};
  if (max_n > 0)
    hipLaunchKernelGGL(k_bow_words, dim3((max_n + 255) / 256, nframes), dim3(256), 0, s, vd, b);
  set_smem_attr((const void*)k_bow_vector, (size_t)kBowMaxFeat * 12);
  hipLaunchKernelGGL(k_bow_vector, dim3(nframes), dim3(256), (size_t)cap * 12, s, vd, b);
  HIP_CHECK(hipGetLastError());
  return ORBPL_OK;
}

int orbv_transform(orbv_vocab* v, int device, const uint8_t* desc, int n, int levelsup,
                   uint32_t* bow_words, double* bow_vals, int* bow_n, int32_t* feat_node) {
  if (!v || (!desc && n > 0) || !bow_words || !bow_vals || !bow_n || (!feat_node && n > 0))
    return arg_fail("orbv_transform: NULL argument");
  if (n < 0 || n > kBowMaxFeat) return arg_fail("orbv_transform: n out of [0, 4096]");
  int rc = orbv_upload(v, device);
  if (rc) return rc;
  HIP_CHECK(hipSetDevice(device));
  std::lock_guard<std::mutex> g(v->host_mu);   // one host transform at a time
  VocCopy* c = v->on(device);
  if (!c->h_desc) {
    // one device block: desc | n | node | word | weight | words | vals | bow_n | err
    const size_t cap = kBowMaxFeat;
    const size_t bytes = cap * 32 + 64 + cap * 4 * 3 + cap * 8 * 2 + cap * 4 + 64;
    HIP_CHECK(hipMalloc(&c->h_desc, bytes));
    char* q = reinterpret_cast<char*>(c->h_desc) + cap * 32;
    c->h_n = reinterpret_cast<int*>(q);
    c->h_bn = c->h_n + 1;
    c->h_err = c->h_n + 2;
    q += 64;
    c->h_node = reinterpret_cast<int32_t*>(q);
    q += cap * 4;
    c->h_word = reinterpret_cast<int32_t*>(q);
    q += cap * 4;
    c->h_words = reinterpret_cast<uint32_t*>(q);
    q += cap * 4;
    c->h_wt = reinterpret_cast<double*>(q);
    q += cap * 8;
    c->h_vals = reinterpret_cast<double*>(q);
    c->host_cap = (int)cap;
  }
  if (n > 0) HIP_CHECK(hipMemcpyAsync(c->h_desc, desc, 32 * (size_t)n, hipMemcpyHostToDevice, c->stream));
  int hdr[3] = {n, 0, 0};
  HIP_CHECK(hipMemcpyAsync(c->h_n, hdr, sizeof(hdr), hipMemcpyHostToDevice, c->stream));
  rc = orbv_transform_batch_device(v, c->h_desc, kBowMaxFeat, c->h_n, 1, n, levelsup, c->h_node,
                                   c->h_word, c->h_wt, c->h_words, c->h_vals, c->h_bn, kBowMaxFeat,
                                   c->h_err, c->stream);
  if (rc) return rc;
  HIP_CHECK(hipMemcpyAsync(hdr, c->h_n, sizeof(hdr), hipMemcpyDeviceToHost, c->stream));
  HIP_CHECK(hipStreamSynchronize(c->stream));
  const int k = hdr[1];
  *bow_n = k;
  if (k > 0) {
    HIP_CHECK(hipMemcpy(bow_words, c->h_words, 4 * (size_t)k, hipMemcpyDeviceToHost));
    HIP_CHECK(hipMemcpy(bow_vals, c->h_vals, 8 * (size_t)k, hipMemcpyDeviceToHost));
  }
  if (n > 0) HIP_CHECK(hipMemcpy(feat_node, c->h_node, 4 * (size_t)n, hipMemcpyDeviceToHost));
  if (hdr[2]) return arg_fail("orbv_transform: feature capacity exceeded");
  return ORBPL_OK;
}

}  // extern "C"
