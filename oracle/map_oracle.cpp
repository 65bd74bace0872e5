// ORACLE — test infrastructure only (see orb_oracle.cpp header). Never linked
// into the product.
//
// Tracking::Track with the reference's map model: a CPU
// restatement of, per RGB-D frame,
//   Track()                     Tracking.cc:283-599
//   StereoInitialization        Tracking.cc:608-727
//   TrackReferenceKeyFrame      Tracking.cc:942-1032
//   UpdateLastFrame             Tracking.cc:1044-1210 (temporal VO points/lines)
//   TrackWithMotionModel        Tracking.cc:1212-1330
//   TrackLocalMap               Tracking.cc:1332-1420 (UpdateLocalMap :1867-2040,
//                               SearchLocalPoints/Lines :1746-1865)
//   NeedNewKeyFrame             Tracking.cc:1423-1557
//   CreateNewKeyFrame           Tracking.cc:1567-1745
// over a KeyFrame / MapPoint / MapLine model restating KeyFrame.cc (ctor :28-58,
// AddConnection / UpdateBestCovisibles :124-158, GetBestCovisibilityKeyFrames
// :175-183, TrackedMapPoints :284-309, UpdateConnections :363-452), MapPoint.cc
// (ctors, AddObservation, ComputeDistinctiveDescriptors :256-321,
// UpdateNormalAndDepth :344-385) and MapLine.cpp (ctors, AddObservation).
// The per-frame primitives are the oracle's own (orb/line/track oracles).
//
// Pinned:
//   P23 LocalMapping = its ProcessNewKeyFrame (LocalMapping.cc:186-240) run
//       synchronously when Tracking inserts a keyframe: AcceptKeyFrames() true,
//       never stopped, empty queue; no culling / triangulation / fusion / local
//       BA / keyframe culling (back end, out of scope). Relocalization is out of
//       scope: it fails, a LOST stream stays LOST (and resets while the map has
//       <= 5 keyframes, Tracking.cc:558-568).
//   P24 every container the reference orders by pointer (map<KeyFrame*, ..>,
//       set<KeyFrame*>, pair<int, KeyFrame*> ties) is ordered by keyframe id
//       (creation order).
//   P25 UpdateNormalAndDepth's float sums: normal_k += (P - Ow)_k * float(1 /
//       |P - Ow|) with the double norm of P16, the mean divided by float(n).
//   The first frame takes the tracker's reset pose (StereoInitialization's
//   identity when none is given); mMaxFrames = 30 (TUM fps); without a
//   vocabulary TrackReferenceKeyFrame is replaced by the motion model with
//   zero velocity (as the P18 tracker).
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <map>
#include <set>
#include <chrono>
#include <thread>
#include <vector>

#include "oracle_api.h"
#include "pinned_math.h"

namespace mapvo {

constexpr int kKeepLines = 80;
constexpr int kMinFrames = 0;

// ---- float matrix helpers (pinned P6: double accumulation, one rounding) ----
static void gemm44(const float* A, const float* B, float* C) {
  float o[16];
  for (int r = 0; r < 4; r++)
    for (int c = 0; c < 4; c++) {
      double s = (double)A[r * 4] * B[c];
      s += (double)A[r * 4 + 1] * B[4 + c];
      s += (double)A[r * 4 + 2] * B[8 + c];
      s += (double)A[r * 4 + 3] * B[12 + c];
      o[r * 4 + c] = (float)s;
    }
  std::memcpy(C, o, 64);
}
// -Rcw^T tcw (Frame::UpdatePoseMatrices mOw, KeyFrame::SetPose Ow)
static void centre(const float* T, float* Ow) {
  for (int r = 0; r < 3; r++) {
    double s = (double)T[0 * 4 + r] * T[3];
    s += (double)T[1 * 4 + r] * T[7];
    s += (double)T[2 * 4 + r] * T[11];
    Ow[r] = (float)(s * -1.0);
  }
}
// [Rwc | Ow; 0 0 0 1] (KeyFrame::GetPoseInverse, Tracking.cc:480-482's LastTwc)
static void twc(const float* T, float* Ti) {
  float ow[3];
  centre(T, ow);
  for (int r = 0; r < 3; r++) {
    for (int c = 0; c < 3; c++) Ti[r * 4 + c] = T[c * 4 + r];
    Ti[r * 4 + 3] = ow[r];
  }
  Ti[12] = 0; Ti[13] = 0; Ti[14] = 0; Ti[15] = 1;
}
// Frame::UnprojectStereo: mRwc * x3Dc + mOw
static void unproject(const orbpl_camera& c, const float* T, float u, float v, float z, float* w) {
  float ow[3];
  centre(T, ow);
  const float invfx = 1.0f / c.fx, invfy = 1.0f / c.fy;
  const float x3[3] = {(u - c.cx) * z * invfx, (v - c.cy) * z * invfy, z};
  for (int r = 0; r < 3; r++) {
    double s = (double)T[0 * 4 + r] * x3[0];
    s += (double)T[1 * 4 + r] * x3[1];
    s += (double)T[2 * 4 + r] * x3[2];
    w[r] = (float)(s + (double)ow[r]);
  }
}
static int hamming(const uint8_t* a, const uint8_t* b) {
  int d = 0;
  for (int k = 0; k < 32; k++) d += __builtin_popcount((unsigned)(a[k] ^ b[k]));
  return d;
}

// ---- map model ----
struct MapPoint {
  float pos[3];
  float normal[3] = {0, 0, 0};
  float min_dist = 0, max_dist = 0;   // mfMinDistance / mfMaxDistance
  uint8_t desc[32];
  int nobs = 0;
  int ref_kf;                          // mpRefKF (the creating keyframe)
  std::map<int, int> obs;              // observations: keyframe id -> keypoint (P24)
  long last_seen = -1;                 // mnLastFrameSeen
  long track_ref = -1;                 // mnTrackReferenceForFrame
};
struct MapLine {
  float pos[6];
  uint8_t desc[32];
  int nobs = 0;
  std::map<int, int> obs;
  long last_seen = -1, track_ref = -1;
};
struct KeyFrame {
  int id;
  long frame_id;
  float Tcw[16], Ow[3];
  int N = 0, NL = 0;
  std::vector<orbpl_keypoint> kps_un;
  std::vector<float> uright;
  std::vector<uint8_t> desc;
  std::vector<int32_t> fnode;
  std::vector<int> mp;                 // mvpMapPoints: pool id or -1
  std::vector<orbpl_keyline> kl_un;
  std::vector<float> dstart, dend;
  std::vector<uint8_t> ldesc;
  std::vector<int> ml;
  std::map<int, int> conn;             // mConnectedKeyFrameWeights
  std::vector<int> ord;                // mvpOrderedConnectedKeyFrames
  bool first_conn = true;
  int parent = -1;
  std::set<int> children;
  long track_ref = -1;
};
// temporal VO points / lines of UpdateLastFrame (pool ids -2 - index)
struct Temporal {
  float pos[6];
  uint8_t desc[32];
};

struct Frame {
  long id = 0;
  float Tcw[16];
  int N = 0, NL = 0;
  std::vector<orbpl_keypoint> kps_un;
  std::vector<float> uright, depth;
  std::vector<uint8_t> desc;
  std::vector<int32_t> fnode;
  std::vector<float> angle;            // mvKeys angles (SearchByBoW)
  std::vector<int> mp;                 // -1 none, >= 0 pool, <= -2 temporal
  std::vector<uint8_t> outl;
  std::vector<orbpl_keyline> kl_un;
  std::vector<uint8_t> ldesc;
  std::vector<float> dstart, dend;
  std::vector<int> ml;
  std::vector<uint8_t> loutl;
  int ref_kf = -1;
};

enum { kNotInit = 0, kOK = 1, kLost = 2 };

struct Stream {
  int state = kNotInit;
  std::vector<KeyFrame> kfs;
  std::vector<MapPoint> mps;
  std::vector<MapLine> mls;
  std::vector<Temporal> tp, tl;        // mlpTemporalPoints / Lines
  Frame last;
  bool has_last = false;
  bool has_velocity = false;
  float V[16];
  float Tcr[16];                       // mlRelativeFramePoses.back()
  int ref_kf = -1;                     // mpReferenceKF
  long last_kf_frame = 0;              // mnLastKeyFrameId
  long next_id = 0;                    // Frame::nNextId
  std::vector<int> local_kfs;          // mvpLocalKeyFrames (persists)
  float T0[16];
  int out[24];
};

struct MapVO {
  orbpl_orb_params orb;
  orbpl_camera cam;
  int use_lines = 1;
  int flags = 0;
  int stereo = 0;          // System::STEREO (ORBPL_TRACK_STEREO flag)
  int max_frames = 30;     // mMaxFrames = Camera.fps (Tracking.cc:81-87)
  void* voc = nullptr;
  std::vector<float> scale, inv_sigma2;
  float log_scale;
  std::vector<Stream> st;
  // the last step's stage times (CPU baseline instrumentation, ms): the ORB
  // extraction on the calling thread, the LineExtractor on its own thread,
  // the calling thread's wait in join(), the whole step
  double t_orb = 0, t_lines = 0, t_join = 0, t_step = 0;
};

// ---- MapPoint / MapLine methods ----
static void add_obs(MapVO*, Stream& S, int p, int kf, int idx) {
  MapPoint& M = S.mps[p];
  if (M.obs.count(kf)) return;
  M.obs[kf] = idx;
  M.nobs += S.kfs[kf].uright[idx] >= 0 ? 2 : 1;
}
static void add_line_obs(Stream& S, int l, int kf, int idx) {
  MapLine& L = S.mls[l];
  if (L.obs.count(kf)) return;
  L.obs[kf] = idx;
  const KeyFrame& K = S.kfs[kf];
  L.nobs += (K.dstart[idx] >= 0 && K.dend[idx] >= 0) ? 2 : 1;
}
static void compute_distinctive(Stream& S, int p) {
  MapPoint& M = S.mps[p];
  std::vector<const uint8_t*> d;
  for (auto& o : M.obs) d.push_back(&S.kfs[o.first].desc[32 * (size_t)o.second]);
  if (d.empty()) return;
  const size_t N = d.size();
  std::vector<int> D(N * N, 0);
  for (size_t i = 0; i < N; i++)
    for (size_t j = i + 1; j < N; j++) D[i * N + j] = D[j * N + i] = hamming(d[i], d[j]);
  int best = 0x7fffffff, bi = 0;
  for (size_t i = 0; i < N; i++) {
    std::vector<int> v(D.begin() + i * N, D.begin() + (i + 1) * N);
    std::sort(v.begin(), v.end());
    const int median = v[(size_t)(0.5 * (double)(N - 1))];
    if (median < best) {
      best = median;
      bi = (int)i;
    }
  }
  std::memcpy(M.desc, d[bi], 32);
}
static void compute_distinctive_line(Stream& S, int l) {
  MapLine& L = S.mls[l];
  std::vector<const uint8_t*> d;
  for (auto& o : L.obs) d.push_back(&S.kfs[o.first].ldesc[32 * (size_t)o.second]);
  if (d.empty()) return;
  const size_t N = d.size();
  std::vector<int> D(N * N, 0);
  for (size_t i = 0; i < N; i++)
    for (size_t j = i + 1; j < N; j++) D[i * N + j] = D[j * N + i] = hamming(d[i], d[j]);
  int best = 0x7fffffff, bi = 0;
  for (size_t i = 0; i < N; i++) {
    std::vector<int> v(D.begin() + i * N, D.begin() + (i + 1) * N);
    std::sort(v.begin(), v.end());
    const int median = v[(size_t)(0.5 * (double)(N - 1))];
    if (median < best) {
      best = median;
      bi = (int)i;
    }
  }
  std::memcpy(L.desc, d[bi], 32);
}
// P16 norm: double squares of the float components, one sqrt
static double norm3(const float* v) {
  return std::sqrt((double)v[0] * v[0] + (double)v[1] * v[1] + (double)v[2] * v[2]);
}
static void update_normal_depth(MapVO* v, Stream& S, int p) {
  MapPoint& M = S.mps[p];
  if (M.obs.empty()) return;
  float nrm[3] = {0, 0, 0};
  int n = 0;
  for (auto& o : M.obs) {
    const float* Ow = S.kfs[o.first].Ow;
    const float d[3] = {M.pos[0] - Ow[0], M.pos[1] - Ow[1], M.pos[2] - Ow[2]};
    const float inv = (float)(1.0 / norm3(d));
    for (int k = 0; k < 3; k++) nrm[k] = nrm[k] + d[k] * inv;   // P25
    n++;
  }
  const KeyFrame& R = S.kfs[M.ref_kf];
  const float PC[3] = {M.pos[0] - R.Ow[0], M.pos[1] - R.Ow[1], M.pos[2] - R.Ow[2]};
  const float dist = (float)norm3(PC);
  const int level = R.kps_un[M.obs.at(M.ref_kf)].octave;
  const int nl = (int)v->scale.size();
  M.max_dist = dist * v->scale[level];
  M.min_dist = M.max_dist / v->scale[nl - 1];
  const float fn = (float)n;
  for (int k = 0; k < 3; k++) M.normal[k] = nrm[k] / fn;
}

// ---- KeyFrame methods ----
static void update_best_covisibles(KeyFrame& K) {
  std::vector<std::pair<int, int>> v;   // (weight, id): ties by id (P24)
  for (auto& c : K.conn) v.push_back({c.second, c.first});
  std::sort(v.begin(), v.end());
  K.ord.clear();
  for (size_t i = v.size(); i-- > 0;) K.ord.push_back(v[i].second);
}
static void add_connection(KeyFrame& K, int other, int w) {
  auto it = K.conn.find(other);
  if (it != K.conn.end() && it->second == w) return;
  K.conn[other] = w;
  update_best_covisibles(K);
}
static void update_connections(Stream& S, int kf) {
  KeyFrame& K = S.kfs[kf];
  std::map<int, int> counter;
  for (int i = 0; i < K.N; i++) {
    const int p = K.mp[i];
    if (p < 0) continue;
    for (auto& o : S.mps[p].obs)
      if (o.first != K.id) counter[o.first]++;
  }
  if (counter.empty()) return;
  int nmax = 0, kmax = -1;
  const int th = 15;
  std::vector<std::pair<int, int>> pairs;
  for (auto& c : counter) {
    if (c.second > nmax) {
      nmax = c.second;
      kmax = c.first;
    }
    if (c.second >= th) {
      pairs.push_back({c.second, c.first});
      add_connection(S.kfs[c.first], K.id, c.second);
    }
  }
  if (pairs.empty()) {
    pairs.push_back({nmax, kmax});
    add_connection(S.kfs[kmax], K.id, nmax);
  }
  std::sort(pairs.begin(), pairs.end());
  KeyFrame& K2 = S.kfs[kf];   // (no reallocation happened; keep the reference fresh)
  K2.conn = counter;
  K2.ord.clear();
  for (size_t i = pairs.size(); i-- > 0;) K2.ord.push_back(pairs[i].second);
  if (K2.first_conn && K2.id != 0) {
    K2.parent = K2.ord.front();
    S.kfs[K2.parent].children.insert(K2.id);
    K2.first_conn = false;
  }
}
static int tracked_map_points(const Stream& S, const KeyFrame& K, int min_obs) {
  int n = 0;
  for (int i = 0; i < K.N; i++) {
    const int p = K.mp[i];
    if (p < 0) continue;
    if (min_obs > 0) {
      if (S.mps[p].nobs >= min_obs) n++;
    } else {
      n++;
    }
  }
  return n;
}

// KeyFrame(Frame&) (KeyFrame.cc:28-58) + SetPose
static int new_keyframe(Stream& S, const Frame& F) {
  KeyFrame K;
  K.id = (int)S.kfs.size();
  K.frame_id = F.id;
  std::memcpy(K.Tcw, F.Tcw, 64);
  centre(K.Tcw, K.Ow);
  K.N = F.N;
  K.NL = F.NL;
  K.kps_un = F.kps_un;
  K.uright = F.uright;
  K.desc = F.desc;
  K.fnode = F.fnode;
  K.mp = F.mp;
  K.kl_un = F.kl_un;
  K.dstart = F.dstart;
  K.dend = F.dend;
  K.ldesc = F.ldesc;
  K.ml = F.ml;
  S.kfs.push_back(std::move(K));
  return S.kfs.back().id;
}

// LocalMapping::ProcessNewKeyFrame (P23): observations of the keyframe's
// matched points, their normals / descriptors, the covisibility links
static void process_new_keyframe(MapVO* v, Stream& S, int kf) {
  const int N = S.kfs[kf].N;
  for (int i = 0; i < N; i++) {
    const int p = S.kfs[kf].mp[i];
    if (p < 0) continue;
    if (!S.mps[p].obs.count(kf)) {
      add_obs(v, S, p, kf, i);
      update_normal_depth(v, S, p);
      compute_distinctive(S, p);
    }
  }
  update_connections(S, kf);
}

static MapPoint new_point(const float* pos, int kf) {
  MapPoint M;
  std::memcpy(M.pos, pos, 12);
  M.ref_kf = kf;
  return M;
}

// ---- frame helpers ----
// Frame::Frame(RGB-D) (Frame.cc:135-205). flags & kTwoThreads: ORB and the
// LineExtractor on two host threads as the reference (Frame.cc:152-155).
constexpr int kTwoThreads = 1 << 16;
// right != NULL: Frame::Frame(stereo) (Frame.cc:70-131): ORB on both images,
// ComputeStereoMatches on the two pyramids, and the defined stereo line mode
// (P17: LineExtractor on the right image, end-point depths by line matching).
static void extract(MapVO* v, const uint8_t* gray, const float* depth, Frame& F,
                    const uint8_t* right = nullptr) {
  const orbpl_camera& cam = v->cam;
  if (right) depth = nullptr;
  std::vector<orbpl_keyline> kl(kKeepLines);
  std::vector<uint8_t> ld(kKeepLines * 32);
  std::vector<double> coef(kKeepLines * 3);
  int nl = 0, nd = 0;
  using clk = std::chrono::steady_clock;
  auto ms = [](clk::time_point a, clk::time_point b) {
    return std::chrono::duration<double, std::milli>(b - a).count();
  };
  double t_lines = 0;
  auto lines = [&]() {
    const auto a = clk::now();
    oracle_line_extract(gray, cam.width, cam.height, kl.data(), ld.data(), coef.data(), kKeepLines,
                        &nl, &nd);
    t_lines = ms(a, clk::now());
  };
  std::thread lt;
  if (v->use_lines && (v->flags & kTwoThreads)) lt = std::thread(lines);
  const int cap = v->orb.nfeatures * 2 + 64;
  std::vector<orbpl_keypoint> kps(cap);
  std::vector<uint8_t> desc((size_t)cap * 32);
  int n = 0;
  const auto t0 = clk::now();
  oracle_orb_extract(&v->orb, gray, cam.width, cam.height, cam.width, kps.data(), desc.data(), cap,
                     &n, nullptr);
  const auto t1 = clk::now();
  double t_join = 0;
  if (lt.joinable()) {
    lt.join();
    t_join = ms(t1, clk::now());
  } else if (v->use_lines) {
    lines();
  }
  v->t_orb = ms(t0, t1);
  v->t_join = t_join;
  v->t_lines = t_lines;
  kps.resize(n);
  desc.resize((size_t)n * 32);
  F.N = n;
  F.kps_un.resize(n);
  F.depth.resize(n);
  F.uright.resize(n);
  std::vector<int32_t> gc(n);
  oracle_frame_prepare(&cam, kps.data(), n, depth, F.kps_un.data(), F.depth.data(), F.uright.data(),
                       gc.data(), nullptr);
  if (right) {
    const int cap2 = v->orb.nfeatures * 2 + 64;
    std::vector<orbpl_keypoint> kr(cap2);
    std::vector<uint8_t> dr((size_t)cap2 * 32);
    int nr = 0;
    oracle_orb_extract(&v->orb, right, cam.width, cam.height, cam.width, kr.data(), dr.data(), cap2,
                       &nr, nullptr);
    const int L = v->orb.nlevels;
    std::vector<int32_t> lw(L), lh(L);
    std::vector<float> sc(L), isc(L);
    oracle_orb_level_sizes(&v->orb, cam.width, cam.height, lw.data(), lh.data(), nullptr, sc.data(),
                           isc.data());
    size_t tot = 0;
    for (int l = 0; l < L; l++) tot += (size_t)(lw[l] + 38) * (lh[l] + 38);
    std::vector<uint8_t> pl(tot), pr(tot);
    oracle_orb_pyramid(&v->orb, gray, cam.width, cam.height, cam.width, pl.data(), 0);
    oracle_orb_pyramid(&v->orb, right, cam.width, cam.height, cam.width, pr.data(), 0);
    oracle_stereo_matches(&cam, sc.data(), isc.data(), L, lw.data(), lh.data(), pl.data(), pr.data(),
                          kps.data(), desc.data(), n, kr.data(), dr.data(), nr, F.uright.data(),
                          F.depth.data());
  }
  F.desc = desc;
  F.angle.resize(n);
  for (int i = 0; i < n; i++) F.angle[i] = kps[i].angle;
  F.fnode.assign(n, -1);
  if (v->voc) {
    std::vector<uint32_t> bw(n + 1);
    std::vector<double> bv(n + 1), fwt(n + 1);
    std::vector<int32_t> fw(n + 1);
    int bn = 0;
    oracle_voc_transform(v->voc, desc.data(), n, 4, bw.data(), bv.data(), &bn, F.fnode.data(),
                         fw.data(), fwt.data());
  }
  F.mp.assign(n, -1);
  F.outl.assign(n, 0);
  F.NL = 0;
  if (v->use_lines) {
    F.NL = nl;
    F.kl_un.resize(nl);
    F.dstart.resize(nl);
    F.dend.resize(nl);
    std::vector<float> urs(nl), ure(nl);
    oracle_line_frame_prepare(&cam, kl.data(), nl, depth, F.kl_un.data(), F.dstart.data(),
                              F.dend.data(), urs.data(), ure.data());
    F.ldesc.assign(ld.begin(), ld.begin() + (size_t)nl * 32);
    if (right) {
      std::vector<orbpl_keyline> klr(kKeepLines);
      std::vector<uint8_t> ldr(kKeepLines * 32);
      std::vector<double> coefr(kKeepLines * 3);
      int nr = 0, ndr = 0;
      oracle_line_extract(right, cam.width, cam.height, klr.data(), ldr.data(), coefr.data(),
                          kKeepLines, &nr, &ndr);
      oracle_stereo_line_depths(&cam, F.kl_un.data(), F.ldesc.data(), nl, klr.data(), ldr.data(), nr,
                                F.dstart.data(), F.dend.data());
    }
  }
  F.ml.assign(F.NL, -1);
  F.loutl.assign(F.NL, 0);
}

// map point / line lookups (pool or temporal)
static const float* mp_pos(const Stream& S, int m) { return m >= 0 ? S.mps[m].pos : S.tp[-2 - m].pos; }
static const uint8_t* mp_desc(const Stream& S, int m) { return m >= 0 ? S.mps[m].desc : S.tp[-2 - m].desc; }
static int mp_nobs(const Stream& S, int m) { return m >= 0 ? S.mps[m].nobs : 0; }
static const float* ml_pos(const Stream& S, int m) { return m >= 0 ? S.mls[m].pos : S.tl[-2 - m].pos; }
static const uint8_t* ml_desc(const Stream& S, int m) { return m >= 0 ? S.mls[m].desc : S.tl[-2 - m].desc; }
static int ml_nobs(const Stream& S, int m) { return m >= 0 ? S.mls[m].nobs : 0; }

// Optimizer::PoseOptimizationWithLines(&F): edges = the frame's map points /
// lines; outlier flags in / out
static int optimize(MapVO* v, Stream& S, Frame& F) {
  std::vector<uint8_t> has(F.N, 0), hasl(F.NL, 0);
  std::vector<float> xyz((size_t)F.N * 3, 0.f), lobs((size_t)F.NL * 4, 0.f), lxyz((size_t)F.NL * 6, 0.f);
  std::vector<int32_t> loct(F.NL, 0);
  for (int i = 0; i < F.N; i++)
    if (F.mp[i] != -1) {
      has[i] = 1;
      std::memcpy(&xyz[3 * i], mp_pos(S, F.mp[i]), 12);
    }
  for (int j = 0; j < F.NL; j++) {
    const orbpl_keyline& k = F.kl_un[j];
    loct[j] = k.octave;
    lobs[4 * j] = k.startPointX;
    lobs[4 * j + 1] = k.startPointY;
    lobs[4 * j + 2] = k.endPointX;
    lobs[4 * j + 3] = k.endPointY;
    if (F.ml[j] != -1) {
      hasl[j] = 1;
      std::memcpy(&lxyz[6 * j], ml_pos(S, F.ml[j]), 24);
    }
  }
  orbpl_pose_problem P{};
  P.n = F.N;
  P.kps_un = F.kps_un.data();
  P.uright = F.uright.data();
  P.has_mp = has.data();
  P.mp_xyz = xyz.data();
  P.nl = F.NL;
  P.kl_obs = lobs.data();
  P.kl_octave = loct.data();
  P.has_ml = hasl.data();
  P.ml_xyz = lxyz.data();
  P.inv_sigma2 = v->inv_sigma2.data();
  P.nlevels = (int)v->inv_sigma2.size();
  int ninl = 0;
  oracle_pose_optimization_ex(&v->cam, &P,
                              (v->flags & ORBPL_TRACK_FIXED_LINE_JAC) ? ORBPL_POSE_FIXED_LINE_JAC : 0,
                              F.Tcw, F.outl.data(), F.loutl.data(), &ninl);
  return ninl;
}

// outlier discard of TrackWithMotionModel / TrackReferenceKeyFrame
// (Tracking.cc:1276-1315, 999-1029): returns nmatchesMap, line count in *lmap
static int discard(Stream& S, Frame& F, int* lmap) {
  int nmap = 0, lnm = 0;
  for (int i = 0; i < F.N; i++) {
    const int m = F.mp[i];
    if (m == -1) continue;
    if (F.outl[i]) {
      F.mp[i] = -1;
      F.outl[i] = 0;
      if (m >= 0) S.mps[m].last_seen = F.id;
    } else if (mp_nobs(S, m) > 0) {
      nmap++;
    }
  }
  for (int j = 0; j < F.NL; j++) {
    const int m = F.ml[j];
    if (m == -1) continue;
    if (F.loutl[j]) {
      F.ml[j] = -1;
      F.loutl[j] = 0;
      if (m >= 0) S.mls[m].last_seen = F.id;
      lnm--;
    } else if (ml_nobs(S, m) > 0) {
      lnm++;
    }
  }
  *lmap = lnm;
  return nmap;
}

// Tracking::UpdateLastFrame (Tracking.cc:1044-1210)
static void update_last_frame(MapVO* v, Stream& S) {
  Frame& L = S.last;
  gemm44(S.Tcr, S.kfs[L.ref_kf].Tcw, L.Tcw);
  if (S.last_kf_frame == L.id) return;
  std::vector<std::pair<float, int>> vd;
  for (int i = 0; i < L.N; i++)
    if (L.depth[i] > 0) vd.push_back({L.depth[i], i});
  if (vd.empty()) return;
  std::sort(vd.begin(), vd.end());
  int np = 0;
  for (size_t j = 0; j < vd.size(); j++) {
    const int i = vd[j].second;
    const int m = L.mp[i];
    if (m == -1 || mp_nobs(S, m) < 1) {
      Temporal t{};
      unproject(v->cam, L.Tcw, L.kps_un[i].x, L.kps_un[i].y, L.depth[i], t.pos);
      std::memcpy(t.desc, &L.desc[32 * (size_t)i], 32);
      S.tp.push_back(t);
      L.mp[i] = -2 - ((int)S.tp.size() - 1);
    }
    np++;
    if (vd[j].first > v->cam.th_depth && np > 100) break;
  }
  std::vector<std::pair<std::pair<float, float>, int>> vl;
  for (int j = 0; j < L.NL; j++)
    if (L.dstart[j] > 0 && L.dend[j] > 0) vl.push_back({{L.dstart[j], L.dend[j]}, j});
  if (vl.empty()) return;
  std::sort(vl.begin(), vl.end(), [](const std::pair<std::pair<float, float>, int>& a,
                                     const std::pair<std::pair<float, float>, int>& b) {
    return std::max(a.first.first, a.first.second) < std::max(b.first.first, b.first.second);
  });
  int nlines = 0;
  for (size_t k = 0; k < vl.size(); k++) {
    const int j = vl[k].second;
    const int m = L.ml[j];
    if (m == -1 || ml_nobs(S, m) < 1) {
      Temporal t{};
      const orbpl_keyline& kl = L.kl_un[j];
      unproject(v->cam, L.Tcw, kl.startPointX, kl.startPointY, L.dstart[j], t.pos);
      unproject(v->cam, L.Tcw, kl.endPointX, kl.endPointY, L.dstart[j], t.pos + 3);   // Frame.cc:1192
      std::memcpy(t.desc, &L.ldesc[32 * (size_t)j], 32);
      S.tl.push_back(t);
      L.ml[j] = -2 - ((int)S.tl.size() - 1);
    }
    nlines++;
    if (std::max(vl[k].first.first, vl[k].first.second) > v->cam.th_depth && nlines > 45) break;
  }
}

// SearchByProjection(F, LastFrame, th) over the last frame's map points
static int search_last(MapVO* v, Stream& S, Frame& F, float th) {
  const Frame& L = S.last;
  std::vector<uint8_t> has(L.N), out(L.N);
  std::vector<float> xyz((size_t)L.N * 3, 0.f);
  std::vector<uint8_t> desc((size_t)L.N * 32, 0);
  std::vector<int32_t> nobs(L.N, 0), match(F.N, -1);
  for (int i = 0; i < L.N; i++) {
    has[i] = L.mp[i] != -1;
    out[i] = L.outl[i];
    if (!has[i]) continue;
    std::memcpy(&xyz[3 * i], mp_pos(S, L.mp[i]), 12);
    std::memcpy(&desc[32 * (size_t)i], mp_desc(S, L.mp[i]), 32);
    nobs[i] = mp_nobs(S, L.mp[i]);
  }
  orbpl_match_current cur{F.N, F.Tcw, F.kps_un.data(), F.desc.data(), F.uright.data()};
  orbpl_match_last last{L.N, L.Tcw, L.kps_un.data(), has.data(), out.data(), xyz.data(), desc.data(),
                        nobs.data()};
  int nm = 0;
  oracle_search_by_projection_last(&v->cam, v->scale.data(), (int)v->scale.size(), &cur, &last, th,
                                   0, 1, match.data(), &nm);
  for (int i = 0; i < F.N; i++)
    if (match[i] >= 0) F.mp[i] = L.mp[match[i]];
  return nm;
}

// LineMatcher::SearchByProjection(F, LastFrame) (LineMatcher.cpp:72-269)
static int search_last_lines(MapVO* v, Stream& S, Frame& F) {
  const Frame& L = S.last;
  std::vector<uint8_t> has(L.NL), out(L.NL);
  std::vector<float> xyz((size_t)L.NL * 6, 0.f);
  std::vector<uint8_t> desc((size_t)L.NL * 32, 0);
  std::vector<int32_t> match(F.NL, -1);
  for (int j = 0; j < L.NL; j++) {
    has[j] = L.ml[j] != -1;
    out[j] = L.loutl[j];
    if (!has[j]) continue;
    std::memcpy(&xyz[6 * j], ml_pos(S, L.ml[j]), 24);
    std::memcpy(&desc[32 * (size_t)j], ml_desc(S, L.ml[j]), 32);
  }
  int nm = 0;
  oracle_line_search_by_projection_last(&v->cam, F.Tcw, F.NL, F.kl_un.data(), F.ldesc.data(), L.NL,
                                        L.kl_un.data(), has.data(), out.data(), xyz.data(),
                                        desc.data(), match.data(), &nm);
  for (int j = 0; j < F.NL; j++) F.ml[j] = match[j] >= 0 ? L.ml[match[j]] : -1;
  return nm;
}

struct TrackOut {
  int nmatches = 0, ninl = 0, nmap = 0, nlm = 0, lnmap = 0;
};

// Tracking::TrackWithMotionModel (Tracking.cc:1212-1330)
static bool track_motion(MapVO* v, Stream& S, Frame& F, TrackOut& o) {
  update_last_frame(v, S);
  if (S.has_velocity) {
    gemm44(S.V, S.last.Tcw, F.Tcw);
  } else {
    std::memcpy(F.Tcw, S.last.Tcw, 64);   // no vocabulary: zero velocity (pinned)
  }
  std::fill(F.mp.begin(), F.mp.end(), -1);
  std::fill(F.ml.begin(), F.ml.end(), -1);
  const float th = v->stereo ? 7.0f : 15.0f;   // Tracking.cc:1238-1241
  o.nmatches = search_last(v, S, F, th);
  o.nlm = v->use_lines ? search_last_lines(v, S, F) : 0;
  if (o.nmatches < 20) {
    std::fill(F.mp.begin(), F.mp.end(), -1);
    o.nmatches = search_last(v, S, F, 2 * th);
  }
  if (o.nmatches < 20 || (v->use_lines && o.nlm < 15)) return false;
  o.ninl = optimize(v, S, F);
  o.nmap = discard(S, F, &o.lnmap);
  return v->use_lines ? (o.nmap >= 10 || o.lnmap >= 15) : o.nmap >= 10;
}

// Tracking::TrackReferenceKeyFrame (Tracking.cc:942-1032)
static bool track_refkf(MapVO* v, Stream& S, Frame& F, TrackOut& o) {
  const KeyFrame& R = S.kfs[S.ref_kf];
  std::vector<uint8_t> valid(R.N);
  std::vector<float> kang(R.N);
  for (int i = 0; i < R.N; i++) {
    valid[i] = R.mp[i] >= 0;
    kang[i] = R.kps_un[i].angle;
  }
  std::vector<int32_t> bm(F.N, -1);
  int nm = 0;
  oracle_search_by_bow(R.N, R.fnode.data(), valid.data(), R.desc.data(), kang.data(), F.N,
                       F.fnode.data(), F.desc.data(), F.angle.data(), 0.7f, 1, bm.data(), &nm);
  o.nmatches = nm;
  std::memcpy(F.Tcw, S.last.Tcw, 64);
  int nlm = 0;
  if (v->use_lines) {
    // LineMatcher(0.7).SearchByProjection(F, RefKF): the keyframe's map lines
    // against the frame's current line assignments
    std::vector<uint8_t> lv(R.NL);
    std::vector<float> lx((size_t)R.NL * 6, 0.f);
    std::vector<uint8_t> ld((size_t)R.NL * 32, 0);
    for (int j = 0; j < R.NL; j++) {
      lv[j] = R.ml[j] >= 0;
      if (!lv[j]) continue;
      std::memcpy(&lx[6 * j], S.mls[R.ml[j]].pos, 24);
      std::memcpy(&ld[32 * (size_t)j], S.mls[R.ml[j]].desc, 32);
    }
    std::vector<int32_t> cn(F.NL, 0), tm(F.NL, -1);
    for (int j = 0; j < F.NL; j++) cn[j] = F.ml[j] != -1 ? ml_nobs(S, F.ml[j]) : 0;
    int wiped = 0;
    oracle_line_search_by_projection_list(&v->cam, F.Tcw, F.NL, F.kl_un.data(), F.ldesc.data(),
                                          cn.data(), R.NL, lv.data(), lx.data(), ld.data(),
                                          tm.data(), &nlm, &wiped);
    if (wiped) std::fill(F.ml.begin(), F.ml.end(), -1);
    for (int j = 0; j < F.NL; j++)
      if (tm[j] >= 0) F.ml[j] = R.ml[tm[j]];
  }
  o.nlm = nlm;
  o.ninl = o.nmap = o.lnmap = 0;
  if (nm < 15 || (v->use_lines && nlm < 10)) return false;
  for (int i = 0; i < F.N; i++) F.mp[i] = bm[i] >= 0 ? R.mp[bm[i]] : -1;
  o.ninl = optimize(v, S, F);
  o.nmap = discard(S, F, &o.lnmap);
  return o.nmap >= 10 && (!v->use_lines || o.lnmap >= 10);
}

struct LocalOut {
  int nlocal = 0, inl = 0, nllocal = 0, linl = 0, nkfs = 0, npts = 0, nlines = 0;
};

// Tracking::UpdateLocalKeyFrames (Tracking.cc:1929-2040)
static void update_local_keyframes(Stream& S, Frame& F) {
  std::map<int, int> counter;
  for (int i = 0; i < F.N; i++) {
    const int m = F.mp[i];
    if (m < 0) continue;   // temporal points have no observations
    for (auto& o : S.mps[m].obs) counter[o.first]++;
  }
  if (counter.empty()) return;
  int mx = 0, kmax = -1;
  S.local_kfs.clear();
  for (auto& c : counter) {
    if (c.second > mx) {
      mx = c.second;
      kmax = c.first;
    }
    S.local_kfs.push_back(c.first);
    S.kfs[c.first].track_ref = F.id;
  }
  const size_t n0 = S.local_kfs.size();
  for (size_t a = 0; a < n0; a++) {
    if (S.local_kfs.size() > 80) break;
    const KeyFrame& K = S.kfs[S.local_kfs[a]];
    const size_t nn = std::min<size_t>(10, K.ord.size());
    for (size_t b = 0; b < nn; b++) {
      KeyFrame& Nk = S.kfs[K.ord[b]];
      if (Nk.track_ref != F.id) {
        S.local_kfs.push_back(Nk.id);
        Nk.track_ref = F.id;
        break;
      }
    }
    const KeyFrame& K2 = S.kfs[S.local_kfs[a]];
    for (int c : K2.children) {
      KeyFrame& C = S.kfs[c];
      if (C.track_ref != F.id) {
        S.local_kfs.push_back(C.id);
        C.track_ref = F.id;
        break;
      }
    }
    const int par = S.kfs[S.local_kfs[a]].parent;
    if (par >= 0 && S.kfs[par].track_ref != F.id) {
      S.local_kfs.push_back(par);
      S.kfs[par].track_ref = F.id;
      break;
    }
  }
  if (kmax >= 0) {
    S.ref_kf = kmax;
    F.ref_kf = kmax;
  }
}

// Tracking::TrackLocalMap (Tracking.cc:1332-1420)
static bool track_local_map(MapVO* v, Stream& S, Frame& F, LocalOut& o) {
  update_local_keyframes(S, F);
  std::vector<int> lp, ll;
  for (int k : S.local_kfs) {
    const KeyFrame& K = S.kfs[k];
    for (int i = 0; i < K.N; i++) {
      const int p = K.mp[i];
      if (p < 0 || S.mps[p].track_ref == F.id) continue;
      lp.push_back(p);
      S.mps[p].track_ref = F.id;
    }
    for (int j = 0; j < K.NL; j++) {
      const int l = K.ml[j];
      if (l < 0 || S.mls[l].track_ref == F.id) continue;
      ll.push_back(l);
      S.mls[l].track_ref = F.id;
    }
  }
  o.nkfs = (int)S.local_kfs.size();
  // SearchLocalPoints / SearchLocalLines: the frame's own elements are seen
  for (int i = 0; i < F.N; i++)
    if (F.mp[i] >= 0) S.mps[F.mp[i]].last_seen = F.id;
  for (int j = 0; j < F.NL; j++)
    if (F.ml[j] >= 0) S.mls[F.ml[j]].last_seen = F.id;
  // the local elements a search considers (the seen ones are skipped)
  o.npts = 0;
  for (int p : lp) o.npts += S.mps[p].last_seen != F.id;
  o.nlines = 0;
  for (int l : ll) o.nlines += S.mls[l].last_seen != F.id;
  const int M = (int)lp.size();
  std::vector<float> x((size_t)M * 3), nr((size_t)M * 3), dmn(M), dmx(M), px(M), py(M), pxr(M), vc(M);
  std::vector<int32_t> lev(M), mpn(M), cur_nobs(F.N, 0), lm(F.N, -1);
  std::vector<uint8_t> inview(M, 0), ld((size_t)M * 32);
  for (int j = 0; j < M; j++) {
    const MapPoint& P = S.mps[lp[j]];
    std::memcpy(&x[3 * j], P.pos, 12);
    std::memcpy(&nr[3 * j], P.normal, 12);
    dmn[j] = P.min_dist;   // raw mfMinDistance / mfMaxDistance: the in-frustum
    dmx[j] = P.max_dist;   // test applies 0.8f / 1.2f, PredictScale the raw max
    std::memcpy(&ld[32 * (size_t)j], P.desc, 32);
    mpn[j] = P.nobs;
  }
  oracle_frame_is_in_frustum(&v->cam, v->log_scale, (int)v->scale.size(), F.Tcw, M, x.data(),
                             nr.data(), dmn.data(), dmx.data(), 0.5f, inview.data(), px.data(),
                             py.data(), pxr.data(), lev.data(), vc.data());
  int nto = 0;
  for (int j = 0; j < M; j++) {
    if (S.mps[lp[j]].last_seen == F.id) inview[j] = 0;   // skipped: mbTrackInView stays false
    nto += inview[j];
  }
  for (int i = 0; i < F.N; i++) cur_nobs[i] = F.mp[i] != -1 ? mp_nobs(S, F.mp[i]) : 0;
  if (nto > 0) {
    const float th = F.id < 2 ? 5.0f : (v->stereo ? 1.0f : 3.0f);   // Tracking.cc:1801-1809
    orbpl_match_current cur{F.N, F.Tcw, F.kps_un.data(), F.desc.data(), F.uright.data()};
    oracle_search_by_projection_local(&v->cam, v->scale.data(), (int)v->scale.size(), &cur, M,
                                      inview.data(), px.data(), py.data(), pxr.data(), lev.data(),
                                      vc.data(), ld.data(), mpn.data(), cur_nobs.data(), th, 0.8f,
                                      lm.data(), &o.nlocal);
    for (int i = 0; i < F.N; i++)
      if (lm[i] >= 0) F.mp[i] = lp[lm[i]];
  }
  // SearchLocalLines
  if (v->use_lines) {
    const int ML = (int)ll.size();
    std::vector<float> lx((size_t)ML * 6);
    std::vector<uint8_t> ldd((size_t)ML * 32), lv(ML, 0);
    for (int k = 0; k < ML; k++) {
      std::memcpy(&lx[6 * k], S.mls[ll[k]].pos, 24);
      std::memcpy(&ldd[32 * (size_t)k], S.mls[ll[k]].desc, 32);
    }
    oracle_line_is_in_frustum(F.Tcw, ML, lx.data(), lv.data());
    int ntl = 0;
    for (int k = 0; k < ML; k++) {
      if (S.mls[ll[k]].last_seen == F.id) lv[k] = 0;
      ntl += lv[k];
    }
    if (ntl > 0) {
      std::vector<int32_t> cn(F.NL, 0), tm(F.NL, -1);
      for (int j = 0; j < F.NL; j++) cn[j] = F.ml[j] != -1 ? ml_nobs(S, F.ml[j]) : 0;
      int wiped = 0;
      oracle_line_search_by_projection_list(&v->cam, F.Tcw, F.NL, F.kl_un.data(), F.ldesc.data(),
                                            cn.data(), ML, lv.data(), lx.data(), ldd.data(),
                                            tm.data(), &o.nllocal, &wiped);
      if (wiped) std::fill(F.ml.begin(), F.ml.end(), -1);
      for (int j = 0; j < F.NL; j++)
        if (tm[j] >= 0) F.ml[j] = ll[tm[j]];
    }
  }
  optimize(v, S, F);
  o.inl = 0;
  for (int i = 0; i < F.N; i++)
    if (F.mp[i] != -1 && !F.outl[i] && mp_nobs(S, F.mp[i]) > 0) o.inl++;
  o.linl = 0;
  for (int j = 0; j < F.NL; j++)
    if (F.ml[j] != -1 && !F.loutl[j] && ml_nobs(S, F.ml[j]) > 0) o.linl++;
  if (v->stereo) {   // an outlier's map point / line leaves the frame (Tracking.cc:1374-1401)
    for (int i = 0; i < F.N; i++)
      if (F.mp[i] != -1 && F.outl[i]) F.mp[i] = -1;
    for (int j = 0; j < F.NL; j++)
      if (F.ml[j] != -1 && F.loutl[j]) F.ml[j] = -1;
  }
  if (F.id < 0 + v->max_frames && o.inl + o.linl < 60) return false;
  return !(o.inl < 30 && o.linl < 20);
}

// Tracking::NeedNewKeyFrame (Tracking.cc:1423-1557) with the P23 stub
static bool need_new_keyframe(MapVO* v, Stream& S, const Frame& F, int inliers) {
  const int nKFs = (int)S.kfs.size();
  if (F.id < 0 + v->max_frames && nKFs > v->max_frames) return false;
  const int nMinObs = nKFs <= 2 ? 2 : 3;
  const int nRefMatches = tracked_map_points(S, S.kfs[S.ref_kf], nMinObs);
  const bool idle = true;
  int ntc = 0, nntc = 0;
  for (int i = 0; i < F.N; i++)
    if (F.depth[i] > 0 && F.depth[i] < v->cam.th_depth) {
      if (F.mp[i] != -1 && !F.outl[i]) ntc++;
      else nntc++;
    }
  const bool close = ntc < 100 && nntc > 70;
  float thRefRatio = 0.75f;
  if (nKFs < 2) thRefRatio = 0.4f;
  const bool c1a = F.id >= S.last_kf_frame + v->max_frames;
  const bool c1b = F.id >= S.last_kf_frame + kMinFrames && idle;
  const bool c1c = inliers < nRefMatches * 0.25 || close;
  const bool c2 = (inliers < nRefMatches * thRefRatio || close) && inliers > 15;
  return (c1a || c1b || c1c) && c2;
}

// Tracking::CreateNewKeyFrame (Tracking.cc:1567-1745) + ProcessNewKeyFrame
static void create_new_keyframe(MapVO* v, Stream& S, Frame& F) {
  const int kf = new_keyframe(S, F);
  S.ref_kf = kf;
  F.ref_kf = kf;
  std::vector<std::pair<float, int>> vd;
  for (int i = 0; i < F.N; i++)
    if (F.depth[i] > 0) vd.push_back({F.depth[i], i});
  if (!vd.empty()) {
    std::sort(vd.begin(), vd.end());
    int np = 0;
    for (size_t j = 0; j < vd.size(); j++) {
      const int i = vd[j].second;
      bool create = F.mp[i] == -1;
      if (!create && mp_nobs(S, F.mp[i]) < 1) {
        create = true;
        F.mp[i] = -1;
      }
      if (create) {
        float pos[3];
        unproject(v->cam, F.Tcw, F.kps_un[i].x, F.kps_un[i].y, vd[j].first, pos);
        S.mps.push_back(new_point(pos, kf));
        const int p = (int)S.mps.size() - 1;
        add_obs(v, S, p, kf, i);
        S.kfs[kf].mp[i] = p;
        compute_distinctive(S, p);
        update_normal_depth(v, S, p);
        F.mp[i] = p;
      }
      np++;
      if (vd[j].first > v->cam.th_depth && np > 100) break;
    }
  }
  std::vector<std::pair<std::pair<float, float>, int>> vl;
  for (int j = 0; j < F.NL; j++)
    if (F.dstart[j] > 0 && F.dend[j] > 0) vl.push_back({{F.dstart[j], F.dend[j]}, j});
  if (!vl.empty()) {
    std::sort(vl.begin(), vl.end(), [](const std::pair<std::pair<float, float>, int>& a,
                                       const std::pair<std::pair<float, float>, int>& b) {
      return std::max(a.first.first, a.first.second) < std::max(b.first.first, b.first.second);
    });
    int nlines = 0;
    for (size_t k = 0; k < vl.size(); k++) {
      const int j = vl[k].second;
      bool create = F.ml[j] == -1;
      if (!create && ml_nobs(S, F.ml[j]) < 1) {
        create = true;
        F.ml[j] = -1;
      }
      if (create) {
        MapLine L;
        const orbpl_keyline& kl = F.kl_un[j];
        unproject(v->cam, F.Tcw, kl.startPointX, kl.startPointY, F.dstart[j], L.pos);
        unproject(v->cam, F.Tcw, kl.endPointX, kl.endPointY, F.dstart[j], L.pos + 3);
        S.mls.push_back(L);
        const int l = (int)S.mls.size() - 1;
        add_line_obs(S, l, kf, j);
        S.kfs[kf].ml[j] = l;
        compute_distinctive_line(S, l);
        F.ml[j] = l;
      }
      nlines++;
      if (std::max(vl[k].first.first, vl[k].first.second) > v->cam.th_depth && nlines > 45) break;
    }
  }
  process_new_keyframe(v, S, kf);
  S.last_kf_frame = F.id;
}

// Tracking::StereoInitialization (Tracking.cc:608-727)
static bool stereo_initialization(MapVO* v, Stream& S, Frame& F) {
  if (F.N <= 500) return false;
  std::memcpy(F.Tcw, S.T0, 64);
  const int kf = new_keyframe(S, F);
  for (int i = 0; i < F.N; i++) {
    const float z = F.depth[i];
    if (!(z > 0)) continue;
    float pos[3];
    unproject(v->cam, F.Tcw, F.kps_un[i].x, F.kps_un[i].y, z, pos);
    S.mps.push_back(new_point(pos, kf));
    const int p = (int)S.mps.size() - 1;
    add_obs(v, S, p, kf, i);
    compute_distinctive(S, p);
    update_normal_depth(v, S, p);
    S.kfs[kf].mp[i] = p;
    F.mp[i] = p;
  }
  for (int j = 0; j < F.NL; j++) {
    if (!(F.dstart[j] > 0 && F.dend[j] > 0)) continue;
    MapLine L;
    const orbpl_keyline& kl = F.kl_un[j];
    unproject(v->cam, F.Tcw, kl.startPointX, kl.startPointY, F.dstart[j], L.pos);
    unproject(v->cam, F.Tcw, kl.endPointX, kl.endPointY, F.dstart[j], L.pos + 3);
    S.mls.push_back(L);
    const int l = (int)S.mls.size() - 1;
    add_line_obs(S, l, kf, j);
    compute_distinctive_line(S, l);
    S.kfs[kf].ml[j] = l;
    F.ml[j] = l;
  }
  process_new_keyframe(v, S, kf);   // InsertKeyFrame: nothing to add, no connections
  S.last_kf_frame = F.id;
  S.local_kfs.assign(1, kf);
  S.ref_kf = kf;
  F.ref_kf = kf;
  return true;
}

static void reset_stream(Stream& S) {
  const long nid = S.next_id;
  float T0[16];
  std::memcpy(T0, S.T0, 64);
  S = Stream();
  S.next_id = nid;
  std::memcpy(S.T0, T0, 64);
}

static int step(MapVO* v, int s, const uint8_t* gray, const float* depth, float* Tcw_out,
                const uint8_t* right = nullptr) {
  Stream& S = v->st[s];
  Frame F;
  const auto t_start = std::chrono::steady_clock::now();
  struct StepClock {   // the whole step, however it returns
    MapVO* v;
    std::chrono::steady_clock::time_point a;
    ~StepClock() {
      v->t_step = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - a).count();
    }
  } step_clock{v, t_start};
  extract(v, gray, depth, F, right);
  F.id = S.next_id++;
  int* out = S.out;
  std::memset(out, 0, sizeof(S.out));
  out[0] = F.N;
  out[5] = F.NL;
  S.tp.clear();
  S.tl.clear();
  if (S.state == kNotInit) {
    if (stereo_initialization(v, S, F)) {
      S.state = kOK;
      float Twr[16];
      twc(S.kfs[F.ref_kf].Tcw, Twr);
      gemm44(F.Tcw, Twr, S.Tcr);
      S.last = F;
      S.has_last = true;
      out[4] = 1;
      out[12] = 2;
    } else {
      std::memcpy(F.Tcw, S.T0, 64);
    }
    std::memcpy(Tcw_out, F.Tcw, 64);
  } else {
    bool ok = false;
    TrackOut o;
    LocalOut lo;
    bool posed = true;
    if (S.state == kOK) {
      const bool refkf = (v->flags & ORBPL_TRACK_REFKF) && v->voc;
      if ((!S.has_velocity || F.id < 0 + 2) && refkf) {
        out[17] = 1;
        ok = track_refkf(v, S, F, o);
      } else {
        ok = track_motion(v, S, F, o);
        if (!ok && refkf) {
          out[17] = 1;
          ok = track_refkf(v, S, F, o);
        }
      }
    } else {
      posed = false;   // Relocalization (out of scope, P23): fails
    }
    F.ref_kf = S.ref_kf;
    if (ok) ok = track_local_map(v, S, F, lo);
    S.state = ok ? kOK : kLost;
    if (ok) {
      float LastTwc[16];
      twc(S.last.Tcw, LastTwc);
      gemm44(F.Tcw, LastTwc, S.V);
      S.has_velocity = true;
      for (int i = 0; i < F.N; i++)
        if (F.mp[i] != -1 && mp_nobs(S, F.mp[i]) < 1) {
          F.outl[i] = 0;
          F.mp[i] = -1;
        }
      for (int j = 0; j < F.NL; j++)
        if (F.ml[j] != -1 && ml_nobs(S, F.ml[j]) < 1) {
          F.loutl[j] = 0;
          F.ml[j] = -1;
        }
      out[16] = (int)S.tp.size();
      out[23] = (int)S.tl.size();
      S.tp.clear();
      S.tl.clear();
      if (need_new_keyframe(v, S, F, lo.inl)) {
        create_new_keyframe(v, S, F);
        out[12] = 1;
      }
      for (int i = 0; i < F.N; i++)
        if (F.mp[i] != -1 && F.outl[i]) F.mp[i] = -1;
      // Tracking.cc:552-555 clears lines by the point outlier flags
      for (int j = 0; j < F.NL; j++)
        if (F.ml[j] != -1 && j < F.N && F.outl[j]) F.ml[j] = -1;
    }
    out[1] = o.nmatches;
    out[2] = o.ninl;
    out[3] = o.nmap;
    out[4] = ok ? 1 : 0;
    out[6] = o.nlm;
    out[7] = o.lnmap;
    out[8] = lo.nlocal;
    out[9] = lo.inl;
    out[10] = lo.nllocal;
    out[11] = lo.linl;
    out[20] = lo.nkfs;
    out[21] = lo.npts;
    out[22] = lo.nlines;
    if (S.state == kLost && (int)S.kfs.size() <= 5) {
      std::memcpy(Tcw_out, posed ? F.Tcw : S.last.Tcw, 64);
      int keep[24];
      std::memcpy(keep, out, sizeof(keep));   // out is S.out, which the reset clears
      reset_stream(S);
      keep[19] = kNotInit;
      keep[13] = keep[14] = keep[15] = 0;
      std::memcpy(S.out, keep, sizeof(S.out));
      return 0;
    }
    if (F.ref_kf < 0) F.ref_kf = S.ref_kf;
    if (posed) {
      float Twr[16];
      twc(S.kfs[F.ref_kf].Tcw, Twr);
      gemm44(F.Tcw, Twr, S.Tcr);
    } else {
      // no pose (LOST): the trajectory repeats the last relative pose
      gemm44(S.Tcr, S.kfs[S.last.ref_kf].Tcw, F.Tcw);
    }
    std::memcpy(Tcw_out, F.Tcw, 64);
    S.last = F;
  }
  out[13] = (int)S.kfs.size();
  out[14] = (int)S.mps.size();
  out[15] = (int)S.mls.size();
  out[18] = S.ref_kf;
  out[19] = S.state;
  return 0;
}

}  // namespace mapvo

extern "C" {

void* oracle_map_create(const orbpl_orb_params* orb, const orbpl_camera* cam, int n_streams,
                        int flags) {
  mapvo::MapVO* v = new mapvo::MapVO();
  v->orb = *orb;
  v->cam = *cam;
  v->flags = flags;
  v->use_lines = (flags & ORBPL_TRACK_LINES) ? 1 : 0;
  v->stereo = (flags & ORBPL_TRACK_STEREO) ? 1 : 0;
  v->st.resize(n_streams);
  v->scale.resize(orb->nlevels);
  std::vector<float> isc(orb->nlevels);
  oracle_orb_level_sizes(orb, cam->width, cam->height, nullptr, nullptr, nullptr, v->scale.data(),
                         isc.data());
  v->inv_sigma2.resize(orb->nlevels);
  for (int l = 0; l < orb->nlevels; l++) v->inv_sigma2[l] = 1.0f / (v->scale[l] * v->scale[l]);
  v->log_scale = (float)pmath::log_((double)orb->scale_factor);   // P15
  for (auto& S : v->st)
    for (int k = 0; k < 16; k++) S.T0[k] = (k % 5 == 0) ? 1.f : 0.f;
  return v;
}

void oracle_map_destroy(void* h) { delete static_cast<mapvo::MapVO*>(h); }

int oracle_map_reset(void* h, const float* Tcw0) {
  mapvo::MapVO* v = static_cast<mapvo::MapVO*>(h);
  for (size_t s = 0; s < v->st.size(); s++) {
    v->st[s] = mapvo::Stream();
    for (int k = 0; k < 16; k++) v->st[s].T0[k] = Tcw0 ? Tcw0[s * 16 + k] : ((k % 5 == 0) ? 1.f : 0.f);
  }
  return 0;
}

// mVelocity = cv::Mat() for one stream (after initialisation / relocalisation:
// its next frame runs TrackReferenceKeyFrame, Tracking.cc:324-338)
int oracle_map_clear_velocity(void* h, int stream) {
  mapvo::MapVO* v = static_cast<mapvo::MapVO*>(h);
  if (stream < 0 || stream >= (int)v->st.size()) return -1;
  v->st[stream].has_velocity = false;
  return 0;
}

int oracle_map_set_vocabulary(void* h, void* voc) {
  static_cast<mapvo::MapVO*>(h)->voc = voc;
  return 0;
}

// out24: nkeypoints, nmatches, ninliers, nmatches_map, ok, nlines, line_matches,
// line_nmatches_map, local_matches, local_inliers, local_line_matches,
// local_line_inliers, keyframe (1 created, 2 initial), keyframes in map, map
// points, map lines, temporal points, TrackReferenceKeyFrame ran, reference
// keyframe id, state (0 not initialised, 1 OK, 2 LOST), local keyframes, local
// map points, local map lines, temporal lines
int oracle_map_step(void* h, int stream, const uint8_t* gray, const float* depth, float* Tcw_out,
                    int* out24) {
  mapvo::MapVO* v = static_cast<mapvo::MapVO*>(h);
  if (stream < 0 || stream >= (int)v->st.size()) return -1;
  float T[16];
  const int rc = mapvo::step(v, stream, gray, depth, T);
  if (Tcw_out) std::memcpy(Tcw_out, T, 64);
  if (out24) std::memcpy(out24, v->st[stream].out, sizeof(int) * 24);
  return rc;
}

// the stereo step: rectified left / right images (Tracking::GrabImageStereo)
int oracle_map_step_stereo(void* h, int stream, const uint8_t* left, const uint8_t* right,
                           float* Tcw_out, int* out24) {
  mapvo::MapVO* v = static_cast<mapvo::MapVO*>(h);
  if (stream < 0 || stream >= (int)v->st.size() || !right) return -1;
  float T[16];
  const int rc = mapvo::step(v, stream, left, nullptr, T, right);
  if (Tcw_out) std::memcpy(Tcw_out, T, 64);
  if (out24) std::memcpy(out24, v->st[stream].out, sizeof(int) * 24);
  return rc;
}

// Camera.fps: mMaxFrames (0 -> 30, Tracking.cc:81-87)
// the last step's stage times in ms: ORB (calling thread), LineExtractor (its
// own thread, or inline), the calling thread's join wait, the whole step
int oracle_map_stage_times(void* h, double* out4) {
  const mapvo::MapVO* v = static_cast<mapvo::MapVO*>(h);
  out4[0] = v->t_orb;
  out4[1] = v->t_lines;
  out4[2] = v->t_join;
  out4[3] = v->t_step;
  return 0;
}

int oracle_map_set_fps(void* h, float fps) {
  static_cast<mapvo::MapVO*>(h)->max_frames = (int)(fps == 0.0f ? 30.0f : fps);
  return 0;
}

// the stream's map for tests: keyframe count; per keyframe its covisibility
// order (up to cap ids), parent; returns the number of keyframes
int oracle_map_keyframes(void* h, int stream, int* parent, int* ord, int cap, int* nord) {
  const mapvo::Stream& S = static_cast<mapvo::MapVO*>(h)->st[stream];
  const int n = (int)S.kfs.size();
  for (int k = 0; k < n; k++) {
    const mapvo::KeyFrame& K = S.kfs[k];
    if (parent) parent[k] = K.parent;
    if (nord) nord[k] = (int)K.ord.size();
    if (ord)
      for (int j = 0; j < cap; j++) ord[k * cap + j] = j < (int)K.ord.size() ? K.ord[j] : -1;
  }
  return n;
}

// per map point: mean viewing direction, mfMinDistance / mfMaxDistance
int oracle_map_points_geom(void* h, int stream, float* nrm, float* dist2, int cap) {
  const mapvo::Stream& S = static_cast<mapvo::MapVO*>(h)->st[stream];
  const int n = (int)S.mps.size();
  for (int p = 0; p < n && p < cap; p++) {
    if (nrm) std::memcpy(nrm + 3 * (size_t)p, S.mps[p].normal, 12);
    if (dist2) {
      dist2[2 * p] = S.mps[p].min_dist;
      dist2[2 * p + 1] = S.mps[p].max_dist;
    }
  }
  return n;
}

// per map line: observation count, descriptor, end points; returns the count
int oracle_map_lines(void* h, int stream, int* nobs, uint8_t* desc, float* pos6, int cap) {
  const mapvo::Stream& S = static_cast<mapvo::MapVO*>(h)->st[stream];
  const int n = (int)S.mls.size();
  for (int l = 0; l < n && l < cap; l++) {
    if (nobs) nobs[l] = S.mls[l].nobs;
    if (desc) std::memcpy(desc + 32 * (size_t)l, S.mls[l].desc, 32);
    if (pos6) std::memcpy(pos6 + 6 * (size_t)l, S.mls[l].pos, 24);
  }
  return n;
}

// per map point: observation count (nObs) and descriptor; returns the count
int oracle_map_points(void* h, int stream, int* nobs, uint8_t* desc, float* xyz, int cap) {
  const mapvo::Stream& S = static_cast<mapvo::MapVO*>(h)->st[stream];
  const int n = (int)S.mps.size();
  for (int p = 0; p < n && p < cap; p++) {
    if (nobs) nobs[p] = S.mps[p].nobs;
    if (desc) std::memcpy(desc + 32 * (size_t)p, S.mps[p].desc, 32);
    if (xyz) std::memcpy(xyz + 3 * (size_t)p, S.mps[p].pos, 12);
  }
  return n;
}

}  // extern "C"
