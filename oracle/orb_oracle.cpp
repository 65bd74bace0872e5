// ============================================================================
// ORACLE — TEST INFRASTRUCTURE ONLY. NOT PART OF THE PRODUCT PATH.
//
// CPU restatement of the reference ORB extractor
//   /root/reference/src/ORBextractor.cc  (wolfcanli/ORB_SLAM2_Modification_with-
//   point-and-line-feature), plus clean-room restatements of the OpenCV 3.4
//   primitives it calls (copyMakeBorder REFLECT_101, resize INTER_LINEAR 8U,
//   FAST_t<16> + cornerScore<16>, fastAtan2, GaussianBlur 8U fixed point).
//
// Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
// this library, and only as the checker / CPU baseline. The product library
// (orb_slam2_modification_with-point-and-line-feature_amd/csrc) never links it.
//
// PARITY STATUS: "parity unpinned" against the real reference binary. The
// reference cannot be built here (OpenCV 3.4 / contrib / Eigen absent, see
// SURVEY.md §8c) and it ships no golden vectors for this path. Every pinned
// semantic choice is listed in DESIGN.md §"Pinned semantics":
//   P1 FMA contraction off (the reference builds with -std=c++14 ISO mode,
//      where GCC's default is -ffp-contract=off).
//   P2 cos/sin in computeOrbDescriptor = correctly rounded float results,
//      computed as (float)cos((double)angle).
//   P3 DistributeOctTree sort ties broken by node creation order (the
//      reference breaks them on heap addresses, ORBextractor.cc:684).
//   P4 GaussianBlur 8U = OpenCV >= 3.4.2 fixed-point path with the 7-tap
//      sigma=2 kernel {18,34,49,54,49,34,18}/256.
//   P5 resize 8U INTER_LINEAR = OpenCV's legacy 11-bit fixed-point path.
// ============================================================================
#include <cmath>
#include <cstdint>
#include <cstring>
#include <cfloat>
#include <vector>
#include <list>
#include <algorithm>
#include <utility>

#include "oracle_api.h"
#include "pinned_math.h"

namespace oracle {

static const int PATCH_SIZE = 31;       // ORBextractor.cc:72
static const int HALF_PATCH_SIZE = 15;  // ORBextractor.cc:73
static const int EDGE_THRESHOLD = 19;   // ORBextractor.cc:74

static inline int cvRound_f(float v) { return (int)lrintf(v); }
static inline int cvRound_d(double v) { return (int)lrint(v); }
static inline int cvFloor_f(float v) { return (int)std::floor(v); }
static inline int cvFloor_d(double v) { return (int)std::floor(v); }
static inline int cvCeil_d(double v) { return (int)std::ceil(v); }

// ---------------------------------------------------------------------------
// bit_pattern_31_ : the 256 point-pair sampling pattern (ORBextractor.cc:150-408).
// These are numeric constants of the ORB descriptor (Rublee et al. 2011),
// identical to OpenCV's orb.cpp table.
// ---------------------------------------------------------------------------
#include "orb_pattern.inc"

// ---------------------------------------------------------------------------
// ORBextractor::ORBextractor (ORBextractor.cc:410-470)
// ---------------------------------------------------------------------------
struct Extractor {
    int nfeatures;
    double scaleFactor;   // declared double in ORBextractor.h:80
    int nlevels;
    int iniThFAST, minThFAST;
    std::vector<float> mvScaleFactor, mvInvScaleFactor, mvLevelSigma2, mvInvLevelSigma2;
    std::vector<int> mnFeaturesPerLevel;
    std::vector<int> umax;

    Extractor(int _nfeatures, float _scaleFactor, int _nlevels, int _ini, int _min)
        : nfeatures(_nfeatures), scaleFactor(_scaleFactor), nlevels(_nlevels),
          iniThFAST(_ini), minThFAST(_min) {
        mvScaleFactor.resize(nlevels);
        mvLevelSigma2.resize(nlevels);
        mvScaleFactor[0] = 1.0f;
        mvLevelSigma2[0] = 1.0f;
        for (int i = 1; i < nlevels; i++) {
            mvScaleFactor[i] = (float)(mvScaleFactor[i - 1] * scaleFactor);
            mvLevelSigma2[i] = mvScaleFactor[i] * mvScaleFactor[i];
        }
        mvInvScaleFactor.resize(nlevels);
        mvInvLevelSigma2.resize(nlevels);
        for (int i = 0; i < nlevels; i++) {
            mvInvScaleFactor[i] = 1.0f / mvScaleFactor[i];
            mvInvLevelSigma2[i] = 1.0f / mvLevelSigma2[i];
        }
        mnFeaturesPerLevel.resize(nlevels);
        float factor = (float)(1.0f / scaleFactor);
        float nDesired = nfeatures * (1 - factor) /
                         (1 - (float)pow((double)factor, (double)nlevels));
        int sumFeatures = 0;
        for (int level = 0; level < nlevels - 1; level++) {
            mnFeaturesPerLevel[level] = cvRound_f(nDesired);
            sumFeatures += mnFeaturesPerLevel[level];
            nDesired *= factor;
        }
        mnFeaturesPerLevel[nlevels - 1] = std::max(nfeatures - sumFeatures, 0);

        umax.resize(HALF_PATCH_SIZE + 1);
        int v, v0, vmax = (int)std::floor(HALF_PATCH_SIZE * sqrt(2.f) / 2 + 1);
        int vmin = (int)std::ceil(HALF_PATCH_SIZE * sqrt(2.f) / 2);
        const double hp2 = HALF_PATCH_SIZE * HALF_PATCH_SIZE;
        for (v = 0; v <= vmax; ++v) umax[v] = cvRound_d(sqrt(hp2 - v * v));
        for (v = HALF_PATCH_SIZE, v0 = 0; v >= vmin; --v) {
            while (umax[v0] == umax[v0 + 1]) ++v0;
            umax[v] = v0;
            ++v0;
        }
    }
};

// ---------------------------------------------------------------------------
// Padded image (one pyramid level): content w x h at offset (19,19) inside a
// (w+38) x (h+38) buffer, as ComputePyramid builds (ORBextractor.cc:1113-1115).
// ---------------------------------------------------------------------------
struct Level {
    int w = 0, h = 0, pw = 0, ph = 0;
    std::vector<uint8_t> buf;
    uint8_t* at(int x, int y) { return &buf[(size_t)(y + EDGE_THRESHOLD) * pw + (x + EDGE_THRESHOLD)]; }
    const uint8_t* at(int x, int y) const { return &buf[(size_t)(y + EDGE_THRESHOLD) * pw + (x + EDGE_THRESHOLD)]; }
};

// OpenCV borderInterpolate for BORDER_REFLECT_101 (clean-room restatement).
static int reflect101(int p, int len) {
    if (len == 1) return 0;
    while ((unsigned)p >= (unsigned)len) {
        if (p < 0) p = -p;                  // -p - 1 + delta, delta = 1
        else p = len - 1 - (p - len) - 1;   // len - 1 - (p - len) - delta
    }
    return p;
}

// copyMakeBorder(src, dst, 19,19,19,19, REFLECT_101[, ISOLATED]) where dst's
// interior already holds the content (ORBextractor.cc:1122-1128).
static void fill_border(Level& L) {
    for (int py = 0; py < L.ph; py++) {
        int sy = reflect101(py - EDGE_THRESHOLD, L.h);
        for (int px = 0; px < L.pw; px++) {
            int cx = px - EDGE_THRESHOLD, cy = py - EDGE_THRESHOLD;
            if (cx >= 0 && cx < L.w && cy >= 0 && cy < L.h) continue;
            int sx = reflect101(cx, L.w);
            L.buf[(size_t)py * L.pw + px] = *L.at(sx, sy);
        }
    }
}

// OpenCV 3.4 hal::resize, INTER_LINEAR, CV_8UC1, fixed-point (11-bit coefs).
static void resize_linear_8u(const Level& S, Level& D) {
    const int sw = S.w, sh = S.h, dw = D.w, dh = D.h;
    const double inv_scale_x = (double)dw / sw, inv_scale_y = (double)dh / sh;
    const double scale_x = 1. / inv_scale_x, scale_y = 1. / inv_scale_y;
    const int ONE = 2048;
    std::vector<int> xofs(dw), yofs(dh);
    std::vector<short> ialpha(dw * 2), ibeta(dh * 2);
    int xmax = dw;
    for (int dx = 0; dx < dw; dx++) {
        float fx = (float)((dx + 0.5) * scale_x - 0.5);
        int sx = cvFloor_f(fx);
        fx -= sx;
        if (sx < 0) { fx = 0; sx = 0; }
        if (sx + 1 >= sw) {
            xmax = std::min(xmax, dx);
            if (sx >= sw - 1) { fx = 0; sx = sw - 1; }
        }
        xofs[dx] = sx;
        float c0 = 1.f - fx, c1 = fx;
        ialpha[dx * 2] = (short)cvRound_f(c0 * ONE);
        ialpha[dx * 2 + 1] = (short)cvRound_f(c1 * ONE);
    }
    for (int dy = 0; dy < dh; dy++) {
        float fy = (float)((dy + 0.5) * scale_y - 0.5);
        int sy = cvFloor_f(fy);
        fy -= sy;
        yofs[dy] = sy;
        ibeta[dy * 2] = (short)cvRound_f((1.f - fy) * ONE);
        ibeta[dy * 2 + 1] = (short)cvRound_f(fy * ONE);
    }
    std::vector<int> r0(dw), r1(dw);
    auto hresize = [&](const uint8_t* Srow, int* Drow) {
        for (int dx = 0; dx < dw; dx++) {
            int sx = xofs[dx];
            if (dx < xmax) Drow[dx] = Srow[sx] * ialpha[dx * 2] + Srow[sx + 1] * ialpha[dx * 2 + 1];
            else Drow[dx] = Srow[sx] * ONE;
        }
    };
    for (int dy = 0; dy < dh; dy++) {
        int sy0 = yofs[dy];
        int ya = std::min(std::max(sy0, 0), sh - 1);
        int yb = std::min(std::max(sy0 + 1, 0), sh - 1);
        hresize(S.at(0, ya), r0.data());
        hresize(S.at(0, yb), r1.data());
        int b0 = ibeta[dy * 2], b1 = ibeta[dy * 2 + 1];
        uint8_t* out = D.at(0, dy);
        for (int x = 0; x < dw; x++)
            out[x] = (uint8_t)((((b0 * (r0[x] >> 4)) >> 16) + ((b1 * (r1[x] >> 4)) >> 16) + 2) >> 2);
    }
}

// ORBextractor::ComputePyramid (ORBextractor.cc:1107-1132)
static void compute_pyramid(const Extractor& E, const uint8_t* img, int w, int h, int stride,
                            std::vector<Level>& pyr) {
    pyr.assign(E.nlevels, Level());
    for (int level = 0; level < E.nlevels; ++level) {
        float scale = E.mvInvScaleFactor[level];
        Level& L = pyr[level];
        L.w = cvRound_f((float)w * scale);
        L.h = cvRound_f((float)h * scale);
        L.pw = L.w + EDGE_THRESHOLD * 2;
        L.ph = L.h + EDGE_THRESHOLD * 2;
        L.buf.assign((size_t)L.pw * L.ph, 0);
        if (level != 0) {
            resize_linear_8u(pyr[level - 1], L);
        } else {
            for (int y = 0; y < h; y++) memcpy(L.at(0, y), img + (size_t)y * stride, w);
        }
        fill_border(L);
    }
}

// ---------------------------------------------------------------------------
// OpenCV FAST_t<16> / cornerScore<16> restated (features2d/fast.cpp, 3.4).
// Runs on a window [x0,x1) x [y0,y1) of a level; emits window-local corners.
// ---------------------------------------------------------------------------
static const int offsets16[16][2] = {
    {0, 3}, {1, 3}, {2, 2}, {3, 1}, {3, 0}, {3, -1}, {2, -2}, {1, -3},
    {0, -3}, {-1, -3}, {-2, -2}, {-3, -1}, {-3, 0}, {-3, 1}, {-2, 2}, {-1, 3}};

static int corner_score16(const uint8_t* ptr, const int pixel[], int threshold) {
    const int K = 8, N = K * 3 + 1;
    int k, v = ptr[0];
    short d[N];
    for (k = 0; k < N; k++) d[k] = (short)(v - ptr[pixel[k]]);
    int a0 = threshold;
    for (k = 0; k < 16; k += 2) {
        int a = std::min((int)d[k + 1], (int)d[k + 2]);
        a = std::min(a, (int)d[k + 3]);
        if (a <= a0) continue;
        a = std::min(a, (int)d[k + 4]);
        a = std::min(a, (int)d[k + 5]);
        a = std::min(a, (int)d[k + 6]);
        a = std::min(a, (int)d[k + 7]);
        a = std::min(a, (int)d[k + 8]);
        a0 = std::max(a0, std::min(a, (int)d[k]));
        a0 = std::max(a0, std::min(a, (int)d[k + 9]));
    }
    int b0 = -a0;
    for (k = 0; k < 16; k += 2) {
        int b = std::max((int)d[k + 1], (int)d[k + 2]);
        b = std::max(b, (int)d[k + 3]);
        b = std::max(b, (int)d[k + 4]);
        b = std::max(b, (int)d[k + 5]);
        if (b >= b0) continue;
        b = std::max(b, (int)d[k + 6]);
        b = std::max(b, (int)d[k + 7]);
        b = std::max(b, (int)d[k + 8]);
        b0 = std::min(b0, std::max(b, (int)d[k]));
        b0 = std::min(b0, std::max(b, (int)d[k + 9]));
    }
    return -b0 - 1;
}

struct Cand { float x, y, response; };  // KeyPoint(pt, size 7, angle -1, response)

static void fast16_window(const Level& L, int x0, int y0, int x1, int y1, int threshold,
                          std::vector<Cand>& out) {
    out.clear();
    const int rows = y1 - y0, cols = x1 - x0;
    const int K = 8, N = 16 + K + 1;
    const int step = L.pw;
    int pixel[25];
    for (int k = 0; k < 16; k++) pixel[k] = offsets16[k][0] + offsets16[k][1] * step;
    for (int k = 16; k < 25; k++) pixel[k] = pixel[k - 16];
    threshold = std::min(std::max(threshold, 0), 255);
    uint8_t threshold_tab[512];
    for (int i = -255; i <= 255; i++)
        threshold_tab[i + 255] = (uint8_t)(i < -threshold ? 1 : i > threshold ? 2 : 0);
    if (cols <= 0 || rows <= 0) return;
    std::vector<uint8_t> bufv((size_t)cols * 3, 0);
    std::vector<int> cpv((size_t)(cols + 1) * 3, 0);
    uint8_t* buf[3] = {&bufv[0], &bufv[cols], &bufv[2 * cols]};
    int* cpbuf[3] = {&cpv[1], &cpv[cols + 2], &cpv[2 * cols + 3]};
    for (int i = 3; i < rows - 2; i++) {
        const uint8_t* ptr = L.at(x0, y0 + i) + 3;
        uint8_t* curr = buf[(i - 3) % 3];
        int* cornerpos = cpbuf[(i - 3) % 3];
        memset(curr, 0, cols);
        int ncorners = 0;
        if (i < rows - 3) {
            for (int j = 3; j < cols - 3; j++, ptr++) {
                int v = ptr[0];
                const uint8_t* tab = &threshold_tab[0] - v + 255;
                int d = tab[ptr[pixel[0]]] | tab[ptr[pixel[8]]];
                if (d == 0) continue;
                d &= tab[ptr[pixel[2]]] | tab[ptr[pixel[10]]];
                d &= tab[ptr[pixel[4]]] | tab[ptr[pixel[12]]];
                d &= tab[ptr[pixel[6]]] | tab[ptr[pixel[14]]];
                if (d == 0) continue;
                d &= tab[ptr[pixel[1]]] | tab[ptr[pixel[9]]];
                d &= tab[ptr[pixel[3]]] | tab[ptr[pixel[11]]];
                d &= tab[ptr[pixel[5]]] | tab[ptr[pixel[13]]];
                d &= tab[ptr[pixel[7]]] | tab[ptr[pixel[15]]];
                if (d & 1) {
                    int vt = v - threshold, count = 0;
                    for (int k = 0; k < N; k++) {
                        int x = ptr[pixel[k]];
                        if (x < vt) {
                            if (++count > K) {
                                cornerpos[ncorners++] = j;
                                curr[j] = (uint8_t)corner_score16(ptr, pixel, threshold);
                                break;
                            }
                        } else count = 0;
                    }
                }
                if (d & 2) {
                    int vt = v + threshold, count = 0;
                    for (int k = 0; k < N; k++) {
                        int x = ptr[pixel[k]];
                        if (x > vt) {
                            if (++count > K) {
                                cornerpos[ncorners++] = j;
                                curr[j] = (uint8_t)corner_score16(ptr, pixel, threshold);
                                break;
                            }
                        } else count = 0;
                    }
                }
            }
        }
        cornerpos[-1] = ncorners;
        if (i == 3) continue;
        const uint8_t* prev = buf[(i - 4 + 3) % 3];
        const uint8_t* pprev = buf[(i - 5 + 3) % 3];
        cornerpos = cpbuf[(i - 4 + 3) % 3];
        ncorners = cornerpos[-1];
        for (int k = 0; k < ncorners; k++) {
            int j = cornerpos[k];
            int score = prev[j];
            if (score > prev[j + 1] && score > prev[j - 1] && score > pprev[j - 1] &&
                score > pprev[j] && score > pprev[j + 1] && score > curr[j - 1] &&
                score > curr[j] && score > curr[j + 1]) {
                out.push_back(Cand{(float)j, (float)(i - 1), (float)score});
            }
        }
    }
}

// ---------------------------------------------------------------------------
// DistributeOctTree (ORBextractor.cc:539-763) with ExtractorNode::DivideNode
// (:481-537). Literal list-based replay; pinned tie-break P3 via `seq`.
// ---------------------------------------------------------------------------
struct Node {
    int ULx, ULy, URx, URy, BLx, BLy, BRx, BRy;
    std::vector<Cand> vKeys;
    std::list<Node>::iterator lit;
    bool bNoMore = false;
    long seq = 0;
};

static void divide_node(const Node& p, Node& n1, Node& n2, Node& n3, Node& n4) {
    const int halfX = (int)std::ceil(static_cast<float>(p.URx - p.ULx) / 2);
    const int halfY = (int)std::ceil(static_cast<float>(p.BRy - p.ULy) / 2);
    n1.ULx = p.ULx; n1.ULy = p.ULy;
    n1.URx = p.ULx + halfX; n1.URy = p.ULy;
    n1.BLx = p.ULx; n1.BLy = p.ULy + halfY;
    n1.BRx = p.ULx + halfX; n1.BRy = p.ULy + halfY;
    n2.ULx = n1.URx; n2.ULy = n1.URy;
    n2.URx = p.URx; n2.URy = p.URy;
    n2.BLx = n1.BRx; n2.BLy = n1.BRy;
    n2.BRx = p.URx; n2.BRy = p.ULy + halfY;
    n3.ULx = n1.BLx; n3.ULy = n1.BLy;
    n3.URx = n1.BRx; n3.URy = n1.BRy;
    n3.BLx = p.BLx; n3.BLy = p.BLy;
    n3.BRx = n1.BRx; n3.BRy = p.BLy;
    n4.ULx = n3.URx; n4.ULy = n3.URy;
    n4.URx = n2.BRx; n4.URy = n2.BRy;
    n4.BLx = n3.BRx; n4.BLy = n3.BRy;
    n4.BRx = p.BRx; n4.BRy = p.BRy;
    for (const Cand& kp : p.vKeys) {
        if (kp.x < n1.URx) {
            if (kp.y < n1.BRy) n1.vKeys.push_back(kp);
            else n3.vKeys.push_back(kp);
        } else if (kp.y < n1.BRy) n2.vKeys.push_back(kp);
        else n4.vKeys.push_back(kp);
    }
    if (n1.vKeys.size() == 1) n1.bNoMore = true;
    if (n2.vKeys.size() == 1) n2.bNoMore = true;
    if (n3.vKeys.size() == 1) n3.bNoMore = true;
    if (n4.vKeys.size() == 1) n4.bNoMore = true;
}

struct SizePtr {
    int size; long seq; Node* ptr;
    bool operator<(const SizePtr& o) const { return size != o.size ? size < o.size : seq < o.seq; }
};

static std::vector<Cand> distribute_octtree(const std::vector<Cand>& keys, int minX, int maxX,
                                            int minY, int maxY, int N) {
    long seq = 0;
    int nIni = (int)std::round(static_cast<float>(maxX - minX) / (maxY - minY));
    if (nIni < 1) nIni = 1;  // pinned: the reference divides by zero here
    const float hX = static_cast<float>(maxX - minX) / nIni;
    std::list<Node> lNodes;
    std::vector<Node*> vpIniNodes(nIni);
    for (int i = 0; i < nIni; i++) {
        Node ni;
        ni.ULx = (int)(hX * static_cast<float>(i)); ni.ULy = 0;
        ni.URx = (int)(hX * static_cast<float>(i + 1)); ni.URy = 0;
        ni.BLx = ni.ULx; ni.BLy = maxY - minY;
        ni.BRx = ni.URx; ni.BRy = maxY - minY;
        ni.seq = seq++;
        lNodes.push_back(ni);
        vpIniNodes[i] = &lNodes.back();
    }
    for (const Cand& kp : keys) {
        size_t idx = (size_t)(kp.x / hX);
        if (idx >= (size_t)nIni) idx = nIni - 1;  // pinned: reference indexes out of range
        vpIniNodes[idx]->vKeys.push_back(kp);
    }
    auto lit = lNodes.begin();
    while (lit != lNodes.end()) {
        if (lit->vKeys.size() == 1) { lit->bNoMore = true; lit++; }
        else if (lit->vKeys.empty()) lit = lNodes.erase(lit);
        else lit++;
    }
    bool bFinish = false;
    std::vector<SizePtr> vSizeAndPointerToNode;
    auto push_child = [&](Node& c, std::vector<SizePtr>& vec, int* nToExpand) {
        if (!c.vKeys.empty()) {
            c.seq = seq++;
            lNodes.push_front(c);
            if (c.vKeys.size() > 1) {
                if (nToExpand) (*nToExpand)++;
                vec.push_back(SizePtr{(int)c.vKeys.size(), lNodes.front().seq, &lNodes.front()});
                lNodes.front().lit = lNodes.begin();
            }
        }
    };
    while (!bFinish) {
        int prevSize = (int)lNodes.size();
        lit = lNodes.begin();
        int nToExpand = 0;
        vSizeAndPointerToNode.clear();
        while (lit != lNodes.end()) {
            if (lit->bNoMore) { lit++; continue; }
            Node n1, n2, n3, n4;
            divide_node(*lit, n1, n2, n3, n4);
            push_child(n1, vSizeAndPointerToNode, &nToExpand);
            push_child(n2, vSizeAndPointerToNode, &nToExpand);
            push_child(n3, vSizeAndPointerToNode, &nToExpand);
            push_child(n4, vSizeAndPointerToNode, &nToExpand);
            lit = lNodes.erase(lit);
        }
        if ((int)lNodes.size() >= N || (int)lNodes.size() == prevSize) {
            bFinish = true;
        } else if (((int)lNodes.size() + nToExpand * 3) > N) {
            while (!bFinish) {
                prevSize = (int)lNodes.size();
                std::vector<SizePtr> vPrev = vSizeAndPointerToNode;
                vSizeAndPointerToNode.clear();
                std::sort(vPrev.begin(), vPrev.end());
                for (int j = (int)vPrev.size() - 1; j >= 0; j--) {
                    Node n1, n2, n3, n4;
                    divide_node(*vPrev[j].ptr, n1, n2, n3, n4);
                    push_child(n1, vSizeAndPointerToNode, nullptr);
                    push_child(n2, vSizeAndPointerToNode, nullptr);
                    push_child(n3, vSizeAndPointerToNode, nullptr);
                    push_child(n4, vSizeAndPointerToNode, nullptr);
                    lNodes.erase(vPrev[j].ptr->lit);
                    if ((int)lNodes.size() >= N) break;
                }
                if ((int)lNodes.size() >= N || (int)lNodes.size() == prevSize) bFinish = true;
            }
        }
    }
    std::vector<Cand> res;
    for (auto it = lNodes.begin(); it != lNodes.end(); it++) {
        const std::vector<Cand>& v = it->vKeys;
        const Cand* best = &v[0];
        float maxResponse = best->response;
        for (size_t k = 1; k < v.size(); k++)
            if (v[k].response > maxResponse) { best = &v[k]; maxResponse = v[k].response; }
        res.push_back(*best);
    }
    return res;
}

// ---------------------------------------------------------------------------
// fastAtan2 (OpenCV 3.4 core, scalar path) and IC_Angle (ORBextractor.cc:77-104)
// ---------------------------------------------------------------------------
static const float atan2_p1 = 0.9997878412794807f * (float)(180 / M_PI);
static const float atan2_p3 = -0.3258083974640975f * (float)(180 / M_PI);
static const float atan2_p5 = 0.1555786518463281f * (float)(180 / M_PI);
static const float atan2_p7 = -0.04432655554792128f * (float)(180 / M_PI);

float fast_atan2(float y, float x) {
    float ax = std::fabs(x), ay = std::fabs(y);
    float a, c, c2;
    if (ax >= ay) {
        c = ay / (ax + (float)DBL_EPSILON);
        c2 = c * c;
        a = (((atan2_p7 * c2 + atan2_p5) * c2 + atan2_p3) * c2 + atan2_p1) * c;
    } else {
        c = ax / (ay + (float)DBL_EPSILON);
        c2 = c * c;
        a = 90.f - (((atan2_p7 * c2 + atan2_p5) * c2 + atan2_p3) * c2 + atan2_p1) * c;
    }
    if (x < 0) a = 180.f - a;
    if (y < 0) a = 360.f - a;
    return a;
}

static float ic_angle(const Level& L, float px, float py, const std::vector<int>& u_max) {
    int m_01 = 0, m_10 = 0;
    const uint8_t* center = L.at(cvRound_f(px), cvRound_f(py));
    for (int u = -HALF_PATCH_SIZE; u <= HALF_PATCH_SIZE; ++u) m_10 += u * center[u];
    int step = L.pw;
    for (int v = 1; v <= HALF_PATCH_SIZE; ++v) {
        int v_sum = 0;
        int d = u_max[v];
        for (int u = -d; u <= d; ++u) {
            int val_plus = center[u + v * step], val_minus = center[u - v * step];
            v_sum += (val_plus - val_minus);
            m_10 += u * (val_plus + val_minus);
        }
        m_01 += v * v_sum;
    }
    return fast_atan2((float)m_01, (float)m_10);
}

// ---------------------------------------------------------------------------
// GaussianBlur(7x7, sigma 2, REFLECT_101) for 8U, fixed-point path (pinned P4).
// Applied to the isolated level image; REFLECT_101 of the isolated level is
// exactly the padded border built by ComputePyramid.
// ---------------------------------------------------------------------------
static const int GK[7] = {18, 34, 49, 54, 49, 34, 18};

static void gaussian_blur(const Level& S, Level& D) {
    D.w = S.w; D.h = S.h; D.pw = S.pw; D.ph = S.ph;
    D.buf.assign(S.buf.size(), 0);
    std::vector<int> tmp((size_t)S.w * (S.h + 6));
    for (int y = -3; y < S.h + 3; y++) {
        int sy = reflect101(y, S.h);
        for (int x = 0; x < S.w; x++) {
            int acc = 0;
            for (int k = 0; k < 7; k++) acc += GK[k] * S.at(reflect101(x + k - 3, S.w), sy)[0];
            tmp[(size_t)(y + 3) * S.w + x] = acc;
        }
    }
    for (int y = 0; y < S.h; y++)
        for (int x = 0; x < S.w; x++) {
            int acc = 0;
            for (int k = 0; k < 7; k++) acc += GK[k] * tmp[(size_t)(y + k) * S.w + x];
            D.at(x, y)[0] = (uint8_t)std::min(255, (acc + (1 << 15)) >> 16);
        }
}

// computeOrbDescriptor (ORBextractor.cc:108-147). a,b pinned P2.
static const float factorPI = (float)(M_PI / 180.f);

static void orb_descriptor(float kx, float ky, float kangle, const Level& img, uint8_t* desc) {
    float angle = (float)kangle * factorPI;
    float a = pmath::cosf_cr(angle), b = pmath::sinf_cr(angle);
    const uint8_t* center = img.at(cvRound_f(kx), cvRound_f(ky));
    const int step = img.pw;
    const int* pattern = bit_pattern_31_;
    auto get = [&](int idx) {
        float px = (float)pattern[idx * 2], py = (float)pattern[idx * 2 + 1];
        return (int)center[cvRound_f(px * b + py * a) * step + cvRound_f(px * a - py * b)];
    };
    for (int i = 0; i < 32; ++i, pattern += 32) {
        int val = 0;
        for (int t = 0; t < 8; t++) {
            int t0 = get(2 * t), t1 = get(2 * t + 1);
            val |= (t0 < t1) << t;
        }
        desc[i] = (uint8_t)val;
    }
}

struct KP { float x, y, size, angle, response; int octave, class_id; };

// ComputeKeyPointsOctTree (ORBextractor.cc:765-853)
static void keypoints_octtree(const Extractor& E, const std::vector<Level>& pyr,
                              std::vector<std::vector<KP>>& all,
                              std::vector<std::vector<Cand>>* cands_out) {
    all.assign(E.nlevels, {});
    if (cands_out) cands_out->assign(E.nlevels, {});
    const float W = 30;
    for (int level = 0; level < E.nlevels; ++level) {
        const Level& L = pyr[level];
        const int minBorderX = EDGE_THRESHOLD - 3, minBorderY = minBorderX;
        const int maxBorderX = L.w - EDGE_THRESHOLD + 3, maxBorderY = L.h - EDGE_THRESHOLD + 3;
        std::vector<Cand> toDist;
        const float width = (float)(maxBorderX - minBorderX);
        const float height = (float)(maxBorderY - minBorderY);
        const int nCols = (int)(width / W), nRows = (int)(height / W);
        const int wCell = (int)std::ceil(width / nCols), hCell = (int)std::ceil(height / nRows);
        std::vector<Cand> cell;
        for (int i = 0; i < nRows; i++) {
            const float iniY = (float)(minBorderY + i * hCell);
            float maxY = iniY + hCell + 6;
            if (iniY >= maxBorderY - 3) continue;
            if (maxY > maxBorderY) maxY = (float)maxBorderY;
            for (int j = 0; j < nCols; j++) {
                const float iniX = (float)(minBorderX + j * wCell);
                float maxX = iniX + wCell + 6;
                if (iniX >= maxBorderX - 6) continue;
                if (maxX > maxBorderX) maxX = (float)maxBorderX;
                fast16_window(L, (int)iniX, (int)iniY, (int)maxX, (int)maxY, E.iniThFAST, cell);
                if (cell.empty())
                    fast16_window(L, (int)iniX, (int)iniY, (int)maxX, (int)maxY, E.minThFAST, cell);
                for (Cand c : cell) {
                    c.x += j * wCell;
                    c.y += i * hCell;
                    toDist.push_back(c);
                }
            }
        }
        if (cands_out) (*cands_out)[level] = toDist;
        std::vector<Cand> kept = distribute_octtree(toDist, minBorderX, maxBorderX, minBorderY,
                                                    maxBorderY, E.mnFeaturesPerLevel[level]);
        const int scaledPatchSize = (int)(PATCH_SIZE * E.mvScaleFactor[level]);
        for (const Cand& c : kept)
            all[level].push_back(KP{c.x + minBorderX, c.y + minBorderY, (float)scaledPatchSize, -1.f,
                                    c.response, level, -1});
    }
    for (int level = 0; level < E.nlevels; ++level)
        for (KP& k : all[level]) k.angle = ic_angle(pyr[level], k.x, k.y, E.umax);
}

}  // namespace oracle

using namespace oracle;

extern "C" {

int oracle_orb_level_sizes(const orbpl_orb_params* p, int w, int h, int* lw, int* lh,
                           int* nfeat_per_level, float* scale, float* inv_scale) {
    Extractor E(p->nfeatures, p->scale_factor, p->nlevels, p->ini_th_fast, p->min_th_fast);
    for (int l = 0; l < E.nlevels; l++) {
        if (lw) lw[l] = cvRound_f((float)w * E.mvInvScaleFactor[l]);
        if (lh) lh[l] = cvRound_f((float)h * E.mvInvScaleFactor[l]);
        if (nfeat_per_level) nfeat_per_level[l] = E.mnFeaturesPerLevel[l];
        if (scale) scale[l] = E.mvScaleFactor[l];
        if (inv_scale) inv_scale[l] = E.mvInvScaleFactor[l];
    }
    return 0;
}

// Padded pyramid, levels concatenated, each (w+38)*(h+38) bytes row-major.
int oracle_orb_pyramid(const orbpl_orb_params* p, const uint8_t* img, int w, int h, int stride,
                       uint8_t* out, int blurred) {
    Extractor E(p->nfeatures, p->scale_factor, p->nlevels, p->ini_th_fast, p->min_th_fast);
    std::vector<Level> pyr;
    compute_pyramid(E, img, w, h, stride, pyr);
    size_t off = 0;
    for (auto& L : pyr) {
        if (blurred) {
            Level B;
            gaussian_blur(L, B);
            memcpy(out + off, B.buf.data(), B.buf.size());
        } else {
            memcpy(out + off, L.buf.data(), L.buf.size());
        }
        off += L.buf.size();
    }
    return 0;
}

// Pre-octree candidates (vToDistributeKeys) per level, concatenated; packed as
// (x, y, response) float triples relative to minBorder (=16).
int oracle_orb_candidates(const orbpl_orb_params* p, const uint8_t* img, int w, int h, int stride,
                          float* out_xyr, int cap, int* level_counts) {
    Extractor E(p->nfeatures, p->scale_factor, p->nlevels, p->ini_th_fast, p->min_th_fast);
    std::vector<Level> pyr;
    compute_pyramid(E, img, w, h, stride, pyr);
    std::vector<std::vector<KP>> all;
    std::vector<std::vector<Cand>> cands;
    keypoints_octtree(E, pyr, all, &cands);
    int n = 0;
    for (int l = 0; l < E.nlevels; l++) {
        level_counts[l] = (int)cands[l].size();
        for (const Cand& c : cands[l]) {
            if (n < cap) { out_xyr[3 * n] = c.x; out_xyr[3 * n + 1] = c.y; out_xyr[3 * n + 2] = c.response; }
            n++;
        }
    }
    return n > cap ? -1 : n;
}

// ORBextractor::operator() (ORBextractor.cc:1043-1105).
int oracle_orb_extract(const orbpl_orb_params* p, const uint8_t* img, int w, int h, int stride,
                       orbpl_keypoint* kps, uint8_t* desc, int cap, int* n_out, int* level_counts) {
    *n_out = 0;
    if (!img || w <= 0 || h <= 0) return 0;  // _image.empty() -> return
    Extractor E(p->nfeatures, p->scale_factor, p->nlevels, p->ini_th_fast, p->min_th_fast);
    std::vector<Level> pyr;
    compute_pyramid(E, img, w, h, stride, pyr);
    std::vector<std::vector<KP>> all;
    keypoints_octtree(E, pyr, all, nullptr);
    int total = 0;
    for (auto& v : all) total += (int)v.size();
    if (total > cap) return -2;
    int offset = 0;
    for (int level = 0; level < E.nlevels; ++level) {
        std::vector<KP>& kl = all[level];
        if (level_counts) level_counts[level] = (int)kl.size();
        if (kl.empty()) continue;
        Level B;
        gaussian_blur(pyr[level], B);
        for (size_t i = 0; i < kl.size(); i++)
            orb_descriptor(kl[i].x, kl[i].y, kl[i].angle, B, desc + (size_t)(offset + i) * 32);
        if (level != 0) {
            float scale = E.mvScaleFactor[level];
            for (KP& k : kl) { k.x *= scale; k.y *= scale; }
        }
        for (size_t i = 0; i < kl.size(); i++) {
            orbpl_keypoint& o = kps[offset + i];
            o.x = kl[i].x; o.y = kl[i].y; o.size = kl[i].size; o.angle = kl[i].angle;
            o.response = kl[i].response; o.octave = kl[i].octave; o.class_id = kl[i].class_id;
        }
        offset += (int)kl.size();
    }
    *n_out = offset;
    return 0;
}

float oracle_fast_atan2(float y, float x) { return fast_atan2(y, x); }

}  // extern "C"
