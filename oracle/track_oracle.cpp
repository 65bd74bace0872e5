// ============================================================================
// ORACLE — TEST INFRASTRUCTURE ONLY. NOT PART OF THE PRODUCT PATH.
//
// CPU restatement of the per-frame tracking path after extraction:
//   Frame glue      : src/Frame.cc:135-205, 265-287, 432-485, 527-538,
//                     737-764, 847-885, 1065-1117 (+ cv::undistortPoints)
//   ORB matching    : src/ORBmatcher.cc:1710-1879 (SearchByProjection last
//                     frame), :2035-2077 (ComputeThreeMaxima), :2083-2103
//   Pose-only LM    : src/Optimizer.cc:375-619, 2132-2486 with the g2o pieces
//                     Thirdparty/g2o/g2o/core/optimization_algorithm_levenberg.cpp:61-164,
//                     core/sparse_optimizer.cpp:100-113,354-420,
//                     core/base_unary_edge.hpp:43-72, core/robust_kernel_impl.cpp:65-91,
//                     types/types_six_dof_expmap.{h,cpp} (OnlyPose edges),
//                     types/se3quat.h (exp, product, map), include/types_line_expmap.h:66-199
//
// Pinned semantics beyond orb_oracle.cpp (DESIGN.md "Pinned semantics"):
//   P6 cv::Mat float 3x3*3x1 (+c) products = double accumulation of exact
//      float products, rounded to float once (OpenCV GEMMSingleMul, WT=double).
//   P7 EdgeLineOnlyPose::linearizeOplus: row 1 of del_dI is never written in
//      the reference (uninitialised); pinned to 0, row 0 keeps the end-point
//      values the reference leaves there, dI_dLc keeps its +fx*cy sign.
//   P8 6x6 solve: Cholesky (LDL^T without pivoting) instead of Eigen's
//      pivoted LDLT; results agree to rounding (pose tolerance 1e-4).
// parity unpinned against the real reference binary (no fixtures exist).
// ============================================================================
#include <algorithm>
#include <climits>
#include <map>
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <vector>

#include "pinned_math.h"
#include "oracle_api.h"

namespace oracle_track {

// ---------------------------------------------------------------------------
// cv::undistortPoints(src, dst, K, D, noArray(), K) for one point: OpenCV 3.4
// cvUndistortPointsInternal with TermCriteria(COUNT, 5) (clean-room).
// ---------------------------------------------------------------------------
static void undistort_point(const orbpl_camera& c, float px, float py, float* ox, float* oy) {
  const double fx = c.fx, fy = c.fy, cx = c.cx, cy = c.cy;
  const double k[12] = {c.k1, c.k2, c.p1, c.p2, c.k3, 0, 0, 0, 0, 0, 0, 0};
  const double ifx = 1. / fx, ify = 1. / fy;
  double x = px, y = py;
  x = (x - cx) * ifx;
  y = (y - cy) * ify;
  const double x0 = x, y0 = y;
  for (int j = 0; j < 5; j++) {
    double r2 = x * x + y * y;
    double icdist = (1 + ((k[7] * r2 + k[6]) * r2 + k[5]) * r2) / (1 + ((k[4] * r2 + k[1]) * r2 + k[0]) * r2);
    double deltaX = 2 * k[2] * x * y + k[3] * (r2 + 2 * x * x) + k[8] * r2 + k[9] * r2 * r2;
    double deltaY = k[2] * (r2 + 2 * y * y) + 2 * k[3] * x * y + k[10] * r2 + k[11] * r2 * r2;
    x = (x0 - deltaX) * icdist;
    y = (y0 - deltaY) * icdist;
  }
  // RR = P * I = K
  double xx = fx * x + 0.0 * y + cx;
  double yy = 0.0 * x + fy * y + cy;
  double ww = 1. / (0.0 * x + 0.0 * y + 1.0);
  *ox = (float)(xx * ww);
  *oy = (float)(yy * ww);
}

static void image_bounds(const orbpl_camera& c, float* b) {
  if (c.k1 != 0.0f) {
    float ux[4], uy[4];
    const float px[4] = {0.0f, (float)c.width, 0.0f, (float)c.width};
    const float py[4] = {0.0f, 0.0f, (float)c.height, (float)c.height};
    for (int i = 0; i < 4; i++) undistort_point(c, px[i], py[i], &ux[i], &uy[i]);
    b[0] = std::min(ux[0], ux[2]);
    b[1] = std::max(ux[1], ux[3]);
    b[2] = std::min(uy[0], uy[1]);
    b[3] = std::max(uy[2], uy[3]);
  } else {
    b[0] = 0.0f; b[1] = (float)c.width; b[2] = 0.0f; b[3] = (float)c.height;
  }
}

struct Grid {
  float minX, maxX, minY, maxY, invW, invH;
  std::vector<int> cells[ORBPL_GRID_COLS][ORBPL_GRID_ROWS];
};

static void grid_constants(const orbpl_camera& c, Grid& g) {
  float b[4];
  image_bounds(c, b);
  g.minX = b[0]; g.maxX = b[1]; g.minY = b[2]; g.maxY = b[3];
  g.invW = static_cast<float>(ORBPL_GRID_COLS) / static_cast<float>(g.maxX - g.minX);
  g.invH = static_cast<float>(ORBPL_GRID_ROWS) / static_cast<float>(g.maxY - g.minY);
}

static bool pos_in_grid(const Grid& g, float x, float y, int* px, int* py) {
  *px = (int)std::round((x - g.minX) * g.invW);
  *py = (int)std::round((y - g.minY) * g.invH);
  return !(*px < 0 || *px >= ORBPL_GRID_COLS || *py < 0 || *py >= ORBPL_GRID_ROWS);
}

// ---------------------------------------------------------------------------
// SE3 with a unit quaternion, mirroring g2o::SE3Quat / Eigen semantics.
// ---------------------------------------------------------------------------
struct Quat { double w, x, y, z; };
struct SE3 { Quat q; double t[3]; };

static void quat_normalize(Quat& q) {
  double n = std::sqrt(q.w * q.w + q.x * q.x + q.y * q.y + q.z * q.z);
  q.w /= n; q.x /= n; q.y /= n; q.z /= n;
}
static void normalize_rotation(Quat& q) {
  if (q.w < 0) { q.w = -q.w; q.x = -q.x; q.y = -q.y; q.z = -q.z; }
  quat_normalize(q);
}
static Quat quat_from_R(const double m[3][3]) {  // Eigen quaternionbase_assign_impl
  Quat q;
  double t = m[0][0] + m[1][1] + m[2][2];
  if (t > 0) {
    t = std::sqrt(t + 1.0);
    q.w = 0.5 * t;
    t = 0.5 / t;
    q.x = (m[2][1] - m[1][2]) * t;
    q.y = (m[0][2] - m[2][0]) * t;
    q.z = (m[1][0] - m[0][1]) * t;
  } else {
    int i = 0;
    if (m[1][1] > m[0][0]) i = 1;
    if (m[2][2] > m[i][i]) i = 2;
    int j = (i + 1) % 3, k = (j + 1) % 3;
    t = std::sqrt(m[i][i] - m[j][j] - m[k][k] + 1.0);
    double v[3];
    v[i] = 0.5 * t;
    t = 0.5 / t;
    q.w = (m[k][j] - m[j][k]) * t;
    v[j] = (m[j][i] + m[i][j]) * t;
    v[k] = (m[k][i] + m[i][k]) * t;
    q.x = v[0]; q.y = v[1]; q.z = v[2];
  }
  return q;
}
static void quat_to_R(const Quat& q, double R[3][3]) {
  const double tx = 2 * q.x, ty = 2 * q.y, tz = 2 * q.z;
  const double twx = tx * q.w, twy = ty * q.w, twz = tz * q.w;
  const double txx = tx * q.x, txy = ty * q.x, txz = tz * q.x;
  const double tyy = ty * q.y, tyz = tz * q.y, tzz = tz * q.z;
  R[0][0] = 1 - (tyy + tzz); R[0][1] = txy - twz; R[0][2] = txz + twy;
  R[1][0] = txy + twz; R[1][1] = 1 - (txx + tzz); R[1][2] = tyz - twx;
  R[2][0] = txz - twy; R[2][1] = tyz + twx; R[2][2] = 1 - (txx + tyy);
}
static void quat_rotate(const Quat& q, const double v[3], double o[3]) {  // Eigen _transformVector
  double uv[3] = {q.y * v[2] - q.z * v[1], q.z * v[0] - q.x * v[2], q.x * v[1] - q.y * v[0]};
  uv[0] += uv[0]; uv[1] += uv[1]; uv[2] += uv[2];
  double c[3] = {q.y * uv[2] - q.z * uv[1], q.z * uv[0] - q.x * uv[2], q.x * uv[1] - q.y * uv[0]};
  o[0] = v[0] + q.w * uv[0] + c[0];
  o[1] = v[1] + q.w * uv[1] + c[1];
  o[2] = v[2] + q.w * uv[2] + c[2];
}
static Quat quat_mul(const Quat& a, const Quat& b) {
  Quat r;
  r.w = a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z;
  r.x = a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y;
  r.y = a.w * b.y + a.y * b.w + a.z * b.x - a.x * b.z;
  r.z = a.w * b.z + a.z * b.w + a.x * b.y - a.y * b.x;
  return r;
}
static SE3 se3_from_T(const float* T) {  // Converter::toSE3Quat + SE3Quat(R,t)
  double R[3][3];
  for (int r = 0; r < 3; r++)
    for (int c = 0; c < 3; c++) R[r][c] = T[r * 4 + c];
  SE3 s;
  s.q = quat_from_R(R);
  normalize_rotation(s.q);
  s.t[0] = T[3]; s.t[1] = T[7]; s.t[2] = T[11];
  return s;
}
static void se3_to_T(const SE3& s, float* T) {  // to_homogeneous_matrix + toCvMat
  double R[3][3];
  quat_to_R(s.q, R);
  for (int r = 0; r < 3; r++) {
    for (int c = 0; c < 3; c++) T[r * 4 + c] = (float)R[r][c];
    T[r * 4 + 3] = (float)s.t[r];
  }
  T[12] = 0; T[13] = 0; T[14] = 0; T[15] = 1;
}
static void se3_map(const SE3& s, const double X[3], double o[3]) {
  quat_rotate(s.q, X, o);
  o[0] += s.t[0]; o[1] += s.t[1]; o[2] += s.t[2];
}
static SE3 se3_exp(const double u[6]) {  // SE3Quat::exp (se3quat.h:223-257)
  const double w[3] = {u[0], u[1], u[2]}, up[3] = {u[3], u[4], u[5]};
  const double theta = std::sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
  const double O[3][3] = {{0, -w[2], w[1]}, {w[2], 0, -w[0]}, {-w[1], w[0], 0}};
  double O2[3][3];
  for (int r = 0; r < 3; r++)
    for (int c = 0; c < 3; c++) O2[r][c] = O[r][0] * O[0][c] + O[r][1] * O[1][c] + O[r][2] * O[2][c];
  double R[3][3], V[3][3];
  if (theta < 0.00001) {
    for (int r = 0; r < 3; r++)
      for (int c = 0; c < 3; c++) R[r][c] = (r == c ? 1.0 : 0.0) + O[r][c] + O2[r][c];
    memcpy(V, R, sizeof(R));
  } else {
    const double a = std::sin(theta) / theta;
    const double b = (1 - std::cos(theta)) / (theta * theta);
    const double cc = (theta - std::sin(theta)) / (theta * theta * theta);
    for (int r = 0; r < 3; r++)
      for (int c = 0; c < 3; c++) {
        R[r][c] = (r == c ? 1.0 : 0.0) + a * O[r][c] + b * O2[r][c];
        V[r][c] = (r == c ? 1.0 : 0.0) + b * O[r][c] + cc * O2[r][c];
      }
  }
  SE3 s;
  s.q = quat_from_R(R);
  normalize_rotation(s.q);
  for (int r = 0; r < 3; r++) s.t[r] = V[r][0] * up[0] + V[r][1] * up[1] + V[r][2] * up[2];
  return s;
}
static SE3 se3_mul(const SE3& a, const SE3& b) {  // SE3Quat::operator*
  SE3 r = a;
  double rt[3];
  quat_rotate(a.q, b.t, rt);
  r.t[0] += rt[0]; r.t[1] += rt[1]; r.t[2] += rt[2];
  r.q = quat_mul(a.q, b.q);
  normalize_rotation(r.q);
  return r;
}

// Pinned P6: float 3x3 * 3x1 (+ c) as OpenCV gemm with double accumulation.
static void gemm33(const float* T, const float* x, float* out) {  // Rcw*x + tcw
  for (int r = 0; r < 3; r++) {
    double s = (double)T[r * 4] * x[0];
    s += (double)T[r * 4 + 1] * x[1];
    s += (double)T[r * 4 + 2] * x[2];
    out[r] = (float)(s + (double)T[r * 4 + 3]);
  }
}

// ---------------------------------------------------------------------------
// Pose optimisation edges (double, g2o semantics)
// ---------------------------------------------------------------------------
struct Edge {
  int kind;       // 0 mono, 1 stereo, 2 line
  int idx;        // frame index
  double obs[4];
  double X[3];    // point Xw
  double nw[3], vw[3];
  double info;    // invSigma2
  double delta, dsqr_f;  // Huber delta and (float) delta^2
  int level;      // 0 active, 1 outlier
  bool robust;
  double err[3];
  int dim;
};

struct Cam {
  double fx, fy, cx, cy, bf;
  int fixed_line_jac;  // 1: analytic EdgeLineOnlyPose Jacobian (ORBPL_POSE_FIXED_LINE_JAC)
};

static void edge_error(const Edge& e, const Cam& c, const SE3& T, double* err) {
  if (e.kind == 2) {
    double R[3][3];
    quat_to_R(T.q, R);
    const double* t = T.t;
    double Rn[3], Rv[3];
    for (int r = 0; r < 3; r++) {
      Rn[r] = R[r][0] * e.nw[0] + R[r][1] * e.nw[1] + R[r][2] * e.nw[2];
      Rv[r] = R[r][0] * e.vw[0] + R[r][1] * e.vw[1] + R[r][2] * e.vw[2];
    }
    // tcw_hat * Rv
    double tRv[3] = {-t[2] * Rv[1] + t[1] * Rv[2], t[2] * Rv[0] - t[0] * Rv[2], -t[1] * Rv[0] + t[0] * Rv[1]};
    double nc[3] = {Rn[0] + tRv[0], Rn[1] + tRv[1], Rn[2] + tRv[2]};
    double l0 = c.fy * nc[0], l1 = c.fx * nc[1];
    double l2 = -c.fy * c.cx * nc[0] + -c.fx * c.cy * nc[1] + c.fx * c.fy * nc[2];
    double sq = std::sqrt(std::pow(l0, 2) + std::pow(l1, 2));
    err[0] = (e.obs[0] * l0 + e.obs[1] * l1 + l2) / sq;
    err[1] = (e.obs[2] * l0 + e.obs[3] * l1 + l2) / sq;
    return;
  }
  double p[3];
  se3_map(T, e.X, p);
  if (e.kind == 0) {
    double u = p[0] / p[2] * c.fx + c.cx;
    double v = p[1] / p[2] * c.fy + c.cy;
    err[0] = e.obs[0] - u;
    err[1] = e.obs[1] - v;
  } else {
    const float invz = (float)(1.0 / p[2]);
    double u = p[0] * (double)invz * c.fx + c.cx;
    double v = p[1] * (double)invz * c.fy + c.cy;
    double ur = u - c.bf * (double)invz;
    err[0] = e.obs[0] - u;
    err[1] = e.obs[1] - v;
    err[2] = e.obs[2] - ur;
  }
}

static void edge_jacobian(const Edge& e, const Cam& c, const SE3& T, double J[3][6]) {
  if (e.kind == 2) {
    double R[3][3];
    quat_to_R(T.q, R);
    const double* t = T.t;
    double Rn[3], Rv[3];
    for (int r = 0; r < 3; r++) {
      Rn[r] = R[r][0] * e.nw[0] + R[r][1] * e.nw[1] + R[r][2] * e.nw[2];
      Rv[r] = R[r][0] * e.vw[0] + R[r][1] * e.vw[1] + R[r][2] * e.vw[2];
    }
    double tRv[3] = {-t[2] * Rv[1] + t[1] * Rv[2], t[2] * Rv[0] - t[0] * Rv[2], -t[1] * Rv[0] + t[0] * Rv[1]};
    double nc[3] = {Rn[0] + tRv[0], Rn[1] + tRv[1], Rn[2] + tRv[2]};
    double l0 = c.fy * nc[0], l1 = c.fx * nc[1];
    double l2 = -c.fy * c.cx * nc[0] + -c.fx * c.cy * nc[1] + c.fx * c.fy * nc[2];
    double ln = std::sqrt(std::pow(l0, 2) + std::pow(l1, 2));
    auto skew = [](const double v[3], double S[3][3]) {
      S[0][0] = 0; S[0][1] = -v[2]; S[0][2] = v[1];
      S[1][0] = v[2]; S[1][1] = 0; S[1][2] = -v[0];
      S[2][0] = -v[1]; S[2][1] = v[0]; S[2][2] = 0;
    };
    if (c.fixed_line_jac) {
      // Analytic form (--fixed-line-jacobian): with the
      // left perturbation exp(d) T, d = (w, u), the camera Plucker line moves
      // as dn = w x n_c + u x v_c, so dn/dd = [-[n_c]x | -[v_c]x]; the two
      // end-point distances e_i = (x_i l0 + y_i l1 + l2) / |l_01| give
      // de_i/dl = ((x_i - l0 N_i / ln^2) / ln, (y_i - l1 N_i / ln^2) / ln, 1 / ln)
      // and l = K_line n_c with K_line as in computeError (-fx*cy).
      const double N[2] = {e.obs[0] * l0 + e.obs[1] * l1 + l2, e.obs[2] * l0 + e.obs[3] * l1 + l2};
      double dd[2][3];
      for (int r = 0; r < 2; r++) {
        dd[r][0] = (e.obs[2 * r] - (l0 * N[r]) / (ln * ln)) / ln;
        dd[r][1] = (e.obs[2 * r + 1] - (l1 * N[r]) / (ln * ln)) / ln;
        dd[r][2] = 1.0 / ln;
      }
      const double A[3][3] = {{c.fy, 0, 0}, {0, c.fx, 0}, {-c.fy * c.cx, -c.fx * c.cy, c.fx * c.fy}};
      double Sn[3][3], Sv[3][3];
      skew(nc, Sn);
      skew(Rv, Sv);
      double M[2][3];
      for (int r = 0; r < 2; r++)
        for (int k = 0; k < 3; k++) M[r][k] = dd[r][0] * A[0][k] + dd[r][1] * A[1][k] + dd[r][2] * A[2][k];
      for (int r = 0; r < 2; r++)
        for (int k = 0; k < 3; k++) {
          J[r][k] = -(M[r][0] * Sn[0][k] + M[r][1] * Sn[1][k] + M[r][2] * Sn[2][k]);
          J[r][3 + k] = -(M[r][0] * Sv[0][k] + M[r][1] * Sv[1][k] + M[r][2] * Sv[2][k]);
        }
      return;
    }
    double e2 = e.obs[2] * l0 + e.obs[3] * l1 + l2;
    // P7: row 0 holds the end-point values, row 1 pinned to zero
    double dd[2][3] = {{(e.obs[2] - (l0 * e2) / (ln * ln)) / ln, (e.obs[3] - (l1 * e2) / (ln * ln)) / ln, 1.0},
                       {0.0, 0.0, 0.0}};
    const double A[3][3] = {{c.fy, 0, 0}, {0, c.fx, 0}, {-c.fy * c.cx, c.fx * c.cy, c.fx * c.fy}};
    double S1[3][3], S2[3][3];
    skew(Rv, S1);
    skew(tRv, S2);
    double D[3][6];  // rows 0..2 of dLc_ddelta
    for (int r = 0; r < 3; r++)
      for (int k = 0; k < 3; k++) {
        D[r][k] = -1.0 * S1[r][k] - S2[r][k];
        D[r][3 + k] = -1.0 * S1[r][k];
      }
    double M[2][3];
    for (int r = 0; r < 2; r++)
      for (int k = 0; k < 3; k++) M[r][k] = dd[r][0] * A[0][k] + dd[r][1] * A[1][k] + dd[r][2] * A[2][k];
    for (int r = 0; r < 2; r++)
      for (int k = 0; k < 6; k++) J[r][k] = M[r][0] * D[0][k] + M[r][1] * D[1][k] + M[r][2] * D[2][k];
    return;
  }
  double p[3];
  se3_map(T, e.X, p);
  const double x = p[0], y = p[1], invz = 1.0 / p[2], invz_2 = invz * invz;
  J[0][0] = x * y * invz_2 * c.fx;
  J[0][1] = -(1 + (x * x * invz_2)) * c.fx;
  J[0][2] = y * invz * c.fx;
  J[0][3] = -invz * c.fx;
  J[0][4] = 0;
  J[0][5] = x * invz_2 * c.fx;
  J[1][0] = (1 + y * y * invz_2) * c.fy;
  J[1][1] = -x * y * invz_2 * c.fy;
  J[1][2] = -x * invz * c.fy;
  J[1][3] = 0;
  J[1][4] = -invz * c.fy;
  J[1][5] = y * invz_2 * c.fy;
  if (e.kind == 1) {
    J[2][0] = J[0][0] - c.bf * y * invz_2;
    J[2][1] = J[0][1] + c.bf * x * invz_2;
    J[2][2] = J[0][2];
    J[2][3] = J[0][3];
    J[2][4] = 0;
    J[2][5] = J[0][5] - c.bf * invz_2;
  }
}

static double edge_chi2(const Edge& e) {
  double s = 0;
  for (int k = 0; k < e.dim; k++) s += e.err[k] * e.info * e.err[k];
  return s;
}

static void huber(const Edge& e, double chi, double rho[3]) {  // robust_kernel_impl.cpp:78-91
  if (chi <= e.dsqr_f) {
    rho[0] = chi; rho[1] = 1.; rho[2] = 0.;
  } else {
    double sq = std::sqrt(chi);
    rho[0] = 2 * sq * e.delta - e.dsqr_f;
    rho[1] = e.delta / sq;
    rho[2] = -0.5 * rho[1] / chi;
  }
}

struct LM {
  std::vector<Edge>& E;
  const Cam& c;
  SE3 T;
  double lambda = -1, ni = 2;
  int nBad = 0;
  LM(std::vector<Edge>& e, const Cam& cc) : E(e), c(cc) {}

  double active_errors() {
    double chi = 0;
    for (Edge& e : E) {
      if (e.level) continue;
      edge_error(e, c, T, e.err);
      double x2 = edge_chi2(e);
      if (e.robust) {
        double rho[3];
        huber(e, x2, rho);
        chi += rho[0];
      } else {
        chi += x2;
      }
    }
    return chi;
  }

  void build(double H[6][6], double b[6]) {
    memset(H, 0, sizeof(double) * 36);
    memset(b, 0, sizeof(double) * 6);
    for (Edge& e : E) {
      if (e.level) continue;
      double J[3][6];
      edge_jacobian(e, c, T, J);
      double w = 1.0;
      if (e.robust) {
        double rho[3];
        huber(e, edge_chi2(e), rho);
        w = rho[1];
      }
      for (int i = 0; i < 6; i++) {
        double bi = 0;
        for (int k = 0; k < e.dim; k++) bi += J[k][i] * e.info * e.err[k];
        b[i] -= w * bi;
        for (int j = 0; j < 6; j++) {
          double h = 0;
          for (int k = 0; k < e.dim; k++) h += J[k][i] * (w * e.info) * J[k][j];
          H[i][j] += h;
        }
      }
    }
  }

  static bool solve6(const double A[6][6], const double b[6], double x[6]) {
    double L[6][6] = {}, D[6];
    for (int j = 0; j < 6; j++) {
      double d = A[j][j];
      for (int k = 0; k < j; k++) d -= L[j][k] * L[j][k] * D[k];
      D[j] = d;
      if (!(d > 0)) return false;
      for (int i = j + 1; i < 6; i++) {
        double s = A[i][j];
        for (int k = 0; k < j; k++) s -= L[i][k] * L[j][k] * D[k];
        L[i][j] = s / d;
      }
    }
    double y[6];
    for (int i = 0; i < 6; i++) {
      double s = b[i];
      for (int k = 0; k < i; k++) s -= L[i][k] * y[k];
      y[i] = s;
    }
    for (int i = 5; i >= 0; i--) {
      double s = y[i] / D[i];
      for (int k = i + 1; k < 6; k++) s -= L[k][i] * x[k];
      x[i] = s;
    }
    return true;
  }

  // SparseOptimizer::optimize(iterations) with OptimizationAlgorithmLevenberg
  void optimize(int iterations) {
    bool any = false;
    for (Edge& e : E) any |= (e.level == 0);
    if (!any) return;  // "0 vertices to optimize"
    double x[6] = {0, 0, 0, 0, 0, 0};
    for (int it = 0; it < iterations; it++) {
      double currentChi = active_errors();
      const double iniChi = currentChi;
      double H[6][6], b[6];
      build(H, b);
      if (it == 0) {
        double md = 0;
        for (int j = 0; j < 6; j++) md = std::max(std::fabs(H[j][j]), md);
        lambda = 1e-5 * md;
        ni = 2;
        nBad = 0;
      }
      double rho = 0;
      int qmax = 0;
      do {
        SE3 backup = T;
        double Hl[6][6];
        memcpy(Hl, H, sizeof(Hl));
        for (int j = 0; j < 6; j++) Hl[j][j] += lambda;
        bool ok2 = solve6(Hl, b, x);
        T = se3_mul(se3_exp(x), T);
        double tempChi = active_errors();
        if (!ok2) tempChi = std::numeric_limits<double>::max();
        rho = currentChi - tempChi;
        double scale = 0;
        for (int j = 0; j < 6; j++) scale += x[j] * (lambda * x[j] + b[j]);
        scale += 1e-3;
        rho /= scale;
        if (rho > 0 && std::isfinite(tempChi)) {
          double alpha = 1. - std::pow((2 * rho - 1), 3);
          alpha = std::min(alpha, 2. / 3.);
          double sf = std::max(1. / 3., alpha);
          lambda *= sf;
          ni = 2;
          currentChi = tempChi;
        } else {
          lambda *= ni;
          ni *= 2;
          T = backup;
        }
        qmax++;
      } while (rho < 0 && qmax < 10);
      if (qmax == 10 || rho == 0) return;
      if ((iniChi - currentChi) * 1e3 < iniChi) nBad++;
      else nBad = 0;
      if (nBad >= 3) return;
    }
  }
};

}  // namespace oracle_track

using namespace oracle_track;

extern "C" {

int oracle_frame_prepare(const orbpl_camera* cam, const orbpl_keypoint* kps, int n,
                         const float* depth, orbpl_keypoint* kps_un, float* depth_out,
                         float* uright, int32_t* grid_cell, float* bounds) {
  Grid g;
  grid_constants(*cam, g);
  if (bounds) { bounds[0] = g.minX; bounds[1] = g.maxX; bounds[2] = g.minY; bounds[3] = g.maxY; }
  for (int i = 0; i < n; i++) {
    kps_un[i] = kps[i];
    if (cam->k1 != 0.0f) undistort_point(*cam, kps[i].x, kps[i].y, &kps_un[i].x, &kps_un[i].y);
  }
  for (int i = 0; i < n; i++) {
    depth_out[i] = -1;
    uright[i] = -1;
    if (depth) {
      const int v = (int)kps[i].y, u = (int)kps[i].x;
      const float d = depth[(size_t)v * cam->width + u];
      if (d > 0) {
        depth_out[i] = d;
        uright[i] = kps_un[i].x - cam->bf / d;
      }
    }
    int px, py;
    grid_cell[i] = pos_in_grid(g, kps_un[i].x, kps_un[i].y, &px, &py) ? px + ORBPL_GRID_COLS * py : -1;
  }
  return 0;
}

static int desc_dist(const uint8_t* a, const uint8_t* b) {
  int d = 0;
  for (int i = 0; i < 32; i++) d += __builtin_popcount((unsigned)(a[i] ^ b[i]));
  return d;
}

int oracle_search_by_projection_last(const orbpl_camera* cam, const float* scale_factors,
                                     int nlevels, const orbpl_match_current* cur,
                                     const orbpl_match_last* last, float th, int mono,
                                     int check_ori, int32_t* match, int* nmatches_out) {
  const int HISTO_LENGTH = 30, TH_HIGH = 100;
  Grid g;
  grid_constants(*cam, g);
  for (int i = 0; i < cur->n; i++) {
    int px, py;
    if (pos_in_grid(g, cur->kps_un[i].x, cur->kps_un[i].y, &px, &py)) g.cells[px][py].push_back(i);
  }
  std::vector<int> rotHist[HISTO_LENGTH];
  const float factor = HISTO_LENGTH / 360.0f;
  const float* Tc = cur->Tcw;
  const float* Tl = last->Tcw;
  // twc = -Rcw' * tcw ; tlc = Rlw * twc + tlw   (P6)
  float twc[3];
  for (int r = 0; r < 3; r++) {
    double s = (double)Tc[0 * 4 + r] * Tc[3];
    s += (double)Tc[1 * 4 + r] * Tc[7];
    s += (double)Tc[2 * 4 + r] * Tc[11];
    twc[r] = (float)(s * -1.0);
  }
  float tlc[3];
  gemm33(Tl, twc, tlc);
  const float fx = cam->fx, fy = cam->fy, cx = cam->cx, cy = cam->cy;
  const float mbf = cam->bf, mb = cam->bf / cam->fx;
  const bool bForward = tlc[2] > mb && !mono;
  const bool bBackward = -tlc[2] > mb && !mono;
  std::vector<int> mp(cur->n, -1);    // CurrentFrame.mvpMapPoints (last index)
  int nmatches = 0;
  for (int i = 0; i < last->n; i++) {
    if (!last->has_mp[i] || last->outlier[i]) continue;
    float x3Dc[3];
    gemm33(Tc, &last->mp_xyz[3 * i], x3Dc);
    const float xc = x3Dc[0], yc = x3Dc[1];
    const float invzc = (float)(1.0 / x3Dc[2]);
    if (invzc < 0) continue;
    float u = fx * xc * invzc + cx;
    float v = fy * yc * invzc + cy;
    if (u < g.minX || u > g.maxX) continue;
    if (v < g.minY || v > g.maxY) continue;
    int nLastOctave = last->kps_un[i].octave;
    float radius = th * scale_factors[nLastOctave];
    int minLevel, maxLevel;
    if (bForward) { minLevel = nLastOctave; maxLevel = -1; }
    else if (bBackward) { minLevel = 0; maxLevel = nLastOctave; }
    else { minLevel = nLastOctave - 1; maxLevel = nLastOctave + 1; }
    // Frame::GetFeaturesInArea (Frame.cc:432-485)
    std::vector<int> vIdx;
    const float r = radius;
    const int nMinCellX = std::max(0, (int)std::floor((u - g.minX - r) * g.invW));
    const int nMaxCellX = std::min((int)ORBPL_GRID_COLS - 1, (int)std::ceil((u - g.minX + r) * g.invW));
    const int nMinCellY = std::max(0, (int)std::floor((v - g.minY - r) * g.invH));
    const int nMaxCellY = std::min((int)ORBPL_GRID_ROWS - 1, (int)std::ceil((v - g.minY + r) * g.invH));
    if (!(nMinCellX >= ORBPL_GRID_COLS || nMaxCellX < 0 || nMinCellY >= ORBPL_GRID_ROWS || nMaxCellY < 0)) {
      const bool bCheckLevels = (minLevel > 0) || (maxLevel >= 0);
      for (int ix = nMinCellX; ix <= nMaxCellX; ix++)
        for (int iy = nMinCellY; iy <= nMaxCellY; iy++)
          for (int j : g.cells[ix][iy]) {
            const orbpl_keypoint& k = cur->kps_un[j];
            if (bCheckLevels) {
              if (k.octave < minLevel) continue;
              if (maxLevel >= 0 && k.octave > maxLevel) continue;
            }
            const float distx = k.x - u, disty = k.y - v;
            if (std::fabs(distx) < r && std::fabs(disty) < r) vIdx.push_back(j);
          }
    }
    if (vIdx.empty()) continue;
    const uint8_t* dMP = &last->mp_desc[32 * i];
    int bestDist = 256, bestIdx2 = -1;
    for (int i2 : vIdx) {
      if (mp[i2] >= 0 && last->mp_nobs[mp[i2]] > 0) continue;
      if (cur->uright[i2] > 0) {
        const float ur = u - mbf * invzc;
        const float er = std::fabs(ur - cur->uright[i2]);
        if (er > radius) continue;
      }
      const int dist = desc_dist(dMP, &cur->desc[32 * i2]);
      if (dist < bestDist) { bestDist = dist; bestIdx2 = i2; }
    }
    if (bestDist <= TH_HIGH) {
      mp[bestIdx2] = i;
      nmatches++;
      if (check_ori) {
        float rot = last->kps_un[i].angle - cur->kps_un[bestIdx2].angle;
        if (rot < 0.0) rot += 360.0f;
        int bin = (int)std::round(rot * factor);
        if (bin == HISTO_LENGTH) bin = 0;
        rotHist[bin].push_back(bestIdx2);
      }
    }
  }
  if (check_ori) {
    int ind1 = -1, ind2 = -1, ind3 = -1;
    int max1 = 0, max2 = 0, max3 = 0;
    for (int i = 0; i < HISTO_LENGTH; i++) {
      const int s = (int)rotHist[i].size();
      if (s > max1) { max3 = max2; max2 = max1; max1 = s; ind3 = ind2; ind2 = ind1; ind1 = i; }
      else if (s > max2) { max3 = max2; max2 = s; ind3 = ind2; ind2 = i; }
      else if (s > max3) { max3 = s; ind3 = i; }
    }
    if (max2 < 0.1f * (float)max1) { ind2 = -1; ind3 = -1; }
    else if (max3 < 0.1f * (float)max1) { ind3 = -1; }
    for (int i = 0; i < HISTO_LENGTH; i++) {
      if (i != ind1 && i != ind2 && i != ind3)
        for (int k : rotHist[i]) { mp[k] = -1; nmatches--; }
    }
  }
  for (int i = 0; i < cur->n; i++) match[i] = mp[i];
  *nmatches_out = nmatches;
  return 0;
}

int oracle_pose_optimization_ex(const orbpl_camera* cam, const orbpl_pose_problem* P, int flags,
                                float* Tcw, uint8_t* outlier, uint8_t* line_outlier,
                                int* n_inliers) {
  Cam c{cam->fx, cam->fy, cam->cx, cam->cy, cam->bf,
        (flags & ORBPL_POSE_FIXED_LINE_JAC) ? 1 : 0};
  const float deltaMono = std::sqrt(5.991), deltaStereo = std::sqrt(7.815);
  std::vector<Edge> E;
  int nInitial = 0, nLineInitial = 0;
  for (int i = 0; i < P->n; i++) {
    if (!P->has_mp[i]) continue;
    Edge e{};
    e.idx = i;
    e.kind = P->uright[i] < 0 ? 0 : 1;
    e.dim = e.kind == 0 ? 2 : 3;
    nInitial++;
    outlier[i] = 0;
    e.obs[0] = P->kps_un[i].x;
    e.obs[1] = P->kps_un[i].y;
    e.obs[2] = P->uright[i];
    e.info = P->inv_sigma2[P->kps_un[i].octave];
    e.delta = e.kind == 0 ? (double)deltaMono : (double)deltaStereo;
    e.dsqr_f = (double)(float)(e.delta * e.delta);
    e.robust = true;
    for (int k = 0; k < 3; k++) e.X[k] = P->mp_xyz[3 * i + k];
    E.push_back(e);
  }
  const size_t nPointEdges = E.size();
  for (int i = 0; i < P->nl; i++) {
    if (!P->has_ml[i]) continue;
    nLineInitial++;
    if (i < P->n) outlier[i] = 0;  // reference writes mvbOutlier here (Optimizer.cc:2308)
    Edge e{};
    e.idx = i;
    e.kind = 2;
    e.dim = 2;
    for (int k = 0; k < 4; k++) e.obs[k] = P->kl_obs[4 * i + k];
    e.info = P->inv_sigma2[P->kl_octave[i]];
    e.delta = (double)deltaStereo;
    e.dsqr_f = (double)(float)(e.delta * e.delta);
    e.robust = true;
    double sp[3], ep[3];
    for (int k = 0; k < 3; k++) { sp[k] = P->ml_xyz[6 * i + k]; ep[k] = P->ml_xyz[6 * i + 3 + k]; }
    e.nw[0] = sp[1] * ep[2] - sp[2] * ep[1];
    e.nw[1] = sp[2] * ep[0] - sp[0] * ep[2];
    e.nw[2] = sp[0] * ep[1] - sp[1] * ep[0];
    for (int k = 0; k < 3; k++) e.vw[k] = ep[k] - sp[k];
    E.push_back(e);
  }
  if (nInitial < 3 && nLineInitial < 3) { *n_inliers = 0; return 0; }
  const float chi2Mono = 5.991f, chi2Stereo = 7.815f, chi2Line = 7.815f;
  LM lm(E, c);
  int nBad = 0;
  for (int it = 0; it < 4; it++) {
    lm.T = se3_from_T(Tcw);
    lm.optimize(10);
    nBad = 0;
    for (size_t k = 0; k < E.size(); k++) {
      Edge& e = E[k];
      bool was_out = k < nPointEdges ? outlier[e.idx] != 0 : line_outlier[e.idx] != 0;
      if (was_out) edge_error(e, c, lm.T, e.err);
      const float chi2 = (float)edge_chi2(e);
      const float th = e.kind == 0 ? chi2Mono : e.kind == 1 ? chi2Stereo : 2 * chi2Line;
      const bool bad = chi2 > th;
      if (k < nPointEdges) {
        outlier[e.idx] = bad;
        if (bad) nBad++;
      } else {
        line_outlier[e.idx] = bad;
      }
      e.level = bad ? 1 : 0;
      if (it == 2) e.robust = false;
    }
    if (E.size() < 10) break;
  }
  se3_to_T(lm.T, Tcw);
  *n_inliers = nInitial - nBad;
  return 0;
}

int oracle_pose_optimization(const orbpl_camera* cam, const orbpl_pose_problem* P, float* Tcw,
                             uint8_t* outlier, uint8_t* line_outlier, int* n_inliers) {
  return oracle_pose_optimization_ex(cam, P, 0, Tcw, outlier, line_outlier, n_inliers);
}

}  // extern "C"

// ---------------------------------------------------------------------------
// One RGB-D tracking step per stream on the CPU: the same sequence the
// product's orbpl_tracker_step runs (Tracking::TrackWithMotionModel,
// Tracking.cc:1212-1330, with every frame acting as the next keyframe).
// ---------------------------------------------------------------------------
namespace oracle_track {

static void gemm44f(const float* A, const float* B, float* Cm) {
  for (int r = 0; r < 4; r++)
    for (int c = 0; c < 4; c++) {
      double s = (double)A[r * 4] * B[c];
      s += (double)A[r * 4 + 1] * B[4 + c];
      s += (double)A[r * 4 + 2] * B[8 + c];
      s += (double)A[r * 4 + 3] * B[12 + c];
      Cm[r * 4 + c] = (float)s;
    }
}
static void neg_Rt_t(const float* T, float* o) {
  for (int r = 0; r < 3; r++) {
    double s = (double)T[0 * 4 + r] * T[3];
    s += (double)T[1 * 4 + r] * T[7];
    s += (double)T[2 * 4 + r] * T[11];
    o[r] = (float)(s * -1.0);
  }
}
static void pose_inv(const float* T, float* Ti) {
  float ow[3];
  neg_Rt_t(T, ow);
  for (int r = 0; r < 3; r++) {
    for (int c = 0; c < 3; c++) Ti[r * 4 + c] = T[c * 4 + r];
    Ti[r * 4 + 3] = ow[r];
  }
  Ti[12] = 0; Ti[13] = 0; Ti[14] = 0; Ti[15] = 1;
}

struct VOStream {
  bool has_last = false, has_velocity = false;
  float Tcw[16], Tlast[16], Tlast2[16];
  std::vector<orbpl_keypoint> kps_un;
  std::vector<uint8_t> desc, has_mp, outlier;
  std::vector<float> xyz;
  std::vector<int32_t> nobs;
};

struct VO {
  orbpl_orb_params orb;
  orbpl_camera cam;
  std::vector<VOStream> st;
  std::vector<float> scale, inv_sigma2;
};

}  // namespace oracle_track

extern "C" {

void oracle_undistort_point(const orbpl_camera* c, float px, float py, float* ox, float* oy) {
  undistort_point(*c, px, py, ox, oy);
}

void oracle_image_bounds(const orbpl_camera* c, float* b4) { image_bounds(*c, b4); }

void* oracle_vo_create(const orbpl_orb_params* orb, const orbpl_camera* cam, int n_streams) {
  VO* v = new VO();
  v->orb = *orb;
  v->cam = *cam;
  v->st.resize(n_streams);
  for (auto& s : v->st)
    for (int k = 0; k < 16; k++) s.Tcw[k] = (k % 5 == 0) ? 1.f : 0.f;
  v->scale.resize(orb->nlevels);
  std::vector<float> isc(orb->nlevels);
  oracle_orb_level_sizes(orb, cam->width, cam->height, nullptr, nullptr, nullptr, v->scale.data(),
                         isc.data());
  v->inv_sigma2.resize(orb->nlevels);
  for (int l = 0; l < orb->nlevels; l++) v->inv_sigma2[l] = 1.0f / (v->scale[l] * v->scale[l]);
  return v;
}

void oracle_vo_destroy(void* h) { delete static_cast<VO*>(h); }

int oracle_vo_reset(void* h, const float* Tcw0) {
  VO* v = static_cast<VO*>(h);
  for (size_t s = 0; s < v->st.size(); s++) {
    VOStream z{};
    for (int k = 0; k < 16; k++) z.Tcw[k] = Tcw0 ? Tcw0[s * 16 + k] : ((k % 5 == 0) ? 1.f : 0.f);
    v->st[s] = z;
  }
  return 0;
}

// out5: nkeypoints, nmatches, ninliers, nmatches_map, ok ; Tcw_out: 16 floats
int oracle_vo_step(void* h, int stream, const uint8_t* gray, const float* depth, float* Tcw_out,
                   int* out5) {
  VO* v = static_cast<VO*>(h);
  VOStream& S = v->st[stream];
  const orbpl_camera& cam = v->cam;
  const int cap = v->orb.nfeatures * 2 + 64;
  std::vector<orbpl_keypoint> kps(cap);
  std::vector<uint8_t> desc((size_t)cap * 32);
  int n = 0;
  int rc = oracle_orb_extract(&v->orb, gray, cam.width, cam.height, cam.width, kps.data(),
                              desc.data(), cap, &n, nullptr);
  if (rc) return rc;
  kps.resize(n);
  desc.resize((size_t)n * 32);
  std::vector<orbpl_keypoint> ku(n);
  std::vector<float> dep(n), ur(n);
  std::vector<int32_t> gc(n);
  oracle_frame_prepare(&cam, kps.data(), n, depth, ku.data(), dep.data(), ur.data(), gc.data(), nullptr);
  std::vector<int32_t> match(n, -1);
  std::vector<uint8_t> outl(n, 0);
  int nmatches = 0, ninl = 0, nmap = 0;
  if (S.has_last) {
    if (S.has_velocity) {
      float Twl[16], V[16];
      pose_inv(S.Tlast2, Twl);
      gemm44f(S.Tlast, Twl, V);
      gemm44f(V, S.Tlast, S.Tcw);
    } else {
      memcpy(S.Tcw, S.Tlast, 64);
    }
    orbpl_match_current cur{n, S.Tcw, ku.data(), desc.data(), ur.data()};
    orbpl_match_last last{(int)S.kps_un.size(), S.Tlast, S.kps_un.data(), S.has_mp.data(),
                          S.outlier.data(), S.xyz.data(), S.desc.data(), S.nobs.data()};
    oracle_search_by_projection_last(&cam, v->scale.data(), (int)v->scale.size(), &cur, &last, 15.0f,
                                     0, 1, match.data(), &nmatches);
    if (nmatches < 20) {
      std::fill(match.begin(), match.end(), -1);
      oracle_search_by_projection_last(&cam, v->scale.data(), (int)v->scale.size(), &cur, &last,
                                       30.0f, 0, 1, match.data(), &nmatches);
    }
    if (nmatches >= 20) {
      std::vector<uint8_t> has(n, 0);
      std::vector<float> xyz((size_t)n * 3, 0.f);
      for (int i = 0; i < n; i++)
        if (match[i] >= 0) {
          has[i] = 1;
          for (int k = 0; k < 3; k++) xyz[3 * i + k] = S.xyz[3 * match[i] + k];
        }
      orbpl_pose_problem P{};
      P.n = n;
      P.kps_un = ku.data();
      P.uright = ur.data();
      P.has_mp = has.data();
      P.mp_xyz = xyz.data();
      P.nl = 0;
      P.inv_sigma2 = v->inv_sigma2.data();
      P.nlevels = (int)v->inv_sigma2.size();
      oracle_pose_optimization(&cam, &P, S.Tcw, outl.data(), nullptr, &ninl);
    }
    for (int i = 0; i < n; i++)
      if (match[i] >= 0) {
        if (outl[i]) match[i] = -1;
        else nmap++;
      }
  }
  // this frame becomes the keyframe of the next one
  float Ow[3];
  neg_Rt_t(S.Tcw, Ow);
  const float invfx = 1.0f / cam.fx, invfy = 1.0f / cam.fy;
  S.kps_un = ku;
  S.desc = desc;
  S.has_mp.assign(n, 0);
  S.outlier.assign(n, 0);
  S.xyz.assign((size_t)n * 3, 0.f);
  S.nobs.assign(n, 0);
  for (int i = 0; i < n; i++) {
    const float z = dep[i];
    if (z > 0) {
      const float x3[3] = {(ku[i].x - cam.cx) * z * invfx, (ku[i].y - cam.cy) * z * invfy, z};
      for (int r = 0; r < 3; r++) {
        double s = (double)S.Tcw[0 * 4 + r] * x3[0];
        s += (double)S.Tcw[1 * 4 + r] * x3[1];
        s += (double)S.Tcw[2 * 4 + r] * x3[2];
        S.xyz[3 * i + r] = (float)(s + (double)Ow[r]);
      }
      S.has_mp[i] = 1;
      S.nobs[i] = 1;
    }
  }
  const bool ok = S.has_last ? (nmatches >= 20 && nmap >= 10) : true;
  memcpy(S.Tlast2, S.Tlast, 64);
  memcpy(S.Tlast, S.Tcw, 64);
  S.has_velocity = S.has_last;
  S.has_last = true;
  if (Tcw_out) memcpy(Tcw_out, S.Tcw, 64);
  if (out5) {
    out5[0] = n; out5[1] = nmatches; out5[2] = ninl; out5[3] = nmap; out5[4] = ok;
  }
  return 0;
}

// ---------------------------------------------------------------------------
// Tracking::SearchLocalPoints pieces: Frame::IsInFrustum(MapPoint*, 0.5)
// (Frame.cc:345-401) with MapPoint::PredictScale (MapPoint.cc:416-431), and
// ORBmatcher::SearchByProjection(Frame&, const vector<MapPoint*>&, th)
// (ORBmatcher.cc:72-183) with RadiusByViewingCos (:186-193).
// Pinned: P15 logf = (float)log((double)x) (fdlibm, P10);
// P16 cv::norm of a float 3-vector = sqrt of double squares, one rounding;
// Mat::dot of float 3-vectors = float products summed in double (OpenCV's
// scalar tail for len < 4).
// ---------------------------------------------------------------------------
int oracle_frame_is_in_frustum(const orbpl_camera* cam, float log_scale_factor, int nlevels,
                               const float* Tcw, int n, const float* xyz, const float* normal,
                               const float* min_dist, const float* max_dist, float view_cos_limit,
                               uint8_t* in_view, float* proj_x, float* proj_y, float* proj_xr,
                               int32_t* level, float* view_cos) {
  float b[4];
  image_bounds(*cam, b);
  float Ow[3];
  for (int r = 0; r < 3; r++) {
    double s = (double)Tcw[0 * 4 + r] * Tcw[3];
    s += (double)Tcw[1 * 4 + r] * Tcw[7];
    s += (double)Tcw[2 * 4 + r] * Tcw[11];
    Ow[r] = (float)(s * -1.0);
  }
  for (int i = 0; i < n; i++) {
    in_view[i] = 0;
    proj_x[i] = proj_y[i] = proj_xr[i] = view_cos[i] = 0.f;
    level[i] = -1;
    float Pc[3];
    gemm33(Tcw, xyz + 3 * i, Pc);
    if (Pc[2] < 0.0f) continue;
    const float invz = 1.0f / Pc[2];
    const float u = cam->fx * Pc[0] * invz + cam->cx;
    const float v = cam->fy * Pc[1] * invz + cam->cy;
    if (u < b[0] || u > b[1]) continue;
    if (v < b[2] || v > b[3]) continue;
    const float PO[3] = {xyz[3 * i] - Ow[0], xyz[3 * i + 1] - Ow[1], xyz[3 * i + 2] - Ow[2]};
    const float dist = (float)std::sqrt((double)PO[0] * PO[0] + (double)PO[1] * PO[1] +
                                        (double)PO[2] * PO[2]);
    // GetMin/MaxDistanceInvariance (MapPoint.cc:387-397) of the raw
    // mfMinDistance / mfMaxDistance the arrays hold
    if (dist < 0.8f * min_dist[i] || dist > 1.2f * max_dist[i]) continue;
    const float* Pn = normal + 3 * i;
    double dot = 0;
    for (int k = 0; k < 3; k++) dot += (double)(float)(PO[k] * Pn[k]);
    const float vc = (float)(dot / (double)dist);
    if (vc < view_cos_limit) continue;
    const float ratio = max_dist[i] / dist;   // MapPoint::PredictScale: mfMaxDistance / dist (MapPoint.cc:421)
    int ns = (int)std::ceil((float)pmath::log_((double)ratio) / log_scale_factor);
    if (ns < 0) ns = 0;
    else if (ns >= nlevels) ns = nlevels - 1;
    in_view[i] = 1;
    proj_x[i] = u;
    proj_xr[i] = u - cam->bf * invz;
    proj_y[i] = v;
    level[i] = ns;
    view_cos[i] = vc;
  }
  return 0;
}

int oracle_search_by_projection_local(const orbpl_camera* cam, const float* scale_factors,
                                      int nlevels, const orbpl_match_current* cur, int nmp,
                                      const uint8_t* in_view, const float* proj_x,
                                      const float* proj_y, const float* proj_xr,
                                      const int32_t* level, const float* view_cos,
                                      const uint8_t* mp_desc, const int32_t* mp_nobs,
                                      const int32_t* cur_nobs, float th, float nnratio,
                                      int32_t* match, int* nmatches_out) {
  (void)nlevels;
  const int TH_HIGH = 100;
  Grid g;
  grid_constants(*cam, g);
  for (int i = 0; i < cur->n; i++) {
    int px, py;
    if (pos_in_grid(g, cur->kps_un[i].x, cur->kps_un[i].y, &px, &py)) g.cells[px][py].push_back(i);
  }
  // Observations() of the map point currently in F.mvpMapPoints[idx]
  std::vector<int> obs(cur->n);
  for (int i = 0; i < cur->n; i++) {
    obs[i] = cur_nobs ? cur_nobs[i] : 0;
    match[i] = -1;
  }
  const bool bFactor = th != 1.0;
  int nmatches = 0;
  for (int i = 0; i < nmp; i++) {
    if (!in_view[i]) continue;
    const int nPredictedLevel = level[i];
    float r = (view_cos[i] > 0.998) ? 2.5f : 4.0f;
    if (bFactor) r *= th;
    const float rad = r * scale_factors[nPredictedLevel];
    const float x = proj_x[i], y = proj_y[i];
    const int minLevel = nPredictedLevel - 1, maxLevel = nPredictedLevel;
    std::vector<int> vIdx;
    const int nMinCellX = std::max(0, (int)std::floor((x - g.minX - rad) * g.invW));
    const int nMaxCellX = std::min((int)ORBPL_GRID_COLS - 1, (int)std::ceil((x - g.minX + rad) * g.invW));
    const int nMinCellY = std::max(0, (int)std::floor((y - g.minY - rad) * g.invH));
    const int nMaxCellY = std::min((int)ORBPL_GRID_ROWS - 1, (int)std::ceil((y - g.minY + rad) * g.invH));
    if (!(nMinCellX >= ORBPL_GRID_COLS || nMaxCellX < 0 || nMinCellY >= ORBPL_GRID_ROWS || nMaxCellY < 0)) {
      const bool bCheckLevels = (minLevel > 0) || (maxLevel >= 0);
      for (int ix = nMinCellX; ix <= nMaxCellX; ix++)
        for (int iy = nMinCellY; iy <= nMaxCellY; iy++)
          for (int j : g.cells[ix][iy]) {
            const orbpl_keypoint& k = cur->kps_un[j];
            if (bCheckLevels) {
              if (k.octave < minLevel) continue;
              if (maxLevel >= 0 && k.octave > maxLevel) continue;
            }
            const float distx = k.x - x, disty = k.y - y;
            if (std::fabs(distx) < rad && std::fabs(disty) < rad) vIdx.push_back(j);
          }
    }
    if (vIdx.empty()) continue;
    const uint8_t* dMP = mp_desc + 32 * i;
    int bestDist = 256, bestLevel = -1, bestDist2 = 256, bestLevel2 = -1, bestIdx = -1;
    for (int idx : vIdx) {
      if (obs[idx] > 0) continue;
      if (cur->uright[idx] > 0) {
        const float er = std::fabs(proj_xr[i] - cur->uright[idx]);
        if (er > r * scale_factors[nPredictedLevel]) continue;
      }
      const int dist = desc_dist(dMP, cur->desc + 32 * idx);
      if (dist < bestDist) {
        bestDist2 = bestDist;
        bestDist = dist;
        bestLevel2 = bestLevel;
        bestLevel = cur->kps_un[idx].octave;
        bestIdx = idx;
      } else if (dist < bestDist2) {
        bestLevel2 = cur->kps_un[idx].octave;
        bestDist2 = dist;
      }
    }
    if (bestDist <= TH_HIGH) {
      if (bestLevel == bestLevel2 && bestDist > nnratio * bestDist2) continue;
      match[bestIdx] = i;
      obs[bestIdx] = mp_nobs[i];
      nmatches++;
    }
  }
  *nmatches_out = nmatches;
  return 0;
}

// ORBmatcher::SearchByBoW(KeyFrame*, Frame&, vector<MapPoint*>&)
// (ORBmatcher.cc:247-410). The DBoW2 FeatureVectors are given as one node id
// per feature (-1: no node); DBoW2 adds features to a node in index order,
// so a node's list is its features in increasing index. kf_valid[i] = the
// keyframe's map point i exists and is not bad. match[j] = keyframe feature
// index whose map point is assigned to frame feature j, or -1.
int oracle_search_by_bow(int nkf, const int32_t* kf_node, const uint8_t* kf_valid,
                         const uint8_t* kf_desc, const float* kf_angle, int nf,
                         const int32_t* f_node, const uint8_t* f_desc, const float* f_angle,
                         float nnratio, int check_ori, int32_t* match, int* nmatches_out) {
  const int HISTO_LENGTH = 30, TH_LOW = 50;
  std::map<int, std::vector<int>> fvKF, fvF;
  for (int i = 0; i < nkf; i++)
    if (kf_node[i] >= 0) fvKF[kf_node[i]].push_back(i);
  for (int j = 0; j < nf; j++)
    if (f_node[j] >= 0) fvF[f_node[j]].push_back(j);
  for (int j = 0; j < nf; j++) match[j] = -1;
  std::vector<int> rotHist[HISTO_LENGTH];
  const float factor = HISTO_LENGTH / 360.0f;
  int nmatches = 0;
  auto KFit = fvKF.begin(), Fit = fvF.begin();
  while (KFit != fvKF.end() && Fit != fvF.end()) {
    if (KFit->first == Fit->first) {
      for (int iKF : KFit->second) {
        if (!kf_valid[iKF]) continue;
        int bestDist1 = 256, bestIdxF = -1, bestDist2 = 256;
        for (int iF : Fit->second) {
          if (match[iF] >= 0) continue;
          const int dist = desc_dist(kf_desc + 32 * iKF, f_desc + 32 * iF);
          if (dist < bestDist1) {
            bestDist2 = bestDist1;
            bestDist1 = dist;
            bestIdxF = iF;
          } else if (dist < bestDist2) {
            bestDist2 = dist;
          }
        }
        if (bestDist1 <= TH_LOW) {
          if (static_cast<float>(bestDist1) < nnratio * static_cast<float>(bestDist2)) {
            match[bestIdxF] = iKF;
            if (check_ori) {
              float rot = kf_angle[iKF] - f_angle[bestIdxF];
              if (rot < 0.0) rot += 360.0f;
              int bin = (int)std::round(rot * factor);
              if (bin == HISTO_LENGTH) bin = 0;
              rotHist[bin].push_back(bestIdxF);
            }
            nmatches++;
          }
        }
      }
      ++KFit;
      ++Fit;
    } else if (KFit->first < Fit->first) {
      KFit = fvKF.lower_bound(Fit->first);
    } else {
      Fit = fvF.lower_bound(KFit->first);
    }
  }
  if (check_ori) {
    int max1 = 0, max2 = 0, max3 = 0, ind1 = -1, ind2 = -1, ind3 = -1;
    for (int i = 0; i < HISTO_LENGTH; i++) {
      const int sz = (int)rotHist[i].size();
      if (sz > max1) {
        max3 = max2; max2 = max1; max1 = sz; ind3 = ind2; ind2 = ind1; ind1 = i;
      } else if (sz > max2) {
        max3 = max2; max2 = sz; ind3 = ind2; ind2 = i;
      } else if (sz > max3) {
        max3 = sz; ind3 = i;
      }
    }
    if (max2 < 0.1f * (float)max1) {
      ind2 = -1; ind3 = -1;
    } else if (max3 < 0.1f * (float)max1) {
      ind3 = -1;
    }
    for (int i = 0; i < HISTO_LENGTH; i++) {
      if (i == ind1 || i == ind2 || i == ind3) continue;
      for (int j : rotHist[i]) {
        match[j] = -1;
        nmatches--;
      }
    }
  }
  *nmatches_out = nmatches;
  return 0;
}

// Frame::ComputeStereoMatches (Frame.cc:886-1063): ORB descriptor search
// along the right image's row bands, SAD refinement on the pyramid level
// (11x11 window, +-5 columns), parabolic sub-pixel fit, median-based
// outlier rejection. Pyramids are the padded levels of oracle_orb_pyramid
// ((w+38)x(h+38), content at (19, 19)). The SAD of integer-valued float
// windows is exact in any summation order, so it is computed in integers.
int oracle_stereo_matches(const orbpl_camera* cam, const float* scale, const float* inv_scale,
                          int nlevels, const int32_t* lw, const int32_t* lh, const uint8_t* pyrL,
                          const uint8_t* pyrR, const orbpl_keypoint* kl, const uint8_t* dl, int n,
                          const orbpl_keypoint* kr, const uint8_t* dr, int nr, float* uright,
                          float* depth) {
  const int TH_HIGH = 100, TH_LOW = 50;
  std::vector<size_t> loff(nlevels);
  size_t off = 0;
  for (int l = 0; l < nlevels; l++) {
    loff[l] = off;
    off += (size_t)(lw[l] + 38) * (lh[l] + 38);
  }
  auto pix = [&](const uint8_t* pyr, int l, int x, int y) -> int {
    return pyr[loff[l] + (size_t)(y + 19) * (lw[l] + 38) + x + 19];
  };
  for (int i = 0; i < n; i++) uright[i] = depth[i] = -1.0f;
  const int thOrbDist = (TH_HIGH + TH_LOW) / 2;
  const int nRows = lh[0];
  std::vector<std::vector<int>> rows(nRows);
  for (int iR = 0; iR < nr; iR++) {
    const float kpY = kr[iR].y;
    const float r = 2.0f * scale[kr[iR].octave];
    const int maxr = (int)std::ceil(kpY + r);
    const int minr = (int)std::floor(kpY - r);
    for (int yi = minr; yi <= maxr; yi++)
      if (yi >= 0 && yi < nRows) rows[yi].push_back(iR);
  }
  const float mb = cam->bf / cam->fx, mbf = cam->bf;
  const float minZ = mb, minD = 0, maxD = mbf / minZ;
  std::vector<std::pair<int, int>> vDistIdx;
  for (int iL = 0; iL < n; iL++) {
    const orbpl_keypoint& kpL = kl[iL];
    const int levelL = kpL.octave;
    const float vL = kpL.y, uL = kpL.x;
    const int row = (int)vL;
    if (row < 0 || row >= nRows || rows[row].empty()) continue;
    const float minU = uL - maxD, maxU = uL - minD;
    if (maxU < 0) continue;
    int bestDist = TH_HIGH;
    int bestIdxR = 0;
    for (int iR : rows[row]) {
      const orbpl_keypoint& kpR = kr[iR];
      if (kpR.octave < levelL - 1 || kpR.octave > levelL + 1) continue;
      const float uR = kpR.x;
      if (uR >= minU && uR <= maxU) {
        const int dist = desc_dist(dl + 32 * iL, dr + 32 * iR);
        if (dist < bestDist) {
          bestDist = dist;
          bestIdxR = iR;
        }
      }
    }
    if (bestDist >= thOrbDist) continue;
    const float uR0 = kr[bestIdxR].x;
    const float scaleFactor = inv_scale[kpL.octave];
    const float scaleduL = std::round(kpL.x * scaleFactor);
    const float scaledvL = std::round(kpL.y * scaleFactor);
    const float scaleduR0 = std::round(uR0 * scaleFactor);
    const int w = 5, L = 5;
    const int l = kpL.octave;
    const int cuL = (int)scaleduL, cvL = (int)scaledvL, cuR = (int)scaleduR0;
    const float iniu = scaleduR0 + L - w;
    const float endu = scaleduR0 + L + w + 1;
    if (iniu < 0 || endu >= lw[l]) continue;
    // windows outside the level (the reference's ROI would assert) are skipped
    if (cvL - w < 0 || cvL + w >= lh[l] || cuL - w < 0 || cuL + w >= lw[l] || cuR - L - w < 0)
      continue;
    const int cL = pix(pyrL, l, cuL, cvL);
    int bestD = INT_MAX, bestincR = 0;
    float vDists[2 * 5 + 1];
    for (int incR = -L; incR <= L; incR++) {
      const int cR = pix(pyrR, l, cuR + incR, cvL);
      int sad = 0;
      for (int yy = -w; yy <= w; yy++)
        for (int xx = -w; xx <= w; xx++) {
          const int a = pix(pyrL, l, cuL + xx, cvL + yy) - cL;
          const int b = pix(pyrR, l, cuR + incR + xx, cvL + yy) - cR;
          sad += std::abs(a - b);
        }
      const float dist = (float)sad;
      if (dist < bestD) {
        bestD = (int)dist;
        bestincR = incR;
      }
      vDists[L + incR] = dist;
    }
    if (bestincR == -L || bestincR == L) continue;
    const float dist1 = vDists[L + bestincR - 1];
    const float dist2 = vDists[L + bestincR];
    const float dist3 = vDists[L + bestincR + 1];
    const float deltaR = (dist1 - dist3) / (2.0f * (dist1 + dist3 - 2.0f * dist2));
    if (deltaR < -1 || deltaR > 1) continue;
    float bestuR = scale[kpL.octave] * ((float)scaleduR0 + (float)bestincR + deltaR);
    float disparity = (uL - bestuR);
    if (disparity >= minD && disparity < maxD) {
      if (disparity <= 0) {
        disparity = 0.01;
        bestuR = uL - 0.01;
      }
      depth[iL] = mbf / disparity;
      uright[iL] = bestuR;
      vDistIdx.push_back(std::make_pair(bestD, iL));
    }
  }
  if (vDistIdx.empty()) return 0;
  std::sort(vDistIdx.begin(), vDistIdx.end());
  const float median = vDistIdx[vDistIdx.size() / 2].first;
  const float thDist = 1.5f * 1.4f * median;
  for (int i = (int)vDistIdx.size() - 1; i >= 0; i--) {
    if (vDistIdx[i].first < thDist) break;
    uright[vDistIdx[i].second] = -1;
    depth[vDistIdx[i].second] = -1;
  }
  return 0;
}

}  // extern "C"
