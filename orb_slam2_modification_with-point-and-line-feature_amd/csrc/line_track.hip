// Per-frame line tracking on gfx950 (restated in oracle/line_track_oracle.cpp):
//   k_line_prepare : Frame::UndistortKeyLines (Frame.cc:769-845) and the line
//                    part of ComputeStereoFromRGBD (Frame.cc:1090-1116)
//   k_line_match   : LineMatcher::SearchByProjection(Frame&, const Frame&)
//                    (LineMatcher.cpp:72-269): last-frame MapLines projected
//                    and Liang-Barsky clipped in parallel, then every
//                    (projected, current) pair tested by LineMatching in
//                    parallel; the last passing projected line of each
//                    current line wins and every pass counts, as in the
//                    reference's double loop; one relaxed retry
//   line map update: lives in k_finish (track_kernels.hip)
#include <hip/hip_runtime.h>

#include "line_common.h"
#include "lsd_kernels.h"
#include "track_common.h"
#include "track_kernels.h"

namespace orbpl {

__global__ void __launch_bounds__(64) k_line_prepare(TrackConsts c, LineTrackArgs a) {
  trk_priority();
  const int s = blockIdx.x, lane = threadIdx.x;
  const int nl = a.nl[s];
  const long long lb = (long long)s * kLineKeep;
  const int W = c.width, H = c.height;
  const float* depth = a.depth ? a.depth + (long long)s * a.depth_pitch : nullptr;
  for (int j = lane; j < nl; j += 64) {
    const orbpl_keyline k0 = a.kl[lb + j];
    orbpl_keyline k = k0;
    if (c.k1 != 0.0f) {
      float x, y;
      undistort_point_d(c, k0.startPointX, k0.startPointY, &x, &y);
      k.startPointX = x;
      k.startPointY = y;
      undistort_point_d(c, k0.endPointX, k0.endPointY, &x, &y);
      k.endPointX = x;
      k.endPointY = y;
      k.sPointInOctaveX = k.startPointX;
      k.sPointInOctaveY = k.startPointY;
      k.ePointInOctaveX = k.endPointX;
      k.ePointInOctaveY = k.endPointY;
      refresh_keyline(k, W, H);
    }
    a.kl_un[lb + j] = k;
    // imDepth.at<float>(int(v), int(u)) on the distorted end points (P14)
    auto at = [&](float v, float u) -> float {
      const long long idx = (long long)(int)v * W + (int)u;
      return (depth && idx >= 0 && idx < (long long)W * H) ? depth[idx] : 0.f;
    };
    const float ds = at(k0.startPointY, k0.startPointX);
    const float de = at(k0.endPointY, k0.endPointX);
    a.dstart[lb + j] = ds > 0 ? ds : -1.f;
    a.dend[lb + j] = de > 0 ? de : -1.f;
    if (a.ur_start) {
      a.ur_start[lb + j] = ds > 0 ? k.startPointX - c.bf / ds : -1.f;
      a.ur_end[lb + j] = de > 0 ? k.endPointX - c.bf / de : -1.f;
    }
    a.lmatch[lb + j] = -1;
    a.loutlier[lb + j] = 0;
  }
}

namespace {

// std::min / std::max: (b < a) ? b : a and (a < b) ? b : a
template <typename T>
__device__ __forceinline__ T smin(T a, T b) { return (b < a) ? b : a; }
template <typename T>
__device__ __forceinline__ T smax(T a, T b) { return (a < b) ? b : a; }

__device__ bool liang_barsky(const double line[4], double out[4], const float b[4]) {
  const double sx = line[0], sy = line[1], ex = line[2], ey = line[3];
  double p[4], q[4];
  p[0] = sx - ex;
  p[1] = ex - sx;
  p[2] = sy - ey;
  p[3] = ey - sy;
  q[0] = sx - b[0];
  q[1] = b[2] - sx;
  q[2] = sy - b[1];
  q[3] = b[3] - sy;
  if (p[0] == 0) {
    if (q[0] <= 0 || q[2] <= 0) return false;
  }
  if (p[2] == 0) {
    if (q[2] >= 0 || q[3] >= 0) return false;
  }
  double u_min = 0, u_max = 1;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const double u = q[i] / p[i];
    if (p[i] < 0) {
      if (u_min < u) u_min = u;
    } else {
      if (u_max > u) u_max = u;
    }
  }
  if (u_max >= u_min) {
    out[0] = sx + round(u_min * (ex - sx));
    out[1] = sy + round(u_min * (ey - sy));
    out[2] = sx + round(u_max * (ex - sx));
    out[3] = sy + round(u_max * (ey - sy));
    return true;
  }
  return false;
}

__device__ bool line_overlap(const orbpl_keyline& a, const orbpl_keyline& b, double th) {
  const double d1_x = fabsf(a.startPointX - a.endPointX);
  const double d2_x = fabsf(b.startPointX - b.endPointX);
  const double min_x = smin(smin(a.startPointX, a.endPointX), smin(b.startPointX, b.endPointX));
  const double max_x = smax(smax(a.startPointX, a.endPointX), smax(b.startPointX, b.endPointX));
  const double d1_y = fabsf(a.startPointY - a.endPointY);
  const double d2_y = fabsf(b.startPointY - b.endPointY);
  const double min_y = smin(smin(a.startPointY, a.endPointY), smin(b.startPointY, b.endPointY));
  const double max_y = smax(smax(a.startPointY, a.endPointY), smax(b.startPointY, b.endPointY));
  if (d1_x == 0 || d2_x == 0) {
    if ((d1_y + d2_y - max_y + min_y) / smin(d1_y, d2_y) >= th) return true;
  }
  if (d1_y == 0 || d2_y == 0) {
    if ((d1_x + d2_x - max_x + min_x) / smin(d1_x, d2_x) >= th) return true;
  }
  if ((d1_x + d2_x - max_x + min_x) / smin(d1_x, d2_x) >= th) {
    if (d1_y + d2_y + min_y >= max_y) return true;
    if (max_y - min_y - d1_y - d2_y < 0.3 * smin(d1_y, d2_y)) return true;
  } else if ((d1_x + d2_x - max_x + min_x) / smin(d1_x, d2_x) < th &&
             (max_x - min_x - d1_x - d2_x) < 0.3 * smin(d1_x, d2_x)) {
    if ((d1_y + d2_y - max_y + min_y) / smin(d1_y, d2_y) >= th) return true;
  }
  return false;
}

__device__ double reprojection_error(const orbpl_keyline& l1, const orbpl_keyline& l2) {
  const double s0 = l1.startPointX, s1 = l1.startPointY, s2 = 1;
  const double e0 = l1.endPointX, e1 = l1.endPointY, e2 = 1;
  const double c0 = s1 * e2 - s2 * e1, c1 = s2 * e0 - s0 * e2, c2 = s0 * e1 - s1 * e0;
  const double nrm = sqrt(c0 * c0 + c1 * c1);
  const double ds = ((double)l2.startPointX * c0 + (double)l2.startPointY * c1 + 1.0 * c2) / nrm;
  const double de = ((double)l2.endPointX * c0 + (double)l2.endPointY * c1 + 1.0 * c2) / nrm;
  return sqrt(ds * ds + de * de);
}

__device__ bool line_matching(const orbpl_keyline& k1, const orbpl_keyline& k2, const uint4* d1,
                              const uint4* d2, const double off0, const double off1,
                              const double off2, const double off3) {
  const double kPi = 3.14159265358979323846;
  int dist = 0;
#pragma unroll
  for (int q = 0; q < 2; q++) {
    const uint4 a = d1[q], b = d2[q];
    dist += __popc(a.x ^ b.x) + __popc(a.y ^ b.y) + __popc(a.z ^ b.z) + __popc(a.w ^ b.w);
  }
  if (dist > 45 + off3) return false;
  if (fabsf(k1.angle - k2.angle) > 15.0 * kPi / 180.0 + off0 * kPi / 180.0) return false;
  if (smin(k1.lineLength, k2.lineLength) / smax(k1.lineLength, k2.lineLength) < 0.45 + off1)
    return false;
  if (!line_overlap(k1, k2, 0.5 + off2)) return false;
  if (reprojection_error(k1, k2) > 45) return false;
  return true;
}

}  // namespace

// Project map line X (6 floats) with T (row-major 3x4 double copy), clip
// to the image bounds and rebuild the KeyLine (LineMatcher.cpp:118-193,
// UpdateKeyLineData :1601-1624). Returns false when the line is not seen.
__device__ bool project_map_line(const TrackConsts& c, const double T[12], const float* X,
                                 orbpl_keyline& k) {
  double cs[3], ce[3];
#pragma unroll
  for (int r = 0; r < 3; r++) {
    cs[r] = (T[r * 4] * (double)X[0] + T[r * 4 + 1] * (double)X[1] + T[r * 4 + 2] * (double)X[2]) + T[r * 4 + 3];
    ce[r] = (T[r * 4] * (double)X[3] + T[r * 4 + 1] * (double)X[4] + T[r * 4 + 2] * (double)X[5]) + T[r * 4 + 3];
  }
  if (cs[2] < 0 && ce[2] < 0) return false;
  double lp[4];
  bool have = false;
  if (cs[2] < 0.0 || ce[2] < 0.0) {
    const double lambda = -1.0 * cs[2] / (cs[2] - ce[2]);
    const double xc = cs[0] + lambda * (cs[0] - ce[0]);
    const double yc = cs[1] + lambda * (cs[1] - ce[1]);
    if (cs[2] < 0.0) {
      const float u_end = c.fx * ce[0] / ce[2] + c.cx;
      const float v_end = c.fy * ce[1] / ce[2] + c.cy;
      lp[0] = xc; lp[1] = yc; lp[2] = u_end; lp[3] = v_end;
    } else {
      const float u_start = c.fx * cs[0] / cs[2] + c.cx;
      const float v_start = c.fy * cs[1] / cs[2] + c.cy;
      lp[0] = u_start; lp[1] = v_start; lp[2] = xc; lp[3] = yc;
    }
    have = true;
  }
  if (cs[2] > 0.0 && ce[2] > 0.0) {
    const float u_start = c.fx * cs[0] / cs[2] + c.cx;
    const float v_start = c.fy * cs[1] / cs[2] + c.cy;
    const float u_end = c.fx * ce[0] / ce[2] + c.cx;
    const float v_end = c.fy * ce[1] / ce[2] + c.cy;
    lp[0] = u_start; lp[1] = v_start; lp[2] = u_end; lp[3] = v_end;
    have = true;
  }
  if (!have) return false;
  double nl4[4];
  const float bounds[4] = {c.minX, c.minY, c.maxX, c.maxY};
  if (!liang_barsky(lp, nl4, bounds)) return false;
  k.startPointX = (float)nl4[0];
  k.startPointY = (float)nl4[1];
  k.endPointX = (float)nl4[2];
  k.endPointY = (float)nl4[3];
  k.sPointInOctaveX = (float)nl4[0];
  k.sPointInOctaveY = (float)nl4[1];
  k.ePointInOctaveX = (float)nl4[2];
  k.ePointInOctaveY = (float)nl4[3];
  refresh_keyline(k, c.width, c.height);
  return true;
}

// One 256-thread block per stream.
__global__ void __launch_bounds__(256) k_line_match(TrackConsts c, LineTrackArgs a,
                                                     StreamState* st) {
  trk_priority();
  __shared__ orbpl_keyline s_kl[kLineKeep];
  __shared__ int s_src[kLineKeep];
  __shared__ int s_np;
  __shared__ unsigned s_ok[kLineKeep][(kLineKeep + 31) / 32];
  __shared__ int s_cnt;
  const int s = blockIdx.x, t = threadIdx.x;
  const StreamState& S = st[s];
  if (!S.has_last) {
    if (t == 0) st[s].nlmatches = 0;
    return;
  }
  const long long lb = (long long)s * kLineKeep;
  const int ncur = min(a.nl[s], kLineKeep), nlast = min(a.last_nl[s], kLineKeep);
  const int W = c.width, H = c.height;
  // ---- project the last frame's map lines with the predicted pose ----
  bool valid = false;
  orbpl_keyline k{};
  if (t < nlast && t < kLineKeep && a.last_has_ml[lb + t] && !a.last_loutlier[lb + t]) {
    double T[12];
#pragma unroll
    for (int q = 0; q < 12; q++) T[q] = S.Tcw[q];
    const float* X = a.last_ml_xyz + (lb + t) * 6;
    double cs[3], ce[3];
#pragma unroll
    for (int r = 0; r < 3; r++) {
      cs[r] = (T[r * 4] * (double)X[0] + T[r * 4 + 1] * (double)X[1] + T[r * 4 + 2] * (double)X[2]) + T[r * 4 + 3];
      ce[r] = (T[r * 4] * (double)X[3] + T[r * 4 + 1] * (double)X[4] + T[r * 4 + 2] * (double)X[5]) + T[r * 4 + 3];
    }
    double lp[4];
    bool have = false;
    if (!(cs[2] < 0 && ce[2] < 0)) {
      if (cs[2] < 0.0 || ce[2] < 0.0) {
        const double lambda = -1.0 * cs[2] / (cs[2] - ce[2]);
        const double xc = cs[0] + lambda * (cs[0] - ce[0]);
        const double yc = cs[1] + lambda * (cs[1] - ce[1]);
        if (cs[2] < 0.0) {
          const float u_end = c.fx * ce[0] / ce[2] + c.cx;
          const float v_end = c.fy * ce[1] / ce[2] + c.cy;
          lp[0] = xc; lp[1] = yc; lp[2] = u_end; lp[3] = v_end;
        } else {
          const float u_start = c.fx * cs[0] / cs[2] + c.cx;
          const float v_start = c.fy * cs[1] / cs[2] + c.cy;
          lp[0] = u_start; lp[1] = v_start; lp[2] = xc; lp[3] = yc;
        }
        have = true;
      }
      if (cs[2] > 0.0 && ce[2] > 0.0) {
        const float u_start = c.fx * cs[0] / cs[2] + c.cx;
        const float v_start = c.fy * cs[1] / cs[2] + c.cy;
        const float u_end = c.fx * ce[0] / ce[2] + c.cx;
        const float v_end = c.fy * ce[1] / ce[2] + c.cy;
        lp[0] = u_start; lp[1] = v_start; lp[2] = u_end; lp[3] = v_end;
        have = true;
      }
    }
    double nl4[4];
    const float bounds[4] = {c.minX, c.minY, c.maxX, c.maxY};
    if (have && liang_barsky(lp, nl4, bounds)) {
      k = a.last_kl_un[lb + t];
      k.startPointX = (float)nl4[0];
      k.startPointY = (float)nl4[1];
      k.endPointX = (float)nl4[2];
      k.endPointY = (float)nl4[3];
      k.sPointInOctaveX = (float)nl4[0];
      k.sPointInOctaveY = (float)nl4[1];
      k.ePointInOctaveX = (float)nl4[2];
      k.ePointInOctaveY = (float)nl4[3];
      refresh_keyline(k, W, H);
      valid = true;
    }
  }
  // compaction keeps the projected lines in last-frame index order
  __shared__ int s_wc[4];
  const unsigned long long m = __ballot(valid);
  if ((t & 63) == 0) s_wc[t >> 6] = __popcll(m);
  __syncthreads();
  int pos = __popcll(m & ((1ull << (t & 63)) - 1ull));
  for (int w = 0; w < (t >> 6); w++) pos += s_wc[w];
  if (valid) {
    s_kl[pos] = k;
    s_src[pos] = t;
  }
  if (t == 0) s_np = s_wc[0] + s_wc[1] + s_wc[2] + s_wc[3];
  __syncthreads();
  const int np = s_np;
  const uint4* cur_desc = reinterpret_cast<const uint4*>(a.desc + lb * 32);
  const uint4* last_desc = reinterpret_cast<const uint4*>(a.last_desc + lb * 32);
  int total = 0;
  for (int pass = 0; pass < 2; pass++) {
    const double o0 = pass ? 10.0 : 0, o1 = pass ? -0.1 : 0, o2 = pass ? -0.1 : 0, o3 = pass ? 5 : 0;
    for (int w = t; w < kLineKeep * ((kLineKeep + 31) / 32); w += 256) (&s_ok[0][0])[w] = 0;
    if (t == 0) s_cnt = 0;
    __syncthreads();
    for (int pr = t; pr < ncur * np; pr += 256) {
      const int j = pr / np, i = pr - j * np;
      const orbpl_keyline kc = a.kl_un[lb + j];
      if (line_matching(s_kl[i], kc, last_desc + 2 * s_src[i], cur_desc + 2 * j, o0, o1, o2, o3))
        atomicOr(&s_ok[j][i >> 5], 1u << (i & 31));
    }
    __syncthreads();
    int cnt = 0;
    if (t < ncur) {
      int last = -1;
      for (int w = 0; w < (kLineKeep + 31) / 32; w++) {
        const unsigned b = s_ok[t][w];
        cnt += __popc(b);
        if (b) last = w * 32 + 31 - __clz(b);
      }
      a.lmatch[lb + t] = last >= 0 ? s_src[last] : -1;
    }
    atomicAdd(&s_cnt, cnt);
    __syncthreads();
    total = s_cnt;
    // retry with relaxed thresholds (LineMatcher.cpp:235-261); 0/0 is not < 0.2
    if (pass == 0 && !(total * 1.0 / ncur < 0.2)) break;
    __syncthreads();
  }
  if (t == 0) st[s].nlmatches = total;
}

void launch_line_prepare(const TrackConsts& c, const LineTrackArgs& a, int nstreams,
                         hipStream_t s) {
  hipLaunchKernelGGL(k_line_prepare, dim3(nstreams), dim3(64), 0, s, c, a);
}

void launch_line_match(const TrackConsts& c, const LineTrackArgs& a, StreamState* st,
                       int nstreams, hipStream_t s) {
  hipLaunchKernelGGL(k_line_match, dim3(nstreams), dim3(256), 0, s, c, a, st);
}

// Stereo line depths (the defined mode P17, oracle_stereo_line_depths): one
// 128-thread block per stereo pair, the right KeyLines and LBD rows in LDS,
// thread i scans the right lines for left line i in index order with the
// same double / float operation sequence as the oracle.
__global__ void __launch_bounds__(128) k_stereo_lines(TrackConsts c, StereoLineArgs a) {
  trk_priority();
  __shared__ orbpl_keyline s_kr[kLineKeep];
  __shared__ uint4 s_dr[kLineKeep * 2];
  const int s = blockIdx.x, t = threadIdx.x;
  const long long lb = (long long)s * kLineKeep;
  const int nl = a.nl[s], nr = min(a.nr[s], kLineKeep);
  for (int j = t; j < nr; j += 128) s_kr[j] = a.kr[lb + j];
  for (int j = t; j < nr * 2; j += 128)
    s_dr[j] = reinterpret_cast<const uint4*>(a.desc_r + lb * 32)[j];
  __syncthreads();
  if (t >= nl) return;
  const double kPi = 3.14159265358979323846;
  const float maxD = c.bf / c.mb;
  const orbpl_keyline ka = a.kl[lb + t];
  const uint4* da = reinterpret_cast<const uint4*>(a.desc + (lb + t) * 32);
  const uint4 a0 = da[0], a1 = da[1];
  float bs = -1.0f, be = -1.0f;
  const double ady = (double)ka.endPointY - ka.startPointY;
  if (fabs(ady) >= 0.25 * ka.lineLength) {
    const double ay0 = smin(ka.startPointY, ka.endPointY), ay1 = smax(ka.startPointY, ka.endPointY);
    int best = 46;
    for (int j = 0; j < nr; j++) {
      const uint4 b0 = s_dr[2 * j], b1 = s_dr[2 * j + 1];
      const int dist = __popc(a0.x ^ b0.x) + __popc(a0.y ^ b0.y) + __popc(a0.z ^ b0.z) +
                       __popc(a0.w ^ b0.w) + __popc(a1.x ^ b1.x) + __popc(a1.y ^ b1.y) +
                       __popc(a1.z ^ b1.z) + __popc(a1.w ^ b1.w);
      if (dist > 45 || dist >= best) continue;
      const orbpl_keyline& kb = s_kr[j];
      if (fabs((double)ka.angle - (double)kb.angle) > 10.0 * kPi / 180.0) continue;
      if (smin(ka.lineLength, kb.lineLength) / smax(ka.lineLength, kb.lineLength) < 0.45f) continue;
      const double bdy = (double)kb.endPointY - kb.startPointY;
      if (fabs(bdy) < 0.25 * kb.lineLength) continue;
      const double by0 = smin(kb.startPointY, kb.endPointY), by1 = smax(kb.startPointY, kb.endPointY);
      const double ov = smin(ay1, by1) - smax(ay0, by0);
      if (ov < 0.5 * smin(ay1 - ay0, by1 - by0)) continue;
      const double slope = ((double)kb.endPointX - kb.startPointX) / bdy;
      const double xs = kb.startPointX + ((double)ka.startPointY - kb.startPointY) * slope;
      const double xe = kb.startPointX + ((double)ka.endPointY - kb.startPointY) * slope;
      const float ds = (float)((double)ka.startPointX - xs);
      const float de = (float)((double)ka.endPointX - xe);
      if (!(ds > 0.0f && ds < maxD && de > 0.0f && de < maxD)) continue;
      best = dist;
      bs = c.bf / ds;
      be = c.bf / de;
    }
  }
  a.dstart[lb + t] = bs;
  a.dend[lb + t] = be;
}

void launch_stereo_lines(const TrackConsts& c, const StereoLineArgs& a, int nstreams,
                         hipStream_t s) {
  hipLaunchKernelGGL(k_stereo_lines, dim3(nstreams), dim3(128), 0, s, c, a);
}


// LineMatcher::SearchByProjection(Frame&, const vector<MapLine*>&) and
// (Frame&, KeyFrame*) (LineMatcher.cpp:755-952, 527-721): any number of map
// lines. One 256-thread block: the valid map lines are projected and
// compacted in order into global scratch, then every (projected, current)
// pair is tested; per current line the last passing projected line wins
// (atomicMax), every pass counts.
__device__ __forceinline__ void line_list_stream(const TrackConsts& c, LineListArgs a, const int b) {
  if (a.ncur_arr) {  // batched: stream b
    const long long co = (long long)b * a.cur_pitch, mo = (long long)b * a.ml_pitch;
    a.ncur = a.ncur_arr[b];
    a.nml = a.nml_arr[b];
    a.Tcw += (long long)b * a.pose_stride;
    a.cur_kl_un += co;
    a.cur_desc += co * 32;
    if (a.cur_nobs) a.cur_nobs += co;
    a.match += co;
    a.valid += mo;
    a.ml_xyz6 += mo * 6;
    a.ml_desc += mo * 32;
    a.proj_kl += mo;
    a.proj_src += mo;
    a.nmatches += (long long)b * a.nm_stride;
    if (a.wiped) a.wiped += (long long)b * a.nm_stride;
  }
  __shared__ int s_wc[4];
  __shared__ int s_nto;
  if (a.ncur_arr && !a.refkf) {
    // SearchLocalLines calls the matcher only when some local line is in the
    // frustum (nToMatch > 0, Tracking.cc:1851)
    if (threadIdx.x == 0) s_nto = 0;
    __syncthreads();
    int v = 0;
    for (int i = threadIdx.x; i < a.nml; i += 256) v |= a.valid[i];
    if (v) s_nto = 1;
    __syncthreads();
    if (!s_nto) {
      for (int j = threadIdx.x; j < a.ncur; j += 256) a.match[j] = -1;
      if (threadIdx.x == 0) {
        *a.nmatches = 0;
        if (a.wiped) *a.wiped = 0;
      }
      return;
    }
  }
  __shared__ int s_np, s_cnt;
  __shared__ int s_last[kLineKeep];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  double T[12];
#pragma unroll
  for (int q = 0; q < 12; q++) T[q] = a.Tcw[q];
  if (t == 0) s_np = 0;
  __syncthreads();
  for (int base = 0; base < a.nml; base += 256) {
    const int i = base + t;
    orbpl_keyline k{};
    const bool ok = i < a.nml && a.valid[i] && project_map_line(c, T, a.ml_xyz6 + (long long)i * 6, k);
    const unsigned long long m = __ballot(ok);
    if (lane == 0) s_wc[wave] = __popcll(m);
    __syncthreads();
    int pos = s_np + __popcll(m & ((1ull << lane) - 1ull));
    for (int w = 0; w < wave; w++) pos += s_wc[w];
    if (ok) {
      a.proj_kl[pos] = k;
      a.proj_src[pos] = i;
    }
    __syncthreads();
    if (t == 0) s_np += s_wc[0] + s_wc[1] + s_wc[2] + s_wc[3];
    __syncthreads();
  }
  const int np = s_np, ncur = min(a.ncur, kLineKeep);
  const uint4* cur_desc = reinterpret_cast<const uint4*>(a.cur_desc);
  const uint4* ml_desc = reinterpret_cast<const uint4*>(a.ml_desc);
  int total = 0, wiped = 0;
  for (int pass = 0; pass < 2; pass++) {
    const double o0 = pass ? 10.0 : 0, o1 = pass ? -0.1 : 0, o2 = pass ? -0.1 : 0, o3 = pass ? 5 : 0;
    for (int j = t; j < ncur; j += 256) s_last[j] = -1;
    if (t == 0) s_cnt = 0;
    __syncthreads();
    int cnt = 0;
    for (long long pr = t; pr < (long long)ncur * np; pr += 256) {
      const int j = (int)(pr / np), i = (int)(pr - (long long)j * np);
      if (pass == 0 && a.cur_nobs && a.cur_nobs[j] > 0) continue;
      const orbpl_keyline kp = a.proj_kl[i];
      const orbpl_keyline kc = a.cur_kl_un[j];
      if (line_matching(kp, kc, ml_desc + 2 * a.proj_src[i], cur_desc + 2 * j, o0, o1, o2, o3)) {
        atomicMax(&s_last[j], i);
        cnt++;
      }
    }
    if (cnt) atomicAdd(&s_cnt, cnt);
    __syncthreads();
    total = s_cnt;
    wiped = pass;
    if (pass == 0 && !(total * 1.0 / ncur < 0.2)) break;
    __syncthreads();
  }
  for (int j = t; j < ncur; j += 256) a.match[j] = s_last[j] >= 0 ? a.proj_src[s_last[j]] : -1;
  if (t == 0) {
    *a.nmatches = total;
    if (a.wiped) *a.wiped = wiped;
  }
}

// batched: one workgroup per stream, or (a.list) a small grid looping over
// the streams a list names
__global__ void __launch_bounds__(256) k_line_match_list(TrackConsts c, LineListArgs a) {
  trk_priority();
  if (a.list) {
    const int n = *a.list_n;
    for (int b = blockIdx.x; b < n; b += gridDim.x) {
      line_list_stream(c, a, a.list[b]);
      __syncthreads();
    }
  } else {
    line_list_stream(c, a, blockIdx.x);
  }
}

// The reference's harness overloads of SearchByProjection that also return
// new_kls and match_indices (LineMatcher.cpp:272-487 = mode 0, last frame;
// :954-1170 = mode 1, local map; restated in oracle_line_search_pairs). One
// 256-thread block: the valid map lines are projected, clipped and rebuilt in
// map-line order (mode 0 on a copy of base_kl[i], mode 1 on a zeroed KeyLine),
// every (projected, current) pair's LineMatching verdict is a bit in global
// scratch, then one thread walks the bits in the reference's loop order
// (current j, projected i) with its Observations() bookkeeping: mode 0 skips a
// pair once line j holds a map line with Observations() > 0 (tested per pair,
// on the map line held at that moment), mode 1 skips line j when it starts
// with one. Retry: mode 0 matches * 1.0 / NL < 0.2, mode 1 matches <= 0.2 NL;
// the retry wipes every assignment (and the pairs) and walks the relaxed bits.
__global__ void __launch_bounds__(256) k_line_pairs(TrackConsts c, LinePairArgs a) {
  trk_priority();
  __shared__ int s_wc[4];
  __shared__ int s_np, s_retry;
  __shared__ int s_cnobs[kLineKeep];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  double T[12];
#pragma unroll
  for (int q = 0; q < 12; q++) T[q] = a.Tcw[q];
  if (t == 0) s_np = 0;
  const int ncur = min(a.ncur, kLineKeep);
  for (int j = t; j < ncur; j += 256) s_cnobs[j] = a.cur_nobs ? a.cur_nobs[j] : 0;
  __syncthreads();
  for (int base = 0; base < a.nml; base += 256) {
    const int i = base + t;
    orbpl_keyline k{};
    if (i < a.nml && a.mode == 0 && a.base_kl) k = a.base_kl[i];
    const bool ok = i < a.nml && a.valid[i] && project_map_line(c, T, a.ml_xyz6 + (long long)i * 6, k);
    const unsigned long long m = __ballot(ok);
    if (lane == 0) s_wc[wave] = __popcll(m);
    __syncthreads();
    int pos = s_np + __popcll(m & ((1ull << lane) - 1ull));
    for (int w = 0; w < wave; w++) pos += s_wc[w];
    if (ok) {
      a.proj_kl[pos] = k;
      a.proj_src[pos] = i;
    }
    __syncthreads();
    if (t == 0) s_np += s_wc[0] + s_wc[1] + s_wc[2] + s_wc[3];
    __syncthreads();
  }
  const int np = s_np, words = (np + 31) >> 5;
  const uint4* cur_desc = reinterpret_cast<const uint4*>(a.cur_desc);
  const uint4* ml_desc = reinterpret_cast<const uint4*>(a.ml_desc);
  int npairs = 0;
  for (int pass = 0; pass < 2; pass++) {
    const double o0 = pass ? 10.0 : 0, o1 = pass ? -0.1 : 0, o2 = pass ? -0.1 : 0, o3 = pass ? 5 : 0;
    for (int w = t; w < ncur * words; w += 256) a.okbits[w] = 0u;
    __syncthreads();
    for (long long pr = t; pr < (long long)ncur * np; pr += 256) {
      const int j = (int)(pr / np), i = (int)(pr - (long long)j * np);
      if (line_matching(a.proj_kl[i], a.cur_kl_un[j], ml_desc + 2 * a.proj_src[i], cur_desc + 2 * j,
                        o0, o1, o2, o3))
        atomicOr(a.okbits + (long long)j * words + (i >> 5), 1u << (i & 31));
    }
    __threadfence_block();
    __syncthreads();
    if (t == 0) {
      if (pass) for (int j = 0; j < ncur; j++) s_cnobs[j] = 0;   // mvpMapLines wiped
      int cnt = 0;
      npairs = 0;
      for (int j = 0; j < ncur; j++) {
        a.match[j] = -1;
        if (a.mode == 1 && s_cnobs[j] > 0) continue;
        for (int w = 0; w < words; w++) {
          unsigned b = a.okbits[(long long)j * words + w];
          while (b) {
            const int i = w * 32 + __builtin_ctz(b);
            b &= b - 1u;
            if (a.mode == 0 && s_cnobs[j] > 0) continue;
            const int src = a.proj_src[i];
            a.match[j] = src;
            s_cnobs[j] = a.ml_nobs ? a.ml_nobs[src] : 0;
            if (npairs < a.pair_cap) {
              a.pairs[2 * npairs] = i;
              a.pairs[2 * npairs + 1] = j;
            }
            npairs++;
            cnt++;
          }
        }
      }
      s_retry = pass == 0 && (a.mode == 0 ? (cnt * 1.0 / ncur < 0.2) : (cnt <= 0.2 * ncur));
      *a.nmatches = cnt;
      *a.npairs = npairs;
      *a.wiped = pass;
      *a.nproj = np;
    }
    __syncthreads();
    if (!s_retry) break;
    __syncthreads();
  }
}

void launch_line_pairs(const TrackConsts& c, const LinePairArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(k_line_pairs, dim3(1), dim3(256), 0, s, c, a);
}

// LineMatcher::SearchByProjection(Frame&, KeyFrame*, vector<MapLine*>&)
// (LineMatcher.cpp:492-525; oracle_line_match_bf_knn): thread q finds query
// q's two nearest train descriptors (knnMatch k = 2: the smaller distance
// first, ties to the lower train index), then one thread assigns in query
// order where best / second < 0.75 (float), a later query overwriting.
__global__ void __launch_bounds__(256) k_line_bf_knn(int nq, const uint8_t* __restrict__ qdesc,
                                                     int nt, const uint8_t* __restrict__ tdesc,
                                                     int* __restrict__ out, int* __restrict__ nm) {
  trk_priority();
  __shared__ int s_best[256];
  __shared__ unsigned char s_ok[256];
  const int q = threadIdx.x;
  for (int j = q; j < nt; j += 256) out[j] = -1;
  if (q < nq) {
    const uint4* a = reinterpret_cast<const uint4*>(qdesc) + 2 * q;
    const uint4 a0 = a[0], a1 = a[1];
    int b = -1, s = -1, db = 0, ds = 0;
    for (int j = 0; j < nt; j++) {
      const uint4* p = reinterpret_cast<const uint4*>(tdesc) + 2 * j;
      const uint4 p0 = p[0], p1 = p[1];
      const int d = __popc(a0.x ^ p0.x) + __popc(a0.y ^ p0.y) + __popc(a0.z ^ p0.z) +
                    __popc(a0.w ^ p0.w) + __popc(a1.x ^ p1.x) + __popc(a1.y ^ p1.y) +
                    __popc(a1.z ^ p1.z) + __popc(a1.w ^ p1.w);
      if (b < 0 || d < db) {
        s = b;
        ds = db;
        b = j;
        db = d;
      } else if (s < 0 || d < ds) {
        s = j;
        ds = d;
      }
    }
    s_best[q] = b;
    s_ok[q] = s >= 0 && (float)db / (float)ds < 0.75f;
  }
  __syncthreads();
  if (q == 0) {
    int n = 0;
    for (int k = 0; k < nq; k++)
      if (s_ok[k]) {
        out[s_best[k]] = k;
        n++;
      }
    *nm = n;
  }
}

void launch_line_bf_knn(int nq, const uint8_t* qdesc, int nt, const uint8_t* tdesc, int* out,
                        int* nm, hipStream_t s) {
  hipLaunchKernelGGL(k_line_bf_knn, dim3(1), dim3(256), 0, s, nq, qdesc, nt, tdesc, out, nm);
}

// Frame::IsInFrustum(MapLine*) (Frame.cc:403-430)
__global__ void k_line_in_frustum(const float* __restrict__ Tcw, int n, const float* __restrict__ xyz6,
                                  uint8_t* __restrict__ in_view) {
  trk_priority();
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  float z[2];
#pragma unroll
  for (int e = 0; e < 2; e++) {
    const float* X = xyz6 + (long long)i * 6 + 3 * e;
    double s = (double)Tcw[8] * X[0];
    s += (double)Tcw[9] * X[1];
    s += (double)Tcw[10] * X[2];
    z[e] = (float)(s + (double)Tcw[11]);
  }
  in_view[i] = !(z[0] < 0.0f && z[1] < 0.0f);
}

void launch_line_match_list(const TrackConsts& c, const LineListArgs& a, hipStream_t s,
                            int nstreams) {
  const int grid = !a.ncur_arr ? 1 : a.list ? (nstreams < kListGrid ? nstreams : kListGrid) : nstreams;
  hipLaunchKernelGGL(k_line_match_list, dim3(grid), dim3(256), 0, s, c, a);
}

__global__ void k_line_in_frustum_b(const float* __restrict__ Tcw, int pose_stride,
                                    const int* __restrict__ n_arr, long long pitch,
                                    const float* __restrict__ xyz6, uint8_t* __restrict__ in_view) {
  trk_priority();
  const int b = blockIdx.y;
  const long long o = (long long)b * pitch;
  const float* T = Tcw + (long long)b * pose_stride;
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n_arr[b]) return;
  float z[2];
#pragma unroll
  for (int e = 0; e < 2; e++) {
    const float* X = xyz6 + (o + i) * 6 + 3 * e;
    double s = (double)T[8] * X[0];
    s += (double)T[9] * X[1];
    s += (double)T[10] * X[2];
    z[e] = (float)(s + (double)T[11]);
  }
  in_view[o + i] = !(z[0] < 0.0f && z[1] < 0.0f);
}

void launch_line_in_frustum_batched(const float* Tcw, int pose_stride, const int* n_arr,
                                    long long pitch, const float* xyz6, uint8_t* in_view,
                                    int nstreams, hipStream_t s) {
  if (pitch <= 0) return;
  hipLaunchKernelGGL(k_line_in_frustum_b, dim3((unsigned)((pitch + 255) / 256), nstreams), dim3(256), 0,
                     s, Tcw, pose_stride, n_arr, pitch, xyz6, in_view);
}

void launch_line_in_frustum(const float* Tcw, int n, const float* xyz6, uint8_t* in_view,
                            hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_line_in_frustum, dim3((n + 255) / 256), dim3(256), 0, s, Tcw, n, xyz6, in_view);
}

}  // namespace orbpl
