// Frame::ComputeStereoMatches (Frame.cc:886-1063) on gfx950, restated in
// oracle/track_oracle.cpp (oracle_stereo_matches). One 256-thread workgroup
// per stereo pair of the batch (blockIdx.x = frame):
//   1. row bands: every right keypoint is entered, in index order, in the
//      lists of the rows floor(y - 2 s) .. ceil(y + 2 s) (counting sort in
//      LDS, lists kept in increasing index like vRowIndices);
//   2. thread per left keypoint: best Hamming distance along its row band
//      (octave +-1, disparity window), then the 11x11 SAD search over +-5
//      columns on the pyramid level, the parabola fit and the depth;
//   3. the sorted (SAD, index) list's median and the 1.5*1.4*median cut
//      (bitonic sort in LDS).
// The reference converts the windows to float and subtracts the centre
// pixel; every value is an integer, so the SAD is computed in integers.
#include <hip/hip_runtime.h>

#include <climits>

#include "orb_geom.h"
#include "track_common.h"
#include "track_kernels.h"

namespace orbpl {

namespace {

constexpr int kStereoKp = 4096;
constexpr int kStereoRows = 1024;

__device__ __forceinline__ int ham32(const uint8_t* a, const uint8_t* b) {
  const uint4 a0 = *reinterpret_cast<const uint4*>(a);
  const uint4 a1 = *reinterpret_cast<const uint4*>(a + 16);
  const uint4 b0 = *reinterpret_cast<const uint4*>(b);
  const uint4 b1 = *reinterpret_cast<const uint4*>(b + 16);
  return __popc(a0.x ^ b0.x) + __popc(a0.y ^ b0.y) + __popc(a0.z ^ b0.z) + __popc(a0.w ^ b0.w) +
         __popc(a1.x ^ b1.x) + __popc(a1.y ^ b1.y) + __popc(a1.z ^ b1.z) + __popc(a1.w ^ b1.w);
}

__device__ void bitonic_u32(uint32_t* a, int n) {
  for (int k = 2; k <= n; k <<= 1)
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < n; i += blockDim.x) {
        const int l = i ^ j;
        if (l > i) {
          const uint32_t x = a[i], y = a[l];
          if (((i & k) == 0) ? (x > y) : (x < y)) {
            a[i] = y;
            a[l] = x;
          }
        }
      }
      __syncthreads();
    }
}

}  // namespace

__global__ void __launch_bounds__(256) k_stereo(StereoArgs a) {
  __shared__ int row_start[kStereoRows + 1];
  __shared__ int row_fill[kStereoRows];
  __shared__ uint32_t keys[kStereoKp];
  __shared__ int s_cnt, s_wsum[4];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int f = blockIdx.x;
  // this frame's slice of the batch (locals: the kernel argument stays
  // read-only, so its level table is never copied to scratch)
  const long long fo = (long long)f * a.kp_pitch;
  const KeyPointD* __restrict__ a_kl = a.kl + fo;
  const KeyPointD* __restrict__ a_kr = a.kr + fo;
  const uint8_t* __restrict__ a_dl = a.dl + fo * 32;
  const uint8_t* __restrict__ a_dr = a.dr + fo * 32;
  float* __restrict__ a_uright = a.uright + fo;
  float* __restrict__ a_depth = a.depth + fo;
  int* __restrict__ a_sad = a.sad + fo;
  const uint8_t* a_pyrL = a.pyrL + (long long)f * a.pyr_pitch;
  const uint8_t* a_pyrR = a.pyrR + (long long)f * a.pyr_pitch;
  uint16_t* __restrict__ a_entries = a.entries + (long long)f * a.entry_cap;
  const int n = min(a.n_arr ? a.n_arr[f] : a.n, kStereoKp);
  const int nr = min(a.nr_arr ? a.nr_arr[f] : a.nr, kStereoKp);
  const int nRows = a.nrows;
  // ---- 1. row bands ----
  for (int i = t; i <= kStereoRows; i += 256) row_start[i] = 0;
  __syncthreads();
  for (int iR = t; iR < nr; iR += 256) {
    const KeyPointD k = a_kr[iR];
    const float r = 2.0f * a.scale[k.octave];
    const int maxr = (int)ceilf(k.y + r), minr = (int)floorf(k.y - r);
    for (int yi = max(minr, 0); yi <= min(maxr, nRows - 1); yi++) atomicAdd(&row_start[yi], 1);
  }
  __syncthreads();
  {  // exclusive scan of kStereoRows counts, 4 per thread
    int loc[4], sum = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      loc[k] = row_start[t * 4 + k];
      sum += loc[k];
    }
    int incl = sum;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int u = __shfl_up(incl, o, 64);
      if (lane >= o) incl += u;
    }
    if (lane == 63) s_wsum[wave] = incl;
    __syncthreads();
    int run = incl - sum;
    for (int w = 0; w < wave; w++) run += s_wsum[w];
#pragma unroll
    for (int k = 0; k < 4; k++) {
      row_start[t * 4 + k] = run;
      row_fill[t * 4 + k] = run;
      run += loc[k];
    }
    if (t == 255) row_start[kStereoRows] = run;
    __syncthreads();
  }
  const int total = row_start[kStereoRows];
  if (total > a.entry_cap) {
    if (t == 0) *a.err = 1;
    return;
  }
  for (int iR = t; iR < nr; iR += 256) {
    const KeyPointD k = a_kr[iR];
    const float r = 2.0f * a.scale[k.octave];
    const int maxr = (int)ceilf(k.y + r), minr = (int)floorf(k.y - r);
    for (int yi = max(minr, 0); yi <= min(maxr, nRows - 1); yi++)
      a_entries[atomicAdd(&row_fill[yi], 1)] = (uint16_t)iR;
  }
  __syncthreads();
  for (int row = t; row < nRows; row += 256) {  // increasing index within a row
    const int b = row_start[row], e = row_start[row + 1];
    for (int q = b + 1; q < e; q++) {
      const uint16_t v = a_entries[q];
      int r = q - 1;
      while (r >= b && a_entries[r] > v) {
        a_entries[r + 1] = a_entries[r];
        r--;
      }
      a_entries[r + 1] = v;
    }
  }
  if (t == 0) s_cnt = 0;
  __syncthreads();
  // ---- 2. per left keypoint ----
  const float mbf = a.mbf, minZ = a.mb, minD = 0, maxD = mbf / minZ;
  for (int iL = t; iL < n; iL += 256) {
    a_uright[iL] = -1.0f;
    a_depth[iL] = -1.0f;
    a_sad[iL] = -1;
    const KeyPointD kpL = a_kl[iL];
    const int levelL = kpL.octave;
    const float vL = kpL.y, uL = kpL.x;
    const int row = (int)vL;
    if (row < 0 || row >= nRows) continue;
    const int rb = row_start[row], re = row_start[row + 1];
    if (rb == re) continue;
    const float minU = uL - maxD, maxU = uL - minD;
    if (maxU < 0) continue;
    int bestDist = 100, bestIdxR = 0;
    const uint8_t* dL = a_dl + (long long)iL * 32;
    for (int q = rb; q < re; q++) {
      const int iR = a_entries[q];
      const KeyPointD kpR = a_kr[iR];
      if (kpR.octave < levelL - 1 || kpR.octave > levelL + 1) continue;
      const float uR = kpR.x;
      if (uR >= minU && uR <= maxU) {
        const int dist = ham32(dL, a_dr + (long long)iR * 32);
        if (dist < bestDist) {
          bestDist = dist;
          bestIdxR = iR;
        }
      }
    }
    if (bestDist >= (100 + 50) / 2) continue;
    const float uR0 = a_kr[bestIdxR].x;
    const float scaleFactor = a.inv_scale[levelL];
    const float scaleduL = roundf(kpL.x * scaleFactor);
    const float scaledvL = roundf(kpL.y * scaleFactor);
    const float scaleduR0 = roundf(uR0 * scaleFactor);
    const int w = 5, L = 5;
    const LevelGeom& G = a.lv[levelL];
    const int cuL = (int)scaleduL, cvL = (int)scaledvL, cuR = (int)scaleduR0;
    const float iniu = scaleduR0 + L - w;
    const float endu = scaleduR0 + L + w + 1;
    if (iniu < 0 || endu >= G.w) continue;
    if (cvL - w < 0 || cvL + w >= G.h || cuL - w < 0 || cuL + w >= G.w || cuR - L - w < 0) continue;
    const uint8_t* PL = a_pyrL + content_off(G, 0, 0);
    const uint8_t* PR = a_pyrR + content_off(G, 0, 0);
    const int cL = PL[(long long)cvL * G.pitch + cuL];
    int sads[11];
#pragma unroll
    for (int k = 0; k < 11; k++) sads[k] = 0;
    for (int yy = -w; yy <= w; yy++) {
      const uint8_t* rl = PL + (long long)(cvL + yy) * G.pitch + cuL - w;
      const uint8_t* rr = PR + (long long)(cvL + yy) * G.pitch + cuR - L - w;
      int lv[11], rv[21];
#pragma unroll
      for (int xx = 0; xx < 11; xx++) lv[xx] = (int)rl[xx] - cL;
#pragma unroll
      for (int xx = 0; xx < 21; xx++) rv[xx] = rr[xx];
#pragma unroll
      for (int k = 0; k < 11; k++) {
        const int cR = PR[(long long)cvL * G.pitch + cuR - L + k];
        int s = 0;
#pragma unroll
        for (int xx = 0; xx < 11; xx++) s += abs(lv[xx] - (rv[k + xx] - cR));
        sads[k] += s;
      }
    }
    int bestD = INT_MAX, bestincR = 0;
    float vDists[11];
#pragma unroll
    for (int k = 0; k < 11; k++) {
      const float dist = (float)sads[k];
      if (dist < bestD) {
        bestD = (int)dist;
        bestincR = k - L;
      }
      vDists[k] = dist;
    }
    if (bestincR == -L || bestincR == L) continue;
    float dist1 = 0, dist2 = 0, dist3 = 0;
#pragma unroll
    for (int k = 1; k < 10; k++)
      if (k == L + bestincR) {
        dist1 = vDists[k - 1];
        dist2 = vDists[k];
        dist3 = vDists[k + 1];
      }
    const float deltaR = (dist1 - dist3) / (2.0f * (dist1 + dist3 - 2.0f * dist2));
    if (deltaR < -1 || deltaR > 1) continue;
    float bestuR = a.scale[levelL] * ((float)scaleduR0 + (float)bestincR + deltaR);
    float disparity = (uL - bestuR);
    if (disparity >= minD && disparity < maxD) {
      if (disparity <= 0) {
        disparity = 0.01f;
        bestuR = (float)((double)uL - 0.01);
      }
      a_depth[iL] = mbf / disparity;
      a_uright[iL] = bestuR;
      a_sad[iL] = bestD;
      atomicAdd(&s_cnt, 1);
    }
  }
  __syncthreads();
  // ---- 3. median of the stored SADs and the outlier cut ----
  const int cnt = s_cnt;
  if (cnt == 0) return;
  for (int i = t; i < kStereoKp; i += 256) {
    const int d = i < n ? a_sad[i] : -1;
    keys[i] = d >= 0 ? ((uint32_t)d << 12) | (uint32_t)i : 0xFFFFFFFFu;
  }
  __syncthreads();
  bitonic_u32(keys, kStereoKp);
  const float median = (float)(int)(keys[cnt / 2] >> 12);
  const float thDist = 1.5f * 1.4f * median;
  for (int iL = t; iL < n; iL += 256) {
    const int d = a_sad[iL];
    if (d >= 0 && !(d < thDist)) {
      a_uright[iL] = -1.0f;
      a_depth[iL] = -1.0f;
    }
  }
}

void launch_stereo(const StereoArgs& a, int batch, hipStream_t s) {
  hipLaunchKernelGGL(k_stereo, dim3(batch), dim3(256), 0, s, a);
}

}  // namespace orbpl
