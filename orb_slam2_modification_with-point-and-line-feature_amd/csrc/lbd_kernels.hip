// KeyLines, 80-longest selection, LBD descriptors and line coefficients on
// gfx950: the rest of LineExtractor::ExtractLineSegment
// (/root/reference/src/LineExtractor.cpp:20-72) after LSD.
//
//   k_keylines : LSDDetector::detectImpl KeyLine fields (class_id = detection
//                index, LineIterator pixel count with clipLine), then the
//                reference's std::sort by response (libstdc++ introsort
//                replayed serially — n is a few hundred) and resize(80)
//   k_sobel    : BinaryDescriptor::computeSobel: dx/dy (Sobel 3x3, 16S) of the
//                GaussianBlur(5x5, 1) image (k_lsd_blur with the 5-tap kernel)
//   k_lbd      : BinaryDescriptor::computeLBD + binaryConversion, one wave per
//                line: lane h accumulates row h of the 63-row support region
//                in the reference's order; band sums, statistics and the
//                32 band-pair comparisons follow serially
//   coefficients: Eigen s.cross(e).normalized() (LineExtractor.cpp:62-72)
// Restated in oracle/lsd_oracle.cpp (oracle_line_extract).
#include <hip/hip_runtime.h>

#include "lsd_kernels.h"
#include "lsd_math.h"
#include "orbpl_math.h"
#include "line_common.h"

namespace orbpl {

namespace {

__device__ __forceinline__ int refl(int i, int n) {
  if (n == 1) return 0;
  while (i < 0 || i >= n) i = i < 0 ? -i : 2 * n - 2 - i;
  return i;
}

// ---- libstdc++ std::sort on an index array, comp(a, b) = key[a] > key[b] ----
__device__ __forceinline__ bool kgt(const float* key, int a, int b) { return key[a] > key[b]; }

__device__ void iswap(int* v, int a, int b) {
  const int t = v[a];
  v[a] = v[b];
  v[b] = t;
}

__device__ void move_median_first(int* v, const float* key, int result, int a, int b, int c) {
  if (kgt(key, v[a], v[b])) {
    if (kgt(key, v[b], v[c])) iswap(v, result, b);
    else if (kgt(key, v[a], v[c])) iswap(v, result, c);
    else iswap(v, result, a);
  } else if (kgt(key, v[a], v[c])) {
    iswap(v, result, a);
  } else if (kgt(key, v[b], v[c])) {
    iswap(v, result, c);
  } else {
    iswap(v, result, b);
  }
}

__device__ int unguarded_partition(int* v, const float* key, int first, int last, int pivot) {
  while (true) {
    while (kgt(key, v[first], v[pivot])) ++first;
    --last;
    while (kgt(key, v[pivot], v[last])) --last;
    if (!(first < last)) return first;
    iswap(v, first, last);
    ++first;
  }
}

__device__ void adjust_heap_i(int* v, const float* key, int base, int hole, int len, int value) {
  const int top = hole;
  int second = hole;
  while (second < (len - 1) / 2) {
    second = 2 * (second + 1);
    if (kgt(key, v[base + second], v[base + second - 1])) second--;
    v[base + hole] = v[base + second];
    hole = second;
  }
  if ((len & 1) == 0 && second == (len - 2) / 2) {
    second = 2 * (second + 1);
    v[base + hole] = v[base + second - 1];
    hole = second - 1;
  }
  int parent = (hole - 1) / 2;
  while (hole > top && key[v[base + parent]] > key[value]) {
    v[base + hole] = v[base + parent];
    hole = parent;
    parent = (hole - 1) / 2;
  }
  v[base + hole] = value;
}

__device__ void heap_sort_i(int* v, const float* key, int base, int len) {
  if (len < 2) return;
  for (int parent = (len - 2) / 2;; parent--) {
    adjust_heap_i(v, key, base, parent, len, v[base + parent]);
    if (parent == 0) break;
  }
  for (int last = len; last > 1;) {
    --last;
    const int val = v[base + last];
    v[base + last] = v[base];
    adjust_heap_i(v, key, base, 0, last, val);
  }
}

__device__ void std_sort_desc(int* v, const float* key, int n) {
  if (n <= 1) return;
  int st_f[64], st_l[64], st_d[64];
  int sp = 0;
  st_f[sp] = 0;
  st_l[sp] = n;
  st_d[sp] = 2 * (31 - __clz(n));
  sp++;
  while (sp > 0) {
    sp--;
    int f = st_f[sp], l = st_l[sp], d = st_d[sp];
    while (l - f > 16) {
      if (d == 0) {
        heap_sort_i(v, key, f, l - f);
        break;
      }
      --d;
      const int mid = f + (l - f) / 2;
      move_median_first(v, key, f, f + 1, mid, l - 1);
      const int cut = unguarded_partition(v, key, f + 1, l, f);
      st_f[sp] = cut;
      st_l[sp] = l;
      st_d[sp] = d;
      sp++;
      l = cut;
    }
  }
  // __final_insertion_sort: never crosses a partition boundary
  for (int i = 1; i < n; i++) {
    const int val = v[i];
    int j = i;
    while (j > 0 && key[val] > key[v[j - 1]]) {
      v[j] = v[j - 1];
      j--;
    }
    v[j] = val;
  }
}

}  // namespace

// One 64-thread block per frame.
__global__ void __launch_bounds__(64) k_keylines(LsdGeom g, LsdScratch sc, LineOut o) {
  __shared__ int s_idx[kLsdMaxLines];
  __shared__ float s_key[kLsdMaxLines];
  const int f = blockIdx.x, lane = threadIdx.x;
  const int n = sc.nlines[f];
  const float* L = sc.lines + (long long)f * kLsdMaxLines * 4;
  orbpl_keyline* K = o.kl_all + (long long)f * kLsdMaxLines;
  const float maxwh = (float)max(g.W, g.H);
  for (int k = lane; k < n; k += 64) {
    const float4 e = *reinterpret_cast<const float4*>(L + 4 * k);
    orbpl_keyline kl;
    kl.startPointX = e.x * 1.0f;
    kl.startPointY = e.y * 1.0f;
    kl.endPointX = e.z * 1.0f;
    kl.endPointY = e.w * 1.0f;
    kl.sPointInOctaveX = e.x;
    kl.sPointInOctaveY = e.y;
    kl.ePointInOctaveX = e.z;
    kl.ePointInOctaveY = e.w;
    const double ddx = (double)(e.x - e.z), ddy = (double)(e.y - e.w);
    kl.lineLength = (float)sqrt(ddx * ddx + ddy * ddy);
    kl.numOfPixels = line_iterator_count(g.W, g.H, e.x, e.y, e.z, e.w);
    kl.angle = (float)lsdm::atan2_((double)(kl.endPointY - kl.startPointY),
                                   (double)(kl.endPointX - kl.startPointX));
    kl.class_id = k;
    kl.octave = 0;
    kl.size = (kl.endPointX - kl.startPointX) * (kl.endPointY - kl.startPointY);
    kl.response = kl.lineLength / maxwh;
    kl.pt_x = (kl.endPointX + kl.startPointX) / 2;
    kl.pt_y = (kl.endPointY + kl.startPointY) / 2;
    K[k] = kl;
    s_idx[k] = k;
    s_key[k] = kl.response;
  }
  __syncthreads();
  if (n > kLineKeep && lane == 0) std_sort_desc(s_idx, s_key, n);
  __syncthreads();
  const int keep = min(n, kLineKeep);
  orbpl_keyline* out = o.kl + (long long)f * kLineKeep;
  double* coef = o.coef + (long long)f * kLineKeep * 3;
  for (int i = lane; i < keep; i += 64) {
    const orbpl_keyline kl = K[s_idx[i]];
    out[i] = kl;
    // Eigen Vector3d(s, 1).cross(Vector3d(e, 1)).normalized()
    const double s0 = kl.startPointX, s1 = kl.startPointY, s2 = 1.0;
    const double e0 = kl.endPointX, e1 = kl.endPointY, e2 = 1.0;
    double c0 = s1 * e2 - s2 * e1, c1 = s2 * e0 - s0 * e2, c2 = s0 * e1 - s1 * e0;
    const double nrm = sqrt(c0 * c0 + c1 * c1 + c2 * c2);
    if (nrm > 0) {
      c0 /= nrm;
      c1 /= nrm;
      c2 /= nrm;
    }
    coef[3 * i] = c0;
    coef[3 * i + 1] = c1;
    coef[3 * i + 2] = c2;
  }
  if (lane == 0) o.n[f] = keep;
}

// Sobel 3x3 (CV_16S, REFLECT_101) of the 5x5-blurred image.
__global__ void __launch_bounds__(256) k_sobel(int W, int H, const uint8_t* __restrict__ blur5,
                                               int16_t* __restrict__ dx, int16_t* __restrict__ dy) {
  const int f = blockIdx.y;
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= W * H) return;
  const int y = i / W, x = i - y * W;
  const uint8_t* G = blur5 + (long long)f * W * H;
  auto px = [&](int xx, int yy) { return (int)G[refl(yy, H) * W + refl(xx, W)]; };
  const int gx = (px(x + 1, y - 1) - px(x - 1, y - 1)) + 2 * (px(x + 1, y) - px(x - 1, y)) +
                 (px(x + 1, y + 1) - px(x - 1, y + 1));
  const int gy = (px(x - 1, y + 1) - px(x - 1, y - 1)) + 2 * (px(x, y + 1) - px(x, y - 1)) +
                 (px(x + 1, y + 1) - px(x + 1, y - 1));
  dx[(long long)f * W * H + i] = (int16_t)gx;
  dy[(long long)f * W * H + i] = (int16_t)gy;
}

// computeLBD for one KeyLine per wave (4 lines per 256-thread block).
__global__ void __launch_bounds__(256) k_lbd(int W, int H, const int16_t* __restrict__ pdx_all,
                                             const int16_t* __restrict__ pdy_all, LbdWeights wts,
                                             LineOut o) {
  constexpr int kBW = 7, kNB = 9, kRows = kBW * kNB;
  __shared__ float s_row[4][kRows][4];
  __shared__ float s_band[4][8][kNB];
  __shared__ float s_d[4][kNB * 8];
  const int f = blockIdx.y, wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int li = blockIdx.x * 4 + wave;
  if (li >= o.n[f]) return;
  const orbpl_keyline kl = o.kl[(long long)f * kLineKeep + li];
  const int16_t* pdx = pdx_all + (long long)f * W * H;
  const int16_t* pdy = pdy_all + (long long)f * W * H;
  const short halfHeight = (kRows - 1) / 2;
  const short imageWidth = (short)(W - 1), imageHeight = (short)(H - 1);
  const short lengthOfLSP = (short)kl.numOfPixels;
  const short halfWidth = (lengthOfLSP - 1) / 2;
  const float midX = (float)(0.5 * (kl.sPointInOctaveX + kl.ePointInOctaveX));
  const float midY = (float)(0.5 * (kl.sPointInOctaveY + kl.ePointInOctaveY));
  float dL0, dL1;
  {
    // cos/sin of a float in [-pi, pi], correctly rounded (pinned P2)
    const float a = kl.angle < 0 ? -kl.angle : kl.angle;
    float c, s;
    cr_cos_sin(a, &c, &s);
    dL0 = c;
    dL1 = copysignf(s, kl.angle);  // sin is odd (also for -0)
  }
  const float dO0 = -dL1, dO1 = dL0;
  if (lane < kRows) {
    float sCorX0 = -dL0 * halfWidth + dL1 * halfHeight + midX;
    float sCorY0 = -dL1 * halfWidth - dL0 * halfHeight + midY;
    for (int h = 0; h < lane; h++) {
      sCorX0 -= dL1;
      sCorY0 += dL0;
    }
    // the row's walk along the line, kLbdU steps per round: the positions
    // (the reference's running sCorX / sCorY sums, in order) and all their
    // dx / dy loads first, then the accumulation in step order (each step's
    // loads used to wait for the previous step's)
    constexpr int kLbdU = 8;
    float sCorX = sCorX0, sCorY = sCorY0;
    float pLr = 0, nLr = 0, pOr = 0, nOr = 0;
    for (int w0 = 0; w0 < lengthOfLSP; w0 += kLbdU) {
      short dxs[kLbdU], dys[kLbdU];
#pragma unroll
      for (int u = 0; u < kLbdU; u++) {
        short t = (short)roundf(sCorX);
        const short xCor = (t < 0) ? 0 : (t > imageWidth) ? imageWidth : t;
        t = (short)roundf(sCorY);
        const short yCor = (t < 0) ? 0 : (t > imageHeight) ? imageHeight : t;
        dxs[u] = pdx[yCor * W + xCor];
        dys[u] = pdy[yCor * W + xCor];
        sCorX += dL0;
        sCorY += dL1;
      }
#pragma unroll
      for (int u = 0; u < kLbdU; u++) {
        if (w0 + u < lengthOfLSP) {
          const short dx = dxs[u], dy = dys[u];
          const float gDL = dx * dL0 + dy * dL1;
          const float gDO = dx * dO0 + dy * dO1;
          if (gDL > 0) pLr += gDL;
          else nLr -= gDL;
          if (gDO > 0) pOr += gDO;
          else nOr -= gDO;
        }
      }
    }
    const float c = wts.gG[lane];
    s_row[wave][lane][0] = c * pLr;
    s_row[wave][lane][1] = c * nLr;
    s_row[wave][lane][2] = c * pOr;
    s_row[wave][lane][3] = c * nOr;
  }
  __builtin_amdgcn_wave_barrier();
  if (lane != 0) return;
  // serial part (lane 0): band sums in LDS (indexed by the row's band)
  float(*B)[kNB] = s_band[wave];
  for (int q = 0; q < 8; q++)
    for (int b = 0; b < kNB; b++) B[q][b] = 0.f;
  for (int hID = 0; hID < kRows; hID++) {
    const float pLr = s_row[wave][hID][0], nLr = s_row[wave][hID][1];
    const float pOr = s_row[wave][hID][2], nOr = s_row[wave][hID][3];
    const float pL2r = pLr * pLr, nL2r = nLr * nLr, pO2r = pOr * pOr, nO2r = nOr * nOr;
    auto acc = [&](int b, float c) {
      B[0][b] += c * pLr;
      B[1][b] += c * nLr;
      B[2][b] += c * c * pL2r;
      B[3][b] += c * c * nL2r;
      B[4][b] += c * pOr;
      B[5][b] += c * nOr;
      B[6][b] += c * c * pO2r;
      B[7][b] += c * c * nO2r;
    };
    int b = hID / kBW;
    acc(b, wts.gL[hID % kBW + kBW]);
    b--;
    if (b >= 0) acc(b, wts.gL[hID % kBW + 2 * kBW]);
    b = b + 2;
    if (b < kNB) acc(b, wts.gL[hID % kBW]);
  }
  float* d = s_d[wave];
  const float invN2 = (float)(1.0 / (kBW * 2.0)), invN3 = (float)(1.0 / (kBW * 3.0));
  for (int b = 0; b < kNB; b++) {
    const float invN = (b == 0 || b == kNB - 1) ? invN2 : invN3;
    float t = B[0][b] * invN;
    d[b * 8 + 0] = t;
    d[b * 8 + 4] = sqrtf(B[2][b] * invN - t * t);
    t = B[1][b] * invN;
    d[b * 8 + 1] = t;
    d[b * 8 + 5] = sqrtf(B[3][b] * invN - t * t);
    t = B[4][b] * invN;
    d[b * 8 + 2] = t;
    d[b * 8 + 6] = sqrtf(B[6][b] * invN - t * t);
    t = B[5][b] * invN;
    d[b * 8 + 3] = t;
    d[b * 8 + 7] = sqrtf(B[7][b] * invN - t * t);
  }
  float tempM = 0, tempS = 0;
  for (int b = 0; b < kNB; b++) {
    const float* v = d + 8 * b;
    tempM += v[0] * v[0];
    tempM += v[1] * v[1];
    tempM += v[2] * v[2];
    tempM += v[3] * v[3];
    tempS += v[4] * v[4];
    tempS += v[5] * v[5];
    tempS += v[6] * v[6];
    tempS += v[7] * v[7];
  }
  tempM = 1 / sqrtf(tempM);
  tempS = 1 / sqrtf(tempS);
  for (int b = 0; b < kNB; b++) {
    float* v = d + 8 * b;
    for (int q = 0; q < 4; q++) v[q] = v[q] * tempM;
    for (int q = 4; q < 8; q++) v[q] = v[q] * tempS;
  }
  for (int i = 0; i < kNB * 8; i++)
    if ((double)d[i] > 0.4) d[i] = (float)0.4;
  float tempSum = 0;
  for (int i = 0; i < kNB * 8; i++) tempSum += d[i] * d[i];
  tempSum = 1 / sqrtf(tempSum);
  for (int i = 0; i < kNB * 8; i++) d[i] = d[i] * tempSum;
  // band pairs of BinaryDescriptor::computeImpl (first 32 of its table)
  const int comb[32][2] = {{0, 1}, {0, 2}, {0, 3}, {0, 4}, {0, 5}, {0, 6}, {1, 2}, {1, 3},
                           {1, 4}, {1, 5}, {1, 6}, {2, 3}, {2, 4}, {2, 5}, {2, 6}, {2, 7},
                           {2, 8}, {3, 4}, {3, 5}, {3, 6}, {3, 7}, {3, 8}, {4, 5}, {4, 6},
                           {4, 7}, {4, 8}, {5, 6}, {5, 7}, {5, 8}, {6, 7}, {6, 8}, {7, 8}};
  uint8_t* out = o.desc + ((long long)f * kLineKeep + li) * 32;
  uint32_t w[8] = {};
#pragma unroll
  for (int c = 0; c < 32; c++) {
    uint32_t r = 0;
#pragma unroll
    for (int i = 0; i < 8; i++)
      if (d[8 * comb[c][0] + i] > d[8 * comb[c][1] + i]) r |= 1u << i;
    w[c >> 2] |= r << (8 * (c & 3));
  }
  uint4* o4 = reinterpret_cast<uint4*>(out);
  o4[0] = make_uint4(w[0], w[1], w[2], w[3]);
  o4[1] = make_uint4(w[4], w[5], w[6], w[7]);
}

void launch_keylines(const LsdGeom& g, const LsdScratch& sc, const LineOut& o, int batch,
                     hipStream_t s) {
  hipLaunchKernelGGL(k_keylines, dim3(batch), dim3(64), 0, s, g, sc, o);
}

// BinaryDescriptor's 5x5 sigma-1 GaussianBlur (k_lsd_blur's fixed point) and
// computeSobel fused per 64x32 tile: the tile's input with both halos (blur 2
// + Sobel 1, REFLECT_101) in LDS, the blur at the tile's pixels and their
// Sobel neighbours, then dx / dy. The blurred image never goes to HBM. The
// Sobel taps outside the image read the blur at REFLECT_101 coordinates; with
// a symmetric kernel that is the blur of the reflected input, which is what
// the tile computes at those virtual coordinates.
constexpr int kBsTW = 64, kBsTH = 32, kBsR = 2;
__global__ void __launch_bounds__(256) k_blur_sobel(LsdGeom g5, const uint8_t* __restrict__ img,
                                                    int stride, long long frame_pitch,
                                                    int16_t* __restrict__ dx,
                                                    int16_t* __restrict__ dy) {
  constexpr int kIW = kBsTW + 2 + 2 * kBsR, kIH = kBsTH + 2 + 2 * kBsR;   // 70 x 38
  constexpr int kBW = kBsTW + 2, kBH = kBsTH + 2;                          // 66 x 34
  __shared__ uint8_t s_in[kIH][kIW];
  __shared__ uint16_t s_h[kIH][kBW];
  __shared__ uint8_t s_b[kBH][kBW + 2];
  const int f = blockIdx.z, t = threadIdx.x;
  const int x0 = blockIdx.x * kBsTW, y0 = blockIdx.y * kBsTH;
  const int W = g5.W, H = g5.H;
  const uint8_t* src = img + (long long)f * frame_pitch;
  for (int i = t; i < kIH * kIW; i += 256) {
    const int r = i / kIW, c = i - r * kIW;
    s_in[r][c] = src[(long long)refl(y0 - 1 - kBsR + r, H) * stride + refl(x0 - 1 - kBsR + c, W)];
  }
  __syncthreads();
  for (int i = t; i < kIH * kBW; i += 256) {
    const int r = i / kBW, c = i - r * kBW;
    int acc = 0;
#pragma unroll
    for (int j = 0; j < 2 * kBsR + 1; j++) acc += g5.gk[j] * s_in[r][c + j];
    s_h[r][c] = (uint16_t)acc;
  }
  __syncthreads();
  for (int i = t; i < kBH * kBW; i += 256) {
    const int r = i / kBW, c = i - r * kBW;
    int acc = 0;
#pragma unroll
    for (int j = 0; j < 2 * kBsR + 1; j++) acc += g5.gk[j] * (int)s_h[r + j][c];
    s_b[r][c] = (uint8_t)min(255, (acc + (1 << 15)) >> 16);
  }
  __syncthreads();
  const long long fo = (long long)f * W * H;
  for (int i = t; i < kBsTH * kBsTW; i += 256) {
    const int r = i / kBsTW, c = i - r * kBsTW;
    const int x = x0 + c, y = y0 + r;
    if (x >= W || y >= H) continue;
    // s_b[r + 1 + dy][c + 1 + dx] = blur at (x + dx, y + dy)
    auto B = [&](int ddx, int ddy) { return (int)s_b[r + 1 + ddy][c + 1 + ddx]; };
    const int gx = (B(1, -1) - B(-1, -1)) + 2 * (B(1, 0) - B(-1, 0)) + (B(1, 1) - B(-1, 1));
    const int gy = (B(-1, 1) - B(-1, -1)) + 2 * (B(0, 1) - B(0, -1)) + (B(1, 1) - B(1, -1));
    dx[fo + (long long)y * W + x] = (int16_t)gx;
    dy[fo + (long long)y * W + x] = (int16_t)gy;
  }
}

void launch_blur_sobel(const LsdGeom& g5, const uint8_t* img, int stride, long long frame_pitch,
                       int16_t* dx, int16_t* dy, int batch, hipStream_t s) {
  dim3 grid((g5.W + kBsTW - 1) / kBsTW, (g5.H + kBsTH - 1) / kBsTH, batch);
  hipLaunchKernelGGL(k_blur_sobel, grid, dim3(256), 0, s, g5, img, stride, frame_pitch, dx, dy);
}

void launch_sobel(int W, int H, const uint8_t* blur5, int16_t* dx, int16_t* dy, int batch,
                  hipStream_t s) {
  hipLaunchKernelGGL(k_sobel, dim3((W * H + 255) / 256, batch), dim3(256), 0, s, W, H, blur5, dx,
                     dy);
}

void launch_lbd(int W, int H, const int16_t* dx, const int16_t* dy, const LbdWeights& w,
                const LineOut& o, int batch, hipStream_t s) {
  hipLaunchKernelGGL(k_lbd, dim3(kLineKeep / 4, batch), dim3(256), 0, s, W, H, dx, dy, w, o);
}

}  // namespace orbpl
