// Host runtime and C-ABI of the line-feature path (include/orbpl.h, lsdx_*):
// LineExtractor::ExtractLineSegment (/root/reference/src/LineExtractor.cpp:12-74).
// One lsdx_ctx = one device + one HIP stream + scratch for max_batch frames of
// one image geometry.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cmath>
#include <cstring>
#include <vector>

#include "../../include/orbpl.h"
#include "lsd_kernels.h"
#include "lsd_math.h"
#include "orbpl_runtime.h"

using namespace orbpl;

#define HIP_CHECK(expr)                                              \
  do {                                                               \
    hipError_t _e = (expr);                                          \
    if (_e != hipSuccess) return orbpl::hip_fail(_e, #expr, __LINE__); \
  } while (0)

namespace {

// getGaussianKernelBitExact rounded to 8.8 fixed point (GaussianBlur 8U).
void gauss_kernel_fixed(int n, double sigma, int* k) {
  const double scale2X = -0.125 / (sigma * sigma);
  const int n2 = (n - 1) / 2;
  double vals[16];
  double sum = 0;
  for (int i = 0, x = 1 - n; i < n2; i++, x += 2) {
    vals[i] = lsdm::exp_((double)(x * x) * scale2X);
    sum += vals[i];
  }
  sum = sum * 2 + 1.0;
  const double mul1 = 1.0 / sum;
  int s2 = 0;
  for (int i = 0; i < n2; i++) {
    const int t = (int)std::lrint(vals[i] * mul1 * 256.0);
    k[i] = k[n - 1 - i] = t;
    s2 += t;
  }
  k[n2] = 256 - 2 * s2;
}

// interpolationLinear coefficients (resize_bitExact): offsets, 8.8 c1, range.
void lin_tab(double inv_scale, int ssize, int dsize, int* ofs, int* c1, int* mn, int* mx) {
  const double scale = 1.0 / inv_scale;
  int minofst = 0, maxofst = dsize;
  for (int d = 0; d < dsize; d++) {
    const double fval = scale * ((double)d + 0.5) - 0.5;
    const int ival = (int)std::floor(fval);
    ofs[d] = 0;
    c1[d] = 0;
    if (ival >= 0 && ssize > 1) {
      if (ival < ssize - 1) {
        ofs[d] = ival;
        c1[d] = (int)std::lrint((fval - (double)ival) * 256.0);
      } else {
        ofs[d] = ssize - 1;
        maxofst = std::min(maxofst, d);
      }
    } else {
      minofst = std::max(minofst, d + 1);
    }
  }
  *mn = minofst;
  *mx = maxofst;
}

}  // namespace

struct lsdx_ctx {
  int device = 0, max_batch = 0, W = 0, H = 0;
  LsdGeom g{};
  LsdGeom g5{};          // the same geometry with BinaryDescriptor's 5x5 sigma 1 blur
  LsdScratch sc{};
  LineOut lo{};
  LbdWeights lw{};
  uint8_t* blur5 = nullptr;
  int16_t* sdx = nullptr;
  int16_t* sdy = nullptr;
  hipStream_t stream = nullptr;
  int* d_tabs = nullptr;
  uint8_t* d_in = nullptr;
  int last_batch = 0;
  bool serial_grow = false;  // lsdx_set_serial_grow: wave-serial seed loop
  bool fused_prep = false;   // k_lsd_prep (the tiles' source spans fit; ksize 7)
  std::vector<void*> allocs;
};

static int lx_alloc(lsdx_ctx* c, void** p, size_t bytes) {
  hipError_t e = hipMalloc(p, bytes ? bytes : 1);
  if (e != hipSuccess) return hip_fail(e, "hipMalloc", __LINE__);
  c->allocs.push_back(*p);
  return ORBPL_OK;
}

namespace orbpl {
int lsd_geometry(int W, int H, LsdGeom* out) {
  if (W < 16 || H < 16 || W > 4096 || H > 4096) return arg_fail("image size out of range [16, 4096]");
  LsdGeom g{};
  g.W = W;
  g.H = H;
  const double scale = 0.8, sigma_scale = 0.6, quant = 2.0, ang_th = 22.5;
  g.sw = (int)std::lrint(W * scale);
  g.sh = (int)std::lrint(H * scale);
  if (g.sw > 65535 || g.sh > 65535) return arg_fail("image too large");
  g.n = (g.sw - 1) * (g.sh - 1);
  if (g.n >= (1 << 22)) return arg_fail("image too large for the LSD pixel order (2^22 pixels)");
  const double sigma = sigma_scale / scale;
  const unsigned h = (unsigned)std::ceil(sigma * std::sqrt(2 * 3.0 * lsdm::log_(10.0)));
  g.ksize = 1 + 2 * (int)h;
  if (g.ksize > 7) return arg_fail("unexpected LSD Gaussian size");
  gauss_kernel_fixed(g.ksize, sigma, g.gk);
  g.prec = 3.14159265358979323846 * ang_th / 180;
  g.p = ang_th / 180;
  g.rho = quant / lsdm::sin_(g.prec);
  g.log_nt = 5 * (lsdm::log10_(double(g.sw)) + lsdm::log10_(double(g.sh))) / 2 + lsdm::log10_(11.0);
  g.min_reg_size = (int)(size_t)(-g.log_nt / lsdm::log10_(g.p));
  g.seg_cap = g.n / 17 + 2;
  g.chunk_cap = g.n / kLsdSortChunk + g.seg_cap + 2;
  g.leaf_cap = g.n / 2 + 2;
  // the global levels only partition segments above the deferral bound
  // (>= 1024 elements): at most 2 n / 1024 chunks of 1024 per level
  g.mask_cap = 2 * (g.n / 1024) + 8;
  *out = g;
  return ORBPL_OK;
}
}  // namespace orbpl

namespace orbpl {
// Detection (and, with `out`, KeyLines + LBD) of `batch` frames on stream `s`.
// The tracker calls this with its own per-frame output buffers and stream;
// `ev_mid` (optional) is recorded between LSD and the LineExtractor stages.
int lsdx_run(lsdx_ctx* c, const uint8_t* d_imgs, int batch, int stride, int64_t frame_pitch,
             const LineOut* out, hipStream_t s, hipEvent_t ev_mid, const hipEvent_t* ev_stage) {
  // ev_stage (optional, 5 events): after blur/resize/grad, after the
  // pseudo-ordering sort, after the seed loop, after KeyLines, after LBD
  const LsdGeom& g = c->g;
  HIP_CHECK(hipMemsetAsync(c->sc.maxq, 0, (size_t)batch * 4, s));
  HIP_CHECK(hipMemsetAsync(c->sc.err, 0, (size_t)batch * 4, s));
  if (c->fused_prep) {
    launch_lsd_prep(g, c->d_tabs, d_imgs, stride, frame_pitch, c->sc.scaled, c->sc.deg, c->sc.q,
                    c->sc.sd, c->sc.maxq, batch, s);
  } else {
    launch_lsd_blur(g, d_imgs, stride, frame_pitch, c->sc.blur, batch, s);
    launch_lsd_resize(g, c->d_tabs, c->sc.blur, c->sc.scaled, batch, s);
    launch_lsd_grad(g, c->sc.scaled, c->sc.deg, c->sc.q, c->sc.sd, c->sc.maxq, batch, s);
  }
  if (ev_stage) HIP_CHECK(hipEventRecord(ev_stage[0], s));
  launch_lsd_sort(g, c->sc, batch, s);
  if (ev_stage) HIP_CHECK(hipEventRecord(ev_stage[1], s));
  launch_lsd_grow(g, c->sc, batch, s, c->serial_grow);
  if (ev_stage) HIP_CHECK(hipEventRecord(ev_stage[2], s));
  launch_lsd_validate(g, c->sc, batch, s);
  if (ev_mid) HIP_CHECK(hipEventRecord(ev_mid, s));
  if (out) {
    LineOut o = *out;
    o.kl_all = c->lo.kl_all;  // per-frame scratch of the full detection
    launch_keylines(c->g, c->sc, o, batch, s);
    if (ev_stage) HIP_CHECK(hipEventRecord(ev_stage[3], s));
    const char* e = getenv("ORBPL_BLUR_SOBEL");   // "0": separate blur + Sobel (A/B)
    if (c->g5.ksize == 5 && !(e && e[0] == '0')) {
      launch_blur_sobel(c->g5, d_imgs, stride, frame_pitch, c->sdx, c->sdy, batch, s);
    } else {
      launch_lsd_blur(c->g5, d_imgs, stride, frame_pitch, c->blur5, batch, s);
      launch_sobel(c->W, c->H, c->blur5, c->sdx, c->sdy, batch, s);
    }
    launch_lbd(c->W, c->H, c->sdx, c->sdy, c->lw, o, batch, s);
    if (ev_stage) HIP_CHECK(hipEventRecord(ev_stage[4], s));
  }
  HIP_CHECK(hipGetLastError());
  return ORBPL_OK;
}

// Device-side capacity flags of the last `batch` frames (caller synchronised).
int lsdx_check(lsdx_ctx* c, int batch) {
  std::vector<int> err(batch);
  HIP_CHECK(hipMemcpy(err.data(), c->sc.err, err.size() * 4, hipMemcpyDeviceToHost));
  for (int e : err)
    if (e) {
      arg_fail("LSD scratch capacity exceeded on device");
      return ORBPL_ERR_OVERFLOW;
    }
  return ORBPL_OK;
}
}  // namespace orbpl

extern "C" {

int lsdx_destroy(lsdx_ctx* c) {
  if (!c) return ORBPL_OK;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  for (void* p : c->allocs) (void)hipFree(p);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
  return ORBPL_OK;
}

int lsdx_create(int width, int height, int max_batch, int device, lsdx_ctx** out) {
  if (!out || max_batch <= 0) return arg_fail("bad argument");
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
    arg_fail("no HIP device visible");
    return ORBPL_ERR_NODEVICE;
  }
  if (device < 0 || device >= ndev) return arg_fail("device index out of range");
  lsdx_ctx* c = new lsdx_ctx();
  c->device = device;
  c->max_batch = max_batch;
  c->W = width;
  c->H = height;
  int rc = lsd_geometry(width, height, &c->g);
  if (rc) {
    delete c;
    return rc;
  }
  if (hipSetDevice(device) != hipSuccess ||
      hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
    delete c;
    return hip_fail(hipErrorUnknown, "hipStreamCreate", __LINE__);
  }
  const LsdGeom& g = c->g;
  const size_t B = max_batch, n = g.n, px = (size_t)g.sw * g.sh;
  LsdScratch& s = c->sc;
#define LA(ptr, bytes)                                     \
  do {                                                     \
    int _r = lx_alloc(c, (void**)&(ptr), (bytes));         \
    if (_r) { lsdx_destroy(c); return _r; }                \
  } while (0)
  LA(c->d_in, B * width * height);
  LA(s.blur, B * width * height);
  LA(s.scaled, B * px);
  LA(s.deg, B * (size_t)lsd_deg_words(g.sw, g.sh) * 4);
  LA(s.q, B * px * 4);
  LA(s.maxq, B * 4);
  LA(s.A, B * n * 4);
  LA(s.Lpos, B * n * 4);
  LA(s.Rpos, B * n * 4);
  LA(s.seg0, B * g.seg_cap * sizeof(int4));
  LA(s.seg1, B * g.seg_cap * sizeof(int4));
  LA(s.heap, B * g.seg_cap * sizeof(int4));
  LA(s.seg_i, B * 8 * g.seg_cap * 4);
  LA(s.chunk_i, B * 4 * g.chunk_cap * 4);
  LA(s.leaves, B * g.leaf_cap * sizeof(int2));
  LA(s.sort_masks, B * (size_t)g.mask_cap * 32 * 8);
  LA(s.reg, B * px * 3 * 4);
  LA(s.lines, B * kLsdMaxLines * 4 * 4);
  LA(s.nlines, B * 4);
  LA(s.err, B * 4);
  LA(s.prof, B * 8 * 8);
  LA(s.cand, B * kLsdMaxCand * 12 * 8);
  LA(s.ncand, B * 4);
  LA(s.cand_line, B * kLsdMaxCand * 4 * 4);
  LA(s.cand_ok, B * kLsdMaxCand * 4);
  LA(s.sd, B * (size_t)lsd_sd_frame_words(g.sw, g.sh) * 8);
  LA(s.lbuf, lsd_spec_lane_frames(B) * kSpecLanes * kLaneCap * sizeof(uint4));
  LA(s.sort_local, B * g.seg_cap * sizeof(int4));
  LA(s.sort_nlocal, B * 4);
  LA(s.sort_kt, B * 4);
  LA(s.sort_nge, B * 4);
  s.lgam_n = g.sw * g.sh + 1;   // a rectangle holds at most every pixel
  LA(s.lgam, (size_t)s.lgam_n * 8);
  LA(c->d_tabs, (size_t)(2 * g.sw + 2 * g.sh) * 4);
  LA(c->blur5, B * width * height);
  LA(c->sdx, B * width * height * 2);
  LA(c->sdy, B * width * height * 2);
  LA(c->lo.kl_all, B * kLsdMaxLines * sizeof(orbpl_keyline));
  LA(c->lo.kl, B * kLineKeep * sizeof(orbpl_keyline));
  LA(c->lo.desc, B * kLineKeep * 32);
  LA(c->lo.coef, B * kLineKeep * 3 * 8);
  LA(c->lo.n, B * 4);
#undef LA
  c->g5 = c->g;
  c->g5.ksize = 5;
  gauss_kernel_fixed(5, 1.0, c->g5.gk);
  // BinaryDescriptor::BinaryDescriptor: F_l (3 bands of width 7) and F_g (63
  // rows) Gaussian weights, integer centre / sigma, cast to float in use
  {
    double u = (7 * 3 - 1) / 2;
    double sigma = (7 * 2 + 1) / 2;
    double inv = -1 / (2 * sigma * sigma);
    for (int i = 0; i < 21; i++) c->lw.gL[i] = (float)lsdm::exp_((i - u) * (i - u) * inv);
    u = (9 * 7 - 1) / 2;
    sigma = u;
    inv = -1 / (2 * sigma * sigma);
    for (int i = 0; i < 63; i++) c->lw.gG[i] = (float)lsdm::exp_((i - u) * (i - u) * inv);
  }
  std::vector<int> tabs(2 * g.sw + 2 * g.sh);
  lin_tab(0.8, width, g.sw, tabs.data(), tabs.data() + g.sw, &c->g.rx0, &c->g.rx1);
  lin_tab(0.8, height, g.sh, tabs.data() + 2 * g.sw, tabs.data() + 2 * g.sw + g.sh, &c->g.ry0,
          &c->g.ry1);
  // the NFA's log_gamma table: filled and waited for here, so the first
  // k_lsd_validate on the context's non-blocking streams reads a finished table
  launch_lgamma_table(const_cast<double*>(s.lgam), s.lgam_n, nullptr);
  {
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipStreamSynchronize(nullptr);
    if (e != hipSuccess) {
      lsdx_destroy(c);
      return hip_fail(e, "k_lgamma_table", __LINE__);
    }
  }
  if (hipMemcpy(c->d_tabs, tabs.data(), tabs.size() * 4, hipMemcpyHostToDevice) != hipSuccess) {
    lsdx_destroy(c);
    return hip_fail(hipErrorUnknown, "hipMemcpy", __LINE__);
  }
  // k_lsd_prep's per-tile source spans (the resize taps of a tile's scaled
  // pixels + 1) must fit its LDS tile
  {
    auto span = [](const int* ofs, int d0, int d1, int mn, int mx, int last, int* lo, int* hi) {
      *lo = 1 << 30;
      *hi = -1;
      for (int d = d0; d < d1; d++) {
        const int a = d < mn ? 0 : (d >= mx ? last : ofs[d]);
        const int b = d < mn ? 0 : (d >= mx ? last : ofs[d] + 1);
        *lo = std::min(*lo, a);
        *hi = std::max(*hi, b);
      }
    };
    bool ok = c->g.ksize == 2 * kPrR + 1;
    for (int x0 = 0; ok && x0 < c->g.sw; x0 += kPrTW) {
      int lo, hi;
      span(tabs.data(), x0, std::min(x0 + kPrTW + 1, c->g.sw), c->g.rx0, c->g.rx1,
           tabs[c->g.sw - 1], &lo, &hi);
      ok = hi - lo + 1 <= kPrSC;
    }
    for (int y0 = 0; ok && y0 < c->g.sh; y0 += kPrTH) {
      int lo, hi;
      span(tabs.data() + 2 * c->g.sw, y0, std::min(y0 + kPrTH + 1, c->g.sh), c->g.ry0, c->g.ry1,
           height - 1, &lo, &hi);
      ok = hi - lo + 1 <= kPrSR;
    }
    const char* e = getenv("ORBPL_LSD_PREP");   // "0": the three-kernel path (A/B)
    c->fused_prep = ok && !(e && e[0] == '0');
  }
  *out = c;
  return ORBPL_OK;
}

int lsdx_detect_batch_device(lsdx_ctx* c, const uint8_t* d_imgs, int batch, int stride,
                             int64_t frame_pitch) {
  if (!c || !d_imgs || batch <= 0 || batch > c->max_batch) return arg_fail("bad argument");
  if (stride < c->W) return arg_fail("stride < width");
  HIP_CHECK(hipSetDevice(c->device));
  int rc = orbpl::lsdx_run(c, d_imgs, batch, stride, frame_pitch, nullptr, c->stream, nullptr);
  if (rc) return rc;
  c->last_batch = batch;
  return ORBPL_OK;
}

int lsdx_extract_batch_device(lsdx_ctx* c, const uint8_t* d_imgs, int batch, int stride,
                              int64_t frame_pitch) {
  if (!c || !d_imgs || batch <= 0 || batch > c->max_batch) return arg_fail("bad argument");
  if (stride < c->W) return arg_fail("stride < width");
  HIP_CHECK(hipSetDevice(c->device));
  int rc = orbpl::lsdx_run(c, d_imgs, batch, stride, frame_pitch, &c->lo, c->stream, nullptr);
  if (rc) return rc;
  c->last_batch = batch;
  return ORBPL_OK;
}

int lsdx_get_keylines(lsdx_ctx* c, int frame, orbpl_keyline* kl, uint8_t* desc, double* coef,
                      int cap, int* n_out) {
  if (!c || !n_out || frame < 0 || frame >= c->last_batch) return arg_fail("bad argument");
  int rc = lsdx_synchronize(c);
  if (rc) return rc;
  int n = 0;
  HIP_CHECK(hipMemcpy(&n, c->lo.n + frame, 4, hipMemcpyDeviceToHost));
  *n_out = n;
  if (n > cap) {
    arg_fail("keyline buffer too small");
    return ORBPL_ERR_CAPACITY;
  }
  const size_t o = (size_t)frame * kLineKeep;
  if (n > 0) {
    if (kl) HIP_CHECK(hipMemcpy(kl, c->lo.kl + o, n * sizeof(orbpl_keyline), hipMemcpyDeviceToHost));
    if (desc) HIP_CHECK(hipMemcpy(desc, c->lo.desc + o * 32, (size_t)n * 32, hipMemcpyDeviceToHost));
    if (coef) HIP_CHECK(hipMemcpy(coef, c->lo.coef + o * 3, (size_t)n * 24, hipMemcpyDeviceToHost));
  }
  return ORBPL_OK;
}

int lsdx_extract(lsdx_ctx* c, const uint8_t* img, int width, int height, int stride,
                 orbpl_keyline* kl, uint8_t* desc, double* coef, int cap, int* n_out) {
  if (!c || !img || !n_out) return arg_fail("NULL argument");
  if (width != c->W || height != c->H) return arg_fail("image size differs from the context");
  HIP_CHECK(hipSetDevice(c->device));
  HIP_CHECK(hipMemcpy2DAsync(c->d_in, width, img, stride, width, height, hipMemcpyHostToDevice,
                             c->stream));
  int rc = lsdx_extract_batch_device(c, c->d_in, 1, width, (int64_t)width * height);
  if (rc) return rc;
  return lsdx_get_keylines(c, 0, kl, desc, coef, cap, n_out);
}

int lsdx_device_outputs(lsdx_ctx* c, orbpl_keyline** d_kl, uint8_t** d_desc, double** d_coef,
                        int** d_n) {
  if (!c) return arg_fail("NULL context");
  if (d_kl) *d_kl = c->lo.kl;
  if (d_desc) *d_desc = c->lo.desc;
  if (d_coef) *d_coef = c->lo.coef;
  if (d_n) *d_n = c->lo.n;
  return ORBPL_OK;
}

int lsdx_set_serial_grow(lsdx_ctx* c, int on) {
  if (!c) return arg_fail("NULL context");
  int rc = lsdx_synchronize(c);
  if (rc) return rc;
  c->serial_grow = on != 0;
  return ORBPL_OK;
}

int lsdx_synchronize(lsdx_ctx* c) {
  if (!c) return arg_fail("NULL context");
  HIP_CHECK(hipSetDevice(c->device));
  HIP_CHECK(hipStreamSynchronize(c->stream));
  return c->last_batch > 0 ? orbpl::lsdx_check(c, c->last_batch) : ORBPL_OK;
}

int lsdx_get_lines(lsdx_ctx* c, int frame, float* lines, int cap, int* n_out) {
  if (!c || !n_out || frame < 0 || frame >= c->last_batch) return arg_fail("bad argument");
  int rc = lsdx_synchronize(c);
  if (rc) return rc;
  int n = 0;
  HIP_CHECK(hipMemcpy(&n, c->sc.nlines + frame, 4, hipMemcpyDeviceToHost));
  *n_out = n;
  if (n > cap) {
    arg_fail("line buffer too small");
    return ORBPL_ERR_CAPACITY;
  }
  if (n > 0 && lines)
    HIP_CHECK(hipMemcpy(lines, c->sc.lines + (size_t)frame * kLsdMaxLines * 4, (size_t)n * 16,
                        hipMemcpyDeviceToHost));
  return ORBPL_OK;
}

int lsdx_detect(lsdx_ctx* c, const uint8_t* img, int width, int height, int stride, float* lines,
                int cap, int* n_out) {
  if (!c || !img || !n_out) return arg_fail("NULL argument");
  if (width != c->W || height != c->H) return arg_fail("image size differs from the context");
  HIP_CHECK(hipSetDevice(c->device));
  HIP_CHECK(hipMemcpy2DAsync(c->d_in, width, img, stride, width, height, hipMemcpyHostToDevice,
                             c->stream));
  int rc = lsdx_detect_batch_device(c, c->d_in, 1, width, (long long)width * height);
  if (rc) return rc;
  return lsdx_get_lines(c, 0, lines, cap, n_out);
}

int lsdx_get_stages(lsdx_ctx* c, int frame, uint8_t* scaled, float* deg, uint32_t* order,
                    int* sw, int* sh, int* n_order) {
  if (!c || frame < 0 || frame >= c->last_batch) return arg_fail("bad argument");
  int rc = lsdx_synchronize(c);
  if (rc) return rc;
  const LsdGeom& g = c->g;
  const size_t px = (size_t)g.sw * g.sh;
  if (sw) *sw = g.sw;
  if (sh) *sh = g.sh;
  if (n_order) *n_order = g.n;
  if (scaled) HIP_CHECK(hipMemcpy(scaled, c->sc.scaled + frame * px, px, hipMemcpyDeviceToHost));
  if (deg) {
    // the plane is tiled on the device (lsd_deg_index); row-major here
    const long long dw = lsd_deg_words(g.sw, g.sh);
    std::vector<float> t((size_t)dw);
    HIP_CHECK(hipMemcpy(t.data(), c->sc.deg + frame * dw, (size_t)dw * 4, hipMemcpyDeviceToHost));
    const int dtw = lsd_deg_tw(g.sw);
    for (int y = 0; y < g.sh; y++)
      for (int x = 0; x < g.sw; x++) deg[(size_t)y * g.sw + x] = t[lsd_deg_index(x, y, dtw)];
  }
  if (order) {
    std::vector<uint32_t> a(g.n);
    HIP_CHECK(hipMemcpy(a.data(), c->sc.A + (size_t)frame * g.n, (size_t)g.n * 4,
                        hipMemcpyDeviceToHost));
    const int w1 = g.sw - 1;
    for (int i = 0; i < g.n; i++) {
      const int idx = (int)(a[i] & 0x3FFFFFu);
      order[i] = (uint32_t)(idx % w1) | ((uint32_t)(idx / w1) << 16);
    }
  }
  return ORBPL_OK;
}

// Debug: per-frame phase cycle counters of the seed loop (grow, fit+refine,
// rect_improve, total, region pixels, regions, candidate regions, lines).
int lsdx_debug_profile(lsdx_ctx* c, long long* out8) {
  if (!c || !out8 || c->last_batch <= 0) return arg_fail("bad argument");
  int rc = lsdx_synchronize(c);
  if (rc) return rc;
  std::vector<long long> p((size_t)c->last_batch * 8);
  HIP_CHECK(hipMemcpy(p.data(), c->sc.prof, p.size() * 8, hipMemcpyDeviceToHost));
  for (int k = 0; k < 8; k++) {
    long long s = 0;
    for (int f = 0; f < c->last_batch; f++) s += p[(size_t)f * 8 + k];
    out8[k] = s / c->last_batch;
  }
  return ORBPL_OK;
}

// Test hook: the device introsort replica on caller keys (values 0..1023);
// perm receives the sorted record indices.
int orbpl_test_introsort(const int* keys, int n, int* perm) {
  if (!keys || !perm || n <= 0 || n >= (1 << 22)) return arg_fail("bad argument");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
    arg_fail("no HIP device visible");
    return ORBPL_ERR_NODEVICE;
  }
  for (int i = 0; i < n; i++)
    if (keys[i] < 0 || keys[i] > 1023) return arg_fail("keys must be in [0, 1023]");
  LsdScratch sc{};
  const int seg_cap = n / 17 + 2, chunk_cap = n / kLsdSortChunk + seg_cap + 2, leaf_cap = n / 2 + 2;
  std::vector<void*> al;
  auto A = [&](void** p, size_t b) {
    hipError_t e = hipMalloc(p, b ? b : 1);
    if (e == hipSuccess) al.push_back(*p);
    return e;
  };
  int* d_keys = nullptr;
  hipError_t e = hipSuccess;
  e = e ? e : A((void**)&d_keys, (size_t)n * 4);
  e = e ? e : A((void**)&sc.A, (size_t)n * 4);
  e = e ? e : A((void**)&sc.Lpos, (size_t)n * 4);
  e = e ? e : A((void**)&sc.Rpos, (size_t)n * 4);
  e = e ? e : A((void**)&sc.seg0, (size_t)seg_cap * sizeof(int4));
  e = e ? e : A((void**)&sc.seg1, (size_t)seg_cap * sizeof(int4));
  e = e ? e : A((void**)&sc.heap, (size_t)seg_cap * sizeof(int4));
  e = e ? e : A((void**)&sc.seg_i, (size_t)8 * seg_cap * 4);
  e = e ? e : A((void**)&sc.chunk_i, (size_t)4 * chunk_cap * 4);
  e = e ? e : A((void**)&sc.leaves, (size_t)leaf_cap * sizeof(int2));
  e = e ? e : A((void**)&sc.sort_masks, (size_t)(2 * (n / 1024) + 8) * 32 * 8);
  e = e ? e : A((void**)&sc.err, 4);
  e = e ? e : A((void**)&sc.sort_local, (size_t)seg_cap * sizeof(int4));
  e = e ? e : A((void**)&sc.sort_nlocal, 4);
  e = e ? e : A((void**)&sc.sort_kt, 4);
  e = e ? e : A((void**)&sc.sort_nge, 4);
  int rc = ORBPL_OK, err = 0;
  std::vector<uint32_t> a(n);
  if (e == hipSuccess) e = hipMemcpy(d_keys, keys, (size_t)n * 4, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemset(sc.err, 0, 4);
  if (e == hipSuccess) {
    launch_lsd_sort_keys(n, d_keys, sc, nullptr);
    e = hipDeviceSynchronize();
  }
  if (e == hipSuccess) e = hipMemcpy(a.data(), sc.A, (size_t)n * 4, hipMemcpyDeviceToHost);
  if (e == hipSuccess) e = hipMemcpy(&err, sc.err, 4, hipMemcpyDeviceToHost);
  if (e != hipSuccess) rc = hip_fail(e, "introsort test", __LINE__);
  else if (err) rc = (arg_fail("sort scratch overflow"), ORBPL_ERR_OVERFLOW);
  for (void* p : al) (void)hipFree(p);
  if (rc == ORBPL_OK)
    for (int i = 0; i < n; i++) perm[i] = (int)(a[i] & 0x3FFFFFu);
  return rc;
}

}  // extern "C"
