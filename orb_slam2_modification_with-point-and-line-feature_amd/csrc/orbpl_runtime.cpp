// Host runtime and C-ABI (include/orbpl.h) of the ORB extraction path.
// One orbx_ctx = one device + one HIP stream + device buffers sized for
// max_batch frames of one image geometry.
#include <dirent.h>
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <unistd.h>
#include <mutex>
#include <map>
#include <set>
#include <cctype>
#include <string>
#include <utility>
#include <vector>

#include "../../include/orbpl.h"
#include "orb_kernels.h"
#include "orbpl_runtime.h"

namespace orbpl {

// Hardware queues: the HIP runtime maps a process's streams onto
// GPU_MAX_HW_QUEUES queues (4 by default, read once, when the runtime starts);
// a tracker drives up to eight streams, which then share queues and serialise
// (DESIGN.md §4 Tracker). At library load the constructor below records what
// the runtime will really use and changes the environment only where that is
// safe and wanted:
//   * the runtime already started (the process holds /dev/kfd open: torch or
//     another HIP library initialised first): nothing is changed, the queue
//     count is the variable's value then (4 when unset);
//   * ORBPL_HW_QUEUES=<n> (n > 0): the caller asks for n queues - set;
//   * GPU_MAX_HW_QUEUES unset: filled in with 16 (a process whose first HIP
//     user is this library: the reference's process with the drop-ins);
//   * GPU_MAX_HW_QUEUES set by the user (the GPU box's 4, say): left alone.
// The split switches (track_runtime.cpp) read the recorded count, never the
// environment. ORBPL_ASSUME_RUNTIME_STARTED=1 makes the constructor treat the
// runtime as started (the CPU test of the first case has no /dev/kfd).
int g_hw_queues = 4;            // queues the runtime runs (or will run) with
int g_runtime_started = 0;      // the runtime was up before this library loaded
int g_queues_set_by_lib = 0;    // the constructor wrote GPU_MAX_HW_QUEUES

static bool kfd_open() {
  const char* force = getenv("ORBPL_ASSUME_RUNTIME_STARTED");
  if (force) return force[0] == '1';
  // every open descriptor, whatever its number
  DIR* d = opendir("/proc/self/fd");
  if (!d) return false;
  const int self = dirfd(d);
  char path[300], target[256];
  bool found = false;
  while (const dirent* e = readdir(d)) {
    if (e->d_name[0] == '.' || atoi(e->d_name) == self) continue;
    snprintf(path, sizeof(path), "/proc/self/fd/%s", e->d_name);
    const ssize_t n = readlink(path, target, sizeof(target) - 1);
    if (n <= 0) continue;
    target[n] = 0;
    if (strcmp(target, "/dev/kfd") == 0) { found = true; break; }
  }
  closedir(d);
  return found;
}

__attribute__((constructor)) static void record_hw_queues() {
  const char* q = getenv("GPU_MAX_HW_QUEUES");
  const int before = q && atoi(q) > 0 ? atoi(q) : 4;
  g_hw_queues = before;
  g_runtime_started = kfd_open() ? 1 : 0;
  if (g_runtime_started) return;
  const char* want = getenv("ORBPL_HW_QUEUES");
  int n = 0;
  if (want) n = atoi(want);     // an explicit request (0: leave the setting alone)
  else if (!q) n = 16;          // unset: fill in
  if (n <= 0) return;
  if (n > 32) n = 32;
  char buf[16];
  snprintf(buf, sizeof(buf), "%d", n);
  setenv("GPU_MAX_HW_QUEUES", buf, 1);
  g_hw_queues = n;
  g_queues_set_by_lib = 1;
}

int hw_queues() { return g_hw_queues; }

static thread_local std::string g_last_error;

void set_error(const char* fmt, const char* a, int line) {
  char buf[512];
  snprintf(buf, sizeof(buf), fmt, a, line);
  g_last_error = buf;
}

int hip_fail(hipError_t e, const char* what, int line) {
  char buf[512];
  snprintf(buf, sizeof(buf), "%s failed (line %d): %s", what, line, hipGetErrorString(e));
  g_last_error = buf;
  return ORBPL_ERR_HIP;
}

int arg_fail(const char* msg) {
  g_last_error = msg;
  return ORBPL_ERR_ARG;
}

bool once_per_device(const void* key) {
  static std::mutex mu;
  static std::set<std::pair<const void*, int>> seen;
  int dev = 0;
  (void)hipGetDevice(&dev);
  std::lock_guard<std::mutex> lk(mu);
  return seen.insert({key, dev}).second;
}

void set_smem_attr(const void* fn, size_t bytes) {
  if (once_per_device(fn))
    (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
}

int device_cu_count() {
  static std::mutex mu;
  static std::map<int, int> cus;
  int dev = 0;
  (void)hipGetDevice(&dev);
  std::lock_guard<std::mutex> lk(mu);
  auto it = cus.find(dev);
  if (it != cus.end()) return it->second;
  int n = 0;
  if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
    n = 256;
  cus[dev] = n;
  return n;
}

}  // namespace orbpl

using namespace orbpl;

struct orbx_ctx {
  orbpl_orb_params params{};
  int device = 0;
  int max_batch = 0;
  OrbHostGeom hg;
  hipStream_t stream = nullptr;
  hipEvent_t ev[6] = {};
  // level pipeline (hardware queues >= 8, ORBPL_LEVEL_PIPE=0 turns it off):
  // the pyramid runs as one launch per group of levels on `stream` and the
  // FAST launch of each group on `fstream` once that group is written, so
  // FAST of the early levels (2/3 of its work) runs beside the pyramid's
  // chain of later levels instead of after it
  hipStream_t fstream = nullptr;
  hipEvent_t ev_group[kMaxLevels] = {};   // pyramid group g written (stream)
  hipEvent_t ev_fjoin = nullptr;          // every FAST launch done (fstream)
  hipEvent_t ev_kern[kKernelBrackets] = {};   // FAST / octree / orientation launch brackets
  int ngroups = 1;
  int group_end[kMaxLevels] = {};         // group g = levels [end[g-1], end[g])
  bool timed = false;
  OrbGeom* d_geom = nullptr;
  CellGeom* d_cells = nullptr;
  int* d_rs = nullptr;
  PyrBand* d_bands = nullptr;
  long long* d_pyr_prof = nullptr;   // ORBPL_PYR_PROFILE: k_pyramid phase stamps
  int pyr_bands = 0;           // 0 = choose per batch (ORBPL_PYR_BANDS overrides)
  int group_bands[kFastGroups] = {0, 0, 0, 0};   // per level group (0 = nb above)
  uint8_t* d_in = nullptr;
  uint8_t* d_pyr = nullptr;
  uint8_t* d_blur = nullptr;
  uint32_t* d_cell_cands = nullptr;
  int* d_cell_counts = nullptr;
  uint32_t* d_kcand = nullptr;
  int* d_knode = nullptr;
  uint32_t* d_kp_list = nullptr;
  int* d_kp_count = nullptr;
  orbpl_keypoint_dev* d_out_kps = nullptr;
  uint8_t* d_out_desc = nullptr;
  int* d_out_n = nullptr;
  int* d_err = nullptr;
  int last_batch = 0;
};

#define HIP_CHECK(expr)                                              \
  do {                                                               \
    hipError_t _e = (expr);                                          \
    if (_e != hipSuccess) return orbpl::hip_fail(_e, #expr, __LINE__); \
  } while (0)

extern "C" {

const char* orbpl_last_error(void) { return orbpl::g_last_error.c_str(); }

const char* orbpl_version(void) { return "orbpl gfx950 r4"; }

int orbpl_hw_queue_state(int* queues, int* runtime_started, int* set_by_library,
                         int* lsd_split_1024) {
  if (queues) *queues = orbpl::g_hw_queues;
  if (runtime_started) *runtime_started = orbpl::g_runtime_started;
  if (set_by_library) *set_by_library = orbpl::g_queues_set_by_lib;
  if (lsd_split_1024) *lsd_split_1024 = orbpl::lsd_split_decision(1024) ? 1 : 0;
  return ORBPL_OK;
}

int orbpl_device_count(int* n) {
  if (!n) return arg_fail("n is NULL");
  int c = 0;
  hipError_t e = hipGetDeviceCount(&c);
  if (e != hipSuccess) {
    *n = 0;
    hip_fail(e, "hipGetDeviceCount", __LINE__);
    return ORBPL_ERR_NODEVICE;
  }
  *n = c;
  return c > 0 ? ORBPL_OK : ORBPL_ERR_NODEVICE;
}

int orbpl_dev_malloc(int device, int64_t bytes, void** out) {
  if (!out || bytes < 0) return arg_fail("bad argument");
  HIP_CHECK(hipSetDevice(device));
  HIP_CHECK(hipMalloc(out, (size_t)(bytes > 0 ? bytes : 1)));
  return ORBPL_OK;
}

int orbpl_dev_free(int device, void* ptr) {
  HIP_CHECK(hipSetDevice(device));
  if (ptr) HIP_CHECK(hipFree(ptr));
  return ORBPL_OK;
}

int orbpl_host_alloc(int64_t bytes, void** out) {
  if (!out || bytes < 0) return arg_fail("bad argument");
  HIP_CHECK(hipHostMalloc(out, (size_t)(bytes > 0 ? bytes : 1), hipHostMallocDefault));
  return ORBPL_OK;
}

int orbpl_host_free(void* ptr) {
  if (ptr) HIP_CHECK(hipHostFree(ptr));
  return ORBPL_OK;
}

int orbpl_memcpy_htod(int device, void* dst, const void* src, int64_t bytes) {
  HIP_CHECK(hipSetDevice(device));
  if (bytes > 0) HIP_CHECK(hipMemcpy(dst, src, (size_t)bytes, hipMemcpyHostToDevice));
  return ORBPL_OK;
}

int orbpl_memcpy_dtoh(int device, void* dst, const void* src, int64_t bytes) {
  HIP_CHECK(hipSetDevice(device));
  if (bytes > 0) HIP_CHECK(hipMemcpy(dst, src, (size_t)bytes, hipMemcpyDeviceToHost));
  return ORBPL_OK;
}

int orbpl_memset_d(int device, void* dst, int value, int64_t bytes) {
  HIP_CHECK(hipSetDevice(device));
  if (bytes > 0) HIP_CHECK(hipMemset(dst, value, (size_t)bytes));
  return ORBPL_OK;
}

int orbpl_device_synchronize(int device) {
  HIP_CHECK(hipSetDevice(device));
  HIP_CHECK(hipDeviceSynchronize());
  return ORBPL_OK;
}

int orbpl_descriptor_distance(const uint8_t* a, const uint8_t* b) {
  // ORBmatcher::DescriptorDistance (ORBmatcher.cc:2083-2103): popcount of XOR
  int d = 0;
  for (int i = 0; i < 4; i++) {
    uint64_t x, y;
    memcpy(&x, a + 8 * i, 8);
    memcpy(&y, b + 8 * i, 8);
    d += __builtin_popcountll(x ^ y);
  }
  return d;
}

static void free_ctx(orbx_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  void* ptrs[] = {c->d_geom, c->d_cells, c->d_rs, c->d_bands, c->d_pyr_prof, c->d_in, c->d_pyr, c->d_blur, c->d_cell_cands,
                  c->d_cell_counts, c->d_kcand, c->d_knode, c->d_kp_list, c->d_kp_count,
                  c->d_out_kps, c->d_out_desc, c->d_out_n, c->d_err};
  for (void* p : ptrs)
    if (p) (void)hipFree(p);
  for (auto& e : c->ev)
    if (e) (void)hipEventDestroy(e);
  for (auto& e : c->ev_group)
    if (e) (void)hipEventDestroy(e);
  for (auto& e : c->ev_kern)
    if (e) (void)hipEventDestroy(e);
  if (c->ev_fjoin) (void)hipEventDestroy(c->ev_fjoin);
  if (c->fstream) {
    (void)hipStreamSynchronize(c->fstream);
    (void)hipStreamDestroy(c->fstream);
  }
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

int orbx_create(const orbpl_orb_params* p, int width, int height, int max_batch, int device,
                orbx_ctx** out) {
  if (!p || !out) return arg_fail("NULL argument");
  *out = nullptr;
  if (width <= 0 || height <= 0 || max_batch <= 0) return arg_fail("bad size/batch");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
    orbpl::g_last_error = "no HIP device visible";
    return ORBPL_ERR_NODEVICE;
  }
  if (device < 0 || device >= ndev) return arg_fail("device index out of range");
  orbx_ctx* c = new orbx_ctx();
  c->params = *p;
  c->device = device;
  c->max_batch = max_batch;
  const char* err = nullptr;
  int rc = build_orb_geometry(p->nfeatures, p->scale_factor, p->nlevels, width, height, &c->hg, &err);
  if (rc != ORBPL_OK) {
    delete c;
    return arg_fail(err ? err : "geometry");
  }
  const OrbGeom& g = c->hg.g;
  auto fail = [&](hipError_t e, const char* what) {
    int r = hip_fail(e, what, __LINE__);
    free_ctx(c);
    return r;
  };
#define CK(expr)                            \
  do {                                      \
    hipError_t _e = (expr);                 \
    if (_e != hipSuccess) return fail(_e, #expr); \
  } while (0)
  CK(hipSetDevice(device));
  // ORBPL_EXTRACT_CU_RESERVE=k (A/B): the extraction stream's kernels leave
  // the last k CUs of every 32-CU group (an XCD) to the other streams, so a
  // tracking workgroup that needs a whole SIMD's registers is placed at once
  // instead of after the extraction kernel beside it drains. Measured 18-20 %
  // slower on the headline for k = 1, 2, 4 (tools/gpu_r04_l.sh): off
  const char* resv = getenv("ORBPL_EXTRACT_CU_RESERVE");
  const int reserve = resv ? atoi(resv) : 0;
  int ncu = 0;
  if (reserve > 0 && reserve < 32 &&
      hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess &&
      ncu >= 32) {
    std::vector<uint32_t> mask((ncu + 31) / 32, 0u);
    for (int cu = 0; cu < ncu; cu++)
      if ((cu & 31) < 32 - reserve) mask[cu >> 5] |= 1u << (cu & 31);
    CK(hipExtStreamCreateWithCUMask(&c->stream, (uint32_t)mask.size(), mask.data()));
  } else {
    CK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
  }
  for (auto& e : c->ev) CK(hipEventCreate(&e));
  for (auto& e : c->ev_kern) CK(hipEventCreate(&e));
  {
    // level groups: [0,1) [1,2) [2,3) [3,n) by default (FAST work per level
    // ~ 1 / 1.44^l of level 0's: the first three groups hold 69 % of it);
    // ORBPL_LEVEL_PIPE=0: one pyramid launch and one FAST launch (no fstream)
    const char* lp = getenv("ORBPL_LEVEL_PIPE");
    const bool pipe = lp ? lp[0] != '0' : orbpl::hw_queues() >= 8;
    const int nl = c->hg.g.nlevels;
    c->ngroups = 0;
    if (pipe) {
      // ORBPL_LEVEL_GROUPS="1/2/3": the group ends (ascending, < nlevels;
      // any non-digit separates them)
      const char* ge = getenv("ORBPL_LEVEL_GROUPS");
      const std::string spec = ge ? ge : "1/2/3";
      for (size_t pos = 0; pos < spec.size() && c->ngroups < kFastGroups - 1;) {
        if (!isdigit((unsigned char)spec[pos])) {
          pos++;
          continue;
        }
        const int e = atoi(spec.c_str() + pos);
        while (pos < spec.size() && isdigit((unsigned char)spec[pos])) pos++;
        if (e > (c->ngroups ? c->group_end[c->ngroups - 1] : 0) && e < nl) c->group_end[c->ngroups++] = e;
      }
    }
    c->group_end[c->ngroups++] = nl;
    if (c->ngroups > 1) {
      CK(hipStreamCreateWithFlags(&c->fstream, hipStreamNonBlocking));
      for (int i = 0; i < c->ngroups; i++)
        CK(hipEventCreateWithFlags(&c->ev_group[i], hipEventDisableTiming));
      CK(hipEventCreateWithFlags(&c->ev_fjoin, hipEventDisableTiming));
    }
  }
  const size_t B = (size_t)max_batch;
  CK(hipMalloc(&c->d_geom, sizeof(OrbGeom)));
  CK(hipMalloc(&c->d_cells, sizeof(CellGeom) * std::max<size_t>(1, c->hg.cells.size())));
  CK(hipMalloc(&c->d_rs, sizeof(int) * c->hg.rs.size()));
  CK(hipMalloc(&c->d_bands, sizeof(PyrBand) * c->hg.bands.size()));
  CK(hipMalloc(&c->d_in, B * (size_t)width * height));
  CK(hipMalloc(&c->d_pyr, B * (size_t)g.pyr_bytes));
  CK(hipMalloc(&c->d_blur, B * (size_t)g.blur_bytes));
  CK(hipMalloc(&c->d_cell_cands, B * (size_t)std::max(1, g.ncells_total) * g.cell_slots * 4));
  CK(hipMalloc(&c->d_cell_counts, B * (size_t)std::max(1, g.ncells_total) * 4));
  CK(hipMalloc(&c->d_kcand, B * (size_t)std::max(1, g.cand_cap_total) * 4));
  CK(hipMalloc(&c->d_knode, B * (size_t)std::max(1, g.cand_cap_total) * 4));
  CK(hipMalloc(&c->d_kp_list, B * (size_t)g.kp_cap_total * 4));
  CK(hipMalloc(&c->d_kp_count, B * (size_t)g.nlevels * 4));
  CK(hipMalloc(&c->d_out_kps, B * (size_t)g.kp_cap_total * sizeof(orbpl_keypoint_dev)));
  CK(hipMalloc(&c->d_out_desc, B * (size_t)g.kp_cap_total * 32));
  CK(hipMalloc(&c->d_out_n, B * 4));
  CK(hipMalloc(&c->d_err, 4));
  CK(hipMemsetAsync(c->d_err, 0, 4, c->stream));
  CK(hipMemsetAsync(c->d_pyr, 0, B * (size_t)g.pyr_bytes, c->stream));
  CK(hipMemsetAsync(c->d_blur, 0, B * (size_t)g.blur_bytes, c->stream));
  CK(hipMemcpyAsync(c->d_geom, &g, sizeof(OrbGeom), hipMemcpyHostToDevice, c->stream));
  if (!c->hg.cells.empty())
    CK(hipMemcpyAsync(c->d_cells, c->hg.cells.data(), sizeof(CellGeom) * c->hg.cells.size(),
                      hipMemcpyHostToDevice, c->stream));
  CK(hipMemcpyAsync(c->d_rs, c->hg.rs.data(), sizeof(int) * c->hg.rs.size(), hipMemcpyHostToDevice,
                    c->stream));
  CK(hipMemcpyAsync(c->d_bands, c->hg.bands.data(), sizeof(PyrBand) * c->hg.bands.size(),
                    hipMemcpyHostToDevice, c->stream));
  if (const char* e = getenv("ORBPL_PYR_BANDS")) {
    const int b = atoi(e);
    if (b == 1 || b == 2 || b == 4 || b == 8) c->pyr_bands = b;
  }
  // ORBPL_PYR_GROUP_BANDS="1/1/1/4": row bands of each level group's
  // pyramid launch (A/B; a group's launch only reads complete lower levels,
  // so its bands need not match the other groups')
  if (const char* e = getenv("ORBPL_PYR_GROUP_BANDS")) {
    int gi = 0;
    for (const char* q = e; *q && gi < kFastGroups;) {
      if (!isdigit((unsigned char)*q)) {
        q++;
        continue;
      }
      const int b = atoi(q);
      while (isdigit((unsigned char)*q)) q++;
      c->group_bands[gi++] = (b == 1 || b == 2 || b == 4 || b == 8) ? b : 0;
    }
  }
  if (getenv("ORBPL_PYR_PROFILE")) {
    CK(hipMalloc(&c->d_pyr_prof, 8 * (1 + 4 * kMaxLevels)));
    CK(hipMemsetAsync(c->d_pyr_prof, 0, 8 * (1 + 4 * kMaxLevels), c->stream));
  }
  CK(upload_pattern(c->stream));
  CK(hipStreamSynchronize(c->stream));
#undef CK
  *out = c;
  return ORBPL_OK;
}

// Debug (ORBPL_PYR_PROFILE set at create): k_pyramid phase times of block
// (band 0, frame 0) in the last launch, ns, 4 per level: content, side
// borders, mirror rows, blur.
int orbx_debug_pyr_profile(orbx_ctx* c, long long* out, int cap, int* n) {
  if (!c || !out || !n) return arg_fail("bad argument");
  if (!c->d_pyr_prof) return arg_fail("ORBPL_PYR_PROFILE was not set when the context was created");
  HIP_CHECK(hipStreamSynchronize(c->stream));
  const int L = c->hg.g.nlevels;
  std::vector<long long> p(1 + 4 * kMaxLevels);
  HIP_CHECK(hipMemcpy(p.data(), c->d_pyr_prof, p.size() * 8, hipMemcpyDeviceToHost));
  *n = std::min(cap, 4 * L);
  for (int i = 0; i < *n; i++) out[i] = (p[i + 1] - p[i]) * 10;   // wall clock: 100 MHz
  return ORBPL_OK;
}

// Debug (ORBPL_OCT_PROFILE set): k_octree per-level block of frame 0 in the
// last launch, 8 values per level: setup ns, pass loop ns, -, retain ns,
// passes, candidates, final list size, -.
int orbx_debug_octree_profile(orbx_ctx* c, long long* out128) {
  if (!c || !out128) return arg_fail("bad argument");
  HIP_CHECK(hipStreamSynchronize(c->stream));
  if (read_octree_profile(out128)) return arg_fail("octree profile unavailable");
  for (int l = 0; l < 16; l++)
    for (int k : {0, 1, 2, 3}) out128[8 * l + k] *= 10;
  // level slots 8..15 are unused by 8-level pyramids: the orient/desc phases
  // of frame 0's first keypoint go to out128[120..125] (ns)
  long long od[6];
  if (read_od_profile(od) == 0)
    for (int k = 0; k < 6; k++) out128[120 + k] = od[k] * 10;
  return ORBPL_OK;
}

int orbx_destroy(orbx_ctx* c) {
  free_ctx(c);
  return ORBPL_OK;
}

int orbx_get_scale_info(const orbx_ctx* c, int* nlevels, float* scale, float* inv_scale,
                        float* sigma2, float* inv_sigma2) {
  if (!c) return arg_fail("NULL ctx");
  const int n = c->hg.g.nlevels;
  if (nlevels) *nlevels = n;
  for (int i = 0; i < n; i++) {
    if (scale) scale[i] = c->hg.scale[i];
    if (inv_scale) inv_scale[i] = c->hg.inv_scale[i];
    if (sigma2) sigma2[i] = c->hg.sigma2[i];
    if (inv_sigma2) inv_sigma2[i] = c->hg.inv_sigma2[i];
  }
  return ORBPL_OK;
}

int orbx_get_level_info(const orbx_ctx* c, int* w, int* h, int* nf) {
  if (!c) return arg_fail("NULL ctx");
  for (int i = 0; i < c->hg.g.nlevels; i++) {
    if (w) w[i] = c->hg.g.lv[i].w;
    if (h) h[i] = c->hg.g.lv[i].h;
    if (nf) nf[i] = c->hg.g.lv[i].nfeat;
  }
  return ORBPL_OK;
}

int orbx_max_keypoints(const orbx_ctx* c) { return c ? c->hg.g.kp_cap_total : 0; }

int orbx_describe(const orbpl_orb_params* p, int width, int height, int* lw, int* lh, int* nf,
                  float* scale, int* max_kps) {
  if (!p) return arg_fail("NULL params");
  OrbHostGeom hg;
  const char* err = nullptr;
  int rc = build_orb_geometry(p->nfeatures, p->scale_factor, p->nlevels, width, height, &hg, &err);
  if (rc != ORBPL_OK) return arg_fail(err ? err : "geometry");
  for (int i = 0; i < hg.g.nlevels; i++) {
    if (lw) lw[i] = hg.g.lv[i].w;
    if (lh) lh[i] = hg.g.lv[i].h;
    if (nf) nf[i] = hg.g.lv[i].nfeat;
    if (scale) scale[i] = hg.scale[i];
  }
  if (max_kps) *max_kps = hg.g.kp_cap_total;
  return ORBPL_OK;
}

}  // extern "C"

namespace orbpl {
hipStream_t orbx_stream(orbx_ctx* c) { return c->stream; }

// Whole extraction pipeline on the ctx stream; images already in device memory.
constexpr int kLevelPipeMinBatch = 64;

int orbx_run(orbx_ctx* c, const uint8_t* d_imgs, int batch, int stride, long long frame_pitch,
             orbpl_keypoint_dev* d_kps, uint8_t* d_desc, int kp_pitch, int* d_n,
             hipEvent_t* ext_events, hipEvent_t* ext_kernels) {
  const OrbGeom& g = c->hg.g;
  hipStream_t s = c->stream;
  c->timed = ext_events == nullptr;
  hipEvent_t* ev = ext_events ? ext_events : c->ev;
  hipEvent_t* evk = ext_kernels ? ext_kernels : (ext_events ? nullptr : c->ev_kern);
  HIP_CHECK(hipEventRecord(ev[0], s));
  // row bands per frame: enough blocks for ~4 per CU (256 CUs), at most 8
  int nb = c->pyr_bands;
  if (!nb) {
    nb = 1;
    while (nb < kPyrMaxBands && nb * batch < 1024) nb *= 2;
  }
  // kernel brackets: FAST / octree / orientation+descriptor launch of group gi
  // at evk[2 (K G + gi)] .. + 1 (K = 0, 1, 2), unused pairs back to back
  auto bracket = [&](int kind, int gi, int end, hipStream_t st) -> hipError_t {
    return evk ? hipEventRecord(evk[2 * (kind * kFastGroups + gi) + end], st) : hipSuccess;
  };
  // small batches run the levels in one launch each: at batch 1 the 16
  // launches and cross-stream events of the pipeline cost more latency than
  // the overlap returns (points batch 1: 1.56 vs 1.51 ms)
  const bool pipe = c->ngroups > 1 && batch >= kLevelPipeMinBatch;
  const int ngroups = pipe ? c->ngroups : 1;
  hipStream_t fs = pipe ? c->fstream : s;
  // Level groups (one group without the pipeline): group gi's pyramid launch
  // on `s`, then its FAST, octree and orientation + descriptor launches on the
  // FAST stream - FAST reads only the group's levels, the octree of a level
  // only its FAST cells, and the orientation of a level's keypoints the
  // counts of that and the lower levels (in stream order). The next group's
  // pyramid launch writes only its own levels.
  int l0 = 0;
  for (int gi = 0; gi < ngroups; gi++) {
    const int l1 = pipe ? c->group_end[gi] : g.nlevels;
    const int nbg = pipe && c->group_bands[gi] ? c->group_bands[gi] : nb;
    launch_pyramid(g, c->d_geom, d_imgs, stride, frame_pitch, c->d_pyr, c->d_blur, c->d_rs,
                   c->d_bands + pyr_band_base(nbg), nbg, batch, c->d_pyr_prof, l0, l1, s);
    if (pipe) {
      HIP_CHECK(hipEventRecord(c->ev_group[gi], s));
      HIP_CHECK(hipStreamWaitEvent(fs, c->ev_group[gi], 0));
    } else {
      HIP_CHECK(hipEventRecord(ev[1], s));
      // the blur is fused into k_pyramid: the blur stage interval stays empty
      HIP_CHECK(hipEventRecord(ev[2], s));
    }
    HIP_CHECK(bracket(0, gi, 0, fs));
    launch_fast(g, c->d_geom, c->d_cells, c->d_pyr, c->d_cell_cands, c->d_cell_counts,
                c->params.ini_th_fast, c->params.min_th_fast, batch, l0, l1, fs);
    HIP_CHECK(bracket(0, gi, 1, fs));
    if (!pipe) HIP_CHECK(hipEventRecord(ev[3], s));
    HIP_CHECK(bracket(1, gi, 0, fs));
    launch_octree(g, c->d_geom, c->d_cell_cands, c->d_cell_counts, c->d_kcand, c->d_knode,
                  c->d_kp_list, c->d_kp_count, c->d_err, batch, l0, l1, fs);
    HIP_CHECK(bracket(1, gi, 1, fs));
    if (!pipe) HIP_CHECK(hipEventRecord(ev[4], s));
    l0 = l1;
  }
  // orientation + descriptors of every level in one launch after the last
  // group's octree (per-group launches measured 1.2 % slower: 148.3-149.0k
  // vs 150.2-150.7k frames/s, `profiles/r05/pipeline_overlap_ab.txt` item 16)
  HIP_CHECK(bracket(2, 0, 0, fs));
  launch_orient_desc(g, c->d_geom, c->d_pyr, c->d_blur, c->d_kp_list, c->d_kp_count, d_kps, d_desc,
                     kp_pitch, d_n, batch, 0, g.nlevels, fs);
  HIP_CHECK(bracket(2, 0, 1, fs));
  for (int kind = 0; kind < 3; kind++)
    for (int gi = kind == 2 ? 1 : ngroups; gi < kFastGroups; gi++) {
      HIP_CHECK(bracket(kind, gi, 0, fs));
      HIP_CHECK(bracket(kind, gi, 1, fs));
    }
  if (pipe) {
    HIP_CHECK(hipEventRecord(ev[1], s));
    HIP_CHECK(hipEventRecord(ev[2], s));
    HIP_CHECK(hipEventRecord(c->ev_fjoin, fs));
    HIP_CHECK(hipStreamWaitEvent(s, c->ev_fjoin, 0));
    HIP_CHECK(hipEventRecord(ev[3], s));
    HIP_CHECK(hipEventRecord(ev[4], s));
  }
  HIP_CHECK(hipEventRecord(ev[5], s));
  HIP_CHECK(hipGetLastError());
  c->last_batch = batch;
  return ORBPL_OK;
}
}  // namespace orbpl

extern "C" {

int orbx_synchronize(orbx_ctx* c) {
  if (!c) return arg_fail("NULL ctx");
  HIP_CHECK(hipSetDevice(c->device));
  HIP_CHECK(hipStreamSynchronize(c->stream));
  int flag = 0;
  HIP_CHECK(hipMemcpy(&flag, c->d_err, 4, hipMemcpyDeviceToHost));
  if (flag) {
    HIP_CHECK(hipMemset(c->d_err, 0, 4));
    char buf[128];
    snprintf(buf, sizeof(buf), "kernel capacity overflow (flags 0x%x)", flag);
    orbpl::g_last_error = buf;
    return ORBPL_ERR_OVERFLOW;
  }
  return ORBPL_OK;
}

int orbx_extract(orbx_ctx* c, const uint8_t* img, int width, int height, int stride,
                 orbpl_keypoint* kps, uint8_t* desc, int cap, int* n) {
  if (!c || !n) return arg_fail("NULL argument");
  *n = 0;
  if (!img || width <= 0 || height <= 0) return ORBPL_OK;  // _image.empty() -> return
  if (width != c->hg.g.W || height != c->hg.g.H)
    return arg_fail("image size differs from the size given to orbx_create");
  if (stride < width) return arg_fail("stride < width");
  HIP_CHECK(hipSetDevice(c->device));
  const OrbGeom& g = c->hg.g;
  HIP_CHECK(hipMemcpy2DAsync(c->d_in, width, img, stride, width, height, hipMemcpyHostToDevice,
                             c->stream));
  int rc = orbx_run(c, c->d_in, 1, width, (long long)width * height, c->d_out_kps, c->d_out_desc,
                    g.kp_cap_total, c->d_out_n);
  if (rc) return rc;
  int cnt = 0;
  HIP_CHECK(hipMemcpyAsync(&cnt, c->d_out_n, 4, hipMemcpyDeviceToHost, c->stream));
  rc = orbx_synchronize(c);
  if (rc) return rc;
  if (cnt > cap) {
    orbpl::g_last_error = "keypoint buffer too small";
    *n = cnt;
    return ORBPL_ERR_CAPACITY;
  }
  if (cnt > 0) {
    if (kps)
      HIP_CHECK(hipMemcpyAsync(kps, c->d_out_kps, (size_t)cnt * sizeof(orbpl_keypoint),
                               hipMemcpyDeviceToHost, c->stream));
    if (desc)
      HIP_CHECK(hipMemcpyAsync(desc, c->d_out_desc, (size_t)cnt * 32, hipMemcpyDeviceToHost,
                               c->stream));
    HIP_CHECK(hipStreamSynchronize(c->stream));
  }
  *n = cnt;
  return ORBPL_OK;
}

int orbx_extract_batch_device(orbx_ctx* c, const uint8_t* d_imgs, int batch, int stride,
                              int64_t frame_pitch, orbpl_keypoint* d_kps, uint8_t* d_desc,
                              int kp_pitch, int32_t* d_n) {
  if (!c || !d_imgs || !d_kps || !d_desc || !d_n) return arg_fail("NULL argument");
  if (batch <= 0 || batch > c->max_batch) return arg_fail("batch out of range");
  if (stride < c->hg.g.W) return arg_fail("stride < width");
  if (kp_pitch < 1) return arg_fail("kp_pitch < 1");
  HIP_CHECK(hipSetDevice(c->device));
  return orbx_run(c, d_imgs, batch, stride, (long long)frame_pitch,
                  reinterpret_cast<orbpl_keypoint_dev*>(d_kps), d_desc, kp_pitch, d_n);
}

}  // extern "C"

namespace orbpl {
// Device view of a context's padded pyramid of batch frame `frame` (internal).
int orbx_device_pyramid(orbx_ctx* c, int frame, const uint8_t** base, const OrbGeom** geom,
                        hipStream_t* stream) {
  if (!c || frame < 0 || frame >= c->max_batch) return arg_fail("bad argument");
  *base = c->d_pyr + (size_t)frame * c->hg.g.pyr_bytes;
  *geom = &c->hg.g;
  *stream = c->stream;
  return ORBPL_OK;
}
}  // namespace orbpl

extern "C" {
int orbx_get_pyramid(orbx_ctx* c, int frame, int level, int padded, int blurred, uint8_t* out,
                     int out_cap, int* w, int* h) {
  if (!c) return arg_fail("NULL ctx");
  const OrbGeom& g = c->hg.g;
  if (level < 0 || level >= g.nlevels || frame < 0 || frame >= c->max_batch)
    return arg_fail("level/frame out of range");
  const LevelGeom& L = g.lv[level];
  if (blurred) padded = 0;  // the blurred working image has no border (content only)
  const int ow = padded ? L.pw : L.w, oh = padded ? L.ph : L.h;
  if (w) *w = ow;
  if (h) *h = oh;
  if (!out) return ORBPL_OK;
  if (out_cap < ow * oh) return ORBPL_ERR_CAPACITY;
  HIP_CHECK(hipSetDevice(c->device));
  HIP_CHECK(hipStreamSynchronize(c->stream));
  const uint8_t* base;
  int pitch;
  if (blurred) {
    base = c->d_blur + (size_t)frame * g.blur_bytes + L.boff;
    pitch = L.bpitch;
  } else {
    base = c->d_pyr + (size_t)frame * g.pyr_bytes +
           (padded ? padded_off(L, 0, 0) : content_off(L, 0, 0));
    pitch = L.pitch;
  }
  HIP_CHECK(hipMemcpy2D(out, ow, base, pitch, ow, oh, hipMemcpyDeviceToHost));
  return ORBPL_OK;
}

int orbx_get_candidates(orbx_ctx* c, float* xyr, int cap, int* level_counts, int* total) {
  if (!c || !total) return arg_fail("NULL argument");
  const OrbGeom& g = c->hg.g;
  HIP_CHECK(hipSetDevice(c->device));
  HIP_CHECK(hipStreamSynchronize(c->stream));
  std::vector<int> counts(std::max(1, g.ncells_total));
  std::vector<uint32_t> cands((size_t)std::max(1, g.ncells_total) * g.cell_slots);
  HIP_CHECK(hipMemcpy(counts.data(), c->d_cell_counts, 4 * (size_t)g.ncells_total, hipMemcpyDeviceToHost));
  HIP_CHECK(hipMemcpy(cands.data(), c->d_cell_cands, 4 * cands.size(), hipMemcpyDeviceToHost));
  int n = 0;
  for (int l = 0; l < g.nlevels; l++) {
    const LevelGeom& L = g.lv[l];
    int lc = 0;
    for (int ci = 0; ci < L.ncells; ci++) {
      const int cell = L.cell_base + ci;
      for (int k = 0; k < counts[cell]; k++) {
        uint32_t v = cands[(size_t)cell * g.cell_slots + k];
        if (n < cap && xyr) {
          xyr[3 * n] = (float)cand_x(v);
          xyr[3 * n + 1] = (float)cand_y(v);
          xyr[3 * n + 2] = (float)cand_s(v);
        }
        n++;
        lc++;
      }
    }
    if (level_counts) level_counts[l] = lc;
  }
  *total = n;
  return n > cap ? ORBPL_ERR_CAPACITY : ORBPL_OK;
}

int orbx_last_stage_ms(const orbx_ctx* c, float* ms5) {
  if (!c || !ms5) return arg_fail("NULL argument");
  if (!c->timed) return arg_fail("no extraction recorded yet");
  HIP_CHECK(hipSetDevice(c->device));
  HIP_CHECK(hipEventSynchronize(c->ev[5]));
  for (int i = 0; i < 5; i++) HIP_CHECK(hipEventElapsedTime(&ms5[i], c->ev[i], c->ev[i + 1]));
  // FAST, octree, orientation + descriptors: the kernel time of their level
  // group launches (beside the pyramid's later levels when the level
  // pipeline is on), without the waits between them
  for (int kind = 0; kind < 3; kind++) {
    ms5[2 + kind] = 0.f;
    for (int k = 0; k < kFastGroups; k++) {
      float m = 0.f;
      HIP_CHECK(hipEventElapsedTime(&m, c->ev_kern[2 * (kind * kFastGroups + k)],
                                    c->ev_kern[2 * (kind * kFastGroups + k) + 1]));
      ms5[2 + kind] += m;
    }
  }
  return ORBPL_OK;
}

}  // extern "C"
