// FETCH_SIZE calibration on gfx950 (MI355X_MICROARCH.md, HBM: "other access
// widths are uncalibrated: calibrate on a known byte count in your own access
// pattern"). Each kernel reads every byte of a 1 GiB buffer (4x the 256 MiB
// Infinity Cache, so the bytes come from HBM) exactly once, in the access
// shape of the LSD kernels: per-lane gathers of 4 / 8 / 16 bytes where the
// lanes of one wave instruction hit different 128-byte lines in a scattered
// order, plus the coalesced 16-B stream the guide calibrates. A last kernel
// reads ONE 16-B piece of each line (the isolated-gather case): its known
// request count gives the counter's bytes per isolated request.
//   rocprofv3 --pmc FETCH_SIZE -- ./fetch_calib  (then tools/calib/fetch_calib.py)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

constexpr size_t kBytes = size_t(1) << 30;
constexpr size_t kLines = kBytes / 128;

// line index of the g-th line in a scattered order (odd multiplier mod 2^k is
// a permutation of the lines)
__device__ __forceinline__ size_t scatter_line(size_t g) {
  return (g * 2654435761ull) & (kLines - 1);
}

// coalesced: lane i of a wave reads bytes [16 (base + i), +16)
__global__ void k_stream16(const uint4* __restrict__ p, uint32_t* out) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t acc = 0;
  for (; i < kBytes / 16; i += (size_t)gridDim.x * blockDim.x) {
    uint4 v = p[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

// W-byte gathers: a wave instruction covers 64*W bytes = (64*W/128) whole
// lines, lines taken in scattered order; every line read exactly once
template <int W>
__global__ void k_gather(const uint8_t* __restrict__ p, uint32_t* out) {
  constexpr int kLanesPerLine = 128 / W;
  constexpr int kLinesPerInst = 64 / kLanesPerLine;
  const int lane = threadIdx.x & 63;
  const size_t wave = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const size_t nwaves = ((size_t)gridDim.x * blockDim.x) >> 6;
  uint32_t acc = 0;
  for (size_t g = wave * kLinesPerInst; g < kLines; g += nwaves * kLinesPerInst) {
    const size_t line = scatter_line(g + lane / kLanesPerLine);
    const uint8_t* a = p + line * 128 + (lane % kLanesPerLine) * W;
    if (W == 16) {
      uint4 v = *reinterpret_cast<const uint4*>(a);
      acc ^= v.x ^ v.y ^ v.z ^ v.w;
    } else if (W == 8) {
      uint2 v = *reinterpret_cast<const uint2*>(a);
      acc ^= v.x ^ v.y;
    } else {
      acc ^= *reinterpret_cast<const uint32_t*>(a);
    }
  }
  if (acc == 0x12345678u) out[0] = acc;
}

// one 16-B piece of every line, lanes on 64 different lines
__global__ void k_sparse16(const uint8_t* __restrict__ p, uint32_t* out) {
  size_t g = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t acc = 0;
  for (; g < kLines; g += (size_t)gridDim.x * blockDim.x) {
    uint4 v = *reinterpret_cast<const uint4*>(p + scatter_line(g) * 128);
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

__global__ void k_fill(uint4* p) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i < kBytes / 16; i += (size_t)gridDim.x * blockDim.x)
    p[i] = make_uint4((uint32_t)i, (uint32_t)(i >> 3), 7u, 11u);
}

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e = (x);                                                    \
    if (e != hipSuccess) {                                                 \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));               \
      return 1;                                                            \
    }                                                                      \
  } while (0)

int main() {
  uint8_t* buf = nullptr;
  uint8_t* flush = nullptr;
  uint32_t* out = nullptr;
  CK(hipMalloc(&buf, kBytes));
  CK(hipMalloc(&flush, kBytes));
  CK(hipMalloc(&out, 64));
  const dim3 grid(4096), block(256);
  hipLaunchKernelGGL(k_fill, grid, block, 0, 0, reinterpret_cast<uint4*>(buf));
  // each measured kernel runs behind a 1 GiB write of another buffer, so the
  // Infinity Cache holds none of the measured buffer's lines
  auto evict = [&]() { hipLaunchKernelGGL(k_fill, grid, block, 0, 0, reinterpret_cast<uint4*>(flush)); };
  for (int rep = 0; rep < 3; rep++) {
    evict();
    hipLaunchKernelGGL(k_stream16, grid, block, 0, 0, reinterpret_cast<const uint4*>(buf), out);
    evict();
    hipLaunchKernelGGL(k_gather<16>, grid, block, 0, 0, buf, out);
    evict();
    hipLaunchKernelGGL(k_gather<8>, grid, block, 0, 0, buf, out);
    evict();
    hipLaunchKernelGGL(k_gather<4>, grid, block, 0, 0, buf, out);
    evict();
    hipLaunchKernelGGL(k_sparse16, grid, block, 0, 0, buf, out);
  }
  CK(hipDeviceSynchronize());
  printf("fetch_calib: %zu bytes per full kernel, %zu lines (k_sparse16 requests)\n", kBytes, kLines);
  CK(hipFree(buf));
  CK(hipFree(flush));
  CK(hipFree(out));
  return 0;
}
