// Prints the device's wall-clock and shader clock rates as reported, and the
// rates measured: a one-wave kernel spins for a fixed number of wall_clock64()
// (then clock64()) ticks, timed with HIP events. The unit of the in-kernel
// stamps of the profiling builds (-DORBPL_LOCAL_PROF, ORBPL_POSE_PROFILE).
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void spin_wall(long long ticks, long long* out) {
  const long long t0 = wall_clock64();
  long long t = t0;
  while (t - t0 < ticks) t = wall_clock64();
  if (threadIdx.x == 0) out[0] = t - t0;
}

__global__ void spin_clock(long long ticks, long long* out) {
  const long long t0 = clock64();
  long long t = t0;
  while (t - t0 < ticks) t = clock64();
  if (threadIdx.x == 0) out[0] = t - t0;
}

int main() {
  int wall = 0, clk = 0;
  if (hipDeviceGetAttribute(&wall, hipDeviceAttributeWallClockRate, 0) != hipSuccess) return 1;
  if (hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0) != hipSuccess) return 1;
  std::printf("reported: wall clock %d kHz, shader clock %d kHz\n", wall, clk);
  long long* d = nullptr;
  if (hipMalloc(&d, sizeof(long long)) != hipSuccess) return 1;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int which = 0; which < 2; which++) {
    const long long ticks = which == 0 ? 10000000LL : 200000000LL;
    for (int rep = 0; rep < 2; rep++) {
      hipEventRecord(e0, 0);
      if (which == 0) hipLaunchKernelGGL(spin_wall, dim3(1), dim3(64), 0, 0, ticks, d);
      else hipLaunchKernelGGL(spin_clock, dim3(1), dim3(64), 0, 0, ticks, d);
      hipEventRecord(e1, 0);
      if (hipEventSynchronize(e1) != hipSuccess) return 1;
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      long long got = 0;
      hipMemcpy(&got, d, sizeof(got), hipMemcpyDeviceToHost);
      std::printf("%s: %lld ticks in %.3f ms -> %.1f MHz\n", which == 0 ? "wall_clock64" : "clock64",
                  got, ms, got / (ms * 1e3));
    }
  }
  hipFree(d);
  return 0;
}
