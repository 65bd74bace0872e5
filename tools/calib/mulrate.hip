// Issue rate of v_mul_lo_u32 vs v_mul_u32_u24 vs v_add_u32 on gfx950: 8
// independent chains per lane, one wave per SIMD (1024 waves), kernel time.
#include <hip/hip_runtime.h>
#include <cstdio>
#define CH(op)                                                                 \
  __global__ void k_##op(uint32_t* out, uint32_t seed, int iters) {           \
    uint32_t a0 = seed + threadIdx.x, a1 = a0 ^ 1, a2 = a0 ^ 2, a3 = a0 ^ 3,   \
             a4 = a0 ^ 4, a5 = a0 ^ 5, a6 = a0 ^ 6, a7 = a0 ^ 7, m = seed | 1; \
    for (int i = 0; i < iters; i++) {                                          \
      asm volatile(#op " %0, %0, %8\n" #op " %1, %1, %8\n" #op " %2, %2, %8\n" \
                   #op " %3, %3, %8\n" #op " %4, %4, %8\n" #op " %5, %5, %8\n" \
                   #op " %6, %6, %8\n" #op " %7, %7, %8\n"                     \
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4),         \
                     "+v"(a5), "+v"(a6), "+v"(a7)                              \
                   : "v"(m));                                                  \
    }                                                                          \
    out[blockIdx.x * 64 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7; \
  }
CH(v_mul_lo_u32)
CH(v_mul_u32_u24)
CH(v_add_u32)
CH(v_mul_hi_u32)
template <class K>
float run(K k, uint32_t* d, int iters) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipLaunchKernelGGL(k, dim3(1024), dim3(64), 0, 0, d, 3u, iters);
  hipEventRecord(a);
  hipLaunchKernelGGL(k, dim3(1024), dim3(64), 0, 0, d, 3u, iters);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  return ms;
}
int main() {
  uint32_t* d;
  hipMalloc(&d, 1024 * 64 * 4);
  const int it = 20000;
  const double n = 8.0 * it;   // instructions per wave
  float t;
  t = run(k_v_add_u32, d, it);
  printf("v_add_u32      %.3f ms  %.2f cycles/instr/wave @2.4GHz\n", t, t * 1e-3 * 2.4e9 / n);
  t = run(k_v_mul_u32_u24, d, it);
  printf("v_mul_u32_u24  %.3f ms  %.2f cycles/instr/wave @2.4GHz\n", t, t * 1e-3 * 2.4e9 / n);
  t = run(k_v_mul_lo_u32, d, it);
  printf("v_mul_lo_u32   %.3f ms  %.2f cycles/instr/wave @2.4GHz\n", t, t * 1e-3 * 2.4e9 / n);
  t = run(k_v_mul_hi_u32, d, it);
  printf("v_mul_hi_u32   %.3f ms  %.2f cycles/instr/wave @2.4GHz\n", t, t * 1e-3 * 2.4e9 / n);
  hipFree(d);
  return 0;
}
