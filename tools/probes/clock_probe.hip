// Effective shader clock of a lone resident wave (the per-event scorers' situation):
// a dependent FMA chain timed with s_memtime (shader clock) and s_memrealtime (100 MHz).
// Also a second pass with the other 255 CUs busy, to see whether load changes the clock.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void chain(float* out, unsigned long long* t, int iters) {
  float x = threadIdx.x * 1e-3f, y = 1.0001f;
  const unsigned long long c0 = __builtin_amdgcn_s_memtime();
  const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int k = 0; k < 16; ++k) x = fmaf(x, y, 1e-7f);
  }
  const unsigned long long c1 = __builtin_amdgcn_s_memtime();
  const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    t[0] = c1 - c0;
    t[1] = r1 - r0;
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

int main() {
  float* out;
  unsigned long long* t;
  hipMalloc(&out, 1024 * 64 * sizeof(float));
  hipMalloc(&t, 2 * sizeof(unsigned long long));
  unsigned long long h[2];
  for (int blocks : {1, 1, 256, 1024}) {
    const int iters = 20000;
    hipLaunchKernelGGL(chain, dim3(blocks), dim3(64), 0, 0, out, t, iters);
    hipDeviceSynchronize();
    hipMemcpy(h, t, sizeof(h), hipMemcpyDeviceToHost);
    const double fmas = 16.0 * iters;
    const double us = h[1] / 100.0;
    printf("{\"blocks\": %d, \"shader_cycles\": %llu, \"realtime_us\": %.2f, \"clock_ghz\": %.3f, "
           "\"cycles_per_dep_fma\": %.2f, \"ns_per_dep_fma\": %.3f}\n",
           blocks, h[0], us, h[0] / (us * 1e3), h[0] / fmas, us * 1e3 / fmas);
  }
  return 0;
}
