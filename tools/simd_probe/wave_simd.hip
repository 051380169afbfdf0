// Which SIMD does each wave of a workgroup land on?  Reads HW_ID.SIMD_ID (bits 5:4) per wave
// for 8-wave (512-thread) workgroups, one workgroup per CU, and prints the wave -> SIMD map of
// the first few workgroups.  Used to place the row / tile waves of ae_minibatch_pipe_kernel.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ __launch_bounds__(512) void wave_simd(int* out) {
  extern __shared__ int big[];   // 96 KB: one workgroup per CU
  const int wave = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    const unsigned hw = __builtin_amdgcn_s_getreg((1 << 11) | (4 << 6) | 4);   // HW_ID[5:4] = SIMD_ID
    const unsigned cu = __builtin_amdgcn_s_getreg((3 << 11) | (8 << 6) | 4);   // HW_ID[11:8] = CU_ID
    out[blockIdx.x * 16 + wave] = (int)hw;
    out[blockIdx.x * 16 + 8 + wave] = (int)cu;
    big[wave] = (int)hw;
  }
}

int main() {
  const int nb = 64;
  int* d;
  if (hipMalloc(&d, nb * 16 * sizeof(int)) != hipSuccess) return 1;
  if (hipFuncSetAttribute(reinterpret_cast<const void*>(wave_simd), hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024) != hipSuccess) return 1;
  hipLaunchKernelGGL(wave_simd, dim3(nb), dim3(512), 96 * 1024, 0, d);
  if (hipDeviceSynchronize() != hipSuccess) return 1;
  int h[nb * 16];
  if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 1;
  int same = 0;
  for (int b = 0; b < nb; ++b) {
    bool rr = true;
    for (int w = 0; w < 8; ++w) rr = rr && h[b * 16 + w] == (h[b * 16] + w) % 4;
    same += rr;
    if (b < 6) {
      printf("wg %d cu %d: simd of waves 0-7 =", b, h[b * 16 + 8]);
      for (int w = 0; w < 8; ++w) printf(" %d", h[b * 16 + w]);
      printf("\n");
    }
  }
  printf("round-robin (simd = simd0 + wave mod 4) in %d of %d workgroups\n", same, nb);
  return 0;
}
