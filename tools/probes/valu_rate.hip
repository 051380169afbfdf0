// VALU / transcendental / MFMA issue rate per SIMD at 1..8 waves per SIMD (gfx950).
// Question it answers (profiles/r06/SUMMARY.md §1): does a SIMD issue a wave64 VALU every
// 2 cycles once two or more waves are resident, or every 4 as one wave alone does?  The AE
// headline kernel's per-trip time sits at ONE wave's issue stream with 3 waves per SIMD.
// Waves per SIMD are set by dynamic LDS (160 KiB / k per 256-thread workgroup, one wave per
// SIMD each); every wave stamps s_memtime around its loop.  Output: cycles per instruction
// per SIMD = wave cycles / (k * instructions per wave).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef __attribute__((__vector_size__(8 * sizeof(short)))) short s16x8;
typedef __attribute__((__vector_size__(4 * sizeof(float)))) float f32x4;

#define FMA(r) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(r) : "v"(x), "v"(y))
#define EXP(r) asm volatile("v_exp_f32 %0, %0" : "+v"(r))
#define CVT(r, s) asm volatile("v_cvt_pk_bf16_f32 %0, %0, %1" : "+v"(r) : "v"(s))

template <int MODE>
__global__ __launch_bounds__(256) void probe(int iters, float x, float y, float* out, long long* cyc) {
  extern __shared__ float lds[];
  float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = acc0;
  s16x8 av = {1, 2, 3, 4, 5, 6, 7, 8}, bv = av;
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
    if constexpr (MODE == 0) {   // 16 independent FMAs (8 chains x 2)
      FMA(a0); FMA(a1); FMA(a2); FMA(a3); FMA(a4); FMA(a5); FMA(a6); FMA(a7);
      FMA(a0); FMA(a1); FMA(a2); FMA(a3); FMA(a4); FMA(a5); FMA(a6); FMA(a7);
    } else if constexpr (MODE == 1) {   // 16 dependent FMAs (one chain)
      FMA(a0); FMA(a0); FMA(a0); FMA(a0); FMA(a0); FMA(a0); FMA(a0); FMA(a0);
      FMA(a0); FMA(a0); FMA(a0); FMA(a0); FMA(a0); FMA(a0); FMA(a0); FMA(a0);
    } else if constexpr (MODE == 2) {   // 8 independent v_exp_f32 + 8 FMAs
      EXP(a0); FMA(a1); EXP(a2); FMA(a3); EXP(a4); FMA(a5); EXP(a6); FMA(a7);
      EXP(a1); FMA(a0); EXP(a3); FMA(a2); EXP(a5); FMA(a4); EXP(a7); FMA(a6);
    } else if constexpr (MODE == 3) {   // 2 independent 16x16x32 bf16 MFMAs + 14 FMAs (the AE kernel's mix)
      acc0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, acc0, 0, 0, 0);
      FMA(a0); FMA(a1); FMA(a2); FMA(a3); FMA(a4); FMA(a5); FMA(a6);
      acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, acc1, 0, 0, 0);
      FMA(a7); FMA(a0); FMA(a1); FMA(a2); FMA(a3); FMA(a4); FMA(a5);
    } else if constexpr (MODE == 4) {   // 16 independent cvt_pk_bf16
      CVT(a0, a1); CVT(a1, a2); CVT(a2, a3); CVT(a3, a4); CVT(a4, a5); CVT(a5, a6); CVT(a6, a7); CVT(a7, a0);
      CVT(a0, a1); CVT(a1, a2); CVT(a2, a3); CVT(a3, a4); CVT(a4, a5); CVT(a5, a6); CVT(a6, a7); CVT(a7, a0);
    } else {   // 4 dependent chains of 4 FMAs each, chains interleaved (ILP 4)
      FMA(a0); FMA(a1); FMA(a2); FMA(a3); FMA(a0); FMA(a1); FMA(a2); FMA(a3);
      FMA(a0); FMA(a1); FMA(a2); FMA(a3); FMA(a0); FMA(a1); FMA(a2); FMA(a3);
    }
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  const float r = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + acc0[0] + acc1[1] + acc0[3];
  if (threadIdx.x == 0) lds[0] = r;
  out[blockIdx.x * 256 + threadIdx.x] = r;
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 4 + (threadIdx.x >> 6)] = t1 - t0;
}

template <int MODE>
static void run(const char* name, int cus, int iters) {
  float* out;
  long long* cyc;
  const int maxk = 8;
  if (hipMalloc(&out, (size_t)cus * maxk * 256 * 4) != hipSuccess) exit(1);
  if (hipMalloc(&cyc, (size_t)cus * maxk * 4 * 8) != hipSuccess) exit(1);
  if (hipFuncSetAttribute(reinterpret_cast<const void*>(probe<MODE>), hipFuncAttributeMaxDynamicSharedMemorySize,
                          160 * 1024) != hipSuccess)
    exit(1);
  for (int k = 1; k <= maxk; ++k) {
    const int lds = (160 * 1024 / k) & ~255;
    const int nb = cus * k;
    hipLaunchKernelGGL(probe<MODE>, dim3(nb), dim3(256), lds, 0, iters, 1.0001f, 0.5f, out, cyc);   // warm-up
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0, 0);
    hipLaunchKernelGGL(probe<MODE>, dim3(nb), dim3(256), lds, 0, iters, 1.0001f, 0.5f, out, cyc);
    (void)hipEventRecord(e1, 0);
    if (hipDeviceSynchronize() != hipSuccess) exit(1);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    long long* h = (long long*)malloc((size_t)nb * 4 * 8);
    (void)hipMemcpy(h, cyc, (size_t)nb * 4 * 8, hipMemcpyDeviceToHost);
    double s = 0;
    for (int i = 0; i < nb * 4; ++i) s += (double)h[i];
    s /= nb * 4;
    const double instr = 16.0 * iters;
    printf("%-22s waves/SIMD %d: wave cycles %.0f  cycles per instr per SIMD %.2f  per wave %.2f  wall %.3f ms\n", name,
           k, s, s / (k * instr), s / instr, ms);
    free(h);
  }
  (void)hipFree(out);
  (void)hipFree(cyc);
}

int main(int argc, char** argv) {
  int dev = 0, cus = 0;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const int iters = argc > 1 ? atoi(argv[1]) : 20000;
  run<0>("fma_indep16", cus, iters);
  run<1>("fma_dep1", cus, iters);
  run<5>("fma_ilp4", cus, iters);
  run<2>("exp8_fma8", cus, iters);
  run<3>("mfma2_fma14", cus, iters);
  run<4>("cvt_pk16", cus, iters);
  return 0;
}
