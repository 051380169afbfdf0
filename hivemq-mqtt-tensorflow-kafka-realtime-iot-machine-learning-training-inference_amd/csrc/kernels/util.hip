// Small utility kernels: lane-exchange self-test (checks the permlane-swap
// helpers the fused kernels rely on against their defining semantics).
#include "sml_common.h"

using namespace sml;

namespace {
__global__ void lane_xor_probe_kernel(float* out) {
  const int lane = threadIdx.x & 63;
  const float v = (float)lane;
  out[lane] = xor16(v, lane);
  out[64 + lane] = xor32(v, lane);
}
}  // namespace

namespace sml {
hipError_t lane_xor_probe_launch(float* out, hipStream_t stream) {
  hipLaunchKernelGGL(lane_xor_probe_kernel, dim3(1), dim3(64), 0, stream, out);
  return hipGetLastError();
}
}  // namespace sml
