// Keras / TF ResourceApplyAdam on one parameter, shared by every device Adam (reduce_adam_kernel,
// slab_adam_kernel in ae_fused.hip; slab_sum2_kernel's fused update in dense.hip).  The roundings are
// pinned with explicit fmaf so the kernels that share it -- operands loaded late, prefetched, or
// gathered through a slab map -- give bit-identical parameters whatever the compiler would contract.
#pragma once

namespace sml {

// bias-corrected step size at step t (t >= 1)
__device__ __forceinline__ float adam_lr_t(float lr, float b1, float b2, float t) {
  return lr * sqrtf(1.0f - powf(b2, t)) / (1.0f - powf(b1, t));
}

__device__ __forceinline__ void adam_update(float tot, float m0, float v0, float p0, float lr_t, float b1, float b2,
                                            float eps, float gscale, float& mm, float& vv, float& pn) {
  const float gr = tot * gscale;
  mm = fmaf(b1, m0, (1.0f - b1) * gr);
  vv = fmaf(b2, v0, ((1.0f - b2) * gr) * gr);
  pn = p0 - (lr_t * mm) / (sqrtf(vv) + eps);
}

}  // namespace sml
