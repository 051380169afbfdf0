// Streams for persistent kernels.
//
// A persistent kernel (the streaming-epoch trainer, the per-event scorers) stays resident
// while work on OTHER streams feeds it (ring copies, doorbells) or while the host does.
// HIP maps streams onto a small number of hardware queues (GPU_MAX_HW_QUEUES, 4 on the
// MI355X boxes) and lets streams share a queue once they are all taken; packets of one
// queue run in order, so a copy that lands in the persistent kernel's queue would wait for
// the kernel that waits for it.  HIP keeps a separate pool of queues per stream priority,
// so these kernels run on a highest-priority stream: nothing else in the framework uses
// that priority, and the normal-priority streams never share its queue.
#pragma once
#include <hip/hip_runtime.h>

namespace sml {

inline hipError_t create_persistent_stream(hipStream_t* s) {
  int least = 0, greatest = 0;
  hipError_t e = hipDeviceGetStreamPriorityRange(&least, &greatest);
  if (e != hipSuccess) return e;
  return hipStreamCreateWithPriority(s, hipStreamNonBlocking, greatest);
}

}  // namespace sml
