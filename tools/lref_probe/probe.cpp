// Standalone timing / phase probe of the reference-LSTM trainer (lstm_ref_train.hip) at
// batch 1, without torch: build.sh compiles the kernel file with -DSML_LREF_PROBE next to
// this driver.  Prints one JSON line: us/step from hipEvents over `launches` launches of
// `steps` Keras steps, and the per-phase shader-clock split measured by wave 0.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "sml_ops.h"

namespace sml {
hipError_t lstm_ref_probe_read(unsigned long long* host8, bool reset);
}

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                    \
    }                                                                                  \
  } while (0)

int main(int argc, char** argv) {
  const int steps = argc > 1 ? std::atoi(argv[1]) : 1000;
  const int launches = argc > 2 ? std::atoi(argv[2]) : 5;
  const int P = sml::lstm_ref_train_params();
  std::mt19937 rng(0);
  std::uniform_real_distribution<float> u(-0.2f, 0.2f), ux(-1.f, 1.f);
  std::vector<float> flat(P), xy((steps + 1) * 18);
  for (auto& w : flat) w = u(rng);
  for (auto& v : xy) v = ux(rng);
  float *dflat, *dm, *dv, *dxy, *dout;
  int64_t* dit;
  CK(hipMalloc(&dflat, P * 4));
  CK(hipMalloc(&dm, P * 4));
  CK(hipMalloc(&dv, P * 4));
  CK(hipMalloc(&dxy, xy.size() * 4));
  CK(hipMalloc(&dout, steps * 2 * 4));
  CK(hipMalloc(&dit, 8));
  CK(hipMemcpy(dflat, flat.data(), P * 4, hipMemcpyHostToDevice));
  CK(hipMemset(dm, 0, P * 4));
  CK(hipMemset(dv, 0, P * 4));
  CK(hipMemset(dit, 0, 8));
  CK(hipMemcpy(dxy, xy.data(), xy.size() * 4, hipMemcpyHostToDevice));
  auto launch = [&]() {
    CK(sml::lstm_ref_train_launch(dflat, dm, dv, dit, dxy, 18, dxy + 18, 18, nullptr, steps, 0, 1, steps, 1, 1e-3f,
                                  0.9f, 0.999f, 1e-7f, dout, nullptr));
  };
  launch();  // warm-up (module load, LDS opt-in)
  CK(hipDeviceSynchronize());
  unsigned long long pr[8];
  CK(sml::lstm_ref_probe_read(pr, true));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0, nullptr));
  for (int i = 0; i < launches; ++i) launch();
  CK(hipEventRecord(e1, nullptr));
  CK(hipEventSynchronize(e1));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, e0, e1));
  CK(sml::lstm_ref_probe_read(pr, false));
  std::vector<float> out(steps * 2);
  CK(hipMemcpy(out.data(), dout, out.size() * 4, hipMemcpyDeviceToHost));
  const double n = pr[4] ? (double)pr[4] : 1.0, tot = (double)(pr[0] + pr[1] + pr[2] + pr[3]);
  std::printf("{\"us_per_step\": %.4f, \"steps\": %d, \"launches\": %d, \"cycles_per_step\": %.1f, "
              "\"chain_busy\": %.1f, \"chain_wait\": %.1f, \"adam_busy\": %.1f, \"adam_wait\": %.1f, \"last_loss\": %.6f}\n",
              ms * 1e3 / (steps * launches), steps, launches, tot / n, pr[0] / n, pr[1] / n, pr[2] / n, pr[3] / n,
              out[2 * (steps - 1)]);
  return 0;
}
