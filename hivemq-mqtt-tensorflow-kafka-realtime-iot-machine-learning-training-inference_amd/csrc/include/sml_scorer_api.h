// C ABI between a device scorer (in _C.so: the persistent AE scorer, runtime/serve.h)
// and the host-only streaming loop (in _io.so: io/scoreloop.h).
//
// The two extension modules are built and loaded independently (_io has no HIP / torch
// dependency), so the loop reaches the scorer through this plain table of function
// pointers: `_C.AEServe.c_api()` returns the table's address, `_io.ScoreLoop` takes it.
// The table lives inside the AEServe binding object, which the Python side keeps alive
// for as long as the loop runs.
#pragma once
#include <cstdint>

extern "C" {

struct SmlScorerApi {
  uint32_t version;   // SML_SCORER_API_VERSION
  int32_t dim;        // features per row
  void* ctx;
  // Score k raw rows [k][dim]: scores[k], anomaly flags[k] and (recon != nullptr) the
  // reconstructions [k][dim].  Returns 0, or non-zero with last_error(ctx) set.
  int (*infer)(void* ctx, const float* rows, int k, float* scores, uint32_t* flags, float* recon,
               double timeout_s);
  const char* (*last_error)(void* ctx);
  // v2: keyed scorers (the LSTM forecaster: per-key windows on the device).  nkeys > 0
  // means every row needs a key in [0, nkeys) and infer_keyed must be used; recon then
  // receives each key's next-event forecast, flags 2 = the key has no previous forecast.
  int64_t nkeys;
  int (*infer_keyed)(void* ctx, const float* rows, const uint32_t* keys, int k, float* scores, uint32_t* flags,
                     float* recon, double timeout_s);
};

}  // extern "C"

#define SML_SCORER_API_VERSION 2u
