// rs_jit.hpp -- bit-sliced kernels compiled at run time for decode / repair
// matrices (rs_jit.cpp).
#pragma once

#include <hip/hip_runtime_api.h>

#include <cstdint>

#include "rs_args.h"

namespace storb_rs {
namespace jit {

// STORB_RS_JIT != 0 (default on; "sync" compiles before the first launch).
bool enabled();
// Whether a (rows x k) matrix moving `bytes` per call is worth a compiled
// kernel (the table kernel measured slower on it, rs_jit.cpp).
bool wanted(uint32_t k, uint32_t rows, uint64_t bytes);
// Launch the compiled kernel of matrix `coef` (a.r x a.k, row-major) with
// a's slots (a.copy[j] != null with a.ncopy: fused assembly) on stream s if
// it is ready; queues its compilation otherwise. *launched = false means the
// caller runs the table kernel. `device` must be current.
hipError_t try_launch(int device, const ApplyArgs &a, const uint8_t *coef, hipStream_t s,
                      bool *launched);

// Queue the compile of matrix `coef` (rows x k) with the given copy mask,
// or with wait finish it. 1 = ready, -1 = failed, 0 = pending / not wanted.
// Needs no GPU (hipRTC only).
int prepare(uint32_t k, uint32_t rows, const uint8_t *coef, uint64_t copy_mask, bool wait);

}  // namespace jit
}  // namespace storb_rs
