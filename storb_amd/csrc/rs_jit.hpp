// rs_jit.hpp -- bit-sliced kernels compiled at run time for decode / repair
// matrices (rs_jit.cpp).
#pragma once

#include <hip/hip_runtime_api.h>

#include <cstdint>

#include "rs_args.h"

#include <string>

namespace storb_rs {
// code_object_check.cpp: 1 if a kernel of the gfx950 code object makes a
// function call (why names it), 0 if none, -1 if unreadable.
int code_object_calls(const void *co, size_t len, std::string &why);

namespace jit {

// Rows one compiled matrix may have: split into launches of <= kSlotR rows
// (Storb's k = 64 geometry has 32 parity rows).
constexpr uint32_t kMaxRows = 2 * kSlotR;

// STORB_RS_JIT != 0 (default on; "sync" compiles before the first launch).
bool enabled();
// Whether a (rows x k) matrix moving `bytes` per call is worth a compiled
// kernel (the table kernel measured slower on it, rs_jit.cpp).
bool wanted(uint32_t k, uint32_t rows, uint64_t bytes);
// Launch the compiled kernel(s) of matrix `coef` (a.r x a.k, row-major, k <=
// kMaxIn, r <= kMaxRows in row blocks of <= kSlotR) with a's input slots
// (a.copy[j] != null with a.ncopy: fused assembly) and the a.r outputs
// d_out / out_stride (a.out is not read) on stream s if every block is
// ready; queues their compilation otherwise. *launched = false means the
// caller runs the table kernel. `device` must be current.
hipError_t try_launch(int device, const ApplyArgs &a, uint8_t *const *d_out,
                      const size_t *out_stride, const uint8_t *coef, hipStream_t s,
                      bool *launched);

// The streamed single call's form of a matrix's compiled kernel (k > 16,
// <= 8 rows; host_calls.cpp streamed): the workgroups of the one launch
// wait per slice on host-written ready words (rs_stream.hpp). Columns per
// workgroup tile, for sizing the slices.
bool stream_form(uint32_t k, uint32_t rows);
uint32_t stream_cols_per_tile(uint32_t k, uint32_t rows);
// Launch it (a: one stripe, a.r rows, a.out set) if compiled; queue its
// compile otherwise. *launched = false: the caller takes another path.
hipError_t try_launch_stream(int device, const ApplyArgs &a, const uint8_t *coef,
                             const StreamArgs &st, hipStream_t s, bool *launched);

// Queue the compile of matrix `coef` (rows x k) with the given copy mask,
// or with wait finish it. 1 = ready, -1 = failed, 0 = pending / not wanted.
// Needs no GPU (hipRTC only).
int prepare(uint32_t k, uint32_t rows, const uint8_t *coef, uint64_t copy_mask, bool wait);

}  // namespace jit
}  // namespace storb_rs
