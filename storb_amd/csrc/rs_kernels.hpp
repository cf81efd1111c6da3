// rs_kernels.hpp -- launch interface of the GF(2^8) shard kernels.
#pragma once

#include <hip/hip_runtime_api.h>

#include <cstdint>

#include "gf256.hpp"

namespace storb_rs {

// One launch applies a (r x k) coefficient block to k input share slots and
// writes (or XOR-accumulates into) r output share slots, for every stripe.
// Larger matrices are tiled over several launches by the host (apply.cpp).
constexpr int kSlotK = 32;
constexpr int kSlotR = 16;

struct ApplyArgs {
  const uint8_t *in[kSlotK];
  uint64_t in_stride[kSlotK];
  uint8_t *out[kSlotR];
  uint64_t out_stride[kSlotR];
  const PermTab *ptab;  // r*k nibble tables, row-major [row][col]
  const uint8_t *btab;  // r*k 256-byte product tables (LDS variant)
  uint32_t k, r;
  uint64_t block;       // bytes per share
  uint32_t nstripes;
  uint32_t accumulate;  // 1: out ^= result (column tiling), 0: out = result
};

enum class Variant { Perm = 1, Lds = 2 };

// True when every slot base / stride and the share size are 16-B aligned,
// i.e. the dwordx4 kernels apply; otherwise the byte kernel runs.
bool vector_ok(const ApplyArgs &a);

hipError_t launch_apply(const ApplyArgs &a, Variant v, hipStream_t s);

hipError_t launch_fill_splitmix(uint8_t *d, uint64_t obj_len, uint32_t nobj,
                                uint64_t obj_stride, uint64_t seed_base,
                                hipStream_t s);

}  // namespace storb_rs
