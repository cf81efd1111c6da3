// rs_kernels.hpp -- launch interface of the GF(2^8) shard kernels.
#pragma once

#include <hip/hip_runtime_api.h>
#ifdef __HIPCC__
#include <hip/hip_runtime.h>
#endif

#include <atomic>
#include <cstdint>

#include "gf256.hpp"
#include "rs_args.h"

// Store policy of the shard kernels (rs_device.hpp, rs_bitslice.hpp): 1 =
// non-temporal stores (measured fastest in steady state), 0 = default
// write-back stores (kept for the comparison in tools/kbench_tune.hip).
#ifndef STORB_RS_NT_STORES
#define STORB_RS_NT_STORES 1
#endif

namespace storb_rs {

// ApplyArgs, kSlotK / kSlotR, kCopyMaxK: rs_args.h (shared with the JIT).

enum class Variant { Perm = 1, Lds = 2 };

// Workgroups resident per CU. The streaming kernels issue all their loads
// up front; with every slot of a CU filled (8 workgroups of 256 lanes) more
// DRAM pages are open at once than the HBM3E channels serve well, and
// capping the resident workgroups streams faster (tools/kbench_tune.hip
// "occ", profiles/r1_occupancy.txt). The cap is imposed by reserving LDS:
// a workgroup asks for 160 KiB / cap, so cap fit on a CU and cap + 1 do not.
// (The caps were swept in round 1 with a run-time override,
// the removed occ_sweep script, profiles/r1_occupancy.txt; the override is gone.)
constexpr size_t kLdsPerCu = 160u << 10;
inline int wg_cap(int tuned) { return tuned; }
// Dynamic LDS to request so at most `cap` workgroups with `static_lds`
// bytes of static LDS each are resident on a CU (0 = no cap).
inline size_t cap_lds(int cap, size_t static_lds) {
  if (cap <= 0) return 0;
  const size_t per = kLdsPerCu / static_cast<size_t>(cap) / 1024 * 1024;
  return per > static_lds ? per - static_lds : 0;
}

#ifdef __HIPCC__
// Launch kernel Kern with `dyn` bytes of dynamic LDS (the resident-workgroup
// cap); above 64 KiB each kernel must opt in once.
template <auto Kern, class... Args>
hipError_t launch_lds(uint64_t blocks, int threads, size_t dyn, hipStream_t s,
                      const Args &...a) {
  if (dyn > (64u << 10)) {
    static std::atomic<size_t> opted{0};  // per kernel instantiation
    if (opted.load(std::memory_order_relaxed) < dyn) {
      const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(Kern),
                                               hipFuncAttributeMaxDynamicSharedMemorySize,
                                               static_cast<int>(dyn));
      if (e != hipSuccess) return e;
      opted.store(dyn, std::memory_order_relaxed);
    }
  }
  hipLaunchKernelGGL(Kern, dim3(blocks), dim3(threads), dyn, s, a...);
  return hipGetLastError();
}
#endif

// Smallest power of two >= v: the kernel bucket for k.
inline int pow2_bucket(uint32_t v) {
  int b = 1;
  while (b < static_cast<int>(v)) b <<= 1;
  return b;
}

// Kernel bucket for r output rows = the padded row count (tab_rows) of the
// coefficient tables: exact up to 8 rows (no wasted v_perm work for the
// odd erasure counts decode produces), 16 above.
inline int rows_bucket(uint32_t r) { return r <= 8 ? static_cast<int>(r) : 16; }

// True when every slot base / stride and the share size are 16-B aligned,
// i.e. the dwordx4 kernels apply; otherwise the byte kernel runs.
bool vector_ok(const ApplyArgs &a);

hipError_t launch_apply(const ApplyArgs &a, Variant v, hipStream_t s);
// One launch of per-stripe descriptors (DescArgs, rs_args.h): k <= kSlotK,
// r <= kSlotR, 16-B aligned pointers and shares (the host checks).
hipError_t launch_apply_desc(const DescArgs &a, hipStream_t s);

// Bit-sliced encoders with the generator compiled in (rs_bitslice.hpp) for
// the (k, n) Storb's large objects use. a.in / a.out hold the k data and
// n - k parity slots; needs vector_ok(a).
bool bitslice_supported(uint32_t k, uint32_t n);
hipError_t launch_encode_bitslice(const ApplyArgs &a, uint32_t n, hipStream_t s);
// Streamed single-call form (StreamArgs): (16, 24) and (32, 48); columns per
// workgroup tile (0: no streamed encoder for the geometry).
uint32_t bitslice_stream_cols_per_tile(uint32_t k, uint32_t n);
hipError_t launch_encode_bitslice_stream(const ApplyArgs &a, uint32_t n, const StreamArgs &st,
                                         hipStream_t s);

hipError_t launch_blake3_batch(const uint8_t *in, uint64_t len, uint32_t count,
                               uint64_t stride, uint8_t *out, hipStream_t s);
// Every share of nstripes stripes in one launch: len bytes of data share t <
// k of stripe s at data + s * data_stride + t * pitch, of parity share t >= k
// at parity + s * parity_stride + (t - k) * pitch; digest of (s, t) at out +
// (s * n + t) * 32.
hipError_t launch_blake3_stripes(const uint8_t *data, uint64_t data_stride, const uint8_t *parity,
                                 uint64_t parity_stride, uint64_t pitch, uint32_t k, uint32_t n,
                                 uint64_t len, uint32_t nstripes, uint8_t *out, hipStream_t s);
// `shares` consecutive shares of each stripe (at base + s * stride + t * pitch),
// digest of (s, t) at out + (s * out_per + out_off + t) * 32.
hipError_t launch_blake3_stripes_part(const uint8_t *base, uint64_t stride, uint64_t pitch,
                                      uint32_t shares, uint32_t out_per, uint32_t out_off,
                                      uint64_t len, uint32_t nstripes, uint8_t *out,
                                      hipStream_t s);

// Encode with the blake3 digest of every share in the same pass
// (rs_encode_hash.hip). Stripe s: data share j at data + s*data_stride +
// j*block, parity share i at parity + s*parity_stride + i*block, digest of
// share t (data then parity) at hashes + (s*n + t)*32. 16-B aligned.
constexpr int kEHMaxTabs = 8;
struct EncHashArgs {
  const uint8_t *data;
  uint64_t data_stride;
  uint8_t *parity;
  uint64_t parity_stride;
  uint8_t *hashes;
  uint64_t block;
  uint64_t share_stride;  // data share j of a stripe at data + s*data_stride + j*share_stride
  uint32_t nstripes, nchunks, seg_log2, pad;
  uint32_t tab[kEHMaxTabs][5];  // [j*(n-k) + i]: perm_tab(parity coefficient)
};
// (k, n) in {(2, 3), (4, 6)} -- Storb's geometries for chunks up to 1 MiB --
// and block a multiple of 1 KiB up to 256 KiB.
bool encode_hash_supported(uint32_t k, uint32_t n, uint64_t block);
hipError_t launch_encode_hash(const EncHashArgs &a, uint32_t k, uint32_t n, hipStream_t s);

// The streamed single-call kernel (rs_stream.hip): k <= 32, 1 <= r <= 8,
// one stripe, dwordx4-aligned slots; hipErrorInvalidValue otherwise.
hipError_t launch_apply_stream(const ApplyArgs &a, const StreamArgs &st, hipStream_t s);
// dst (device) <- src (device-accessible, e.g. page-locked host), 16-B
// aligned, bytes % 16 == 0, by a kernel on stream s.
hipError_t launch_copy16(void *dst, const void *src, uint64_t bytes, hipStream_t s);
hipError_t launch_fill_splitmix(uint8_t *d, uint64_t obj_len, uint32_t nobj,
                                uint64_t obj_stride, uint64_t seed_base,
                                hipStream_t s);

}  // namespace storb_rs
