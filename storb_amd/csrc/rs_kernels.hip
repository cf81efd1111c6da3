// rs_kernels.hip -- dispatch, the any-alignment byte kernel and the
// synthetic-input fill kernel. The dwordx4 kernels and their design notes
// are in rs_device.hpp; their instantiations in rs_perm_k*.hip / rs_lds.hip.
#include <cstdlib>

#include <algorithm>

#include "rs_device.hpp"

namespace storb_rs {

// Any alignment, any share size: each lane owns 4 consecutive bytes. Only
// taken when a caller's device layout is not 16-B aligned (the host API
// always stages into an aligned layout).
__global__ __launch_bounds__(kThreads) void rs_apply_bytes(const ApplyArgs a) {
  const uint64_t words = (a.block + 3) >> 2;
  const uint64_t tps = (words + kThreads - 1) / kThreads;
  const uint64_t stripe = blockIdx.x / tps;
  const uint64_t w = (blockIdx.x - stripe * tps) * kThreads + threadIdx.x;
  if (w >= words) return;
  const uint64_t off = w * 4;
  const uint32_t nb =
      a.block - off >= 4 ? 4u : static_cast<uint32_t>(a.block - off);
  uint32_t acc[kSlotR];
#pragma unroll
  for (int i = 0; i < kSlotR; i++) acc[i] = 0;
  for (uint32_t j = 0; j < a.k; j++) {
    const uint8_t *p = a.in[j] + stripe * a.in_stride[j] + off;
    uint32_t d = 0;
    for (uint32_t b = 0; b < nb; b++) d |= static_cast<uint32_t>(p[b]) << (8 * b);
    const uint32_t s0 = d & 0x07070707u;
    const uint32_t s1 = (d >> 3) & 0x07070707u;
    const uint32_t s2 = (d >> 6) & 0x03030303u;
#pragma unroll
    for (int i = 0; i < kSlotR; i++)
      if (i < static_cast<int>(a.r))
        acc[i] ^= gf_mul_perm(a.ptab[j * a.tab_rows + i], s0, s1, s2);
  }
#pragma unroll
  for (int i = 0; i < kSlotR; i++) {
    if (i >= static_cast<int>(a.r)) continue;
    uint8_t *q = a.out[i] + stripe * a.out_stride[i] + off;
    for (uint32_t b = 0; b < nb; b++) {
      const uint8_t v = static_cast<uint8_t>(acc[i] >> (8 * b));
      q[b] = a.accumulate ? static_cast<uint8_t>(q[b] ^ v) : v;
    }
  }
}

__device__ __forceinline__ uint64_t splitmix(uint64_t seed, uint64_t i) {
  uint64_t z = seed + (i + 1) * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__global__ __launch_bounds__(kThreads) void fill_splitmix_kernel(
    uint8_t *d, uint64_t obj_len, uint32_t nobj, uint64_t obj_stride,
    uint64_t seed_base, int aligned8) {
  const uint64_t words = (obj_len + 7) >> 3;
  const uint64_t total = words * nobj;
  for (uint64_t g = blockIdx.x * static_cast<uint64_t>(kThreads) + threadIdx.x;
       g < total; g += static_cast<uint64_t>(gridDim.x) * kThreads) {
    const uint64_t o = g / words, w = g - o * words;
    const uint64_t z = splitmix(seed_base + o, w);
    uint8_t *p = d + o * obj_stride + w * 8;
    if (aligned8 && (w + 1) * 8 <= obj_len) {
      *reinterpret_cast<uint64_t *>(p) = z;
    } else {
      const uint64_t nb = obj_len - w * 8 < 8 ? obj_len - w * 8 : 8;
      for (uint64_t b = 0; b < nb; b++) p[b] = static_cast<uint8_t>(z >> (8 * b));
    }
  }
}

bool vector_ok(const ApplyArgs &a) {
  if (a.block % 16) return false;
  for (uint32_t j = 0; a.ncopy && j < a.k; j++)
    if ((reinterpret_cast<uintptr_t>(a.copy[j]) | a.copy_stride[j]) % 16) return false;
  for (uint32_t j = 0; j < a.k; j++)
    if ((reinterpret_cast<uintptr_t>(a.in[j]) | a.in_stride[j]) % 16) return false;
  for (uint32_t i = 0; i < a.r; i++)
    if ((reinterpret_cast<uintptr_t>(a.out[i]) | a.out_stride[i]) % 16) return false;
  return true;
}

hipError_t launch_apply(const ApplyArgs &a, Variant v, hipStream_t s) {
  if (a.k == 0 || a.k > kSlotK || a.r > kSlotR ||
      a.tab_rows != static_cast<uint32_t>(rows_bucket(a.r ? a.r : 1)))
    return hipErrorInvalidValue;
  // Fused assembly runs only in the dwordx4 register-table kernels; the host
  // (copy_fusable) checks that before asking for it.
  if (a.ncopy && (a.k > kCopyMaxK || v != Variant::Perm || !vector_ok(a)))
    return hipErrorInvalidValue;
  if (a.r == 0 && !a.ncopy) return hipErrorInvalidValue;
  if (a.block == 0 || a.nstripes == 0) return hipSuccess;
  if (!vector_ok(a)) {
    const uint64_t words = (a.block + 3) >> 2;
    const uint64_t blocks = ((words + kThreads - 1) / kThreads) * a.nstripes;
    if (blocks > 0x7FFFFFFFull) return hipErrorInvalidConfiguration;
    hipLaunchKernelGGL(rs_apply_bytes, dim3(blocks), dim3(kThreads), 0, s, a);
    return hipGetLastError();
  }
  // The LDS variant holds r*k*256 B of tables; beyond 16x8 it would cap
  // occupancy, so larger blocks always take the register-table kernel.
  if (v == Variant::Lds && a.k <= 16 && a.r <= 8 && a.btab != nullptr)
    return dispatch_lds(a, s);
  switch (pow2_bucket(a.k)) {
    case 1: return dispatch_perm_k1(a, s);
    case 2: return dispatch_perm_k2(a, s);
    case 4: return dispatch_perm_k4(a, s);
    case 8: return dispatch_perm_k8(a, s);
    case 16: return dispatch_perm_k16(a, s);
    default: return dispatch_perm_k32(a, s);
  }
}

hipError_t launch_apply_desc(const DescArgs &a, hipStream_t s) {
  if (a.k == 0 || a.k > kSlotK || a.r > kSlotR || (a.copy && a.k > kCopyMaxK) ||
      (a.r == 0 && !a.copy) || a.block % 16 || a.tpw == 0 || (a.mix && a.r != kMixR) ||
      a.rec_qwords != 1 + a.k + a.r + (a.copy ? a.k : 0))
    return hipErrorInvalidValue;
  if (a.block == 0 || a.nitems == 0) return hipSuccess;
  switch (pow2_bucket(a.k)) {
    case 1: return dispatch_desc_k1(a, s);
    case 2: return dispatch_desc_k2(a, s);
    case 4: return dispatch_desc_k4(a, s);
    case 8: return dispatch_desc_k8(a, s);
    case 16: return dispatch_desc_k16(a, s);
    default: return dispatch_desc_k32(a, s);
  }
}

// Descriptor upload (decode_stripes.cpp apply_desc): page-locked host
// memory -> device, read over PCIe by a kernel on the launch stream. An SDMA
// copy (hipMemcpyAsync) in front of the decode kernels kept them waiting on
// the copy engine's start-up and completion signalling.
__global__ __launch_bounds__(kThreads) void copy_u32x4_kernel(u32x4 *dst, const u32x4 *src,
                                                              uint64_t n) {
  for (uint64_t i = blockIdx.x * static_cast<uint64_t>(kThreads) + threadIdx.x; i < n;
       i += static_cast<uint64_t>(gridDim.x) * kThreads)
    dst[i] = __builtin_nontemporal_load(src + i);
}

hipError_t launch_copy16(void *dst, const void *src, uint64_t bytes, hipStream_t s) {
  if (bytes % 16 || (reinterpret_cast<uintptr_t>(dst) | reinterpret_cast<uintptr_t>(src)) % 16)
    return hipErrorInvalidValue;
  const uint64_t n = bytes / 16;
  if (n == 0) return hipSuccess;
  const uint64_t blocks = std::min<uint64_t>(256, (n + kThreads - 1) / kThreads);
  hipLaunchKernelGGL(copy_u32x4_kernel, dim3(blocks), dim3(kThreads), 0, s,
                     static_cast<u32x4 *>(dst), static_cast<const u32x4 *>(src), n);
  return hipGetLastError();
}

hipError_t launch_fill_splitmix(uint8_t *d, uint64_t obj_len, uint32_t nobj,
                                uint64_t obj_stride, uint64_t seed_base,
                                hipStream_t s) {
  if (obj_len == 0 || nobj == 0) return hipSuccess;
  const uint64_t total = ((obj_len + 7) >> 3) * nobj;
  uint64_t blocks = (total + kThreads - 1) / kThreads;
  if (blocks > 8192) blocks = 8192;
  const int aligned8 =
      ((reinterpret_cast<uintptr_t>(d) | obj_stride) % 8) == 0 ? 1 : 0;
  hipLaunchKernelGGL(fill_splitmix_kernel, dim3(blocks), dim3(kThreads), 0, s, d,
                     obj_len, nobj, obj_stride, seed_base, aligned8);
  return hipGetLastError();
}

}  // namespace storb_rs
