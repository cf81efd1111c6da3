// rs_device.hpp -- device-side templates of the GF(2^8) shard kernels.
//
// What the reference computes here: zfec's addmul loop (fec.c, ported by
// zfec-rs @3f3a3720 and called from crates/storb_base/src/piece.rs:329 for
// encode and :384-386 for decode): out_r[b] = XOR_j M[r][j] * in_j[b] over
// GF(2^8), byte-wise. Encode uses M = the parity rows of the systematic
// generator, decode uses the rows of the inverted survivor matrix that
// rebuild the missing data shares. Both are this one streaming kernel.
//
// Design (DESIGN.md "Kernels"):
//  * HBM-bound byte work, no MFMA. Every lane streams 16 B (dwordx4) of each
//    of the k input shares at the same column, so each wave-instruction
//    moves one contiguous, fully coalesced 1 KiB per share.
//  * Multiplication by a constant c is GF(2)-linear in the data byte x, so
//    c*x = T0[x & 7] ^ T1[(x >> 3) & 7] ^ T2[x >> 6]. T0/T1 are 8-entry and
//    T2 4-entry byte tables that fit one v_perm_b32 each: 3 v_perm_b32 +
//    ~1.5 v_xor per dword per coefficient, with the per-dword selectors
//    (two masks, two shifts) shared by every output row. The tables are
//    wave-uniform and live in SGPRs (s_load from the coefficient buffer),
//    so the kernel touches no LDS at all and has no bank conflicts.
//  * Variant LDS (rs_apply_lds) stages classic 256-byte product tables in
//    LDS and looks each byte up with ds_read_u8 -- the textbook GPU layout,
//    kept as the measured comparison point for the register-table variant.
//  * The grid is nstripes x tiles; a tile is 256 lanes x U dwordx4 columns.
//    Full tiles (the common case) run without per-lane bounds checks.
#pragma once

#include <hip/hip_runtime.h>

#include "rs_kernels.hpp"

namespace storb_rs {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

static constexpr int kThreads = 256;

template <int KM>
struct Unroll {
  // Columns per lane: enough dwordx4 loads in flight without blowing the
  // register budget as k grows.
  static constexpr int U = KM <= 4 ? 2 : 1;
};

__device__ __forceinline__ uint32_t gf_mul_perm(const PermTab &t, uint32_t s0,
                                                uint32_t s1, uint32_t s2) {
  return __builtin_amdgcn_perm(t.t0hi, t.t0lo, s0) ^
         __builtin_amdgcn_perm(t.t1hi, t.t1lo, s1) ^
         __builtin_amdgcn_perm(0u, t.t2, s2);
}

template <int KM, int RM, bool EXACT, bool GUARD>
__device__ __forceinline__ void perm_tile(const ApplyArgs &a, uint32_t k,
                                          uint32_t r, uint32_t cols,
                                          uint32_t stripe, uint32_t c0) {
  constexpr int U = Unroll<KM>::U;
  u32x4 x[KM][U];
#pragma unroll
  for (int j = 0; j < KM; j++) {
    if (EXACT || j < static_cast<int>(k)) {
      const u32x4 *p = reinterpret_cast<const u32x4 *>(
          a.in[j] + static_cast<uint64_t>(stripe) * a.in_stride[j]);
#pragma unroll
      for (int u = 0; u < U; u++) {
        const uint32_t c = c0 + u * kThreads;
        if (GUARD)
          x[j][u] = c < cols ? p[c] : u32x4{0, 0, 0, 0};
        else
          x[j][u] = p[c];
      }
    }
  }

  u32x4 acc[RM][U];
#pragma unroll
  for (int i = 0; i < RM; i++)
#pragma unroll
    for (int u = 0; u < U; u++) acc[i][u] = u32x4{0, 0, 0, 0};

#pragma unroll
  for (int j = 0; j < KM; j++) {
    if (!(EXACT || j < static_cast<int>(k))) continue;
#pragma unroll
    for (int u = 0; u < U; u++) {
#pragma unroll
      for (int w = 0; w < 4; w++) {
        const uint32_t d = x[j][u][w];
        const uint32_t s0 = d & 0x07070707u;
        const uint32_t s1 = (d >> 3) & 0x07070707u;
        const uint32_t s2 = (d >> 6) & 0x03030303u;
#pragma unroll
        for (int i = 0; i < RM; i++) {
          if (!(EXACT || i < static_cast<int>(r))) continue;
          const PermTab &t = a.ptab[i * k + j];
          acc[i][u][w] ^= gf_mul_perm(t, s0, s1, s2);
        }
      }
    }
  }

#pragma unroll
  for (int i = 0; i < RM; i++) {
    if (!(EXACT || i < static_cast<int>(r))) continue;
    u32x4 *q = reinterpret_cast<u32x4 *>(
        a.out[i] + static_cast<uint64_t>(stripe) * a.out_stride[i]);
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint32_t c = c0 + u * kThreads;
      if (!GUARD || c < cols) {
        u32x4 v = acc[i][u];
        if (a.accumulate) v ^= q[c];
        q[c] = v;
      }
    }
  }
}

template <int KM, int RM, bool EXACT>
__global__ __launch_bounds__(kThreads) void rs_apply_perm(const ApplyArgs a) {
  constexpr uint32_t TILE = kThreads * Unroll<KM>::U;
  const uint32_t k = EXACT ? KM : a.k;
  const uint32_t r = EXACT ? RM : a.r;
  const uint32_t cols = static_cast<uint32_t>(a.block >> 4);
  const uint32_t tps = (cols + TILE - 1) / TILE;
  const uint32_t stripe = blockIdx.x / tps;
  const uint32_t base = (blockIdx.x - stripe * tps) * TILE;
  if (base + TILE <= cols)
    perm_tile<KM, RM, EXACT, false>(a, k, r, cols, stripe, base + threadIdx.x);
  else
    perm_tile<KM, RM, EXACT, true>(a, k, r, cols, stripe, base + threadIdx.x);
}

template <int KM, int RM>
__global__ __launch_bounds__(kThreads) void rs_apply_lds(const ApplyArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds_tab[];
  constexpr int U = Unroll<KM>::U;
  constexpr uint32_t TILE = kThreads * U;
  const uint32_t k = a.k, r = a.r;
  const uint32_t cols = static_cast<uint32_t>(a.block >> 4);
  const uint32_t tps = (cols + TILE - 1) / TILE;
  const uint32_t stripe = blockIdx.x / tps;
  const uint32_t c0 = (blockIdx.x - stripe * tps) * TILE + threadIdx.x;

  // Stage the r*k product tables (256 B each) into LDS, 16 B per lane.
  const uint32_t tab16 = r * k * 16;
  for (uint32_t t = threadIdx.x; t < tab16; t += kThreads)
    reinterpret_cast<u32x4 *>(lds_tab)[t] =
        reinterpret_cast<const u32x4 *>(a.btab)[t];

  u32x4 x[KM][U];
#pragma unroll
  for (int j = 0; j < KM; j++) {
    if (j < static_cast<int>(k)) {
      const u32x4 *p = reinterpret_cast<const u32x4 *>(
          a.in[j] + static_cast<uint64_t>(stripe) * a.in_stride[j]);
#pragma unroll
      for (int u = 0; u < U; u++) {
        const uint32_t c = c0 + u * kThreads;
        x[j][u] = c < cols ? p[c] : u32x4{0, 0, 0, 0};
      }
    }
  }
  __syncthreads();

  u32x4 acc[RM][U];
#pragma unroll
  for (int i = 0; i < RM; i++)
#pragma unroll
    for (int u = 0; u < U; u++) acc[i][u] = u32x4{0, 0, 0, 0};

#pragma unroll
  for (int j = 0; j < KM; j++) {
    if (j >= static_cast<int>(k)) continue;
#pragma unroll
    for (int u = 0; u < U; u++) {
#pragma unroll
      for (int w = 0; w < 4; w++) {
        const uint32_t d = x[j][u][w];
#pragma unroll
        for (int i = 0; i < RM; i++) {
          if (i >= static_cast<int>(r)) continue;
          const uint8_t *row = lds_tab + (i * k + j) * 256u;
          acc[i][u][w] ^= static_cast<uint32_t>(row[d & 0xFF]) |
                          static_cast<uint32_t>(row[(d >> 8) & 0xFF]) << 8 |
                          static_cast<uint32_t>(row[(d >> 16) & 0xFF]) << 16 |
                          static_cast<uint32_t>(row[d >> 24]) << 24;
        }
      }
    }
  }

#pragma unroll
  for (int i = 0; i < RM; i++) {
    if (i >= static_cast<int>(r)) continue;
    u32x4 *q = reinterpret_cast<u32x4 *>(
        a.out[i] + static_cast<uint64_t>(stripe) * a.out_stride[i]);
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint32_t c = c0 + u * kThreads;
      if (c < cols) {
        u32x4 v = acc[i][u];
        if (a.accumulate) v ^= q[c];
        q[c] = v;
      }
    }
  }
}

inline int pow2_bucket(uint32_t v) {  // smallest power of two >= v
  int b = 1;
  while (b < static_cast<int>(v)) b <<= 1;
  return b;
}

template <int KM>
inline uint64_t tile_blocks(const ApplyArgs &a) {
  constexpr uint32_t TILE = kThreads * Unroll<KM>::U;
  const uint64_t cols = a.block >> 4;
  return ((cols + TILE - 1) / TILE) * a.nstripes;
}

template <int KM, int RM>
hipError_t go_perm(const ApplyArgs &a, hipStream_t s) {
  const uint64_t blocks = tile_blocks<KM>(a);
  if (blocks == 0) return hipSuccess;
  if (blocks > 0x7FFFFFFFull) return hipErrorInvalidConfiguration;
  if (a.k == KM && a.r == RM)
    hipLaunchKernelGGL((rs_apply_perm<KM, RM, true>), dim3(blocks), dim3(kThreads),
                       0, s, a);
  else
    hipLaunchKernelGGL((rs_apply_perm<KM, RM, false>), dim3(blocks),
                       dim3(kThreads), 0, s, a);
  return hipGetLastError();
}

template <int KM>
hipError_t go_perm_r(const ApplyArgs &a, hipStream_t s) {
  switch (pow2_bucket(a.r)) {
    case 1: return go_perm<KM, 1>(a, s);
    case 2: return go_perm<KM, 2>(a, s);
    case 4: return go_perm<KM, 4>(a, s);
    case 8: return go_perm<KM, 8>(a, s);
    default: return go_perm<KM, 16>(a, s);
  }
}

// One translation unit per KM bucket (rs_perm_k*.hip) so hipcc can build
// the instantiations in parallel.
hipError_t dispatch_perm_k1(const ApplyArgs &a, hipStream_t s);
hipError_t dispatch_perm_k2(const ApplyArgs &a, hipStream_t s);
hipError_t dispatch_perm_k4(const ApplyArgs &a, hipStream_t s);
hipError_t dispatch_perm_k8(const ApplyArgs &a, hipStream_t s);
hipError_t dispatch_perm_k16(const ApplyArgs &a, hipStream_t s);
hipError_t dispatch_perm_k32(const ApplyArgs &a, hipStream_t s);
hipError_t dispatch_lds(const ApplyArgs &a, hipStream_t s);

}  // namespace storb_rs
