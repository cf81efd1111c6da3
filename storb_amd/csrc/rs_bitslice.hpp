// rs_bitslice.hpp -- bit-sliced encode kernels for Storb's wide geometries.
//
// What the reference computes: zfec's encode (piece.rs:329 -> Fec::encode),
// parity_p = XOR_j enc[k+p][j] * data_j over GF(2^8). Storb chunks an object
// at piece_length(len) (a power of two, upload.rs:209) and sizes every full
// chunk with get_k_and_m (piece.rs:307-317): objects of 1 GiB and up give
// 8-32 MiB chunks, i.e. (k, n) = (16, 24) or (32, 48). For those the
// v_perm_b32 kernel (rs_device.hpp) is VALU-bound: ~5.6 VALU ops per
// (input, output, dword), i.e. ~7.5 ops per HBM byte at RS(16,8).
//
// Here the encode matrix is a compile-time constant (it depends only on k and
// n), so each multiplication by enc[o][j] becomes a fixed 8x8 GF(2) bit
// matrix and the whole encode a fixed XOR network:
//  * Each lane holds 32 bytes of a share (two dwordx4 loads, each a
//    contiguous 1 KiB per wave). A 3-layer SWAPMOVE network turns the 8
//    dwords into 8 bit-planes (plane b = bit b of all 32 bytes): ~4 VALU ops
//    per SWAPMOVE, 12 SWAPMOVEs per input, amortised over every output row.
//  * Method of Four Russians: per input, the 15 XOR combinations of planes
//    0-3 and of planes 4-7 (22 XORs; unused ones are dead code). Every output
//    plane row is then acc ^= LO[row & 15] ^ HI[row >> 4]: ONE v_bitop3_b32
//    per (output, plane, input) for 32 bytes, i.e. 0.25 ops per
//    (input, output, byte) against 1.4 for the v_perm form.
//  * After the last input the output planes are transposed back (the
//    network is an involution) and stored with two dwordx4 stores.
// Bit-exactness against the oracle is tested (tests/test_gpu_parity.py).
#pragma once

#include <hip/hip_runtime.h>

#include <utility>

#include "rs_kernels.hpp"

namespace storb_rs {
namespace bs {

// ---------------------------------------------------------------- constexpr
// GF(2^8) with 0x11D, alpha = 2 (fec.c generate_gf).
struct GFc {
  uint8_t exp[512];
  uint8_t log[256];
};

constexpr GFc make_gf() {
  GFc g{};
  unsigned x = 1;
  for (int i = 0; i < 255; i++) {
    g.exp[i] = static_cast<uint8_t>(x);
    g.log[x] = static_cast<uint8_t>(i);
    x <<= 1;
    if (x & 0x100) x ^= 0x11D;
  }
  for (int i = 255; i < 512; i++) g.exp[i] = g.exp[i - 255];
  return g;
}

constexpr uint8_t gmul(const GFc &g, uint8_t a, uint8_t b) {
  return (a == 0 || b == 0) ? 0 : g.exp[g.log[a] + g.log[b]];
}

constexpr uint8_t ginv(const GFc &g, uint8_t a) { return g.exp[255 - g.log[a]]; }

// enc[k + p][j] in closed (Lagrange) form -- the unique systematic generator
// with evaluation points {0, alpha^0, alpha^1, ...},
// equal to V_bot * V_top^-1 (host gf256.hpp computes it by inversion; the
// GPU tests compare the two through the oracle).
template <int K, int N>
struct Bits {
  // row[p][j][b]: bit b' of row[p][j][b] = bit b of enc[k+p][j] * 2^b'.
  uint8_t row[N - K][K][8];
};

template <int K, int N>
constexpr Bits<K, N> make_bits();

template <int K, int N>
struct Net {
  static constexpr Bits<K, N> bits = make_bits<K, N>();
};

template <int K, int N>
constexpr Bits<K, N> make_bits() {
  const GFc g = make_gf();
  uint8_t xs[N] = {};
  for (int i = 1; i < N; i++) xs[i] = g.exp[i - 1];
  Bits<K, N> out{};
  for (int p = 0; p < N - K; p++) {
    const uint8_t xr = xs[K + p];
    for (int j = 0; j < K; j++) {
      uint8_t num = 1, den = 1;
      for (int l = 0; l < K; l++) {
        if (l == j) continue;
        num = gmul(g, num, static_cast<uint8_t>(xr ^ xs[l]));
        den = gmul(g, den, static_cast<uint8_t>(xs[j] ^ xs[l]));
      }
      const uint8_t c = gmul(g, num, ginv(g, den));
      for (int b = 0; b < 8; b++) {
        uint8_t m = 0;
        for (int bp = 0; bp < 8; bp++)
          if ((gmul(g, c, static_cast<uint8_t>(1u << bp)) >> b) & 1u) m |= 1u << bp;
        out.row[p][j][b] = m;
      }
    }
  }
  return out;
}

// ------------------------------------------------------------------ device
typedef uint32_t v4 __attribute__((ext_vector_type(4)));

// Compile-time loop: f(std::integral_constant<int, I>) for I in [0, N).
// The network's indices must be constants; #pragma unroll gives up on
// bodies this large and falls back to dynamic VGPR indexing.
template <typename F, int... I>
__device__ __forceinline__ void static_for_impl(F &&f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void static_for(F &&f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}

// (m & x) | (~m & y) as one v_bitop3_b32 (truth table over the operand
// constants 0xF0/0xCC/0xAA, as LLVM encodes it). Written as the builtin so
// InstCombine cannot re-split the selects of consecutive layers into extra
// v_and_b32s (it did: +15 ops per transpose).
__device__ __forceinline__ uint32_t sel(uint32_t m, uint32_t x, uint32_t y) {
  return __builtin_amdgcn_bitop3_b32(m, x, y, 0xCA);
}

// Exchange bit S of the position with bit log2(S) of the register index
// between registers lo (index bit clear) and hi (index bit set): 4 VALU ops.
template <int S, uint32_t M>
__device__ __forceinline__ void swapmove(uint32_t &lo, uint32_t &hi) {
  const uint32_t l = lo, h = hi;
  lo = sel(M << S, h << S, l);
  hi = sel(M, l >> S, h);
}

// 8 dwords (32 bytes; byte q of dword r at bit 8q..8q+7 of x[r]) <-> 8
// bit-planes (bit b of byte q of dword r at bit 8q + r of x[b]). The three
// layers act on disjoint index bits, so the network is its own inverse.
__device__ __forceinline__ void transpose8(uint32_t (&x)[8]) {
  swapmove<1, 0x55555555u>(x[0], x[1]);
  swapmove<1, 0x55555555u>(x[2], x[3]);
  swapmove<1, 0x55555555u>(x[4], x[5]);
  swapmove<1, 0x55555555u>(x[6], x[7]);
  swapmove<2, 0x33333333u>(x[0], x[2]);
  swapmove<2, 0x33333333u>(x[1], x[3]);
  swapmove<2, 0x33333333u>(x[4], x[6]);
  swapmove<2, 0x33333333u>(x[5], x[7]);
  swapmove<4, 0x0F0F0F0Fu>(x[0], x[4]);
  swapmove<4, 0x0F0F0F0Fu>(x[1], x[5]);
  swapmove<4, 0x0F0F0F0Fu>(x[2], x[6]);
  swapmove<4, 0x0F0F0F0Fu>(x[3], x[7]);
}

__device__ __forceinline__ uint32_t x3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

__device__ __forceinline__ v4 ld_nt(const v4 *p) { return __builtin_nontemporal_load(p); }
// Stores: default write-back policy unless STORB_RS_NT_STORES (rs_device.hpp).
__device__ __forceinline__ void st_nt(v4 *p, v4 v) {
#if STORB_RS_NT_STORES
  __builtin_nontemporal_store(v, p);
#else
  *p = v;
#endif
}

// One share's 32 bytes (already bit-sliced) folded into the R x 8
// accumulator planes with the Four-Russians tables.
template <int K, int N, int J>
__device__ __forceinline__ void fold_planes(uint32_t (&acc)[N - K][8], const uint32_t (&x)[8]) {
  uint32_t lo[16], hi[16];
  lo[0] = 0;
  hi[0] = 0;
#pragma unroll
  for (int m = 1; m < 16; m++) {
    const int b = __builtin_ctz(m), rest = m & (m - 1);
    lo[m] = rest ? lo[rest] ^ x[b] : x[b];
    hi[m] = rest ? hi[rest] ^ x[4 + b] : x[4 + b];
  }
#pragma unroll
  for (int p = 0; p < N - K; p++) {
#pragma unroll
    for (int b = 0; b < 8; b++) {
      const int row = Net<K, N>::bits.row[p][J][b];
      const int l = row & 15, h = row >> 4;
      if (l && h)
        acc[p][b] = x3(acc[p][b], lo[l], hi[h]);
      else if (l)
        acc[p][b] ^= lo[l];
      else if (h)
        acc[p][b] ^= hi[h];
    }
  }
}

// The loads of one group of G shares: 2 x dwordx4 per share and lane, at the
// lane's two (clamped) column indices ca / cb.
template <int G>
__device__ __forceinline__ void load_group(const ApplyArgs &a, int j0, uint32_t stripe,
                                           uint32_t ca, uint32_t cb, v4 (&buf)[G][2]) {
#pragma unroll
  for (int g = 0; g < G; g++) {
    const v4 *p = reinterpret_cast<const v4 *>(a.in[j0 + g] +
                                               static_cast<uint64_t>(stripe) * a.in_stride[j0 + g]);
    buf[g][0] = ld_nt(p + ca);
    buf[g][1] = ld_nt(p + cb);
  }
}

// Shares are consumed in groups of G; group i+1's loads are issued before
// group i is folded (double buffer), and sched_barriers keep the compiler
// from hoisting every later load above the folds (register blow-up).
template <int R>
__device__ __forceinline__ void fence_acc(uint32_t (&acc)[R][8]) {
#pragma unroll
  for (int p = 0; p < R; p++)
    asm volatile("" : "+v"(acc[p][0]), "+v"(acc[p][1]), "+v"(acc[p][2]), "+v"(acc[p][3]),
                 "+v"(acc[p][4]), "+v"(acc[p][5]), "+v"(acc[p][6]), "+v"(acc[p][7]));
}

// Ragged last tile: lanes past the share end load a clamped (valid) column
// and store nothing. Bit-slicing keeps every byte in its own bit position,
// so the garbage never reaches a stored byte -- one branch-free body for
// full and partial tiles (a separate guarded body doubled the VGPRs).
template <int K, int N, int G>
__device__ __forceinline__ void encode_tile(const ApplyArgs &a, uint32_t stripe, uint32_t v0,
                                            uint32_t cols) {
  constexpr int R = N - K;
  static_assert(K % G == 0, "group size must divide k");
  uint32_t acc[R][8];
#pragma unroll
  for (int p = 0; p < R; p++)
#pragma unroll
    for (int b = 0; b < 8; b++) acc[p][b] = 0;

  v4 buf[2][G][2];
  const uint32_t ca = v0 < cols ? v0 : cols - 1, cb = v0 + 64 < cols ? v0 + 64 : cols - 1;
  load_group<G>(a, 0, stripe, ca, cb, buf[0]);
  static_for<K / G>([&](auto GI) {
    constexpr int gi = decltype(GI)::value;
    if constexpr (gi + 1 < K / G)
      load_group<G>(a, (gi + 1) * G, stripe, ca, cb, buf[(gi + 1) & 1]);
    static_for<G>([&](auto GG) {
      constexpr int g = decltype(GG)::value;
      const v4 &A = buf[gi & 1][g][0], &Bv = buf[gi & 1][g][1];
      uint32_t x[8] = {A[0], A[1], A[2], A[3], Bv[0], Bv[1], Bv[2], Bv[3]};
      // Ordering point: share j's bit-slicing cannot be hoisted above the
      // previous share's fold (volatile asms keep their order), which bounds
      // the live tables to one share.
      asm volatile("" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]),
                   "+v"(x[6]), "+v"(x[7]));
      transpose8(x);
      fold_planes<K, N, gi * G + g>(acc, x);
      // ... and the accumulators pass through the same kind of point after
      // every share, so the Reassociate pass cannot regroup the 16-32 term
      // XOR chains across shares (which kept many shares' tables alive).
      fence_acc(acc);
    });
  });

#pragma unroll
  for (int p = 0; p < R; p++) {
    transpose8(acc[p]);
    v4 *q = reinterpret_cast<v4 *>(a.out[p] + static_cast<uint64_t>(stripe) * a.out_stride[p]);
    const v4 A = {acc[p][0], acc[p][1], acc[p][2], acc[p][3]};
    const v4 Bv = {acc[p][4], acc[p][5], acc[p][6], acc[p][7]};
    if (v0 < cols) st_nt(q + v0, A);
    if (v0 + 64 < cols) st_nt(q + v0 + 64, Bv);
  }
}

// Group size per geometry: whole k in flight where the registers allow it.
template <int K, int N>
struct BsTune {
  // resident workgroups per CU (rs_kernels.hpp wg_cap): RS(16,8) 0.281 ->
  // 0.275 ms at 2 (= 3; tools/occ_sweep.py, profiles/r1_occupancy.txt)
  static constexpr int OCC = K == 16 ? 2 : 0;
  static constexpr int G = K <= 8 ? K : ((N - K) >= 16 ? 2 : 4);
};

// Grid: nstripes x tiles; a tile = 256 lanes x 32 B = 8 KiB of every share.
// Wave w of the tile covers 2 KiB: lane l holds the 16-B columns
// (w*128 + l) and (w*128 + 64 + l) of the tile, so each load and store
// instruction moves one contiguous 1 KiB per wave.
template <int K, int N>
__global__ __launch_bounds__(256) void rs_encode_bitslice(const ApplyArgs a) {
  const uint32_t cols = static_cast<uint32_t>(a.block >> 4);
  const uint32_t tps = (cols + 511) / 512;
  const uint32_t stripe = blockIdx.x / tps;
  const uint32_t tile = blockIdx.x - stripe * tps;
  const uint32_t v0 = tile * 512 + (threadIdx.x >> 6) * 128 + (threadIdx.x & 63);
  encode_tile<K, N, BsTune<K, N>::G>(a, stripe, v0, cols);
}

template <int K, int N>
hipError_t launch_bitslice(const ApplyArgs &a, hipStream_t s) {
  const uint64_t cols = a.block >> 4;
  const uint64_t blocks = ((cols + 511) / 512) * a.nstripes;
  if (blocks == 0) return hipSuccess;
  if (blocks > 0x7FFFFFFFull) return hipErrorInvalidConfiguration;
  return launch_lds<rs_encode_bitslice<K, N>>(blocks, 256,
                                               cap_lds(wg_cap(BsTune<K, N>::OCC), 0), s, a);
}

}  // namespace bs
}  // namespace storb_rs
