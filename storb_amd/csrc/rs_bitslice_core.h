// rs_bitslice_core.h -- bit-sliced GF(2^8) matrix application with the
// matrix compiled in, for any (R x K) matrix type M.
//
// Two users:
//  * rs_bitslice.hpp: the ahead-of-time encoders for Storb's wide
//    full-chunk geometries (k, n) = (16, 24), (32, 48) -- M = the generator's
//    parity rows, computed constexpr;
//  * rs_jit.cpp: decode / repair matrices known only at run time (rows of the
//    inverted survivor matrix, piece.rs:384-386 Fec::decode) -- the host
//    writes M out as a constexpr table and compiles this header with hipRTC,
//    once per matrix, keeping the v_perm kernel for the calls that arrive
//    while it compiles.
// Self-contained (no standard headers) so hipRTC takes it as an in-memory
// header next to rs_args.h.
//
// Method: a lane holds 32 bytes of a share (two dwordx4 loads,
// each a contiguous 1 KiB per wave); a 3-layer SWAPMOVE network turns the 8
// dwords into 8 bit-planes; multiplication by a constant is then a fixed 8x8
// GF(2) bit matrix. Per input the 15 XOR combinations of planes 0-3 and of
// planes 4-7 are formed (Method of Four Russians) and every output plane row
// is acc ^= LO[row & 15] ^ HI[row >> 4]: one v_bitop3_b32 per (output,
// plane, input) for 32 bytes. Outputs go back through the (involutive)
// network before the stores.
//
// M provides: static constexpr int K, R; static constexpr unsigned long long
// copy_mask (bit j: input j is also stored, as loaded, to a.copy[j] -- fused
// assembly of a decode into a separate chunk buffer); static constexpr
// <struct> net with net.row[R][K][8], where bit b' of row[p][j][b] is bit b
// of M[p][j] * 2^b'.
#pragma once

#include "rs_args.h"

#ifndef STORB_RS_NT_STORES
#define STORB_RS_NT_STORES 1
#endif
// 64-bit shifts in two of the transposition's three layers (transpose8).
#ifndef STORB_BS_SHIFT64
#define STORB_BS_SHIFT64 1
#endif

namespace storb_rs {
namespace bs {

typedef uint32_t v4 __attribute__((ext_vector_type(4)));

// Compile-time loop: f(ic<I>) for I in [0, N). The network's indices must
// be constants; #pragma unroll gives up on bodies this large and falls back
// to dynamic VGPR indexing.
template <typename T, T... I>
struct iseq {};
template <int I>
struct ic {
  static constexpr int value = I;
};
template <typename F, int... I>
__device__ __forceinline__ void static_for_impl(F &&f, iseq<int, I...>) {
  (f(ic<I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void static_for(F &&f) {
  static_for_impl(f, __make_integer_seq<iseq, int, N>{});
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
template <int S, uint32_t Mk>
__device__ __forceinline__ void swapmove(uint32_t &lo, uint32_t &hi) {
  const uint32_t l = lo, h = hi;
  lo = sel(Mk << S, h << S, l);
  hi = sel(Mk, l >> S, h);
}

// Two swapmoves at once, (x[i], x[i+D]) and (x[i+1], x[i+1+D]) for even i:
// the two lo registers and the two hi registers each shift as one 64-bit
// value (v_lshrrev_b64 / v_lshlrev_b64 on an aligned register pair, full rate
// on gfx950: tools/valu64_probe.hip). The bits that cross the dword boundary
// land where the masks are zero (Mk's top S bits, (Mk << S)'s low S bits), so
// the selects are unchanged: 6 VALU ops for two swaps instead of 8.
template <int S, uint32_t Mk>
__device__ __forceinline__ void swapmove2(uint32_t &lo0, uint32_t &lo1, uint32_t &hi0,
                                          uint32_t &hi1) {
  const uint64_t l = (static_cast<uint64_t>(lo1) << 32) | lo0;
  const uint64_t h = (static_cast<uint64_t>(hi1) << 32) | hi0;
  // asm: LLVM splits a 64-bit shift whose halves are used apart into
  // v_alignbit + a 32-bit shift (and rebuilds pairs with v_mov / v_or)
  uint64_t hs, ls;
  asm("v_lshlrev_b64 %0, %2, %1" : "=v"(hs) : "v"(h), "n"(S));
  asm("v_lshrrev_b64 %0, %2, %1" : "=v"(ls) : "v"(l), "n"(S));
  const uint32_t l0 = lo0, l1 = lo1, h0 = hi0, h1 = hi1;
  lo0 = sel(Mk << S, static_cast<uint32_t>(hs), l0);
  lo1 = sel(Mk << S, static_cast<uint32_t>(hs >> 32), l1);
  hi0 = sel(Mk, static_cast<uint32_t>(ls), h0);
  hi1 = sel(Mk, static_cast<uint32_t>(ls >> 32), h1);
}

// 8 dwords (32 bytes; byte q of dword r at bit 8q..8q+7 of x[r]) <-> 8
// bit-planes (bit b of byte q of dword r at bit 8q + r of x[b]). The three
// layers act on disjoint index bits, so they commute and the network is its
// own inverse. The index-bit-2 and index-bit-1 layers pair registers that
// sit in aligned pairs (x[0..3] / x[4..7] come from dwordx4 loads) and run as
// swapmove2; the index-bit-0 layer pairs the two halves of one register pair
// and stays 32-bit. 40 VALU ops per transpose (48 with 32-bit shifts only).
__device__ __forceinline__ void transpose8(uint32_t (&x)[8]) {
#if STORB_BS_SHIFT64
  swapmove2<4, 0x0F0F0F0Fu>(x[0], x[1], x[4], x[5]);
  swapmove2<4, 0x0F0F0F0Fu>(x[2], x[3], x[6], x[7]);
  swapmove2<2, 0x33333333u>(x[0], x[1], x[2], x[3]);
  swapmove2<2, 0x33333333u>(x[4], x[5], x[6], x[7]);
#else
  swapmove<4, 0x0F0F0F0Fu>(x[0], x[4]);
  swapmove<4, 0x0F0F0F0Fu>(x[1], x[5]);
  swapmove<4, 0x0F0F0F0Fu>(x[2], x[6]);
  swapmove<4, 0x0F0F0F0Fu>(x[3], x[7]);
  swapmove<2, 0x33333333u>(x[0], x[2]);
  swapmove<2, 0x33333333u>(x[1], x[3]);
  swapmove<2, 0x33333333u>(x[4], x[6]);
  swapmove<2, 0x33333333u>(x[5], x[7]);
#endif
  swapmove<1, 0x55555555u>(x[0], x[1]);
  swapmove<1, 0x55555555u>(x[2], x[3]);
  swapmove<1, 0x55555555u>(x[4], x[5]);
  swapmove<1, 0x55555555u>(x[6], x[7]);
}

__device__ __forceinline__ uint32_t x3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// Loads: non-temporal (shares are read once) unless STORB_BS_LOAD_NT=0
// (the removed k64pair probe, profiles/r2_k64/k64pair.txt: whether cached loads let a
// second reader hit).
#ifndef STORB_BS_LOAD_NT
#define STORB_BS_LOAD_NT 1
#endif
__device__ __forceinline__ v4 ld_nt(const v4 *p) {
#if STORB_BS_LOAD_NT
  return __builtin_nontemporal_load(p);
#else
  return *p;
#endif
}
// Stores: non-temporal unless STORB_RS_NT_STORES=0 (shares are touched once;
// nt stores measured 5-9 % faster in steady state, profiles/r1_store_policy.txt).
__device__ __forceinline__ void st_nt(v4 *p, v4 v) {
#if STORB_RS_NT_STORES
  __builtin_nontemporal_store(v, p);
#else
  *p = v;
#endif
}

// The Four-Russians tables of one share's 32 bytes (already bit-sliced):
// lo[m] / hi[m] = XOR of the planes 0-3 / 4-7 selected by the bits of m.
__device__ __forceinline__ void make_tables(const uint32_t (&x)[8], uint32_t (&lo)[16],
                                            uint32_t (&hi)[16]) {
  lo[0] = 0;
  hi[0] = 0;
#pragma unroll
  for (int m = 1; m < 16; m++) {
    const int b = __builtin_ctz(m), rest = m & (m - 1);
    lo[m] = rest ? lo[rest] ^ x[b] : x[b];
    hi[m] = rest ? hi[rest] ^ x[4 + b] : x[4 + b];
  }
}

// Share J's tables folded into the R x 8 accumulator planes.
template <class M, int J>
__device__ __forceinline__ void fold_tables(uint32_t (&acc)[M::R][8], const uint32_t (&lo)[16],
                                            const uint32_t (&hi)[16]) {
#pragma unroll
  for (int p = 0; p < M::R; p++) {
#pragma unroll
    for (int b = 0; b < 8; b++) {
      const int row = M::net.row[p][J][b];
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

// One share's 32 bytes (already bit-sliced) folded into the R x 8
// accumulator planes with the Four-Russians tables.
template <class M, int J>
__device__ __forceinline__ void fold_planes(uint32_t (&acc)[M::R][8], const uint32_t (&x)[8]) {
  uint32_t lo[16], hi[16];
  make_tables(x, lo, hi);
  fold_tables<M, J>(acc, lo, hi);
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

// Accumulators pass through an empty volatile asm after every share, so the
// Reassociate pass cannot regroup the 16-32 term XOR chains across shares
// (which kept many shares' tables alive: 424 VGPRs at k = 16 without it).
template <int R>
__device__ __forceinline__ void fence_acc(uint32_t (&acc)[R][8]) {
#pragma unroll
  for (int p = 0; p < R; p++)
    asm volatile("" : "+v"(acc[p][0]), "+v"(acc[p][1]), "+v"(acc[p][2]), "+v"(acc[p][3]),
                 "+v"(acc[p][4]), "+v"(acc[p][5]), "+v"(acc[p][6]), "+v"(acc[p][7]));
}

// Shares are consumed in groups of G; group i+1's loads are issued before
// group i is folded (double buffer). Ragged last tile: lanes past the share
// end load a clamped (valid) column and store nothing. Bit-slicing keeps
// every byte in its own bit position, so the garbage never reaches a stored
// byte -- one branch-free body for full and partial tiles.
template <class M, int G>
__device__ __forceinline__ void bs_tile_to(const ApplyArgs &a, uint8_t *const *outp,
                                           const uint64_t *out_stride, uint32_t stripe,
                                           uint32_t v0, uint32_t cols) {
  constexpr int K = M::K, R = M::R;
  static_assert(K % G == 0, "group size must divide k");
  uint32_t acc[R][8];
#pragma unroll
  for (int p = 0; p < R; p++)
#pragma unroll
    for (int b = 0; b < 8; b++) acc[p][b] = 0;

  v4 buf[2][G][2];
  uint32_t ca = v0 < cols ? v0 : cols - 1, cb = v0 + 64 < cols ? v0 + 64 : cols - 1;
  load_group<G>(a, 0, stripe, ca, cb, buf[0]);
  static_for<K / G>([&](auto GI) {
    constexpr int gi = decltype(GI)::value;
    // k > 32: the load addresses pass through an ordering point, so group
    // gi + 1's loads cannot be hoisted above group gi - 1's fold (with 32+
    // groups the scheduler otherwise ran many groups ahead and spilled).
    if constexpr (K > 32) asm volatile("" : "+v"(ca), "+v"(cb));
    if constexpr (gi + 1 < K / G)
      load_group<G>(a, (gi + 1) * G, stripe, ca, cb, buf[(gi + 1) & 1]);
    static_for<G>([&](auto GG) {
      constexpr int g = decltype(GG)::value;
      constexpr int j = gi * G + g;
      const v4 &A = buf[gi & 1][g][0], &Bv = buf[gi & 1][g][1];
      if constexpr (((M::copy_mask >> j) & 1ull) != 0) {
        v4 *c = reinterpret_cast<v4 *>(a.copy[j] + static_cast<uint64_t>(stripe) * a.copy_stride[j]);
        if (v0 < cols) st_nt(c + v0, A);
        if (v0 + 64 < cols) st_nt(c + v0 + 64, Bv);
      }
      uint32_t x[8] = {A[0], A[1], A[2], A[3], Bv[0], Bv[1], Bv[2], Bv[3]};
      // Ordering point: share j's bit-slicing cannot be hoisted above the
      // previous share's fold, which bounds the live tables to one share.
      asm volatile("" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]),
                   "+v"(x[6]), "+v"(x[7]));
      transpose8(x);
      fold_planes<M, j>(acc, x);
      fence_acc(acc);
    });
  });

#pragma unroll
  for (int p = 0; p < R; p++) {
    transpose8(acc[p]);
    v4 *q = reinterpret_cast<v4 *>(outp[p] + static_cast<uint64_t>(stripe) * out_stride[p]);
    const v4 A = {acc[p][0], acc[p][1], acc[p][2], acc[p][3]};
    const v4 Bv = {acc[p][4], acc[p][5], acc[p][6], acc[p][7]};
    if (v0 < cols) st_nt(q + v0, A);
    if (v0 + 64 < cols) st_nt(q + v0 + 64, Bv);
  }
}

template <class M, int G>
__device__ __forceinline__ void bs_tile(const ApplyArgs &a, uint32_t stripe, uint32_t v0,
                                        uint32_t cols) {
  bs_tile_to<M, G>(a, a.out, a.out_stride, stripe, v0, cols);
}

// Grid: nstripes x tiles of bs_cols_per_tile(T) 16-B columns (rs_args.h);
// T lanes per workgroup, each wave covering 2 KiB of every share. SWZ = 1
// rotates the tile order of stripe s by s * (tiles / 8 + 1), so the
// workgroups of neighbouring stripes that run at the same moment stream
// from different offsets of their shares (profiles/r2_wide_probe_2.txt).
// ------------------------------------------------------------ row-split form
// Matrices of more than 16 rows (Storb's k = 64 geometry: 32 parity rows,
// and decodes losing more than 16 shares of it). One lane cannot hold 32 x 8
// accumulator planes, so round 1 ran two 16-row launches that each read and
// bit-sliced every input: 160 bytes moved per 96 algorithmic and the
// transposes done twice. Here the two waves of a 128-lane workgroup cover
// the SAME 2 KiB of every share and split the rows: wave w folds rows
// [w ? RA : 0, w ? R : RA). Each input is loaded and transposed once, by the
// wave that owns it (half of every load group), which publishes its 8
// bit-planes through LDS; both waves fold every input into their own rows.
// One barrier per load group, LDS double-buffered by group parity.

// Rows [R0, R1) of matrix M, as a matrix type of their own.
template <class M, int R0, int R1>
struct RowSlice {
  static constexpr int K = M::K, R = R1 - R0;
  static constexpr unsigned long long copy_mask = M::copy_mask;
  struct Net {
    unsigned char row[R][K][8];
  };
  static constexpr Net make() {
    Net n{};
    for (int p = 0; p < R; p++)
      for (int j = 0; j < K; j++)
        for (int b = 0; b < 8; b++) n.row[p][j][b] = M::net.row[R0 + p][j][b];
    return n;
  }
  static constexpr Net net = make();
};

// Launch shape: kSplitThreads lanes, kSplitGroup, kSplitCap (rs_args.h).
// LDS of one workgroup: [group parity][owner wave][G/2 inputs][2 halves][64 lanes].
template <int G>
struct SplitLds {
  v4 v[2 * 2 * (G / 2) * 2 * 64];
};
static_assert(sizeof(SplitLds<2>) == split_lds_bytes(2) && sizeof(SplitLds<4>) == split_lds_bytes(4),
              "rs_args.h split_lds_bytes");

// Waits for this wave's LDS writes, then the workgroup barrier. A compiler
// memory barrier too: no LDS access moves across it. (Not __syncthreads():
// its workgroup-scope fences also wait for the next group's global loads.)
__device__ __forceinline__ void split_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

template <class M, int G, int W>
__device__ __forceinline__ void bs_split_wave(const ApplyArgs &a, uint32_t stripe, uint32_t v0,
                                              uint32_t cols, uint32_t lane, v4 *lds) {
  constexpr int K = M::K, R = M::R, H = G / 2, RA = (R + 1) / 2;
  static_assert(G % 2 == 0 && K % G == 0, "split groups: an even count dividing k");
  using MW = RowSlice<M, W ? RA : 0, W ? R : RA>;
  constexpr int RW = MW::R;
  uint32_t acc[RW][8];
#pragma unroll
  for (int p = 0; p < RW; p++)
#pragma unroll
    for (int b = 0; b < 8; b++) acc[p][b] = 0;

  v4 buf[2][H][2];
  uint32_t ca = v0 < cols ? v0 : cols - 1, cb = v0 + 64 < cols ? v0 + 64 : cols - 1;
  load_group<H>(a, W * H, stripe, ca, cb, buf[0]);
  static_for<K / G>([&](auto GI) {
    constexpr int gi = decltype(GI)::value;
    if constexpr (K > 32) asm volatile("" : "+v"(ca), "+v"(cb));
    if constexpr (gi + 1 < K / G)
      load_group<H>(a, (gi + 1) * G + W * H, stripe, ca, cb, buf[(gi + 1) & 1]);
    // Own inputs: fused-assembly copy, bit-slice, publish, fold.
    static_for<H>([&](auto HH) {
      constexpr int h = decltype(HH)::value;
      constexpr int j = gi * G + W * H + h;
      const v4 &A = buf[gi & 1][h][0], &Bv = buf[gi & 1][h][1];
      if constexpr (((M::copy_mask >> j) & 1ull) != 0) {
        v4 *c = reinterpret_cast<v4 *>(a.copy[j] + static_cast<uint64_t>(stripe) * a.copy_stride[j]);
        if (v0 < cols) st_nt(c + v0, A);
        if (v0 + 64 < cols) st_nt(c + v0 + 64, Bv);
      }
      uint32_t x[8] = {A[0], A[1], A[2], A[3], Bv[0], Bv[1], Bv[2], Bv[3]};
      asm volatile("" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]),
                   "+v"(x[6]), "+v"(x[7]));
      transpose8(x);
      v4 *slot = lds + ((((gi & 1) * 2 + W) * H + h) * 2) * 64 + lane;
      slot[0] = v4{x[0], x[1], x[2], x[3]};
      slot[64] = v4{x[4], x[5], x[6], x[7]};
      fold_planes<MW, j>(acc, x);
      fence_acc(acc);
    });
    split_barrier();
    // The other wave's inputs of this group, from LDS.
    static_for<H>([&](auto HH) {
      constexpr int h = decltype(HH)::value;
      constexpr int j = gi * G + (1 - W) * H + h;
      const v4 *slot = lds + ((((gi & 1) * 2 + (1 - W)) * H + h) * 2) * 64 + lane;
      const v4 P = slot[0], Q = slot[64];
      uint32_t x[8] = {P[0], P[1], P[2], P[3], Q[0], Q[1], Q[2], Q[3]};
      fold_planes<MW, j>(acc, x);
      fence_acc(acc);
    });
  });

  constexpr int r0 = W ? RA : 0;
#pragma unroll
  for (int p = 0; p < RW; p++) {
    transpose8(acc[p]);
    v4 *q = reinterpret_cast<v4 *>(a.out[r0 + p] + static_cast<uint64_t>(stripe) * a.out_stride[r0 + p]);
    const v4 A = {acc[p][0], acc[p][1], acc[p][2], acc[p][3]};
    const v4 Bv = {acc[p][4], acc[p][5], acc[p][6], acc[p][7]};
    if (v0 < cols) st_nt(q + v0, A);
    if (v0 + 64 < cols) st_nt(q + v0 + 64, Bv);
  }
}

// Grid: nstripes x tiles of kSplitColsPerTile columns, kSplitThreads lanes.
// (Sharing the Four-Russians tables instead of the planes measured slower,
// 366.9 -> 387.9 us at k = 64, profiles/r2_k64/k64split_tables.txt; removed.)
template <class M, int G, int SWZ = 0>
__device__ __forceinline__ void bs_split_body(const ApplyArgs &a) {
  __shared__ SplitLds<G> lds;
  constexpr uint32_t CPT = kSplitColsPerTile;
  const uint32_t cols = static_cast<uint32_t>(a.block >> 4);
  const uint32_t tps = (cols + CPT - 1) / CPT;
  const uint32_t stripe = blockIdx.x / tps;
  uint32_t tile = blockIdx.x - stripe * tps;
  if constexpr (SWZ == 1) tile = (tile + stripe * (tps / 8 + 1)) % tps;
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t v0 = tile * CPT + lane;
  // wave-uniform (an SGPR), so the two row halves are scalar branches
  if (__builtin_amdgcn_readfirstlane(threadIdx.x >> 6) == 0)
    bs_split_wave<M, G, 0>(a, stripe, v0, cols, lane, lds.v);
  else
    bs_split_wave<M, G, 1>(a, stripe, v0, cols, lane, lds.v);
}

// ------------------------------------------------------------ input-split form
// A workgroup of C x W waves covers C x 2 KiB (128 16-B columns per column
// group) of every share. The W waves of a column group cover the SAME 2 KiB
// and split the INPUTS: wave w loads, bit-slices and folds inputs
// [w K/W, (w+1) K/W) into partial planes of all R rows; the partials meet in
// LDS and wave w finishes rows [w R/W, (w+1) R/W) (the other waves' partials
// XORed in, inverse transpose, stores). Same VALU as one wave per tile (each
// input transposed and tabled once, each output transposed once) plus R/W x 8
// XORs per partner wave, but W waves per 2 KiB of each share: a CU keeps
// enough waves to overlap the folds with the loads while fewer bytes -- fewer
// DRAM pages -- are in flight (one-wave tiles need 6 per
// CU, 16 shares x 2 KiB each in flight, and stream below the 4 KiB-per-
// workgroup probe shape).
// LDS per column group: [owner wave d][partner q (W-1)][row of d (R/W)][2 halves][64 lanes] x 16 B.
// (ksplit_lds_bytes: rs_args.h)
template <int C, int W, int R>
struct KsplitLds {
  v4 v[ksplit_lds_bytes(C, W, R) / 16];
};

template <class M, int W, int G, int WI>
__device__ __forceinline__ void bs_ksplit_wave(const ApplyArgs &a, uint32_t stripe, uint32_t v0,
                                               uint32_t cols, uint32_t lane, v4 *lds) {
  constexpr int K = M::K, R = M::R, KW = K / W, RW = R / W, J0 = WI * KW;
  static_assert(K % W == 0 && R % W == 0 && KW % G == 0, "input split: W | k, W | r, G | k / W");
  uint32_t acc[R][8];
#pragma unroll
  for (int p = 0; p < R; p++)
#pragma unroll
    for (int b = 0; b < 8; b++) acc[p][b] = 0;

  v4 buf[2][G][2];
  const uint32_t ca = v0 < cols ? v0 : cols - 1, cb = v0 + 64 < cols ? v0 + 64 : cols - 1;
  load_group<G>(a, J0, stripe, ca, cb, buf[0]);
  static_for<KW / G>([&](auto GI) {
    constexpr int gi = decltype(GI)::value;
    if constexpr (gi + 1 < KW / G)
      load_group<G>(a, J0 + (gi + 1) * G, stripe, ca, cb, buf[(gi + 1) & 1]);
    static_for<G>([&](auto GG) {
      constexpr int g = decltype(GG)::value;
      constexpr int j = J0 + gi * G + g;
      const v4 &A = buf[gi & 1][g][0], &Bv = buf[gi & 1][g][1];
      if constexpr (((M::copy_mask >> j) & 1ull) != 0) {
        v4 *c = reinterpret_cast<v4 *>(a.copy[j] + static_cast<uint64_t>(stripe) * a.copy_stride[j]);
        if (v0 < cols) st_nt(c + v0, A);
        if (v0 + 64 < cols) st_nt(c + v0 + 64, Bv);
      }
      uint32_t x[8] = {A[0], A[1], A[2], A[3], Bv[0], Bv[1], Bv[2], Bv[3]};
      asm volatile("" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]),
                   "+v"(x[6]), "+v"(x[7]));
      transpose8(x);
      fold_planes<M, j>(acc, x);
      fence_acc(acc);
    });
  });

  if constexpr (W > 1) {
    // the partials of the rows the other waves own
    static_for<W>([&](auto DI) {
      constexpr int d = decltype(DI)::value;
      if constexpr (d != WI) {
        constexpr int q = WI < d ? WI : WI - 1;
        static_for<RW>([&](auto RR) {
          constexpr int rr = decltype(RR)::value, p = d * RW + rr;
          v4 *slot = lds + (((d * (W - 1) + q) * RW + rr) * 2) * 64 + lane;
          slot[0] = v4{acc[p][0], acc[p][1], acc[p][2], acc[p][3]};
          slot[64] = v4{acc[p][4], acc[p][5], acc[p][6], acc[p][7]};
        });
      }
    });
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    static_for<W - 1>([&](auto QI) {
      constexpr int q = decltype(QI)::value;
      static_for<RW>([&](auto RR) {
        constexpr int rr = decltype(RR)::value, p = WI * RW + rr;
        const v4 *slot = lds + (((WI * (W - 1) + q) * RW + rr) * 2) * 64 + lane;
        const v4 P = slot[0], Q = slot[64];
        acc[p][0] ^= P[0];
        acc[p][1] ^= P[1];
        acc[p][2] ^= P[2];
        acc[p][3] ^= P[3];
        acc[p][4] ^= Q[0];
        acc[p][5] ^= Q[1];
        acc[p][6] ^= Q[2];
        acc[p][7] ^= Q[3];
      });
    });
  }
  static_for<RW>([&](auto RR) {
    constexpr int p = WI * RW + decltype(RR)::value;
    transpose8(acc[p]);
    v4 *q = reinterpret_cast<v4 *>(a.out[p] + static_cast<uint64_t>(stripe) * a.out_stride[p]);
    const v4 A = {acc[p][0], acc[p][1], acc[p][2], acc[p][3]};
    const v4 Bv = {acc[p][4], acc[p][5], acc[p][6], acc[p][7]};
    if (v0 < cols) st_nt(q + v0, A);
    if (v0 + 64 < cols) st_nt(q + v0 + 64, Bv);
  });
}

// Grid: nstripes x tiles of C x 128 16-B columns, 64 C W lanes (wave i:
// column group i / W, input part i % W).
template <class M, int C, int W, int G, int SWZ = 0>
__device__ __forceinline__ void bs_ksplit_body(const ApplyArgs &a) {
  __shared__ KsplitLds<C, W, M::R> lds;
  constexpr uint32_t CPT = 128 * C;
  const uint32_t cols = static_cast<uint32_t>(a.block >> 4);
  const uint32_t tps = (cols + CPT - 1) / CPT;
  const uint32_t stripe = blockIdx.x / tps;
  uint32_t tile = blockIdx.x - stripe * tps;
  if constexpr (SWZ == 1) tile = (tile + stripe * (tps / 8 + 1)) % tps;
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t cg = wid / W, w = wid - cg * W;
  const uint32_t v0 = tile * CPT + cg * 128 + lane;
  v4 *mine = lds.v + cg * (ksplit_lds_bytes(1, W, M::R) / 16);
  static_for<W>([&](auto WI) {
    constexpr int wi = decltype(WI)::value;
    if (w == wi) bs_ksplit_wave<M, W, G, wi>(a, stripe, v0, cols, lane, mine);
  });
}

template <class M, int G, int T = kBsThreads, int SWZ = 0>
__device__ __forceinline__ void bs_kernel_body(const ApplyArgs &a) {
  constexpr uint32_t CPT = bs_cols_per_tile(T);
  const uint32_t cols = static_cast<uint32_t>(a.block >> 4);
  const uint32_t tps = (cols + CPT - 1) / CPT;
  const uint32_t stripe = blockIdx.x / tps;
  uint32_t tile = blockIdx.x - stripe * tps;
  if constexpr (SWZ == 1) tile = (tile + stripe * (tps / 8 + 1)) % tps;
  const uint32_t v0 = tile * CPT + (threadIdx.x >> 6) * 128 + (threadIdx.x & 63);
  bs_tile<M, G>(a, stripe, v0, cols);
}

}  // namespace bs
}  // namespace storb_rs
