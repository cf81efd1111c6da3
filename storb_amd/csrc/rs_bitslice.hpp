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
// matrix and the whole encode a fixed XOR network -- the bit-sliced method of
// rs_bitslice_core.h (shared with the run-time-compiled decode kernels of
// rs_jit.cpp), 0.25 VALU ops per (input, output, byte) against 1.4 for the
// v_perm form. Bit-exactness against the oracle is tested
// (tests/test_gpu_parity.py).
#pragma once

#include <hip/hip_runtime.h>

#include "rs_bitslice_core.h"
#include "rs_stream.hpp"
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
// The generator's parity rows as the matrix type of rs_bitslice_core.h.
template <int K_, int N_>
struct EncMat {
  static constexpr int K = K_, R = N_ - K_;
  static constexpr unsigned long long copy_mask = 0;
  static constexpr Bits<K_, N_> net = make_bits<K_, N_>();
};

// Launch shape per geometry (rs_args.h bs_shape, or the row-split form
// where bs_split says so -- more than 16 parity rows; none of the two AOT
// geometries today).
template <int K, int N>
struct BsTune {
  static constexpr bool SPLIT = bs_split(K, N - K);
  static constexpr BsShape S = bs_shape(K, N - K);
  static constexpr int T = SPLIT ? kSplitThreads : S.threads, SWZ = SPLIT ? 0 : S.swz;
  static constexpr int OCC = SPLIT ? bs_split_cap(N - K) : S.cap;
  static constexpr int G = SPLIT ? kSplitGroup : bs_group(K, N - K);
  static constexpr uint64_t CPT = SPLIT ? kSplitColsPerTile : bs_cols_per_tile(T);
  static constexpr size_t LDS = SPLIT ? split_lds_bytes(kSplitGroup) : 0;
};

// Input-split workgroups (rs_bitslice_core.h bs_ksplit_body) for the batch
// encoders: C column groups of W waves, G shares per load group, CAP resident
// per CU (LDS and registers cap it lower: (16, 24) holds 3 of its 256-lane
// workgroups per CU). tools/bstune.hip BSTUNE_KSPLIT, three sweeps
// (profiles/r6c_bstune_ksplit.txt, r6e_*): (16, 24) 79.3-80.1 % -> 81.0-81.7 %
// of 8 TB/s (C = 1, W = 4), (32, 48) 74.0 -> 75.4 % (C = 2, W = 2); the same
// shapes with no GF work stream at 81.8 / 75.5 % (r6d_bstune_nogf.txt), the
// one-wave tiles at 80.1 / 77.4 %.
template <int K, int N>
struct KsTune {
  static constexpr KsShape S = ks_shape(K, N - K);  // rs_args.h
  static constexpr bool ON = S.c > 0;
  static constexpr int C = ON ? S.c : 1, W = ON ? S.w : 1, G = ON ? S.g : 1, CAP = S.cap;
  static constexpr uint64_t CPT = 128u * C;
};

template <int K, int N>
__global__ __launch_bounds__((64 * KsTune<K, N>::C * KsTune<K, N>::W)) void rs_encode_bitslice_ks(
    const ApplyArgs a) {
  using S = KsTune<K, N>;
  bs_ksplit_body<EncMat<K, N>, S::C, S::W, S::G, 1>(a);
}

template <int K, int N>
__global__ __launch_bounds__((BsTune<K, N>::T)) __attribute__((amdgpu_waves_per_eu(2))) void
rs_encode_bitslice(const ApplyArgs a) {
  using C = BsTune<K, N>;
  if constexpr (C::SPLIT)
    bs_split_body<EncMat<K, N>, C::G, C::SWZ>(a);
  else
    bs_kernel_body<EncMat<K, N>, C::G, C::T, C::SWZ>(a);
}

// The row-split form for geometries bs_split leaves to one wave per tile
// (the round-2 A/B of it at k = 16 / 32 is in DESIGN.md §4). CAP resident per CU.
template <int K, int N, int CAP>
__global__ __launch_bounds__(kSplitThreads) __attribute__((amdgpu_waves_per_eu(2))) void
rs_encode_bitslice_split(const ApplyArgs a) {
  bs_split_body<EncMat<K, N>, kSplitGroup, 0>(a);
}

// The streamed single call's bit-sliced encoder (rs_stream.hpp): one stripe,
// each workgroup gated on its tile's slice (one wave per tile geometries).
template <int K, int N>
__global__ __launch_bounds__((BsTune<K, N>::T)) __attribute__((amdgpu_waves_per_eu(2))) void
rs_encode_bitslice_stream(const ApplyArgs a, const StreamArgs st) {
  using C = BsTune<K, N>;
  static_assert(!C::SPLIT, "streamed encode: one wave per tile");
  const uint32_t slice = static_cast<uint32_t>(blockIdx.x * C::CPT / st.slice_cols);
  if (!stream_gate(st, slice)) return;
  bs_kernel_body<EncMat<K, N>, C::G, C::T, C::SWZ>(a);
  stream_report(st, slice);
}

template <int K, int N>
hipError_t launch_bitslice_stream(const ApplyArgs &a, const StreamArgs &st, hipStream_t s) {
  using C = BsTune<K, N>;
  const uint64_t blocks = ((a.block >> 4) + C::CPT - 1) / C::CPT;
  if (blocks == 0) return hipSuccess;
  return launch_lds<rs_encode_bitslice_stream<K, N>>(blocks, C::T, cap_lds(wg_cap(C::OCC), C::LDS),
                                                     s, a, st);
}

template <int K, int N, int CAP>
hipError_t launch_bitslice_split(const ApplyArgs &a, hipStream_t s) {
  const uint64_t cols = a.block >> 4;
  const uint64_t blocks = ((cols + kSplitColsPerTile - 1) / kSplitColsPerTile) * a.nstripes;
  if (blocks == 0) return hipSuccess;
  if (blocks > 0x7FFFFFFFull) return hipErrorInvalidConfiguration;
  return launch_lds<rs_encode_bitslice_split<K, N, CAP>>(
      blocks, kSplitThreads, cap_lds(wg_cap(CAP), split_lds_bytes(kSplitGroup)), s, a);
}

template <int K, int N>
hipError_t launch_bitslice(const ApplyArgs &a, hipStream_t s) {
  if constexpr (KsTune<K, N>::ON) {
    using S = KsTune<K, N>;
    const uint64_t blocks = (((a.block >> 4) + S::CPT - 1) / S::CPT) * a.nstripes;
    if (blocks == 0) return hipSuccess;
    if (blocks > 0x7FFFFFFFull) return hipErrorInvalidConfiguration;
    return launch_lds<rs_encode_bitslice_ks<K, N>>(
        blocks, 64 * S::C * S::W, cap_lds(wg_cap(S::CAP), ksplit_lds_bytes(S::C, S::W, N - K)), s,
        a);
  }
  using C = BsTune<K, N>;
  constexpr uint64_t cpt = C::CPT;
  const uint64_t cols = a.block >> 4;
  const uint64_t blocks = ((cols + cpt - 1) / cpt) * a.nstripes;
  if (blocks == 0) return hipSuccess;
  if (blocks > 0x7FFFFFFFull) return hipErrorInvalidConfiguration;
  return launch_lds<rs_encode_bitslice<K, N>>(blocks, C::T, cap_lds(wg_cap(C::OCC), C::LDS), s, a);
}

}  // namespace bs
}  // namespace storb_rs
