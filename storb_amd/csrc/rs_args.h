// rs_args.h -- the launch argument block of the GF(2^8) shard kernels.
//
// Self-contained on purpose: besides the ahead-of-time kernels it is handed
// to hipRTC (as an in-memory header) for the per-matrix bit-sliced kernels
// compiled at run time (rs_jit.cpp), so the JIT kernels read exactly the
// struct the host fills in. No standard headers under hipRTC.
#pragma once

#ifdef __HIPCC_RTC__
typedef unsigned char uint8_t;
typedef unsigned int uint32_t;
typedef unsigned long long uint64_t;
#else
#include <cstdint>
#endif

namespace storb_rs {

struct PermTab;  // gf256.hpp (host side only)

// One launch applies a (r x k) coefficient block to k input share slots and
// writes (or XOR-accumulates into) r output share slots, for every stripe.
// Larger matrices are tiled over several launches by the host (storb_rs.cpp):
// the table kernels take up to kSlotK inputs per launch, the bit-sliced ones
// kMaxIn -- Storb sizes the chunks of objects from ~160 GiB up (128-256 MiB)
// k = 64 (piece.rs:292-317), and a launch that sees every input writes each
// output once instead of XOR-accumulating it over column tiles.
constexpr int kSlotK = 32;
constexpr int kSlotR = 16;
// Output slots of one launch: the table kernel fills kSlotR of them, the
// row-split bit-sliced kernels (rs_bitslice_core.h) up to 32.
constexpr int kMaxOut = 32;
#ifndef STORB_RS_MAX_IN
#define STORB_RS_MAX_IN 64  // (tools: -DSTORB_RS_MAX_IN=32 for a kernel-argument-size A/B)
#endif
constexpr int kMaxIn = STORB_RS_MAX_IN;

// Largest k bucket with COPY instantiations of the table kernel; wider
// decodes copy survivors with hipMemcpy2DAsync before the kernel.
constexpr uint32_t kCopyMaxK = 16;

struct ApplyArgs {
  const uint8_t *in[kMaxIn];
  uint64_t in_stride[kMaxIn];
  uint8_t *out[kMaxOut];
  uint64_t out_stride[kMaxOut];
  const PermTab *ptab;  // nibble tables [col][tab_rows], rows >= r zeroed
  const uint8_t *btab;  // 256-byte product tables, same order (LDS variant)
  uint32_t k, r;
  uint32_t tab_rows;    // row stride of both tables = rows_bucket(r)
  uint64_t block;       // bytes per share
  uint32_t nstripes;
  uint32_t accumulate;  // 1: out ^= result (column tiling), 0: out = result
  // Fused assembly (decode into a separate chunk buffer): input slot j is
  // also stored, as loaded, to copy[j] (null = not copied). ncopy > 0 selects
  // the COPY kernels; r may then be 0 (pure assembly).
  uint32_t ncopy;
  uint8_t *copy[kMaxIn];
  uint64_t copy_stride[kMaxIn];
};

// Per-stripe descriptors: one launch over stripes that each lost different
// shares (Storb's download keeps whichever k + 1 pieces arrive first,
// download.rs:363-451, so the survivor set varies from chunk to chunk). Item
// i of the launch is the record desc + i * rec_qwords (8-byte words):
//   [0]                  offset (in PermTabs) of the item's tables in ptab,
//                        [input][rows_bucket(r)]
//   [1 .. k]             input pointers, slot order
//   [k+1 .. k+r]         output row pointers
//   [k+r+1 .. 2k+r]      (copy != 0) where input j is also stored, 0 = nowhere
// Every item rebuilds r rows with its own matrix and pointers; the stripes
// (and shares) of different items need not be related at all. A workgroup
// covers tpw consecutive tiles of one item.
struct DescArgs {
  const uint64_t *desc;
  const PermTab *ptab;
  uint64_t block;  // bytes per share
  uint32_t k;
  uint32_t r;      // output slots per record (mix: the most rows an item has)
  uint32_t tpw;    // tiles per workgroup
  uint32_t nitems;
  uint32_t copy;
  uint32_t rec_qwords;  // 1 + k + r (+ k with copy)
  // mix = 1: items of different row counts (1..kMixR, 0 with copy) in one
  // launch; item i's count is its record's rec[0] >> 32 and a workgroup runs
  // the tile of that count. cap: resident workgroups per CU (0: the tuned
  // value of the launch's row bucket).
  uint32_t mix;
  uint32_t cap;
};

// Streamed single call (host_calls.cpp): ONE launch over one stripe whose
// page-locked staging the host is still filling, slice by slice, while the
// kernel runs. A workgroup of slice s waits until ready[16 s] == seq (the
// word the host writes once slice s is packed; the wait gives up after
// timeout_ticks of s_memrealtime, 100 MHz, and the workgroup then exits
// without writing), runs its tile, and the last workgroup of the slice --
// the one that brings the device counter cnt[s] to target[s] -- writes
// done[16 s] = seq once every store of the slice is complete. So the launch
// latency overlaps the packing of slice 0, each slice's transfer overlaps
// the packing of the next, and the host unpacks a slice as soon as its word
// turns, with no launch or stream synchronisation per slice.
constexpr int kMaxStreamSlices = 16;
struct StreamArgs {
  const uint32_t *ready;  // page-locked words, 64 B apart (device address)
  uint32_t *done;         // page-locked words, 64 B apart (device address)
  uint32_t *cnt;          // device counters, one per slice
  uint32_t target[kMaxStreamSlices];
  uint32_t seq;
  uint32_t slice_cols;    // 16-B columns per slice, a multiple of the tile
  uint32_t nslices;
  uint32_t pad;
  uint64_t timeout_ticks;
};

// Rows per item a mixed-row descriptor launch takes: a download's chunks
// mostly lost 0-3 data shares (tools/descbench.cpp, bench --erase-pattern
// download); items with more rows get launches of their own.
constexpr uint32_t kMixR = 4;

// Launch shape of the bit-sliced kernels (rs_bitslice_core.h), shared by
// the host launchers and the kernels. Grid: nstripes x tiles; a tile = T
// lanes x 32 B of every share. Wave w of the tile covers 2 KiB: lane l holds
// the 16-B columns (w*128 + l) and (w*128 + 64 + l) of the tile, so each
// load and store instruction moves one contiguous 1 KiB per wave.
namespace bs {
constexpr int kBsThreads = 256;
constexpr unsigned bs_cols_per_tile(int threads) { return 2u * static_cast<unsigned>(threads); }

// Launch shape per (k, rows), from the sweep of workgroup size x tile
// rotation x resident-workgroup cap: over the kernels alone
// (tools/bstune.hip, profiles/r2_bstune_shape*.txt; profiles/r2_wide_probe_2.txt for
// the access shape with no GF work) and on the product's own decode path
// (a removed A/B script, profiles/r2_shape_ab/: bench --config 5/6 --erase E).
// The wide shapes stream best with few bytes in flight per CU and no
// workgroup waiting long on its slowest wave: one-wave workgroups, 6 per CU,
// for 6+ rows at k <= 16 (RS(16,8) encode 0.267 -> 0.257 ms, 8-lost decode
// 0.272 -> 0.257); two-wave workgroups, 3 per CU, for fewer rows (16 in + 2
// out 0.218 -> 0.193 ms, + 4 out 0.243 -> 0.217); 4 per CU for 8+ rows at
// k > 16 (48 streams: RS(32,16) 16-lost decode 0.282 -> 0.276 ms). swz:
// tile rotation per stripe (bs_kernel_body); threads <= 128 with
// amdgpu_waves_per_eu(2) keeps 2 waves per SIMD.
struct BsShape {
  int threads, swz, cap;
};
// k > 32 with few rows (Storb's k = 64 decode with a few miners lost): 2 per
// CU -- bench --config 7 decode (2 lost) 0.1805 ms at 3 per CU -> 0.1744 at
// 2, 0.1958 at 4 (profiles/r2_k64/shape_c7_ab.txt).
constexpr BsShape bs_shape(int K, int R) {
  return K <= 16 ? (R >= 6 ? BsShape{64, 1, 6} : BsShape{128, 0, 3})
                 : (R >= 8 ? BsShape{128, 0, 4} : (K > 32 ? BsShape{128, 0, 2} : BsShape{128, 0, 3}));
}

// Shares per load group (R x 8 accumulators + 2 x G x 8 loaded dwords + 30
// table entries must fit): at k = 16 with 6-8 rows, 8 shares per group
// (196 VGPRs) streams 2 % faster than 4 (141 VGPRs) -- both run 2 waves per
// SIMD (tools/bstune.hip, profiles/r2_bstune.txt); with up to 5 rows (the
// common decodes: a few miners lost) 4 per group in the two-wave
// workgroups is 2-6 % faster than 8 at k = 16 and 32 (16 in + 2 out 193 ->
// 183 us, + 4 out 223 -> 214; k = 32 + 4 out 194 -> 192;
// profiles/r2_bstune_fewrows.txt); 16 rows leave room for 2.
constexpr int bs_group(int K, int R) {
  return K <= 8 ? K
                : (R >= 12 ? (K % 2 == 0 ? 2 : 1)
                           : (R <= 5 && K % 4 == 0
                                  ? 4
                                  : (R <= 8 && K % 8 == 0
                                         ? 8
                                         : (K % 4 == 0 ? 4 : (K % 2 == 0 ? 2 : 1)))));
}

// Row-split kernels (rs_bitslice_core.h bs_split_body): 128 lanes (one row
// half per wave), one input per wave per load group. Used (bs_split)
//  * for 17-32 rows -- Storb's k = 64 encode and decodes losing more than 16
//    shares -- which one wave cannot hold: 4 workgroups per CU (2 waves per
//    SIMD at ~197 VGPRs). the removed k64split probe, k = 64 encode of 8 x 128 MiB
//    chunks: 494.6 us as two 16-row launches -> 348.6 us; 3 per CU 556 us
//    (6 waves per CU), uncapped 391, 2 inputs per wave per group 376
//    (profiles/r2_k64/k64split.txt);
//  * not for 16 rows or fewer: RS(32,16) with 8 rows per wave (127 VGPRs, 6
//    per CU) measured 274.8 -> 267.7 us in isolation
//    (profiles/r2_k64/k64split2.txt) but nothing in the product (bench
//    --config 6 --erase 16: decode 0.2709 ms one wave per tile, 0.2720
//    split, profiles/r2_k64/split_k32_ab.txt); RS(16,8) within noise.
constexpr int kSplitGroup = 2;
constexpr bool bs_split(int K, int R) { return K % kSplitGroup == 0 && R > 16 && R <= 32; }
constexpr int bs_split_cap(int R) { return R > 16 ? 4 : 6; }
constexpr int kSplitThreads = 128;           // two waves, one row half each
constexpr unsigned kSplitColsPerTile = 128;  // 64 lanes x 2 16-B columns
// Static LDS of one workgroup: [group parity][owner wave][G/2 inputs][2 halves][64 lanes] x 16 B.
constexpr unsigned split_lds_bytes(int G) { return 2u * 2u * static_cast<unsigned>(G / 2) * 2u * 64u * 16u; }

// Input-split form (rs_bitslice_core.h bs_ksplit_body): C column groups of W
// waves per workgroup, W waves on the same 2 KiB of every share, each folding
// K / W inputs (G per load group); cap resident per CU. c = 0: not used (one
// wave per tile, bs_shape). Measured (tools/bstune.hip BSTUNE_KSPLIT, every
// variant bit-exact against the one-wave kernel; profiles/r6e_bstune_ksplit.txt
// for the encoders, r6n/bstune_dec.txt for the in-place decodes): RS(16,8)
// encode 79.3-80.1 -> 81.0-81.7 % of 8 TB/s (C 1 W 4), k = 16 decode of 8
// lost 80.7 -> 82.4 % (C 1 W 4), of 4 lost 77.5 -> 80.1 % (C 2 W 2), RS(32,16)
// encode 74.0 -> 75.4 % and k = 32 decode of 16 lost 74.1 -> 76.5 % (C 2 W 2);
// k = 16 decode of 2 lost 82.1 -> 79.5 % and k = 32 of 2 lost equal, so few
// rows keep one wave per tile.
struct KsShape {
  int c, w, g, cap;
};
constexpr int ks_group(int KW) { return KW % 4 == 0 ? 4 : KW % 2 == 0 ? 2 : 1; }
constexpr KsShape ks_shape(int K, int R) {
  return (K <= 16 && R == 8 && K % 4 == 0)   ? KsShape{1, 4, ks_group(K / 4), 4}
         : (K <= 16 && R == 4 && K % 2 == 0) ? KsShape{2, 2, ks_group(K / 2), 3}
         : (K > 16 && R == 16 && K % 2 == 0) ? KsShape{2, 2, ks_group(K / 2), 2}
                                             : KsShape{0, 0, 0, 0};
}
// Static LDS of an input-split workgroup: per column group
// [owner wave][partner (W-1)][row of owner (R/W)][2 halves][64 lanes] x 16 B.
constexpr unsigned ksplit_lds_bytes(int C, int W, int R) {
  return W > 1 ? static_cast<unsigned>(C * W * (W - 1) * (R / W) * 2 * 64 * 16) : 16u;
}

}  // namespace bs

}  // namespace storb_rs
