// blake3.hpp -- BLAKE3 compression shared by the host hasher and the gfx950
// shard-hashing kernel (hash mode, 32-byte output).
//
// Storb's shard identity is blake3(shard bytes): upload.rs:623 hashes every
// piece right after encode_chunk, the miner re-hashes on receipt
// (crates/storb_miner/src/lib.rs:265-283), download re-hashes on retrieve
// (download.rs:158-161); crate blake3 1.8.2 (reference Cargo.lock:1099).
// This is the published algorithm: 7-round BLAKE2s-style compression over
// 64-byte blocks, 1024-byte chunks, left-balanced binary tree.
#pragma once

#include <cstddef>
#include <cstdint>

#ifdef __HIPCC__
#define B3_HD __host__ __device__ __forceinline__
#else
#define B3_HD inline
#endif

namespace storb_rs {
namespace b3 {

constexpr uint32_t kChunkStart = 1, kChunkEnd = 2, kParent = 4, kRoot = 8;
constexpr uint32_t kBlockLen = 64, kChunkLen = 1024;

B3_HD uint32_t iv(int i) {
  constexpr uint32_t v[8] = {0x6A09E667u, 0xBB67AE85u, 0x3C6EF372u, 0xA54FF53Au,
                             0x510E527Fu, 0x9B05688Cu, 0x1F83D9ABu, 0x5BE0CD19u};
  return v[i];
}

B3_HD uint32_t rotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

// Message word used by round r at position i: the per-round permutation
// (2,6,3,10,7,0,4,13,1,11,12,5,9,14,15,8) applied r times, as a constant
// schedule so the unrolled rounds index registers statically.
B3_HD int sched(int r, int i) {
  constexpr unsigned char s[7][16] = {
      {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15},
      {2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8},
      {3, 4, 10, 12, 13, 2, 7, 14, 6, 5, 9, 0, 11, 15, 8, 1},
      {10, 7, 12, 9, 14, 3, 13, 15, 4, 0, 11, 2, 5, 8, 1, 6},
      {12, 13, 9, 11, 15, 10, 14, 8, 7, 2, 5, 3, 0, 1, 6, 4},
      {9, 14, 11, 5, 8, 12, 15, 1, 13, 3, 0, 10, 2, 6, 4, 7},
      {11, 15, 5, 0, 1, 9, 8, 6, 14, 10, 2, 12, 3, 4, 7, 13}};
  return s[r][i];
}

B3_HD void g(uint32_t *s, int a, int b, int c, int d, uint32_t mx, uint32_t my) {
  s[a] = s[a] + s[b] + mx;
  s[d] = rotr(s[d] ^ s[a], 16);
  s[c] = s[c] + s[d];
  s[b] = rotr(s[b] ^ s[c], 12);
  s[a] = s[a] + s[b] + my;
  s[d] = rotr(s[d] ^ s[a], 8);
  s[c] = s[c] + s[d];
  s[b] = rotr(s[b] ^ s[c], 7);
}

// cv (8 words) <- first 8 words of compress(cv, m, counter, len, flags).
B3_HD void compress_cv(uint32_t *cv, const uint32_t *m, uint64_t counter,
                       uint32_t block_len, uint32_t flags) {
  uint32_t s[16] = {cv[0], cv[1], cv[2], cv[3], cv[4], cv[5], cv[6], cv[7],
                    iv(0), iv(1), iv(2), iv(3),
                    static_cast<uint32_t>(counter),
                    static_cast<uint32_t>(counter >> 32), block_len, flags};
#pragma unroll
  for (int r = 0; r < 7; r++) {
    g(s, 0, 4, 8, 12, m[sched(r, 0)], m[sched(r, 1)]);
    g(s, 1, 5, 9, 13, m[sched(r, 2)], m[sched(r, 3)]);
    g(s, 2, 6, 10, 14, m[sched(r, 4)], m[sched(r, 5)]);
    g(s, 3, 7, 11, 15, m[sched(r, 6)], m[sched(r, 7)]);
    g(s, 0, 5, 10, 15, m[sched(r, 8)], m[sched(r, 9)]);
    g(s, 1, 6, 11, 12, m[sched(r, 10)], m[sched(r, 11)]);
    g(s, 2, 7, 8, 13, m[sched(r, 12)], m[sched(r, 13)]);
    g(s, 3, 4, 9, 14, m[sched(r, 14)], m[sched(r, 15)]);
  }
#pragma unroll
  for (int i = 0; i < 8; i++) cv[i] = s[i] ^ s[i + 8];
}

// Parent node: block = left cv || right cv, counter 0, flags PARENT(|ROOT).
B3_HD void parent_cv(uint32_t *out, const uint32_t *l, const uint32_t *r,
                     uint32_t extra_flags) {
  uint32_t m[16];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    m[i] = l[i];
    m[i + 8] = r[i];
  }
#pragma unroll
  for (int i = 0; i < 8; i++) out[i] = iv(i);
  compress_cv(out, m, 0, kBlockLen, kParent | extra_flags);
}

B3_HD uint32_t load_le32(const uint8_t *p) {
  return static_cast<uint32_t>(p[0]) | static_cast<uint32_t>(p[1]) << 8 |
         static_cast<uint32_t>(p[2]) << 16 | static_cast<uint32_t>(p[3]) << 24;
}

// Chaining value of chunk `idx` (`len` <= 1024 bytes at p); root_flag is
// ROOT for a single-chunk message (then cv holds the hash words).
B3_HD void chunk_cv(uint32_t *cv, const uint8_t *p, uint32_t len, uint64_t idx,
                    uint32_t root_flag) {
  const uint32_t nb = len == 0 ? 1 : (len + kBlockLen - 1) / kBlockLen;
#pragma unroll
  for (int i = 0; i < 8; i++) cv[i] = iv(i);
  for (uint32_t b = 0; b < nb; b++) {
    const uint32_t off = b * kBlockLen;
    const uint32_t bl = len - off < kBlockLen ? len - off : kBlockLen;
    uint32_t m[16];
    if (bl == kBlockLen) {
#pragma unroll
      for (int i = 0; i < 16; i++) m[i] = load_le32(p + off + 4 * i);
    } else {
      uint8_t tmp[kBlockLen];
      for (uint32_t i = 0; i < kBlockLen; i++) tmp[i] = i < bl ? p[off + i] : 0;
#pragma unroll
      for (int i = 0; i < 16; i++) m[i] = load_le32(tmp + 4 * i);
    }
    uint32_t flags = (b == 0 ? kChunkStart : 0) | (b + 1 == nb ? kChunkEnd | root_flag : 0);
    compress_cv(cv, m, idx, bl, flags);
  }
}

}  // namespace b3
}  // namespace storb_rs
