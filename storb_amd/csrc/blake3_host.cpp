// blake3_host.cpp -- host BLAKE3 (storb_blake3): the hasher Storb's CPU side
// runs on every shard -- the miner on receipt (crates/storb_miner/src/lib.rs:
// 265-283) and download on retrieve (download.rs:158-161). The reference
// links crate blake3 1.8.2 (Cargo.lock:1099), which hashes full chunks
// several at a time with SIMD; this is the same idea written for the hosts
// that carry MI355X (x86-64 with AVX-512: EPYC Zen 4/5, Xeon SPR+).
//
// Layout: the 16 lanes of a zmm register hold the same state word of 16
// consecutive 1 KiB chunks. Each 64-byte block of the 16 chunks is loaded
// as 16 rows and transposed (16x16 dwords, 64 shuffles) so that message
// word w of every chunk sits in one register; one compression then advances
// all 16 chunk chaining values. Parent nodes are reduced layer by layer, 16
// per compression, with the same transpose (two children = one 64-B row).
// Without AVX-512 the scalar path (blake3.hpp) runs unchanged.
#include <immintrin.h>

#include <array>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/storb_rs.h"
#include "blake3.hpp"

namespace storb_rs {
namespace {

#define B3_AVX512 __attribute__((target("avx512f")))

B3_AVX512 inline void g16(__m512i *s, int a, int b, int c, int d, __m512i mx, __m512i my) {
  s[a] = _mm512_add_epi32(_mm512_add_epi32(s[a], s[b]), mx);
  s[d] = _mm512_ror_epi32(_mm512_xor_si512(s[d], s[a]), 16);
  s[c] = _mm512_add_epi32(s[c], s[d]);
  s[b] = _mm512_ror_epi32(_mm512_xor_si512(s[b], s[c]), 12);
  s[a] = _mm512_add_epi32(_mm512_add_epi32(s[a], s[b]), my);
  s[d] = _mm512_ror_epi32(_mm512_xor_si512(s[d], s[a]), 8);
  s[c] = _mm512_add_epi32(s[c], s[d]);
  s[b] = _mm512_ror_epi32(_mm512_xor_si512(s[b], s[c]), 7);
}

// r[j] = 64-byte row of chunk j  ->  m[w] lane j = dword w of row j.
B3_AVX512 inline void transpose16(const __m512i *r, __m512i *m) {
  __m512i a[16], t[16];
  for (int j = 0; j < 16; j += 2) {  // dword interleave of row pairs
    a[j] = _mm512_unpacklo_epi32(r[j], r[j + 1]);
    a[j + 1] = _mm512_unpackhi_epi32(r[j], r[j + 1]);
  }
  // t[4G + q]: 128-bit lane L holds dword 4L + q of rows 4G .. 4G+3
  for (int G = 0; G < 4; G++) {
    const __m512i *p = a + 4 * G;
    t[4 * G + 0] = _mm512_unpacklo_epi64(p[0], p[2]);
    t[4 * G + 1] = _mm512_unpackhi_epi64(p[0], p[2]);
    t[4 * G + 2] = _mm512_unpacklo_epi64(p[1], p[3]);
    t[4 * G + 3] = _mm512_unpackhi_epi64(p[1], p[3]);
  }
  // 4x4 transpose of 128-bit lanes across t[q], t[4+q], t[8+q], t[12+q]
  for (int q = 0; q < 4; q++) {
    const __m512i u0 = _mm512_shuffle_i32x4(t[q], t[4 + q], 0x44);
    const __m512i u1 = _mm512_shuffle_i32x4(t[q], t[4 + q], 0xEE);
    const __m512i u2 = _mm512_shuffle_i32x4(t[8 + q], t[12 + q], 0x44);
    const __m512i u3 = _mm512_shuffle_i32x4(t[8 + q], t[12 + q], 0xEE);
    m[0 + q] = _mm512_shuffle_i32x4(u0, u2, 0x88);
    m[4 + q] = _mm512_shuffle_i32x4(u0, u2, 0xDD);
    m[8 + q] = _mm512_shuffle_i32x4(u1, u3, 0x88);
    m[12 + q] = _mm512_shuffle_i32x4(u1, u3, 0xDD);
  }
}

// Chaining values of the 16 full chunks at p (chunk indices idx0 .. idx0+15),
// none of them the root.
B3_AVX512 void chunks16_cv(const uint8_t *p, uint64_t idx0, uint32_t (*out)[8]) {
  alignas(64) uint32_t lo[16], hi[16];
  for (int j = 0; j < 16; j++) {
    lo[j] = static_cast<uint32_t>(idx0 + j);
    hi[j] = static_cast<uint32_t>((idx0 + j) >> 32);
  }
  const __m512i ctr_lo = _mm512_load_si512(lo), ctr_hi = _mm512_load_si512(hi);
  __m512i cv[8];
  for (int i = 0; i < 8; i++) cv[i] = _mm512_set1_epi32(static_cast<int>(b3::iv(i)));
  for (uint32_t b = 0; b < b3::kChunkLen / b3::kBlockLen; b++) {
    __m512i r[16], m[16];
    for (int j = 0; j < 16; j++)
      r[j] = _mm512_loadu_si512(p + static_cast<size_t>(j) * b3::kChunkLen + b * b3::kBlockLen);
    transpose16(r, m);
    const uint32_t flags = (b == 0 ? b3::kChunkStart : 0) | (b == 15 ? b3::kChunkEnd : 0);
    __m512i s[16] = {cv[0], cv[1], cv[2], cv[3], cv[4], cv[5], cv[6], cv[7],
                     _mm512_set1_epi32(static_cast<int>(b3::iv(0))),
                     _mm512_set1_epi32(static_cast<int>(b3::iv(1))),
                     _mm512_set1_epi32(static_cast<int>(b3::iv(2))),
                     _mm512_set1_epi32(static_cast<int>(b3::iv(3))),
                     ctr_lo, ctr_hi, _mm512_set1_epi32(static_cast<int>(b3::kBlockLen)),
                     _mm512_set1_epi32(static_cast<int>(flags))};
#pragma unroll
    for (int rd = 0; rd < 7; rd++) {
      g16(s, 0, 4, 8, 12, m[b3::sched(rd, 0)], m[b3::sched(rd, 1)]);
      g16(s, 1, 5, 9, 13, m[b3::sched(rd, 2)], m[b3::sched(rd, 3)]);
      g16(s, 2, 6, 10, 14, m[b3::sched(rd, 4)], m[b3::sched(rd, 5)]);
      g16(s, 3, 7, 11, 15, m[b3::sched(rd, 6)], m[b3::sched(rd, 7)]);
      g16(s, 0, 5, 10, 15, m[b3::sched(rd, 8)], m[b3::sched(rd, 9)]);
      g16(s, 1, 6, 11, 12, m[b3::sched(rd, 10)], m[b3::sched(rd, 11)]);
      g16(s, 2, 7, 8, 13, m[b3::sched(rd, 12)], m[b3::sched(rd, 13)]);
      g16(s, 3, 4, 9, 14, m[b3::sched(rd, 14)], m[b3::sched(rd, 15)]);
    }
    for (int i = 0; i < 8; i++) cv[i] = _mm512_xor_si512(s[i], s[i + 8]);
  }
  alignas(64) uint32_t w[8][16];
  for (int i = 0; i < 8; i++) _mm512_store_si512(w[i], cv[i]);
  for (int j = 0; j < 16; j++)
    for (int i = 0; i < 8; i++) out[j][i] = w[i][j];
}

// 16 parent nodes at once: cvs holds 32 consecutive child CVs (8 words
// each), so parent j's 64-byte block (left || right) is row j of a 16 x 16
// dword matrix -- the same transpose as the chunk blocks.
B3_AVX512 void parents16_cv(const uint32_t *cvs, uint32_t (*out)[8]) {
  __m512i r[16], m[16];
  for (int j = 0; j < 16; j++) r[j] = _mm512_loadu_si512(cvs + 16 * j);
  transpose16(r, m);
  __m512i s[16];
  for (int i = 0; i < 8; i++) s[i] = _mm512_set1_epi32(static_cast<int>(b3::iv(i)));
  for (int i = 0; i < 4; i++) s[8 + i] = _mm512_set1_epi32(static_cast<int>(b3::iv(i)));
  s[12] = _mm512_setzero_si512();
  s[13] = _mm512_setzero_si512();
  s[14] = _mm512_set1_epi32(static_cast<int>(b3::kBlockLen));
  s[15] = _mm512_set1_epi32(static_cast<int>(b3::kParent));
#pragma unroll
  for (int rd = 0; rd < 7; rd++) {
    g16(s, 0, 4, 8, 12, m[b3::sched(rd, 0)], m[b3::sched(rd, 1)]);
    g16(s, 1, 5, 9, 13, m[b3::sched(rd, 2)], m[b3::sched(rd, 3)]);
    g16(s, 2, 6, 10, 14, m[b3::sched(rd, 4)], m[b3::sched(rd, 5)]);
    g16(s, 3, 7, 11, 15, m[b3::sched(rd, 6)], m[b3::sched(rd, 7)]);
    g16(s, 0, 5, 10, 15, m[b3::sched(rd, 8)], m[b3::sched(rd, 9)]);
    g16(s, 1, 6, 11, 12, m[b3::sched(rd, 10)], m[b3::sched(rd, 11)]);
    g16(s, 2, 7, 8, 13, m[b3::sched(rd, 12)], m[b3::sched(rd, 13)]);
    g16(s, 3, 4, 9, 14, m[b3::sched(rd, 14)], m[b3::sched(rd, 15)]);
  }
  alignas(64) uint32_t w[8][16];
  for (int i = 0; i < 8; i++) _mm512_store_si512(w[i], _mm512_xor_si512(s[i], s[i + 8]));
  for (int j = 0; j < 16; j++)
    for (int i = 0; i < 8; i++) out[j][i] = w[i][j];
}

// CV of the complete subtree over chunks [c0, c0 + 2^p) (c0 aligned):
// chunk CVs 16 at a time, then layers of parents 16 at a time; layers
// under 32 nodes and blocks under 16 chunks finish on the scalar path.
void subtree_cv(const uint8_t *data, uint64_t c0, uint64_t size, bool simd,
                std::vector<std::array<uint32_t, 8>> &buf, uint32_t *cv) {
  buf.resize(size);
  uint64_t c = 0;
  if (simd)
    for (; c + 16 <= size; c += 16)
      chunks16_cv(data + (c0 + c) * b3::kChunkLen, c0 + c,
                  reinterpret_cast<uint32_t(*)[8]>(buf[c].data()));
  for (; c < size; c++)
    b3::chunk_cv(buf[c].data(), data + (c0 + c) * b3::kChunkLen, b3::kChunkLen, c0 + c, 0);
  for (uint64_t nodes = size; nodes > 1; nodes >>= 1) {
    uint64_t j = 0;
    if (simd)
      for (; 2 * j + 32 <= nodes; j += 16)
        parents16_cv(buf[2 * j].data(), reinterpret_cast<uint32_t(*)[8]>(buf[j].data()));
    for (; 2 * j < nodes; j++) {
      uint32_t t[8];
      b3::parent_cv(t, buf[2 * j].data(), buf[2 * j + 1].data(), 0);
      std::memcpy(buf[j].data(), t, 32);
    }
  }
  std::memcpy(cv, buf[0].data(), 32);
}

bool have_avx512() {
  static const bool ok = __builtin_cpu_supports("avx512f") &&
                         std::getenv("STORB_B3_SCALAR") == nullptr;
  return ok;
}

}  // namespace

namespace detail {

// The chunks before the last one form the complete subtrees of the binary
// decomposition of n - 1 (largest first) -- exactly the stack a streaming
// hasher holds at that point; each is reduced on its own, then the last
// chunk is folded in right to left and the final parent carries ROOT.
void blake3_host(const uint8_t *data, size_t len, uint8_t out[32]) {
  const uint64_t n = len == 0 ? 1 : (len + b3::kChunkLen - 1) / b3::kChunkLen;
  uint32_t cv[8];
  auto emit = [&](const uint32_t *w) {
    for (int i = 0; i < 8; i++)
      for (int b = 0; b < 4; b++) out[4 * i + b] = static_cast<uint8_t>(w[i] >> (8 * b));
  };
  if (n == 1) {
    b3::chunk_cv(cv, data, static_cast<uint32_t>(len), 0, b3::kRoot);
    emit(cv);
    return;
  }
  const bool simd = have_avx512();
  std::vector<std::array<uint32_t, 8>> stack, buf;
  uint64_t c0 = 0;
  for (int p = 63; p >= 0; p--) {
    const uint64_t size = uint64_t{1} << p;
    if (!((n - 1) & size)) continue;
    std::array<uint32_t, 8> t;
    subtree_cv(data, c0, size, simd, buf, t.data());
    stack.push_back(t);
    c0 += size;
  }
  const uint64_t last = n - 1;
  b3::chunk_cv(cv, data + last * b3::kChunkLen,
               static_cast<uint32_t>(len - last * b3::kChunkLen), last, 0);
  while (!stack.empty()) {
    const std::array<uint32_t, 8> l = stack.back();
    stack.pop_back();
    b3::parent_cv(cv, l.data(), cv, stack.empty() ? b3::kRoot : 0);
  }
  emit(cv);
}

}  // namespace detail
}  // namespace storb_rs
