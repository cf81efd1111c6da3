// blake3.hip -- batched BLAKE3 of shards on gfx950 (one workgroup per shard).
//
// Every Storb shard is blake3-hashed after encode (upload.rs:623) and again
// on the miner and on download. Hashing the shards where they already are
// (HBM, right after the encode kernel) replaces a full host pass over
// n*B bytes per chunk.
//
// Layout of the work: shard of n = ceil(len/1024) chunks, 256 lanes. Lane l
// owns the aligned group of q chunks [l*q, (l+1)*q) (q = smallest power of
// two with 256*q >= n), hashes them one 64-byte block at a time and merges
// its group into one subtree node with a per-lane stack kept in LDS
// ([depth][word][lane], bank-conflict free). Aligned power-of-two groups are
// exactly the subtrees of BLAKE3's left-balanced tree, so the group nodes
// then merge pairwise (odd node carried) in LDS; the last parent gets ROOT.
#include <hip/hip_runtime.h>

#include "blake3.hpp"
#include "rs_kernels.hpp"

namespace storb_rs {

namespace {

constexpr int kB3Threads = 256;
typedef uint32_t u32x4b __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void load_block(uint32_t *m, const uint8_t *p, uint32_t bl,
                                           bool aligned16) {
  if (bl == b3::kBlockLen && aligned16) {
    const u32x4b *q = reinterpret_cast<const u32x4b *>(p);
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const u32x4b v = __builtin_nontemporal_load(q + i);
      m[4 * i] = v[0];
      m[4 * i + 1] = v[1];
      m[4 * i + 2] = v[2];
      m[4 * i + 3] = v[3];
    }
  } else {
#pragma unroll
    for (int i = 0; i < 16; i++) {
      uint32_t w = 0;
#pragma unroll
      for (int b = 0; b < 4; b++) {
        const uint32_t o = 4 * i + b;
        if (o < bl) w |= static_cast<uint32_t>(p[o]) << (8 * b);
      }
      m[i] = w;
    }
  }
}

__device__ void chunk_cv_dev(uint32_t *cv, const uint8_t *p, uint32_t len, uint64_t idx,
                             uint32_t root_flag, bool aligned16) {
  const uint32_t nb = len == 0 ? 1 : (len + b3::kBlockLen - 1) / b3::kBlockLen;
#pragma unroll
  for (int i = 0; i < 8; i++) cv[i] = b3::iv(i);
  for (uint32_t b = 0; b < nb; b++) {
    const uint32_t off = b * b3::kBlockLen;
    const uint32_t bl = len - off < b3::kBlockLen ? len - off : b3::kBlockLen;
    uint32_t m[16];
    load_block(m, p + off, bl, aligned16);
    const uint32_t flags =
        (b == 0 ? b3::kChunkStart : 0) | (b + 1 == nb ? b3::kChunkEnd | root_flag : 0);
    b3::compress_cv(cv, m, idx, bl, flags);
  }
}

__device__ __forceinline__ void put(uint32_t *base, int slot, int lane, const uint32_t *cv) {
#pragma unroll
  for (int w = 0; w < 8; w++) base[(slot * 8 + w) * kB3Threads + lane] = cv[w];
}
__device__ __forceinline__ void get(const uint32_t *base, int slot, int lane, uint32_t *cv) {
#pragma unroll
  for (int w = 0; w < 8; w++) cv[w] = base[(slot * 8 + w) * kB3Threads + lane];
}

__device__ __forceinline__ void store_hash(uint8_t *o, const uint32_t *cv) {
#pragma unroll
  for (int w = 0; w < 8; w++)
#pragma unroll
    for (int b = 0; b < 4; b++) o[4 * w + b] = static_cast<uint8_t>(cv[w] >> (8 * b));
}

__global__ __launch_bounds__(kB3Threads) void blake3_batch_kernel(
    const uint8_t *in, uint64_t len, uint64_t stride, uint8_t *out, uint32_t q_log2,
    uint32_t depth) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds3[];
  const uint8_t *p = in + static_cast<uint64_t>(blockIdx.x) * stride;
  uint8_t *o = out + static_cast<uint64_t>(blockIdx.x) * 32;
  const uint64_t n = len == 0 ? 1 : (len + b3::kChunkLen - 1) / b3::kChunkLen;
  const int lane = threadIdx.x;
  const bool aligned16 = ((reinterpret_cast<uintptr_t>(p)) & 15) == 0;
  if (n == 1) {  // single chunk: it is the root
    if (lane == 0) {
      uint32_t cv[8];
      chunk_cv_dev(cv, p, static_cast<uint32_t>(len), 0, b3::kRoot, aligned16);
      store_hash(o, cv);
    }
    return;
  }
  uint32_t *stack = lds3;                                  // [depth][8][256]
  uint32_t *nodes = lds3 + depth * 8 * kB3Threads;         // [2][8][256]
  const uint64_t q = 1ull << q_log2;
  const uint64_t c0 = static_cast<uint64_t>(lane) * q;
  const uint64_t c1 = c0 + q < n ? c0 + q : n;
  uint32_t cv[8], left[8];
  int sp = 0;
  for (uint64_t c = c0; c < c1; c++) {
    const uint64_t off = c * b3::kChunkLen;
    const uint32_t clen =
        static_cast<uint32_t>(len - off < b3::kChunkLen ? len - off : b3::kChunkLen);
    chunk_cv_dev(cv, p + off, clen, c, 0, aligned16);
    for (uint64_t t = c - c0 + 1; (t & 1) == 0; t >>= 1) {  // complete subtrees merge
      get(stack, --sp, lane, left);
      b3::parent_cv(cv, left, cv, 0);
    }
    put(stack, sp++, lane, cv);
  }
  if (c1 > c0) {  // a partial (last) group folds right to left
    get(stack, --sp, lane, cv);
    while (sp > 0) {
      get(stack, --sp, lane, left);
      b3::parent_cv(cv, left, cv, 0);
    }
    put(nodes, 0, lane, cv);
  }
  __syncthreads();
  uint32_t cnt = static_cast<uint32_t>((n + q - 1) / q);  // >= 2 by the choice of q
  int cur = 0;
  while (cnt > 2) {
    const uint32_t half = cnt / 2;
    uint32_t *src = nodes + cur * 8 * kB3Threads, *dst = nodes + (cur ^ 1) * 8 * kB3Threads;
    if (static_cast<uint32_t>(lane) < half) {
      uint32_t r[8];
      get(src, 0, 2 * lane, left);
      get(src, 0, 2 * lane + 1, r);
      b3::parent_cv(cv, left, r, 0);
      put(dst, 0, lane, cv);
    } else if ((cnt & 1) && static_cast<uint32_t>(lane) == half) {
      get(src, 0, cnt - 1, cv);
      put(dst, 0, lane, cv);
    }
    __syncthreads();
    cur ^= 1;
    cnt = half + (cnt & 1);
  }
  if (lane == 0) {
    uint32_t r[8];
    const uint32_t *src = nodes + cur * 8 * kB3Threads;
    get(src, 0, 0, left);
    get(src, 0, 1, r);
    b3::parent_cv(cv, left, r, b3::kRoot);
    store_hash(o, cv);
  }
}

}  // namespace

// Largest message the LDS tree handles: 256 lanes x 64 chunks = 16 MiB.
constexpr uint64_t kB3MaxLen = 256ull * 64 * b3::kChunkLen;

hipError_t launch_blake3_batch(const uint8_t *in, uint64_t len, uint32_t count,
                               uint64_t stride, uint8_t *out, hipStream_t s) {
  if (count == 0) return hipSuccess;
  if (len > kB3MaxLen) return hipErrorInvalidValue;
  const uint64_t n = len == 0 ? 1 : (len + b3::kChunkLen - 1) / b3::kChunkLen;
  uint32_t q_log2 = 0;
  while ((static_cast<uint64_t>(kB3Threads) << q_log2) < n) q_log2++;
  const uint32_t depth = q_log2 + 1;
  const size_t lds = (static_cast<size_t>(depth) + 2) * 8 * kB3Threads * sizeof(uint32_t);
  hipLaunchKernelGGL(blake3_batch_kernel, dim3(count), dim3(kB3Threads), lds, s, in, len,
                     stride, out, q_log2, depth);
  return hipGetLastError();
}

}  // namespace storb_rs
