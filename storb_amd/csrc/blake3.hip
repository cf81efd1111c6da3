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

// The 7-round compression behind one scalar-argument interface, so the
// chunk, parent and root paths share a call shape whose arguments and result
// stay in VGPRs (array pointers would force the arrays to scratch). It is
// inlined like every device function of the library: the kernels make no
// calls (code_object_check.cpp, tests/test_abi_host.py).
struct CV8 {
  uint32_t w0, w1, w2, w3, w4, w5, w6, w7;
};

__device__ __forceinline__ CV8 compress_dev(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                         uint32_t c4, uint32_t c5, uint32_t c6, uint32_t c7,
                                         uint32_t m0, uint32_t m1, uint32_t m2, uint32_t m3,
                                         uint32_t m4, uint32_t m5, uint32_t m6, uint32_t m7,
                                         uint32_t m8, uint32_t m9, uint32_t m10, uint32_t m11,
                                         uint32_t m12, uint32_t m13, uint32_t m14, uint32_t m15,
                                         uint32_t ctr_lo, uint32_t ctr_hi, uint32_t block_len,
                                         uint32_t flags) {
  uint32_t cv[8] = {c0, c1, c2, c3, c4, c5, c6, c7};
  const uint32_t m[16] = {m0, m1, m2, m3, m4, m5, m6, m7, m8, m9, m10, m11, m12, m13, m14, m15};
  b3::compress_cv(cv, m, (static_cast<uint64_t>(ctr_hi) << 32) | ctr_lo, block_len, flags);
  return CV8{cv[0], cv[1], cv[2], cv[3], cv[4], cv[5], cv[6], cv[7]};
}

__device__ __forceinline__ void compress_call(uint32_t *cv, const uint32_t *m, uint64_t counter,
                                              uint32_t block_len, uint32_t flags) {
  const CV8 r = compress_dev(cv[0], cv[1], cv[2], cv[3], cv[4], cv[5], cv[6], cv[7], m[0], m[1],
                             m[2], m[3], m[4], m[5], m[6], m[7], m[8], m[9], m[10], m[11], m[12],
                             m[13], m[14], m[15], static_cast<uint32_t>(counter),
                             static_cast<uint32_t>(counter >> 32), block_len, flags);
  cv[0] = r.w0;
  cv[1] = r.w1;
  cv[2] = r.w2;
  cv[3] = r.w3;
  cv[4] = r.w4;
  cv[5] = r.w5;
  cv[6] = r.w6;
  cv[7] = r.w7;
}

__device__ __forceinline__ void parent_dev(uint32_t *out, const uint32_t *l, const uint32_t *r,
                                           uint32_t extra_flags) {
  uint32_t m[16];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    m[i] = l[i];
    m[i + 8] = r[i];
  }
#pragma unroll
  for (int i = 0; i < 8; i++) out[i] = b3::iv(i);
  compress_call(out, m, 0, b3::kBlockLen, b3::kParent | extra_flags);
}

// Partial or unaligned block: byte loads, zero padded (rare path).
__device__ __forceinline__ void load_block_bytes(uint32_t *m, const uint8_t *p, uint32_t bl) {
#pragma unroll
  for (int i = 0; i < 16; i++) {
    uint32_t w = 0;
    for (int b = 0; b < 4; b++) {
      const uint32_t o = 4 * i + b;
      if (o < bl) w |= static_cast<uint32_t>(p[o]) << (8 * b);
    }
    m[i] = w;
  }
}

__device__ __forceinline__ void load_block16(u32x4b *v, const uint8_t *p) {
  const u32x4b *q = reinterpret_cast<const u32x4b *>(p);
#pragma unroll
  for (int i = 0; i < 4; i++) v[i] = q[i];  // cached: the 4 loads share lines
}

// Two full, 16-B aligned chunks hashed together: the two compressions per
// block step are independent, which doubles the ILP of BLAKE3's serial G
// chains (one chunk per lane measured ~65 % SQ_WAIT_INST_ANY).
__device__ void chunk_cv_pair(uint32_t *cva, uint32_t *cvb, const uint8_t *pa, uint64_t idx) {
  const uint8_t *pb = pa + b3::kChunkLen;
#pragma unroll
  for (int i = 0; i < 8; i++) cva[i] = cvb[i] = b3::iv(i);
  u32x4b na[4], nb[4];
  load_block16(na, pa);
  load_block16(nb, pb);
  for (uint32_t b = 0; b < b3::kChunkLen / b3::kBlockLen; b++) {
    uint32_t ma[16], mb[16];
#pragma unroll
    for (int i = 0; i < 4; i++)
#pragma unroll
      for (int e = 0; e < 4; e++) {
        ma[4 * i + e] = na[i][e];
        mb[4 * i + e] = nb[i][e];
      }
    if (b + 1 < b3::kChunkLen / b3::kBlockLen) {
      load_block16(na, pa + (b + 1) * b3::kBlockLen);
      load_block16(nb, pb + (b + 1) * b3::kBlockLen);
    }
    const uint32_t flags = (b == 0 ? b3::kChunkStart : 0) | (b == 15 ? b3::kChunkEnd : 0);
    b3::compress_cv(cva, ma, idx, b3::kBlockLen, flags);
    b3::compress_cv(cvb, mb, idx + 1, b3::kBlockLen, flags);
  }
}

// Chunk chaining value; full aligned blocks are software-pipelined: the next
// block's four dwordx4 loads are in flight while the current block is
// compressed.
__device__ void chunk_cv_dev(uint32_t *cv, const uint8_t *p, uint32_t len, uint64_t idx,
                             uint32_t root_flag, bool aligned16) {
  const uint32_t nb = len == 0 ? 1 : (len + b3::kBlockLen - 1) / b3::kBlockLen;
  const uint32_t nfull = aligned16 ? len / b3::kBlockLen : 0;  // fast-path blocks
#pragma unroll
  for (int i = 0; i < 8; i++) cv[i] = b3::iv(i);
  u32x4b nxt[4];
  if (nfull > 0) load_block16(nxt, p);
  for (uint32_t b = 0; b < nb; b++) {
    const uint32_t off = b * b3::kBlockLen;
    const uint32_t bl = len - off < b3::kBlockLen ? len - off : b3::kBlockLen;
    uint32_t m[16];
    if (b < nfull) {
#pragma unroll
      for (int i = 0; i < 4; i++) {
        m[4 * i] = nxt[i][0];
        m[4 * i + 1] = nxt[i][1];
        m[4 * i + 2] = nxt[i][2];
        m[4 * i + 3] = nxt[i][3];
      }
      if (b + 1 < nfull) load_block16(nxt, p + off + b3::kBlockLen);
    } else {
      load_block_bytes(m, p + off, bl);
    }
    const uint32_t flags =
        (b == 0 ? b3::kChunkStart : 0) | (b + 1 == nb ? b3::kChunkEnd | root_flag : 0);
    compress_call(cv, m, idx, bl, flags);
  }
}

__device__ __forceinline__ void put(uint32_t *base, int slot, int lane, const uint32_t *cv,
                                    int T) {
#pragma unroll
  for (int w = 0; w < 8; w++) base[(slot * 8 + w) * T + lane] = cv[w];
}
__device__ __forceinline__ void get(const uint32_t *base, int slot, int lane, uint32_t *cv,
                                    int T) {
#pragma unroll
  for (int w = 0; w < 8; w++) cv[w] = base[(slot * 8 + w) * T + lane];
}

__device__ __forceinline__ void store_hash(uint8_t *o, const uint32_t *cv) {
#pragma unroll
  for (int w = 0; w < 8; w++)
#pragma unroll
    for (int b = 0; b < 4; b++) o[4 * w + b] = static_cast<uint8_t>(cv[w] >> (8 * b));
}

// Shard i of a launch is share t = i % per of stripe s = i / per: shares
// t < k at in0 + s * stride0 + t * pitch (data shares of a chunk, back to
// back), the rest at in1 + s * stride1 + (t - k) * pitch (its parity);
// digest at out + i * 32, i.e. [stripe][share]. A plain batch is per = k = 1.
struct B3Map {
  const uint8_t *in0, *in1;
  uint64_t stride0, stride1, pitch;
  uint32_t per, k;
  uint32_t out_per, out_off;  // digest of (s, t) at out + (s * out_per + out_off + t) * 32
};

__global__ __launch_bounds__(kB3Threads) void blake3_batch_kernel(
    const B3Map mp, uint64_t len, uint8_t *out, uint32_t count, uint32_t q_log2, uint32_t depth,
    uint32_t seg_log2) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds3[];
  // A segment of L = 2^seg_log2 lanes hashes one shard; a workgroup holds
  // T / L segments (small shards pack several to a workgroup, large ones
  // take the whole workgroup, L = T).
  const int T = blockDim.x;
  const int lane = threadIdx.x;
  const int L = 1 << seg_log2;
  const int ls = lane & (L - 1), sbase = lane - ls;
  const uint32_t shard_raw = blockIdx.x * static_cast<uint32_t>(T >> seg_log2) +
                             static_cast<uint32_t>(lane >> seg_log2);
  const bool live = shard_raw < count;
  // Segments past the last shard redo the last one (every lane must reach
  // the barriers below) and store nothing.
  const uint32_t shard = live ? shard_raw : count - 1;
  const uint32_t st = shard / mp.per, t = shard - st * mp.per;
  const uint8_t *p = t < mp.k ? mp.in0 + st * mp.stride0 + static_cast<uint64_t>(t) * mp.pitch
                              : mp.in1 + st * mp.stride1 + static_cast<uint64_t>(t - mp.k) * mp.pitch;
  uint8_t *o = out + (static_cast<uint64_t>(st) * mp.out_per + mp.out_off + t) * 32;
  const uint64_t n = len == 0 ? 1 : (len + b3::kChunkLen - 1) / b3::kChunkLen;
  const bool aligned16 = ((reinterpret_cast<uintptr_t>(p)) & 15) == 0;
  if (n == 1) {  // single chunk: it is the root (one lane per shard, L = 1)
    if (ls == 0 && live) {
      uint32_t cv[8];
      chunk_cv_dev(cv, p, static_cast<uint32_t>(len), 0, b3::kRoot, aligned16);
      store_hash(o, cv);
    }
    return;
  }
  uint32_t *stack = lds3;                          // [depth][8][T]
  uint32_t *nodes = lds3 + depth * 8 * T;          // [2][8][T]
  const uint64_t q = 1ull << q_log2;
  const uint64_t c0 = static_cast<uint64_t>(ls) * q;
  const uint64_t c1 = c0 + q < n ? c0 + q : n;
  uint32_t cv[8], left[8];
  int sp = 0;
  auto push = [&](uint64_t c) {  // merge complete subtrees, then push
    for (uint64_t t = c - c0 + 1; (t & 1) == 0; t >>= 1) {
      get(stack, --sp, lane, left, T);
      parent_dev(cv, left, cv, 0);
    }
    put(stack, sp++, lane, cv, T);
  };
  for (uint64_t c = c0; c < c1;) {
    if (aligned16 && c + 2 <= c1 && (c + 2) * b3::kChunkLen <= len) {
      uint32_t cvb[8];
      chunk_cv_pair(cv, cvb, p + c * b3::kChunkLen, c);
      push(c);
#pragma unroll
      for (int i = 0; i < 8; i++) cv[i] = cvb[i];
      push(c + 1);
      c += 2;
    } else {
      const uint64_t off = c * b3::kChunkLen;
      const uint32_t clen =
          static_cast<uint32_t>(len - off < b3::kChunkLen ? len - off : b3::kChunkLen);
      chunk_cv_dev(cv, p + off, clen, c, 0, aligned16);
      push(c);
      c += 1;
    }
  }
  if (c1 > c0) {  // a partial (last) group folds right to left
    get(stack, --sp, lane, cv, T);
    while (sp > 0) {
      get(stack, --sp, lane, left, T);
      parent_dev(cv, left, cv, 0);
    }
    put(nodes, 0, lane, cv, T);
  }
  __syncthreads();
  // Group nodes merge pairwise within each segment (odd node carried); every
  // segment has the same count, so the loop is uniform across the block.
  uint32_t cnt = static_cast<uint32_t>((n + q - 1) / q);  // >= 2 by the choice of q
  int cur = 0;
  while (cnt > 2) {
    const uint32_t half = cnt / 2;
    uint32_t *src = nodes + cur * 8 * T, *dst = nodes + (cur ^ 1) * 8 * T;
    if (static_cast<uint32_t>(ls) < half) {
      uint32_t r[8];
      get(src, 0, sbase + 2 * ls, left, T);
      get(src, 0, sbase + 2 * ls + 1, r, T);
      parent_dev(cv, left, r, 0);
      put(dst, 0, lane, cv, T);
    } else if ((cnt & 1) && static_cast<uint32_t>(ls) == half) {
      get(src, 0, sbase + cnt - 1, cv, T);
      put(dst, 0, lane, cv, T);
    }
    __syncthreads();
    cur ^= 1;
    cnt = half + (cnt & 1);
  }
  if (ls == 0 && live) {
    uint32_t r[8];
    const uint32_t *src = nodes + cur * 8 * T;
    get(src, 0, sbase, left, T);
    get(src, 0, sbase + 1, r, T);
    parent_dev(cv, left, r, b3::kRoot);
    store_hash(o, cv);
  }
}

}  // namespace

// Largest message the LDS tree handles: 256 lanes x 64 chunks = 16 MiB.
constexpr uint64_t kB3MaxLen = 256ull * 64 * b3::kChunkLen;

static hipError_t launch_b3(const B3Map &mp, uint64_t len, uint32_t count, uint8_t *out,
                            hipStream_t s) {
  if (count == 0) return hipSuccess;
  if (len > kB3MaxLen) return hipErrorInvalidValue;
  const uint64_t n = len == 0 ? 1 : (len + b3::kChunkLen - 1) / b3::kChunkLen;
  // Lanes per shard L: enough that each owns >= 2 chunks (pairs hash
  // interleaved), a power of two; L >= 64 takes a workgroup of L (at most
  // 256) lanes per shard, smaller L packs 256 / L shards into a workgroup
  // (a 16 KiB shard used to leave 3/4 of its wave idle).
  // (n >= 2 needs L >= 2: the root is the parent of the segment's first two
  // group nodes, so a segment must end with at least two of them.)
  uint32_t L = n >= 2 ? 2 : 1;
  while (L < kB3Threads && static_cast<uint64_t>(L) * 2 < n) L <<= 1;
  const int T = L >= 64 ? static_cast<int>(L) : kB3Threads;
  uint32_t seg_log2 = 0;
  while ((1u << seg_log2) < L) seg_log2++;
  uint32_t q_log2 = 0;
  while ((static_cast<uint64_t>(L) << q_log2) < n) q_log2++;
  const uint32_t depth = q_log2 + 1;
  const size_t lds = n == 1 ? 0 : (static_cast<size_t>(depth) + 2) * 8 * T * sizeof(uint32_t);
  const uint32_t per_block = static_cast<uint32_t>(T) / L;
  const uint32_t blocks = (count + per_block - 1) / per_block;
  hipLaunchKernelGGL(blake3_batch_kernel, dim3(blocks), dim3(T), lds, s, mp, len, out, count,
                     q_log2, depth, seg_log2);
  return hipGetLastError();
}

hipError_t launch_blake3_batch(const uint8_t *in, uint64_t len, uint32_t count,
                               uint64_t stride, uint8_t *out, hipStream_t s) {
  return launch_b3(B3Map{in, in, stride, stride, 0, 1, 1, 1, 0}, len, count, out, s);
}

hipError_t launch_blake3_stripes(const uint8_t *data, uint64_t data_stride, const uint8_t *parity,
                                 uint64_t parity_stride, uint64_t pitch, uint32_t k, uint32_t n,
                                 uint64_t len, uint32_t nstripes, uint8_t *out, hipStream_t s) {
  if (n == 0 || k > n || static_cast<uint64_t>(nstripes) * n > 0xFFFFFFFFull)
    return hipErrorInvalidValue;
  return launch_b3(B3Map{data, parity, data_stride, parity_stride, pitch, n, k, n, 0}, len,
                   nstripes * n, out, s);
}

hipError_t launch_blake3_stripes_part(const uint8_t *base, uint64_t stride, uint64_t pitch,
                                      uint32_t shares, uint32_t out_per, uint32_t out_off,
                                      uint64_t len, uint32_t nstripes, uint8_t *out,
                                      hipStream_t s) {
  if (shares == 0 || static_cast<uint64_t>(nstripes) * shares > 0xFFFFFFFFull)
    return hipErrorInvalidValue;
  return launch_b3(B3Map{base, base, stride, stride, pitch, shares, shares, out_per, out_off},
                   len, nstripes * shares, out, s);
}

}  // namespace storb_rs
