// rs_encode_hash.hip -- encode with the blake3 piece ids in the same pass.
//
// Storb hashes every piece right after encode_chunk (upload.rs:623, then
// validator.rs:154,197,273 over the same bytes): SURVEY 8(f)1 asks for the
// hash in the encode kernel's epilogue. The two-kernel path
// (rs_apply_perm + blake3_batch_kernel) reads the k data shares twice and
// the parity shares once more after writing them; here every share byte
// crosses HBM once (k*B read, (n-k)*B written, 32 B of digest per share).
//
// Work layout. BLAKE3 consumes a 1 KiB chunk as 16 sequential 64-byte
// blocks, and the GF(2^8) encode is column-wise, so a lane owns one chunk
// position c of one stripe across all n shares: per block step it loads the
// 64-byte block b of chunk c of each data share, folds it into the (n-k)
// parity blocks (register v_perm tables, as rs_apply_perm), compresses it
// into that data share's chaining value, then stores each parity block and
// compresses it into the parity share's chaining value. No LDS, no barrier
// and no divergence in the chunk phase; a workgroup of 256 lanes covers
// 256 / C stripes of C = B / 1 KiB chunks (C <= 256, i.e. B <= 256 KiB).
// Then the chunk chaining values of each share merge pairwise in LDS (the
// last odd node carried up: that is BLAKE3's left-balanced tree), and the
// final parent, with ROOT, is the digest.
//
// Cost: the hash is VALU-bound (blake3.hip: 689 VALU per 64-byte block), so
// this kernel is too; the fold adds ~(n-k)/n * k * 5 ops per dword.
#include <hip/hip_runtime.h>

#include "blake3.hpp"
#include "rs_device.hpp"

namespace storb_rs {

namespace {

constexpr int kEHThreads = 256;

// The product's chunk-phase shape, from tools/ehbench.hip
// (profiles/r4k_ehbench.txt, config-2 geometry; the two-kernel path takes
// 1.0 ms for the same work, hashing alone 0.60): rolling prefetch (PF 2),
// one share per basic block, chaining values in VGPRs, write-back parity
// stores (ST 1): RS(4,2) 0.683 ms, RS(2,1) 0.634 ms. With non-temporal
// parity stores every variant took 1.25-1.55 ms: the lane's 64-byte pieces
// 1 KiB apart are partial lines, and a non-temporal store is not retired
// until it has gone past L2, so each block step's loads (one in-order vmcnt
// with the stores) waited out the previous step's writes -- 0.37 of the
// VALU issue cycles busy (SQ counters, profiles/r4j_valu_busy.json) against
// 0.94 with the stores removed.
#ifndef EH_PF
#define EH_PF 2
#define EH_GS 1
#define EH_CVL false
#define EH_ST 1
#endif

template <int K, int M>
__device__ __forceinline__ PermTab eh_tab(const EncHashArgs &a, int j, int i) {
  const uint32_t *t = a.tab[j * M + i];
  PermTab p{};
  p.t0lo = t[0];
  p.t0hi = t[1];
  p.t1lo = t[2];
  p.t1hi = t[3];
  p.t2 = t[4];
  return p;
}

// Chunk-phase shape (tools/ehbench.hip sweeps it). PF: 0 = each data block
// loaded right before it is folded, 1 = the next group's blocks loaded
// before the current group is compressed, 2 = rolling, share j's next block
// loaded right after its current one is compressed (before the step's
// parity stores). GS = shares compressed together in one basic block (2:
// two independent compressions for the scheduler to interleave; PF < 2).
// CVL = the chaining values live in LDS (the tree's area) instead of N x 8
// VGPRs. ST: 0 = non-temporal parity stores, 1 = write-back.
template <int K, int M, int PF, int GS, bool CVL, int DIAG = 0, int ST = 0>
__global__ __launch_bounds__(kEHThreads) void rs_encode_hash(const EncHashArgs a) {
  // DIAG (tools/ehbench.hip only, wrong output): 1 = no GF fold, 2 = no
  // parity stores, 3 = neither
  constexpr int N = K + M;
  constexpr int RI = (N + 1) / 2;  // tree items per lane per level (see below)
  static_assert(K % GS == 0, "data shares in whole groups");
  extern __shared__ __attribute__((aligned(16))) uint32_t nodes[];  // [N][8][256]
  const int lane = threadIdx.x;
  const uint32_t C = a.nchunks;
  const int sl = static_cast<int>(a.seg_log2);
  const int Cp = 1 << sl;
  const int spw = kEHThreads >> sl;  // stripes per workgroup
  const int ls = lane & (Cp - 1), seg = lane >> sl;
  const uint32_t stripe = blockIdx.x * static_cast<uint32_t>(spw) + static_cast<uint32_t>(seg);
  const bool live = stripe < a.nstripes;
  uint32_t cv[CVL ? 1 : N][8];
  auto cv_get = [&](int j, uint32_t *o) {
#pragma unroll
    for (int w = 0; w < 8; w++) o[w] = CVL ? nodes[(j * 8 + w) * kEHThreads + lane] : cv[CVL ? 0 : j][w];
  };
  auto cv_put = [&](int j, const uint32_t *v) {
#pragma unroll
    for (int w = 0; w < 8; w++) {
      if constexpr (CVL)
        nodes[(j * 8 + w) * kEHThreads + lane] = v[w];
      else
        cv[j][w] = v[w];
    }
  };

  // ---- chunk phase: lane = chunk ls of stripe `stripe`, all n shares ----
  if (live && static_cast<uint32_t>(ls) < C) {
    const uint8_t *d = a.data + stripe * a.data_stride + static_cast<uint64_t>(ls) * b3::kChunkLen;
    uint8_t *p = a.parity + stripe * a.parity_stride + static_cast<uint64_t>(ls) * b3::kChunkLen;
    {
      uint32_t iv8[8];
#pragma unroll
      for (int w = 0; w < 8; w++) iv8[w] = b3::iv(w);
#pragma unroll
      for (int j = 0; j < N; j++) cv_put(j, iv8);
    }
    auto load_blk = [&](int j, uint32_t b, uint32_t *m) {
      // the four dwordx4 of a block share 128-B lines with the next block:
      // cached loads
      const u32x4 *q =
          reinterpret_cast<const u32x4 *>(d + j * a.share_stride + b * b3::kBlockLen);
#pragma unroll
      for (int e = 0; e < 4; e++) {
        const u32x4 v = q[e];
        m[4 * e] = v[0];
        m[4 * e + 1] = v[1];
        m[4 * e + 2] = v[2];
        m[4 * e + 3] = v[3];
      }
    };
    const uint32_t last_flags = b3::kChunkEnd | (C == 1 ? b3::kRoot : 0u);
    if constexpr (PF == 2) {
      // Rolling prefetch: share j's block b + 1 is loaded into its own
      // buffer right after block b was folded and compressed, i.e. before
      // this step's parity stores. gfx950 counts loads and stores in one
      // in-order vmcnt, so a load issued after a store cannot be waited for
      // without waiting for the store too; issued this way no load ever
      // waits behind the parity stores.
      uint32_t blk[K][16];
#pragma unroll
      for (int j = 0; j < K; j++) load_blk(j, 0, blk[j]);
      for (uint32_t b = 0; b < b3::kChunkLen / b3::kBlockLen; b++) {
        const uint32_t flags = (b == 0 ? b3::kChunkStart : 0u) | (b == 15 ? last_flags : 0u);
        uint32_t par[M > 0 ? M : 1][16];  // (M = 0: hash only)
#pragma unroll
        for (int i = 0; i < M; i++)
#pragma unroll
          for (int w = 0; w < 16; w++) par[i][w] = 0;
#pragma unroll
        for (int j = 0; j < K; j++) {
#pragma unroll
          for (int e = 0; e < 4; e++) {
            if constexpr (DIAG & 1) continue;
            uint32_t s0[4], s1[4], s2[4];
#pragma unroll
            for (int w = 0; w < 4; w++) {
              const uint32_t x = blk[j][4 * e + w];
              s0[w] = x & 0x07070707u;
              s1[w] = (x >> 3) & 0x07070707u;
              s2[w] = (x >> 6) & 0x03030303u;
            }
#pragma unroll
            for (int i = 0; i < M; i++) {
              const PermTab t = eh_tab<K, M>(a, j, i);
#pragma unroll
              for (int w = 0; w < 4; w++)
                par[i][4 * e + w] = gf_madd_perm(par[i][4 * e + w], t, s0[w], s1[w], s2[w]);
            }
            __builtin_amdgcn_sched_barrier(0);
          }
          uint32_t c8[8];
          cv_get(j, c8);
          b3::compress_cv(c8, blk[j], static_cast<uint64_t>(ls), b3::kBlockLen, flags);
          cv_put(j, c8);
          __builtin_amdgcn_sched_barrier(0);
          if (b + 1 < b3::kChunkLen / b3::kBlockLen) load_blk(j, b + 1, blk[j]);
          __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int i = 0; i < M; i++) {
          if constexpr ((DIAG & 2) != 0) continue;
          u32x4 *o = reinterpret_cast<u32x4 *>(p + i * a.block + b * b3::kBlockLen);
#pragma unroll
          for (int e = 0; e < 4; e++) {
            const u32x4 v{par[i][4 * e], par[i][4 * e + 1], par[i][4 * e + 2], par[i][4 * e + 3]};
            if constexpr (ST == 1)
              o[e] = v;
            else
              st_stream(o + e, v);
          }
        }
#pragma unroll
        for (int i = 0; i < M; i++) {
          uint32_t c8[8];
          cv_get(K + i, c8);
          b3::compress_cv(c8, par[i], static_cast<uint64_t>(ls), b3::kBlockLen, flags);
          cv_put(K + i, c8);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
    } else {
    uint32_t cur[GS][16];
    if constexpr (PF)
#pragma unroll
      for (int h = 0; h < GS; h++) load_blk(h, 0, cur[h]);
    for (uint32_t b = 0; b < b3::kChunkLen / b3::kBlockLen; b++) {
      const uint32_t flags = (b == 0 ? b3::kChunkStart : 0u) | (b == 15 ? last_flags : 0u);
      uint32_t par[M > 0 ? M : 1][16];  // (M = 0: hash only)
#pragma unroll
      for (int i = 0; i < M; i++)
#pragma unroll
        for (int w = 0; w < 16; w++) par[i][w] = 0;
#pragma unroll
      for (int g = 0; g < K / GS; g++) {
        if constexpr (!PF)
#pragma unroll
          for (int h = 0; h < GS; h++) load_blk(g * GS + h, b, cur[h]);
        // fold, a dwordx4 at a time (selectors shared by the M rows), then
        // compress: fenced apart, or the scheduler interleaves the two and
        // holds every selector and both working sets at once
#pragma unroll
        for (int h = 0; h < GS; h++)
#pragma unroll
          for (int e = 0; e < 4; e++) {
            if constexpr (DIAG & 1) continue;
            uint32_t s0[4], s1[4], s2[4];
#pragma unroll
            for (int w = 0; w < 4; w++) {
              const uint32_t x = cur[h][4 * e + w];
              s0[w] = x & 0x07070707u;
              s1[w] = (x >> 3) & 0x07070707u;
              s2[w] = (x >> 6) & 0x03030303u;
            }
#pragma unroll
            for (int i = 0; i < M; i++) {
              const PermTab t = eh_tab<K, M>(a, g * GS + h, i);
#pragma unroll
              for (int w = 0; w < 4; w++)
                par[i][4 * e + w] = gf_madd_perm(par[i][4 * e + w], t, s0[w], s1[w], s2[w]);
            }
            __builtin_amdgcn_sched_barrier(0);
          }
        uint32_t nxt[GS][16];
        if constexpr (PF) {  // next group of this block, or the first of the next block
          const int gn = g + 1 < K / GS ? g + 1 : 0;
          const uint32_t bn = g + 1 < K / GS ? b : b + 1;
          if (bn < b3::kChunkLen / b3::kBlockLen)
#pragma unroll
            for (int h = 0; h < GS; h++) load_blk(gn * GS + h, bn, nxt[h]);
        }
#pragma unroll
        for (int h = 0; h < GS; h++) {
          uint32_t c8[8];
          cv_get(g * GS + h, c8);
          b3::compress_cv(c8, cur[h], static_cast<uint64_t>(ls), b3::kBlockLen, flags);
          cv_put(g * GS + h, c8);
        }
        // one group per basic block: unfenced, the scheduler hoists every
        // share's loads and folds and interleaves all the compressions
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (PF)
#pragma unroll
          for (int h = 0; h < GS; h++)
#pragma unroll
            for (int w = 0; w < 16; w++) cur[h][w] = nxt[h][w];
      }
#pragma unroll
      for (int i = 0; i < M; i++) {
        if constexpr ((DIAG & 2) != 0) continue;
        u32x4 *o = reinterpret_cast<u32x4 *>(p + i * a.block + b * b3::kBlockLen);
#pragma unroll
        for (int e = 0; e < 4; e++) {
          const u32x4 v{par[i][4 * e], par[i][4 * e + 1], par[i][4 * e + 2], par[i][4 * e + 3]};
          if constexpr (ST == 1)
            o[e] = v;  // write-back: the store retires into L2
          else
            st_stream(o + e, v);
        }
      }
#pragma unroll
      for (int i = 0; i < M; i++) {
        uint32_t c8[8];
        cv_get(K + i, c8);
        b3::compress_cv(c8, par[i], static_cast<uint64_t>(ls), b3::kBlockLen, flags);
        cv_put(K + i, c8);
        if ((i + 1) % GS == 0) __builtin_amdgcn_sched_barrier(0);
      }
    }
    }  // PF < 2
  }
  auto store_digest = [&](uint32_t s, int j, const uint32_t *h) {
    u32x4 *o = reinterpret_cast<u32x4 *>(a.hashes + (static_cast<uint64_t>(s) * N + j) * 32);
    o[0] = u32x4{h[0], h[1], h[2], h[3]};
    o[1] = u32x4{h[4], h[5], h[6], h[7]};
  };
  if (C == 1) {  // the single chunk is the root (ROOT set on its last block)
    if (live)
#pragma unroll
      for (int j = 0; j < N; j++) {
        uint32_t h[8];
        cv_get(j, h);
        store_digest(stripe, j, h);
      }
    return;
  }

  // ---- tree phase: merge each share's C chunk nodes in LDS ----
  // Level-l node t of share j of segment g sits in column g * (Cp >> l) + t
  // (level 0: the lane's own column). Lanes of dead segments write garbage
  // that only dead segments read; their digests are not stored.
  // (with CVL the chunk values already sit in the lane's own column)
  if constexpr (!CVL)
#pragma unroll
    for (int j = 0; j < N; j++)
#pragma unroll
      for (int w = 0; w < 8; w++) nodes[(j * 8 + w) * kEHThreads + lane] = cv[j][w];
  __syncthreads();
  uint32_t cnt = C;
  int lvl = 0;
  for (;;) {
    const uint32_t half = cnt / 2, nc = half + (cnt & 1);
    const bool last = cnt == 2;
    const uint32_t per_seg = N * nc;
    const uint32_t items = static_cast<uint32_t>(spw) * per_seg;
    const int src_w = Cp >> lvl, dst_w = src_w >> 1;
    // items <= 256 * N / 2 (nc <= Cp >> (lvl + 1)): RI per lane
    uint32_t res[RI][8];
#pragma unroll
    for (int r = 0; r < RI; r++) {
      const uint32_t item = static_cast<uint32_t>(lane) + static_cast<uint32_t>(r) * kEHThreads;
      if (item >= items) continue;
      const uint32_t g = item / per_seg, rem = item - g * per_seg;
      const uint32_t j = rem / nc, t = rem - j * nc;
      const uint32_t *base = nodes + j * 8 * kEHThreads;
      const uint32_t col = g * src_w + 2 * t;
      if (t < half) {
        uint32_t l[8], rr[8];
#pragma unroll
        for (int w = 0; w < 8; w++) {
          l[w] = base[w * kEHThreads + col];
          rr[w] = base[w * kEHThreads + col + 1];
        }
        b3::parent_cv(res[r], l, rr, last ? b3::kRoot : 0u);
        const uint32_t s = blockIdx.x * static_cast<uint32_t>(spw) + g;
        if (last && s < a.nstripes) store_digest(s, static_cast<int>(j), res[r]);
      } else {  // odd node carried to the next level
#pragma unroll
        for (int w = 0; w < 8; w++) res[r][w] = base[w * kEHThreads + col];
      }
    }
    if (last) break;
    __syncthreads();
#pragma unroll
    for (int r = 0; r < RI; r++) {
      const uint32_t item = static_cast<uint32_t>(lane) + static_cast<uint32_t>(r) * kEHThreads;
      if (item >= items) continue;
      const uint32_t g = item / per_seg, rem = item - g * per_seg;
      const uint32_t j = rem / nc, t = rem - j * nc;
      uint32_t *base = nodes + j * 8 * kEHThreads;
#pragma unroll
      for (int w = 0; w < 8; w++) base[w * kEHThreads + g * dst_w + t] = res[r][w];
    }
    __syncthreads();
    cnt = nc;
    lvl++;
  }
}

template <int K, int M, int PF, int GS, bool CVL, int DIAG = 0, int ST = 0>
hipError_t launch_eh(const EncHashArgs &a, hipStream_t s) {
  const int spw = kEHThreads >> a.seg_log2;
  const uint64_t blocks = (a.nstripes + spw - 1) / spw;
  const size_t lds =
      a.nchunks == 1 && !CVL ? 0 : static_cast<size_t>(K + M) * 8 * kEHThreads * 4;
  return launch_lds<rs_encode_hash<K, M, PF, GS, CVL, DIAG, ST>>(blocks, kEHThreads, lds, s, a);
}

}  // namespace

bool encode_hash_supported(uint32_t k, uint32_t n, uint64_t block) {
  const bool shape = (k == 2 && n == 3) || (k == 4 && n == 6);
  return shape && block > 0 && block % b3::kChunkLen == 0 && block / b3::kChunkLen <= kEHThreads;
}

hipError_t launch_encode_hash(const EncHashArgs &a, uint32_t k, uint32_t n, hipStream_t s) {
  if (!encode_hash_supported(k, n, a.block) || a.nchunks != a.block / b3::kChunkLen ||
      (1u << a.seg_log2) < a.nchunks || (1u << a.seg_log2) > kEHThreads)
    return hipErrorInvalidValue;
  if (a.nstripes == 0) return hipSuccess;
  if (k == 2) return launch_eh<2, 1, EH_PF, EH_GS, EH_CVL, 0, EH_ST>(a, s);
  return launch_eh<4, 2, EH_PF, EH_GS, EH_CVL, 0, EH_ST>(a, s);
}

}  // namespace storb_rs
