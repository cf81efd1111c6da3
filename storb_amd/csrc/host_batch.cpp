// host_batch.cpp -- pipelined host batches of the C ABI: the chunk loop of
// upload.rs:418-420 (storb_rs_encode_chunks, with blake3 piece ids:
// storb_rs_encode_chunks_hashed) and of download.rs:453-465
// (storb_rs_decode_chunks), double-buffered over two streams.
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <cstring>
#include <map>
#include <mutex>
#include <vector>

#include "ctx.hpp"

using namespace storb_rs;
using namespace storb_rs::detail;

namespace {

// The staged batch pipelines' device side: H2D on one stream (ctx->pipe[0]),
// kernels on another (ctx->stream), D2H on a third (ctx->pipe[1]), ordered by
// events per double-buffer slot. Batch i on stream i % 2 doing H2D -> kernel
// -> D2H (rounds 1-4) kept the two copy directions from overlapping:
// tools/sdma_probe.hip measured that arrangement at 50 GB/s of PCIe traffic
// against 76 GB/s for per-direction streams (profiles/r5w_sdma_probe.txt).
// Host buffers of slot b (pinned in / out) are reusable once its D2H is
// done (host_wait); device buffer b once its kernels (for the next H2D)
// and its D2H (for the next kernel) are done -- both ordered on the device.
struct Staging {
  storb_rs_ctx *ctx;
  hipStream_t in, k, out;
  bool used[2] = {false, false};
  explicit Staging(storb_rs_ctx *c) : ctx(c), in(c->pipe[0]), k(c->stream), out(c->pipe[1]) {}
  hipError_t init() {
    for (auto &row : ctx->stage_ev)
      for (auto &e : row)
        if (!e) {
          const hipError_t r = hipEventCreateWithFlags(&e, hipEventDisableTiming);
          if (r != hipSuccess) return r;
        }
    return hipSuccess;
  }
  hipEvent_t ev(int which, int b) const { return ctx->stage_ev[which][b]; }
  // Host: slot b's pinned buffers are free (its last D2H has landed).
  hipError_t host_wait(int b) { return used[b] ? hipEventSynchronize(ev(2, b)) : hipSuccess; }
  // Device: the H2D into slot b may start (the last kernel reading it is done).
  hipError_t before_in(int b) { return used[b] ? hipStreamWaitEvent(in, ev(1, b), 0) : hipSuccess; }
  // The kernels of slot b may start after its H2D (and after the last D2H
  // that read slot b's device outputs).
  hipError_t after_in(int b) {
    hipError_t r = hipEventRecord(ev(0, b), in);
    if (r == hipSuccess) r = hipStreamWaitEvent(k, ev(0, b), 0);
    if (r == hipSuccess && used[b]) r = hipStreamWaitEvent(k, ev(2, b), 0);
    return r;
  }
  hipError_t after_k(int b) {
    hipError_t r = hipEventRecord(ev(1, b), k);
    if (r == hipSuccess) r = hipStreamWaitEvent(out, ev(1, b), 0);
    return r;
  }
  hipError_t after_out(int b) {
    used[b] = true;
    return hipEventRecord(ev(2, b), out);
  }
};

}  // namespace

extern "C" {

// Pipelined batch encode: two pinned in/out buffer pairs and two streams.
// While the GPU copies and encodes batch i, the host packs batch i+1 and
// unpacks batch i-1 (hipMemcpyAsync from pinned memory is a true DMA).
// With hashes_out, the blake3 of every share is computed on the device
// right after the encode kernel and only the digests come back.
static int encode_chunks_locked(storb_rs_ctx *ctx, uint32_t k, uint32_t n,
                              const uint8_t *data, size_t chunk_len, uint32_t nchunks,
                              uint8_t *parity_out, uint8_t *hashes_out) {
  if (!valid_params(k, n)) return fail(ctx, STORB_RS_EINVAL, "invalid (k, n)");
  if (chunk_len == 0 || !data) return fail(ctx, STORB_RS_EINVAL, "empty chunk");
  const uint32_t p = n - k;
  if (nchunks == 0) return STORB_RS_OK;
  if (p > 0 && !parity_out) return fail(ctx, STORB_RS_EINVAL, "null parity_out");
  const size_t B = (chunk_len + k - 1) / k;
  if (hashes_out && B > 16ull * 1024 * 1024)
    return fail(ctx, STORB_RS_EINVAL, "blake3: share larger than 16 MiB");
  const size_t S = round_up(B, kAlign);
  const bool packed = (S == B) && (B * k == chunk_len);
  // ~64 MiB of input per batch keeps both DMA directions busy.
  const size_t per = static_cast<size_t>(k) * S;
  uint32_t batch = static_cast<uint32_t>(std::max<size_t>(1, (64ull << 20) / per));
  batch = std::min(batch, nchunks);
  const size_t hash_bytes = hashes_out ? static_cast<size_t>(batch) * n * 32 : 0;
  // Caller buffers that are page-locked (storb_rs_host_alloc / _register)
  // are DMA'd directly: no pack copy in, no unpack copy out.
  const bool in_direct = packed && range_pinned(data, static_cast<size_t>(nchunks) * chunk_len);
  const bool out_direct =
      p > 0 && S == B && range_pinned(parity_out, static_cast<size_t>(nchunks) * p * B);
  // Page-locked caller chunks without piece ids: the kernel reads them (and
  // writes parity) over PCIe directly (zero-copy). Kernel-driven PCIe
  // traffic overlaps both directions, where the SDMA copies of H2D and D2H
  // share one ceiling (57 GB/s total, round 1's PCIe probe; the bench line measures it now): 47 vs 35 GiB/s
  // measured. From pageable chunks the SDMA pipeline stays ahead (34 vs
  // 20 GiB/s: the host's packing competes with the kernel's reads of the
  // same staging), and the hashed path keeps the shares on the device.
  // Piece ids from the encode kernel itself (rs_encode_hash.hip) where the
  // geometry has one: digests land in [c][n] order. Not zero-copy: run on
  // page-locked chunks over PCIe (its lanes read 64-byte pieces 1 KiB
  // apart) it gave 30.9-33.0 GiB/s against 32.9 staged
  // (profiles/r4r_hashed_zc.txt).
  const bool fused = hashes_out && p > 0 && ctx->fused_hash && S == B &&
                     encode_hash_supported(k, n, B);
  const bool zc = ctx->zc_batch && !hashes_out && p > 0 && in_direct;
  DeviceGuard g(ctx->device);
  for (int b = 0; b < 2; b++) {
    if (!in_direct) HIP_TRY(ctx, ctx->pipe_in[b].ensure(per * batch));
    HIP_TRY(ctx, ctx->pipe_out[b].ensure(static_cast<size_t>(p) * S * batch + hash_bytes));
    if (!zc)
      HIP_TRY(ctx, ctx->pipe_dev[b].ensure(static_cast<size_t>(n) * S * batch + hash_bytes));
  }
  const uint32_t nb = (nchunks + batch - 1) / batch;
  HostPool &pool = host_pool(ctx);
  // Whether batch buffer b's digests came from the fused kernel or need the
  // hash launch: try_encode_hash may decline a batch the up-front check let
  // through.
  bool did_fuse[2] = {false, false};
  auto unpack = [&](uint32_t bi) {
    const int b = bi & 1;
    const uint32_t c0 = bi * batch, cn = std::min(batch, nchunks - c0);
    if (p > 0 && !out_direct) {
      if (S == B) {
        pool.copy(parity_out + static_cast<size_t>(c0) * p * B, ctx->pipe_out[b].p,
                  static_cast<size_t>(cn) * p * B, true);
      } else {
        pool.run(static_cast<int>(cn), [&](int c) {
          for (uint32_t i = 0; i < p; i++)
            std::memcpy(parity_out + ((static_cast<size_t>(c0) + c) * p + i) * B,
                        ctx->pipe_out[b].p + (static_cast<size_t>(c) * p + i) * S, B);
        });
      }
    }
    if (hashes_out)  // [c][t] from either the fused kernel or the hash launch
      std::memcpy(hashes_out + static_cast<size_t>(c0) * n * 32,
                  ctx->pipe_out[b].p + static_cast<size_t>(p) * S * batch,
                  static_cast<size_t>(cn) * n * 32);
  };
  Staging st(ctx);
  if (!zc) HIP_TRY(ctx, st.init());
  for (uint32_t bi = 0; bi < nb; bi++) {
    const int b = bi & 1;
    hipStream_t s = zc ? ctx->pipe[b] : st.k;
    // Pinned buffer pair b is free once batch bi-2 has landed (device
    // buffers are reused in device-side event order and need no host wait).
    if (bi >= 2 && !(in_direct && (out_direct || p == 0) && !hashes_out)) {
      HIP_TRY(ctx, zc ? hipStreamSynchronize(s) : st.host_wait(b));
      unpack(bi - 2);
    }
    const uint32_t c0 = bi * batch, cn = std::min(batch, nchunks - c0);
    const uint8_t *hin = in_direct ? data + static_cast<size_t>(c0) * chunk_len
                                   : ctx->pipe_in[b].p;
    if (in_direct) {
      // the H2D below reads the caller's page-locked chunks in place
    } else if (packed) {
      pool.copy(ctx->pipe_in[b].p, data + static_cast<size_t>(c0) * chunk_len, per * cn, true);
    } else {
      pool.run(static_cast<int>(cn), [&](int c) {
        const uint8_t *src = data + (static_cast<size_t>(c0) + c) * chunk_len;
        for (uint32_t j = 0; j < k; j++) {
          const size_t off = static_cast<size_t>(j) * B;
          const size_t cnt = off < chunk_len ? std::min(B, chunk_len - off) : 0;
          uint8_t *dst = ctx->pipe_in[b].p + static_cast<size_t>(c) * per +
                         static_cast<size_t>(j) * S;
          if (cnt) std::memcpy(dst, src + off, cnt);
          std::memset(dst + cnt, 0, S - cnt);
        }
      });
    }
    if (zc) {  // the kernel reads the pinned chunks and writes pinned parity over PCIe
      uint8_t *di, *dq;
      HIP_TRY(ctx, host_dev_ptr(const_cast<uint8_t *>(hin), &di));
      HIP_TRY(ctx, host_dev_ptr(out_direct ? parity_out + static_cast<size_t>(c0) * p * B
                                           : ctx->pipe_out[b].p,
                                &dq));
      std::vector<const uint8_t *> in(k);
      std::vector<uint8_t *> out(p);
      std::vector<size_t> ins(k, per), outs(p, static_cast<size_t>(p) * S);
      for (uint32_t j = 0; j < k; j++) in[j] = di + static_cast<size_t>(j) * S;
      for (uint32_t i = 0; i < p; i++) out[i] = dq + static_cast<size_t>(i) * S;
      const int rc = encode_apply(ctx, k, n, in.data(), ins.data(), out.data(), outs.data(), S,
                                  cn, s);
      if (rc) return rc;
      continue;
    }
    uint8_t *dd = ctx->pipe_dev[b].p;
    uint8_t *dp = dd + per * batch;
    uint8_t *dh = dp + static_cast<size_t>(p) * S * batch;  // digests (if any)
    HIP_TRY(ctx, st.before_in(b));
    HIP_TRY(ctx, hipMemcpyAsync(dd, hin, per * cn, hipMemcpyHostToDevice, st.in));
    HIP_TRY(ctx, st.after_in(b));
    hipError_t fe = hipSuccess;
    did_fuse[b] = fused && try_encode_hash(ctx, k, n, B, cn, dd, per, dp,
                                           static_cast<size_t>(p) * S, dh, s, &fe);
    if (did_fuse[b]) {
      HIP_TRY(ctx, fe);
    } else if (p > 0) {
      std::vector<const uint8_t *> in(k);
      std::vector<uint8_t *> out(p);
      std::vector<size_t> ins(k, per), outs(p, static_cast<size_t>(p) * S);
      for (uint32_t j = 0; j < k; j++) in[j] = dd + static_cast<size_t>(j) * S;
      for (uint32_t i = 0; i < p; i++) out[i] = dp + static_cast<size_t>(i) * S;
      const int rc = encode_apply(ctx, k, n, in.data(), ins.data(), out.data(), outs.data(), S,
                                  cn, s);
      if (rc) return rc;
    }
    size_t back = static_cast<size_t>(p) * S * cn;
    if (hashes_out && !did_fuse[b])  // every share of the batch, one launch, [c][t] digests
      HIP_TRY(ctx, launch_blake3_stripes(dd, per, dp, static_cast<size_t>(p) * S, S, k, n, B, cn,
                                         dh, s));
    HIP_TRY(ctx, st.after_k(b));
    if (back)
      HIP_TRY(ctx, hipMemcpyAsync(out_direct ? parity_out + static_cast<size_t>(c0) * p * B
                                             : ctx->pipe_out[b].p,
                                  dp, back, hipMemcpyDeviceToHost, st.out));
    if (hashes_out)
      HIP_TRY(ctx, hipMemcpyAsync(ctx->pipe_out[b].p + static_cast<size_t>(p) * S * batch, dh,
                                  static_cast<size_t>(cn) * n * 32, hipMemcpyDeviceToHost, st.out));
    HIP_TRY(ctx, st.after_out(b));
  }
  for (uint32_t bi = nb >= 2 ? nb - 2 : 0; bi < nb; bi++) {
    HIP_TRY(ctx, zc ? hipStreamSynchronize(ctx->pipe[bi & 1]) : st.host_wait(bi & 1));
    unpack(bi);
  }
  return STORB_RS_OK;
}

// Pipelined batch decode (the download path, download.rs:453-465, one
// chunk after another today). Every chunk selects its first k shares by
// index (decode_chunk, piece.rs:368-381) -- which shares those are differs
// from chunk to chunk, since Storb keeps the first k + 1 pieces to arrive
// (download.rs:363-451). Chunks whose k data shares are all present are pure
// host copies. The rest go, in order and whatever their erasure patterns, to
// per-stripe descriptor launches (decode_stripes.cpp): one launch per
// missing-row count per batch, each workgroup with its own chunk's pointers
// and matrix.
//  * Zero-copy: page-locked, aligned shares and output (storb_rs_host_alloc /
//    _register): the kernel reads the k survivors over PCIe where they lie
//    and writes only the rebuilt rows into `out`, while the host pool copies
//    the present data shares into `out` (disjoint rows).
//  * Staged: double-buffered pinned batches -- pack the k survivors into
//    pinned staging (present data shares also go straight to `out`), H2D,
//    rebuild the missing rows, D2H them, unpack into `out`.
// Geometries the descriptor kernel does not take (k > 32, > 16 rebuilt rows,
// the LDS comparison variant) run the staged pipeline with one launch per
// pattern group (decode_chunks_grouped).
static int decode_chunks_grouped(storb_rs_ctx *ctx, uint32_t k, size_t block, size_t outlen,
                                 const std::vector<uint32_t> &rest,
                                 const std::vector<const Pattern *> &pats,
                                 const std::vector<const uint8_t *> &slot_ptr, uint8_t *out,
                                 size_t out_stride) {
  HostPool &pool = host_pool(ctx);
  auto put_row = [&](uint32_t c, uint32_t row, const uint8_t *src) {
    const size_t o = static_cast<size_t>(row) * block;
    if (o < outlen)
      copy_nt(out + static_cast<size_t>(c) * out_stride + o, src, std::min(block, outlen - o));
  };
  std::map<const Pattern *, std::vector<uint32_t>> groups;
  for (uint32_t c : rest) groups[pats[c]].push_back(c);
  struct Item {
    const Pattern *pat;
    const uint32_t *chunks;
    uint32_t cn;
  };
  const size_t S = round_up(block, kAlign);
  const size_t per = static_cast<size_t>(k) * S;
  uint32_t batch = static_cast<uint32_t>(std::max<size_t>(1, (64ull << 20) / per));
  std::vector<Item> items;
  uint32_t emax = 0;
  for (auto &g : groups) {
    emax = std::max<uint32_t>(emax, static_cast<uint32_t>(g.first->missing.size()));
    for (size_t i = 0; i < g.second.size(); i += batch)
      items.push_back(Item{g.first, g.second.data() + i,
                           static_cast<uint32_t>(std::min<size_t>(batch, g.second.size() - i))});
  }
  batch = 0;
  for (auto &it : items) batch = std::max(batch, it.cn);
  for (int b = 0; b < 2; b++) {
    HIP_TRY(ctx, ctx->pipe_in[b].ensure(per * batch));
    HIP_TRY(ctx, ctx->pipe_out[b].ensure(static_cast<size_t>(emax) * S * batch));
    HIP_TRY(ctx, ctx->pipe_dev[b].ensure(static_cast<size_t>(k + emax) * S * batch));
  }
  auto unpack = [&](size_t ii) {
    const Item &it = items[ii];
    const uint8_t *src = ctx->pipe_out[ii & 1].p;
    const uint32_t e = static_cast<uint32_t>(it.pat->missing.size());
    pool.run(static_cast<int>(it.cn), [&](int c) {
      for (uint32_t r = 0; r < e; r++)
        put_row(it.chunks[c], it.pat->missing[r], src + (static_cast<size_t>(c) * e + r) * S);
    });
  };
  Staging st(ctx);
  HIP_TRY(ctx, st.init());
  for (size_t ii = 0; ii < items.size(); ii++) {
    const int b = ii & 1;
    hipStream_t s = st.k;
    if (ii >= 2) {  // pinned pair b is free once item ii-2 has landed
      HIP_TRY(ctx, st.host_wait(b));
      unpack(ii - 2);
    }
    const Item &it = items[ii];
    const uint32_t e = static_cast<uint32_t>(it.pat->missing.size());
    uint8_t *hin = ctx->pipe_in[b].p;
    pool.run(static_cast<int>(it.cn), [&](int c) {
      const uint32_t ch = it.chunks[c];
      for (uint32_t sl = 0; sl < k; sl++) {
        const uint8_t *src = slot_ptr[static_cast<size_t>(ch) * k + sl];
        uint8_t *dst = hin + static_cast<size_t>(c) * per + static_cast<size_t>(sl) * S;
        copy_nt(dst, src, block);
        if (S > block) std::memset(dst + block, 0, S - block);
        if (it.pat->slot_idx[sl] == sl) put_row(ch, sl, src);  // present data share
      }
    });
    uint8_t *dd = ctx->pipe_dev[b].p;
    uint8_t *dm = dd + per * it.cn;
    HIP_TRY(ctx, st.before_in(b));
    HIP_TRY(ctx, hipMemcpyAsync(dd, hin, per * it.cn, hipMemcpyHostToDevice, st.in));
    HIP_TRY(ctx, st.after_in(b));
    std::vector<const uint8_t *> in(k);
    std::vector<uint8_t *> o(e);
    std::vector<size_t> ins(k, per), outs(e, static_cast<size_t>(e) * S);
    for (uint32_t j = 0; j < k; j++) in[j] = dd + static_cast<size_t>(j) * S;
    for (uint32_t r = 0; r < e; r++) o[r] = dm + static_cast<size_t>(r) * S;
    const int rc = apply(ctx, k, e, it.pat->coef.data(), in.data(), ins.data(), o.data(),
                         outs.data(), S, it.cn, s);
    if (rc) return rc;
    HIP_TRY(ctx, st.after_k(b));
    HIP_TRY(ctx, hipMemcpyAsync(ctx->pipe_out[b].p, dm, static_cast<size_t>(e) * S * it.cn,
                                hipMemcpyDeviceToHost, st.out));
    HIP_TRY(ctx, st.after_out(b));
  }
  for (size_t ii = items.size() >= 2 ? items.size() - 2 : 0; ii < items.size(); ii++) {
    HIP_TRY(ctx, st.host_wait(ii & 1));
    unpack(ii);
  }
  return STORB_RS_OK;
}

static int decode_chunks_locked(storb_rs_ctx *ctx, uint32_t k, uint32_t n, size_t block,
                                size_t padlen, uint32_t nchunks, const uint8_t *const *shares,
                                const uint32_t *share_idx, const uint32_t *nshares,
                                uint8_t *out, size_t out_stride) {
  if (!valid_params(k, n)) return fail(ctx, STORB_RS_EINVAL, "invalid (k, n)");
  if (nchunks == 0) return STORB_RS_OK;
  if (!shares || !share_idx || !nshares || !out || block == 0 ||
      padlen >= static_cast<size_t>(k) * block)
    return fail(ctx, STORB_RS_EINVAL, "decode_chunks: bad arguments");
  const size_t outlen = static_cast<size_t>(k) * block - padlen;
  if (out_stride == 0) out_stride = outlen;
  if (out_stride < outlen) return fail(ctx, STORB_RS_EINVAL, "decode_chunks: out_stride < chunk");
  trim_patterns(ctx);
  // per chunk: its pattern and its k slot shares (pointers)
  std::vector<const Pattern *> pats(nchunks);
  std::vector<const uint8_t *> slot_ptr(static_cast<size_t>(nchunks) * k);
  std::vector<uint32_t> plain, rest, slot_pos;
  size_t off = 0;
  PatternMemo memo(ctx, k, n);
  for (uint32_t c = 0; c < nchunks; c++) {
    const int rc = memo.get(share_idx + off, nshares[c], &pats[c], slot_pos);
    if (rc) {
      ctx->last_error += " (chunk " + std::to_string(c) + ")";
      return rc;
    }
    for (uint32_t s = 0; s < k; s++) {
      slot_ptr[static_cast<size_t>(c) * k + s] = shares[off + slot_pos[s]];
      if (!slot_ptr[static_cast<size_t>(c) * k + s])
        return fail(ctx, STORB_RS_EINVAL, "decode_chunks: null share");
    }
    off += nshares[c];
    (pats[c]->missing.empty() ? plain : rest).push_back(c);
  }
  HostPool &pool = host_pool(ctx);
  auto sp = [&](uint32_t c, uint32_t sl) { return slot_ptr[static_cast<size_t>(c) * k + sl]; };
  auto put_row = [&](uint32_t c, uint32_t row, const uint8_t *src) {
    const size_t o = static_cast<size_t>(row) * block;
    if (o < outlen)
      copy_nt(out + static_cast<size_t>(c) * out_stride + o, src, std::min(block, outlen - o));
  };
  // Chunks with all k data shares present are a concatenation (zfec does the
  // same). Their host copies overlap the GPU work of the others: slice i of
  // n is copied while the device runs batch i (copy_plain(i, n)).
  auto copy_plain = [&](size_t i, size_t n) {
    const size_t a = plain.size() * i / n, b = plain.size() * (i + 1) / n;
    if (b > a)
      pool.run(static_cast<int>(b - a), [&](int j) {
        for (uint32_t s = 0; s < k; s++) put_row(plain[a + j], s, sp(plain[a + j], s));
      });
  };
  if (rest.empty()) {
    copy_plain(0, 1);
    return STORB_RS_OK;
  }
  DeviceGuard dg(ctx->device);
  const size_t S = round_up(block, kAlign);
  if (!desc_ok(ctx, k, n, S)) {
    copy_plain(0, 1);
    return decode_chunks_grouped(ctx, k, block, outlen, rest, pats, slot_ptr, out, out_stride);
  }
  const size_t W = 2 * static_cast<size_t>(k) + kSlotR;

  // Zero-copy chunks: page-locked caller shares AND output, no padding.
  const bool zc_out = ctx->zc_batch && padlen == 0 && block % kAlign == 0 &&
                      out_stride % kAlign == 0 &&
                      reinterpret_cast<uintptr_t>(out) % kAlign == 0 &&
                      range_pinned(out, static_cast<size_t>(nchunks - 1) * out_stride + outlen);
  std::vector<uint32_t> zc, staged;
  for (uint32_t c : rest) {
    bool ok = zc_out;
    for (uint32_t sl = 0; ok && sl < k; sl++)
      ok = reinterpret_cast<uintptr_t>(sp(c, sl)) % kAlign == 0 && range_pinned(sp(c, sl), block);
    (ok ? zc : staged).push_back(c);
  }
  if (!zc.empty()) {
    // Device address of a page-locked pointer: one hipHostGetDevicePointer
    // per registered range (a range maps linearly), not one per share.
    std::map<const uint8_t *, uint8_t *> dev_base;
    auto dev_ptr = [&](const uint8_t *p, size_t len, uint64_t *d) -> hipError_t {
      const uint8_t *b = pinned_base(p, len);
      if (!b) return hipErrorInvalidValue;
      auto f = dev_base.find(b);
      if (f == dev_base.end()) {
        uint8_t *db = nullptr;
        const hipError_t e = host_dev_ptr(const_cast<uint8_t *>(b), &db);
        if (e != hipSuccess) return e;
        f = dev_base.emplace(b, db).first;
      }
      *d = reinterpret_cast<uint64_t>(f->second + (p - b));
      return hipSuccess;
    };
    std::vector<const Pattern *> zp(zc.size());
    std::vector<uint64_t> ptr(zc.size() * W, 0);
    for (size_t i = 0; i < zc.size(); i++) {
      const uint32_t c = zc[i];
      zp[i] = pats[c];
      for (uint32_t sl = 0; sl < k; sl++) HIP_TRY(ctx, dev_ptr(sp(c, sl), block, &ptr[i * W + sl]));
      uint8_t *ob = out + static_cast<size_t>(c) * out_stride;
      for (size_t r = 0; r < pats[c]->missing.size(); r++)
        HIP_TRY(ctx, dev_ptr(ob + pats[c]->missing[r] * block, block, &ptr[i * W + k + r]));
    }
    int rc = apply_desc(ctx, k, block, false, zp, ptr, ctx->pipe[0]);
    if (rc) return rc;
    std::vector<std::pair<uint32_t, uint32_t>> rows;  // (chunk, present data slot)
    for (uint32_t c : zc)
      for (uint32_t sl = 0; sl < k; sl++)
        if (pats[c]->slot_idx[sl] == sl) rows.emplace_back(c, sl);
    pool.run(static_cast<int>(rows.size()), [&](int i) {  // overlaps the kernels
      put_row(rows[i].first, rows[i].second, sp(rows[i].first, rows[i].second));
    });
    if (staged.empty()) copy_plain(0, 1);  // also under the kernels
    HIP_TRY(ctx, hipStreamSynchronize(ctx->pipe[0]));
  }
  if (staged.empty()) return STORB_RS_OK;

  // Staged: batches of chunks in order, ~64 MiB of survivors each.
  const size_t per = static_cast<size_t>(k) * S;
  const uint32_t batch = static_cast<uint32_t>(
      std::min<size_t>(staged.size(), std::max<size_t>(1, (64ull << 20) / per)));
  uint32_t emax = 0;
  for (uint32_t c : staged) emax = std::max<uint32_t>(emax, static_cast<uint32_t>(pats[c]->missing.size()));
  for (int b = 0; b < 2; b++) {
    HIP_TRY(ctx, ctx->pipe_in[b].ensure(per * batch));
    HIP_TRY(ctx, ctx->pipe_out[b].ensure(static_cast<size_t>(emax) * S * batch));
    HIP_TRY(ctx, ctx->pipe_dev[b].ensure(static_cast<size_t>(k + emax) * S * batch));
  }
  const uint32_t nb = static_cast<uint32_t>((staged.size() + batch - 1) / batch);
  // Rebuilt rows of a batch packed chunk after chunk (row_off: rows before
  // staged chunk i within its batch), so the D2H moves only the rows rebuilt
  // -- download patterns mix chunks that lost 1 and 8 shares; an emax-row
  // pitch copied every chunk's emax rows back.
  std::vector<uint32_t> row_off(staged.size());
  for (size_t i = 0; i < staged.size(); i++)
    row_off[i] = i % batch ? row_off[i - 1] + static_cast<uint32_t>(pats[staged[i - 1]]->missing.size())
                           : 0;
  auto batch_rows = [&](uint32_t c0, uint32_t cn) {
    return static_cast<size_t>(row_off[c0 + cn - 1]) + pats[staged[c0 + cn - 1]]->missing.size();
  };
  auto unpack = [&](uint32_t bi) {
    const uint8_t *src = ctx->pipe_out[bi & 1].p;
    const uint32_t c0 = bi * batch, cn = std::min<uint32_t>(batch, static_cast<uint32_t>(staged.size()) - c0);
    pool.run(static_cast<int>(cn), [&](int c) {
      const uint32_t ch = staged[c0 + c];
      const Pattern &p = *pats[ch];
      for (size_t r = 0; r < p.missing.size(); r++)
        put_row(ch, p.missing[r], src + (static_cast<size_t>(row_off[c0 + c]) + r) * S);
    });
  };
  std::vector<const Pattern *> bp;
  std::vector<uint64_t> ptr;
  Staging st(ctx);
  HIP_TRY(ctx, st.init());
  for (uint32_t bi = 0; bi < nb; bi++) {
    const int b = bi & 1;
    hipStream_t s = st.k;
    if (bi >= 2) {  // pinned pair b is free once batch bi-2 has landed
      HIP_TRY(ctx, st.host_wait(b));
      unpack(bi - 2);
    }
    const uint32_t c0 = bi * batch, cn = std::min<uint32_t>(batch, static_cast<uint32_t>(staged.size()) - c0);
    uint8_t *hin = ctx->pipe_in[b].p;
    pool.run(static_cast<int>(cn), [&](int c) {
      const uint32_t ch = staged[c0 + c];
      for (uint32_t sl = 0; sl < k; sl++) {
        uint8_t *dst = hin + static_cast<size_t>(c) * per + static_cast<size_t>(sl) * S;
        copy_nt(dst, sp(ch, sl), block);
        if (S > block) std::memset(dst + block, 0, S - block);
        if (pats[ch]->slot_idx[sl] == sl) put_row(ch, sl, sp(ch, sl));  // present data share
      }
    });
    uint8_t *dd = ctx->pipe_dev[b].p;
    uint8_t *dm = dd + per * batch;
    HIP_TRY(ctx, st.before_in(b));
    HIP_TRY(ctx, hipMemcpyAsync(dd, hin, per * cn, hipMemcpyHostToDevice, st.in));
    HIP_TRY(ctx, st.after_in(b));
    bp.assign(cn, nullptr);
    ptr.assign(static_cast<size_t>(cn) * W, 0);
    for (uint32_t c = 0; c < cn; c++) {
      const Pattern &p = *pats[staged[c0 + c]];
      bp[c] = &p;
      for (uint32_t sl = 0; sl < k; sl++)
        ptr[c * W + sl] = reinterpret_cast<uint64_t>(dd + static_cast<size_t>(c) * per + sl * S);
      for (size_t r = 0; r < p.missing.size(); r++)
        ptr[c * W + k + r] =
            reinterpret_cast<uint64_t>(dm + (static_cast<size_t>(row_off[c0 + c]) + r) * S);
    }
    // staged shares are S-pitched: the kernel works on S-byte rows
    const int rc = apply_desc(ctx, k, S, false, bp, ptr, s);
    if (rc) return rc;
    HIP_TRY(ctx, st.after_k(b));
    HIP_TRY(ctx, hipMemcpyAsync(ctx->pipe_out[b].p, dm, batch_rows(c0, cn) * S,
                                hipMemcpyDeviceToHost, st.out));
    HIP_TRY(ctx, st.after_out(b));
    copy_plain(bi, nb);  // while the device runs batch bi
  }
  for (uint32_t bi = nb >= 2 ? nb - 2 : 0; bi < nb; bi++) {
    HIP_TRY(ctx, st.host_wait(bi & 1));
    unpack(bi);
  }
  return STORB_RS_OK;
}

// On an early error, batches already queued may still read or write the
// caller's buffers (page-locked ones in place): drain before returning.
static int encode_chunks_impl(storb_rs_ctx *ctx, uint32_t k, uint32_t n, const uint8_t *data,
                              size_t chunk_len, uint32_t nchunks, uint8_t *parity_out,
                              uint8_t *hashes_out) {
  if (!ctx) return STORB_RS_EINVAL;
  std::lock_guard<std::mutex> lk(ctx->mu);
  const int rc = encode_chunks_locked(ctx, k, n, data, chunk_len, nchunks, parity_out, hashes_out);
  if (rc) drain_streams(ctx);
  return rc;
}

int storb_rs_decode_chunks(storb_rs_ctx *ctx, uint32_t k, uint32_t n, size_t block,
                           size_t padlen, uint32_t nchunks, const uint8_t *const *shares,
                           const uint32_t *share_idx, const uint32_t *nshares, uint8_t *out,
                           size_t out_stride) {
  if (!ctx) return STORB_RS_EINVAL;
  std::lock_guard<std::mutex> lk(ctx->mu);
  const int rc = decode_chunks_locked(ctx, k, n, block, padlen, nchunks, shares, share_idx,
                                      nshares, out, out_stride);
  if (rc) drain_streams(ctx);
  return rc;
}

int storb_rs_encode_chunks(storb_rs_ctx *ctx, uint32_t k, uint32_t n, const uint8_t *data,
                           size_t chunk_len, uint32_t nchunks, uint8_t *parity_out) {
  return encode_chunks_impl(ctx, k, n, data, chunk_len, nchunks, parity_out, nullptr);
}

int storb_rs_encode_chunks_hashed(storb_rs_ctx *ctx, uint32_t k, uint32_t n,
                                  const uint8_t *data, size_t chunk_len, uint32_t nchunks,
                                  uint8_t *parity_out, uint8_t *hashes_out) {
  if (!hashes_out) return STORB_RS_EINVAL;
  return encode_chunks_impl(ctx, k, n, data, chunk_len, nchunks, parity_out, hashes_out);
}

}  // extern "C"
