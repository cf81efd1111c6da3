// host_async.cpp -- asynchronous single-chunk host calls of the C ABI.
//
// The reference calls encode_chunk / decode_chunk synchronously inside async
// tasks (upload.rs:418-420 in consume_bytes, download.rs:464 per chunk; SURVEY
// 8(b): "an async variant is a next item"). These entry points let a tokio
// integration await the GPU instead of blocking a worker thread:
//
//   start   validate, stage the input into the op's page-locked slot (the
//           caller may reuse its input as soon as the call returns), queue
//           the kernel on the slot's own stream -- zero-copy: it reads the
//           staging and writes the slot's page-locked output (or the
//           caller's output in place when that is page-locked) over PCIe --
//           and, if asked, a host function that calls notify(user) when the
//           device work is done;
//   test    poll the slot's completion event;
//   finish  wait if needed, copy the outputs into the caller's buffers,
//           return the slot, free the op.
//
// Ops of one context run concurrently, one slot (stream + staging) each; a
// finished op's slot is reused. The math is the synchronous calls' own
// (encode_apply / apply, host_calls.cpp), so the bytes are identical.
#include <hip/hip_runtime_api.h>
#include <unistd.h>

#include <cerrno>

#include <algorithm>
#include <cstring>
#include <mutex>
#include <vector>

#include "ctx.hpp"

using namespace storb_rs;
using namespace storb_rs::detail;

namespace storb_rs {
namespace detail {

constexpr size_t kMaxAsyncSlots = 64;

}  // namespace detail
}  // namespace storb_rs

struct storb_rs_op {
  storb_rs_ctx *ctx = nullptr;
  AsyncSlot *slot = nullptr;  // null: completed at start (no device work)
  int rc = STORB_RS_OK;
  // The context was destroyed before finish (storb_rs_ctx_destroy drained
  // the op's stream and detached it): ctx and slot are gone, rc = ECLOSED.
  bool closed = false;
  storb_rs_notify_fn notify = nullptr;
  void *user = nullptr;
  // Copies finish() makes from the slot's page-locked output: (dst, offset
  // in slot.out, bytes).
  struct Copy {
    uint8_t *dst;
    size_t off, len;
  };
  std::vector<Copy> copies;
};

namespace {

// The notification runs on a HIP runtime thread and owns its own copy of
// (notify, user): nothing it reads depends on *op, which finish() deletes.
struct Notify {
  storb_rs_notify_fn fn;
  void *user;
};

void notify_host_fn(void *p) {
  Notify *n = static_cast<Notify *>(p);
  n->fn(n->user);
  delete n;
}

// A free slot of the context (created on demand, at most kMaxAsyncSlots).
int acquire_slot(storb_rs_ctx *ctx, AsyncSlot **out) {
  std::lock_guard<std::mutex> lk(ctx->async_mu);
  for (auto &s : ctx->async_slots)
    if (!s->busy) {
      s->busy = true;
      *out = s.get();
      return STORB_RS_OK;
    }
  if (ctx->async_slots.size() >= kMaxAsyncSlots)
    return fail(ctx, STORB_RS_EBUSY, "too many unfinished async ops on this context");
  auto s = std::make_unique<AsyncSlot>();
  HIP_TRY(ctx, hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking));
  const hipError_t e = hipEventCreateWithFlags(&s->done, hipEventDisableTiming);
  if (e != hipSuccess) {
    (void)hipStreamDestroy(s->stream);
    return hip_fail(ctx, e, "hipEventCreateWithFlags(async slot)");
  }
  s->busy = true;
  *out = s.get();
  ctx->async_slots.push_back(std::move(s));
  return STORB_RS_OK;
}

// A slot keeps its page-locked staging for the next op up to this size;
// larger buffers (a 128-256 MiB k = 64 chunk) are released when the op is
// finished, so idle slots never pin more than 64 x 2 x kSlotKeep bytes.
constexpr size_t kSlotKeep = 32u << 20;

void release_slot(storb_rs_ctx *ctx, AsyncSlot *s, storb_rs_op *op = nullptr) {
  if (s->in.cap > kSlotKeep) s->in.release();
  if (s->out.cap > kSlotKeep) s->out.release();
  std::lock_guard<std::mutex> lk(ctx->async_mu);
  s->busy = false;
  if (op) ctx->live_ops.erase(op);
}

// Queue the notification, then record completion on the slot's stream: an
// op that tests done has had its notification delivered.
int queue_completion(storb_rs_ctx *ctx, storb_rs_op *op) {
  if (op->notify) {
    Notify *n = new Notify{op->notify, op->user};
    const hipError_t e = hipLaunchHostFunc(op->slot->stream, notify_host_fn, n);
    if (e != hipSuccess) {
      delete n;
      return hip_fail(ctx, e, "hipLaunchHostFunc(notify)");
    }
  }
  HIP_TRY(ctx, hipEventRecord(op->slot->done, op->slot->stream));
  return STORB_RS_OK;
}

bool aligned16(const void *q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; }

int encode_start(storb_rs_ctx *ctx, storb_rs_op *op, uint32_t k, uint32_t n,
                 const uint8_t *data, size_t len, uint8_t *const *parity_out, size_t *block_out,
                 size_t *padlen_out) {
  if (!valid_params(k, n)) return fail(ctx, STORB_RS_EINVAL, "invalid (k, n)");
  if (len == 0 || !data) return fail(ctx, STORB_RS_EINVAL, "empty chunk");
  const size_t B = (len + k - 1) / k, pad = B * k - len;
  if (block_out) *block_out = B;
  if (padlen_out) *padlen_out = pad;
  const uint32_t p = n - k;
  if (p == 0) return STORB_RS_OK;
  if (!parity_out) return fail(ctx, STORB_RS_EINVAL, "null parity_out");
  for (uint32_t i = 0; i < p; i++)
    if (!parity_out[i]) return fail(ctx, STORB_RS_EINVAL, "null parity_out");
  if (k == 1) {  // parity = data (host_calls.cpp encode_one): done at once
    for (uint32_t i = 0; i < p; i++) std::memcpy(parity_out[i], data, len);
    return STORB_RS_OK;
  }
  const size_t S = round_up(B, kAlign);
  bool out_direct = S == B;
  for (uint32_t i = 0; out_direct && i < p; i++)
    out_direct = aligned16(parity_out[i]) && range_pinned(parity_out[i], B);
  DeviceGuard g(ctx->device);
  int rc = acquire_slot(ctx, &op->slot);
  if (rc) return rc;
  AsyncSlot &sl = *op->slot;
  HIP_TRY(ctx, sl.in.ensure(static_cast<size_t>(k) * S));
  if (!out_direct) HIP_TRY(ctx, sl.out.ensure(static_cast<size_t>(p) * S));
  // zero-padded data shares, S-pitched, into the slot's staging
  HostPool &pool = host_pool(ctx);
  const int parts = static_cast<size_t>(k) * S >= (2u << 20) ? static_cast<int>(k) : 1;
  pool.run(parts, [&](int part) {
    for (uint32_t j = static_cast<uint32_t>(part); j < k; j += parts) {
      const size_t src = static_cast<size_t>(j) * B;
      const size_t avail = src < len ? std::min(B, len - src) : 0;
      uint8_t *dst = sl.in.p + static_cast<size_t>(j) * S;
      if (avail) std::memcpy(dst, data + src, avail);
      std::memset(dst + avail, 0, S - avail);
    }
  });
  uint8_t *dd = nullptr, *dp = nullptr;
  HIP_TRY(ctx, host_dev_ptr(sl.in.p, &dd));
  std::vector<const uint8_t *> in(k);
  std::vector<uint8_t *> out(p);
  std::vector<size_t> ins(k, static_cast<size_t>(k) * S), outs(p, static_cast<size_t>(p) * S);
  for (uint32_t j = 0; j < k; j++) in[j] = dd + static_cast<size_t>(j) * S;
  if (out_direct) {
    for (uint32_t i = 0; i < p; i++) HIP_TRY(ctx, host_dev_ptr(parity_out[i], &out[i]));
  } else {
    HIP_TRY(ctx, host_dev_ptr(sl.out.p, &dp));
    for (uint32_t i = 0; i < p; i++) {
      out[i] = dp + static_cast<size_t>(i) * S;
      op->copies.push_back({parity_out[i], static_cast<size_t>(i) * S, B});
    }
  }
  rc = encode_apply(ctx, k, n, in.data(), ins.data(), out.data(), outs.data(), S, 1, sl.stream);
  if (rc) return rc;
  return queue_completion(ctx, op);
}

int decode_start(storb_rs_ctx *ctx, storb_rs_op *op, uint32_t k, uint32_t n,
                 const uint8_t *const *shares, const uint32_t *share_idx, uint32_t nshares,
                 size_t block, size_t padlen, uint8_t *out) {
  if (!valid_params(k, n)) return fail(ctx, STORB_RS_EINVAL, "invalid (k, n)");
  if (!shares || !share_idx || !out || block == 0 ||
      padlen >= static_cast<size_t>(k) * block)
    return fail(ctx, STORB_RS_EINVAL, "decode: bad arguments");
  std::vector<uint32_t> slot_idx, slot_pos, missing;
  int rc = select_shares(ctx, k, n, share_idx, nshares, slot_idx, slot_pos);
  if (rc) return rc;
  for (uint32_t c = 0; c < k; c++)
    if (!shares[slot_pos[c]]) return fail(ctx, STORB_RS_EINVAL, "decode: null share");
  std::vector<uint8_t> coef;
  rc = decode_rows(ctx, k, n, slot_idx, coef, missing);
  if (rc) return rc;
  const size_t outlen = static_cast<size_t>(k) * block - padlen;
  auto put = [&](uint32_t row, const uint8_t *src) {  // row of the chunk, truncated
    const size_t off = static_cast<size_t>(row) * block;
    if (off < outlen) std::memcpy(out + off, src, std::min(block, outlen - off));
  };
  HostPool &pool = host_pool(ctx);
  const int parts = static_cast<size_t>(k) * block >= (1u << 20) ? static_cast<int>(k) : 1;
  if (missing.empty() || k == 1) {  // concatenation / the one share: done at once
    if (k == 1) {
      std::memcpy(out, shares[slot_pos[0]], outlen);
      return STORB_RS_OK;
    }
    pool.run(parts, [&](int part) {
      for (uint32_t s = static_cast<uint32_t>(part); s < k; s += parts) put(s, shares[slot_pos[s]]);
    });
    return STORB_RS_OK;
  }
  const size_t S = round_up(block, kAlign);
  const uint32_t e = static_cast<uint32_t>(missing.size());
  const bool out_direct = S == block && padlen == 0 && aligned16(out) && range_pinned(out, outlen);
  DeviceGuard g(ctx->device);
  rc = acquire_slot(ctx, &op->slot);
  if (rc) return rc;
  AsyncSlot &sl = *op->slot;
  HIP_TRY(ctx, sl.in.ensure(static_cast<size_t>(k) * S));
  if (!out_direct) HIP_TRY(ctx, sl.out.ensure(static_cast<size_t>(e) * S));
  // survivors into staging; present data shares straight into out
  pool.run(parts, [&](int part) {
    for (uint32_t c = static_cast<uint32_t>(part); c < k; c += parts) {
      const uint8_t *src = shares[slot_pos[c]];
      uint8_t *dst = sl.in.p + static_cast<size_t>(c) * S;
      std::memcpy(dst, src, block);
      if (S > block) std::memset(dst + block, 0, S - block);
      if (slot_idx[c] < k) put(c, src);
    }
  });
  uint8_t *base = nullptr;
  std::vector<const uint8_t *> in(k);
  std::vector<uint8_t *> o(e);
  std::vector<size_t> ins(k, static_cast<size_t>(k) * S), outs(e, static_cast<size_t>(e) * S);
  HIP_TRY(ctx, host_dev_ptr(sl.in.p, &base));
  for (uint32_t c = 0; c < k; c++) in[c] = base + static_cast<size_t>(c) * S;
  if (out_direct) {
    HIP_TRY(ctx, host_dev_ptr(out, &base));
    for (uint32_t r = 0; r < e; r++) o[r] = base + static_cast<size_t>(missing[r]) * block;
  } else {
    HIP_TRY(ctx, host_dev_ptr(sl.out.p, &base));
    for (uint32_t r = 0; r < e; r++) {
      o[r] = base + static_cast<size_t>(r) * S;
      const size_t off = static_cast<size_t>(missing[r]) * block;
      if (off < outlen)
        op->copies.push_back({out + off, static_cast<size_t>(r) * S, std::min(block, outlen - off)});
    }
  }
  rc = apply(ctx, k, e, coef.data(), in.data(), ins.data(), o.data(), outs.data(), S, 1,
             sl.stream);
  if (rc) return rc;
  return queue_completion(ctx, op);
}

// Common tail of the two starts: on success hand the op out; an op with no
// device work is complete at once (notify is called before returning); on
// error drain the slot's stream (queued work may still touch the staging)
// and give the slot back.
int finish_start(storb_rs_ctx *ctx, storb_rs_op *op, int rc, storb_rs_op **out) {
  if (rc) {
    if (op->slot) {
      DeviceGuard g(ctx->device);
      (void)hipStreamSynchronize(op->slot->stream);
      release_slot(ctx, op->slot);
    }
    delete op;
    return rc;
  }
  if (!op->slot && op->notify) op->notify(op->user);
  if (op->slot) {
    std::lock_guard<std::mutex> lk(ctx->async_mu);
    ctx->live_ops.insert(op);
  }
  *out = op;
  return STORB_RS_OK;
}

}  // namespace

namespace storb_rs {
namespace detail {

void invalidate_ops(storb_rs_ctx *ctx) {
  std::lock_guard<std::mutex> lk(ctx->async_mu);
  for (storb_rs_op *op : ctx->live_ops) {
    op->closed = true;
    op->rc = STORB_RS_ECLOSED;
    op->ctx = nullptr;
    op->slot = nullptr;
    op->copies.clear();
  }
  ctx->live_ops.clear();
}

}  // namespace detail
}  // namespace storb_rs

extern "C" {

int storb_rs_encode_async(storb_rs_ctx *ctx, uint32_t k, uint32_t n, const uint8_t *data,
                          size_t len, uint8_t *const *parity_out, size_t *block_out,
                          size_t *padlen_out, storb_rs_notify_fn notify, void *user,
                          storb_rs_op **op) {
  if (!ctx || !op) return STORB_RS_EINVAL;
  *op = nullptr;
  storb_rs_op *o = new storb_rs_op;
  o->ctx = ctx;
  o->notify = notify;
  o->user = user;
  int rc;
  {
    std::lock_guard<std::mutex> lk(ctx->mu);
    rc = encode_start(ctx, o, k, n, data, len, parity_out, block_out, padlen_out);
  }
  return finish_start(ctx, o, rc, op);
}

int storb_rs_decode_async(storb_rs_ctx *ctx, uint32_t k, uint32_t n,
                          const uint8_t *const *shares, const uint32_t *share_idx,
                          uint32_t nshares, size_t block, size_t padlen, uint8_t *out,
                          storb_rs_notify_fn notify, void *user, storb_rs_op **op) {
  if (!ctx || !op) return STORB_RS_EINVAL;
  *op = nullptr;
  storb_rs_op *o = new storb_rs_op;
  o->ctx = ctx;
  o->notify = notify;
  o->user = user;
  int rc;
  {
    std::lock_guard<std::mutex> lk(ctx->mu);
    rc = decode_start(ctx, o, k, n, shares, share_idx, nshares, block, padlen, out);
  }
  return finish_start(ctx, o, rc, op);
}

int storb_rs_op_test(const storb_rs_op *op) {
  if (!op) return STORB_RS_EINVAL;
  if (op->closed) return STORB_RS_ECLOSED;
  if (!op->slot) return STORB_RS_OK;
  const hipError_t q = hipEventQuery(op->slot->done);
  if (q == hipSuccess) return STORB_RS_OK;
  if (q == hipErrorNotReady) return STORB_RS_EAGAIN;
  return STORB_RS_EDEVICE;
}

int storb_rs_op_finish(storb_rs_op *op) {
  if (!op) return STORB_RS_EINVAL;
  int rc = op->rc;
  if (op->closed) {  // its context is gone: nothing to wait for or write
    delete op;
    return rc;
  }
  if (op->slot) {
    storb_rs_ctx *ctx = op->ctx;
    DeviceGuard g(ctx->device);
    // The stream: the kernel, the notification and the completion event.
    const hipError_t e = hipStreamSynchronize(op->slot->stream);
    if (e != hipSuccess) {
      rc = STORB_RS_EDEVICE;
    } else {
      const uint8_t *src = op->slot->out.p;
      std::lock_guard<std::mutex> lk(ctx->mu);  // the copy pool serves one caller at a time
      HostPool &pool = host_pool(ctx);
      const int parts = static_cast<int>(op->copies.size());
      size_t total = 0;
      for (auto &c : op->copies) total += c.len;
      if (parts > 1 && total >= (2u << 20))
        pool.run(parts, [&](int i) {
          const auto &c = op->copies[i];
          std::memcpy(c.dst, src + c.off, c.len);
        });
      else
        for (auto &c : op->copies) std::memcpy(c.dst, src + c.off, c.len);
    }
    release_slot(ctx, op->slot, op);
  }
  delete op;
  return rc;
}

// Ready-made notify function: wakes a waiter blocked on (or polling) the
// eventfd / pipe `(int)(intptr_t)user` by writing an 8-byte 1 to it.
void storb_rs_notify_fd(void *user) {
  const uint64_t one = 1;
  const int fd = static_cast<int>(reinterpret_cast<intptr_t>(user));
  ssize_t r;
  do {
    r = write(fd, &one, sizeof(one));
  } while (r < 0 && errno == EINTR);
}

}  // extern "C"
