// host_calls.cpp -- single-chunk host calls of the C ABI: the entry points
// the zfec-rs shim reaches once per chunk (Fec::encode, piece.rs:329;
// Fec::decode, piece.rs:384-386) and host-side repair. Each call runs the
// kernel on page-locked staging mapped into the GPU (zero-copy over PCIe),
// uses page-locked caller buffers in place, and overlaps the staging copies
// of pageable ones with the kernel over column slices.
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <mutex>
#include <sched.h>

#include <thread>
#include <vector>

#include "ctx.hpp"
#include "rs_jit.hpp"
#include "seq.hpp"

using namespace storb_rs;
using namespace storb_rs::detail;

// Stage timestamps of the single calls, only in a build with
// -DSTORB_RS_CALL_TRACE (tools/callprobe.cpp's tracing build); the product
// build compiles the marks away.
#ifdef STORB_RS_CALL_TRACE
#include <chrono>
namespace {
struct Mark {
  const char *what;
  double us;
};
thread_local std::vector<Mark> g_marks;
void tmark(const char *w) {
  g_marks.push_back({w, std::chrono::duration<double, std::micro>(
                            std::chrono::steady_clock::now().time_since_epoch()).count()});
}
}  // namespace
extern "C" int storb_rs_debug_marks(const char **what, double *us, int max) {
  int n = 0;
  for (const Mark &m : g_marks) {
    if (n == max) break;
    what[n] = m.what;
    us[n++] = m.us;
  }
  g_marks.clear();
  return n;
}
#define TMARK(w) tmark(w)
#else
#define TMARK(w) ((void)0)
#endif

namespace storb_rs {
namespace detail {

// Single-call pipeline over column slices of one stripe. A chunk's shares
// are split into q column ranges [off, off+cnt) (16-B multiples); while the
// kernel works on slice t (zero-copy, over PCIe), the host packs slice t+1
// into pinned staging and unpacks slice t-1's outputs, so the staging copies
// of pageable caller buffers overlap the kernel instead of adding to it.
// q = 1 (small chunks) degenerates to pack -> launch -> sync -> unpack.
// Completion of a slice's kernel. A blocking hipEventSynchronize returned
// ~13 us after the kernel had ended (interrupt wake-up; stage marks of
// tools/callprobe.cpp, profiles/r3k_calltrace.txt) -- a quarter of a 1 MiB
// call -- and polling hipEventQuery slowed the calls down instead (runtime
// lock contention: page-locked (4, 6) encode 43.5 -> 60 us). So the stream
// itself writes a sequence number into page-locked memory once the slice's
// kernel has completed (hipStreamWriteValue32, ordered after the kernel like
// any stream operation), and the host spins on that word: no runtime call
// while waiting. After 2 ms of spinning the wait falls back to a blocking
// stream synchronisation (which also reports a device error).
#ifndef STORB_RS_SLICE_EVENTS
static int slice_signal(storb_rs_ctx *ctx, hipStream_t s, int t, uint32_t *seq) {
  if (!ctx->flag_pin.p) {
    HIP_TRY(ctx, ctx->flag_pin.ensure(kMaxSlices * 64));
    std::memset(ctx->flag_pin.p, 0, kMaxSlices * 64);
    HIP_TRY(ctx, host_dev_ptr(ctx->flag_pin.p, &ctx->flag_dev));
  }
  *seq = next_seq(ctx->flag_seq);
  HIP_TRY(ctx, hipStreamWriteValue32(s, ctx->flag_dev + t * 64, *seq, 0));
  return STORB_RS_OK;
}

static int slice_wait(storb_rs_ctx *ctx, hipStream_t s, int t, uint32_t seq) {
  const uint32_t *f = reinterpret_cast<const uint32_t *>(ctx->flag_pin.p + t * 64);
  const auto t0 = std::chrono::steady_clock::now();
  for (unsigned i = 1; __atomic_load_n(f, __ATOMIC_ACQUIRE) != seq; i++) {
#if defined(__x86_64__)
    __builtin_ia32_pause();
#endif
    if ((i & 1023) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(2)) {
      HIP_TRY(ctx, hipStreamSynchronize(s));
      break;
    }
  }
  return STORB_RS_OK;
}
#else  // the A/B baseline: one event per slice, blocking waits
static int slice_signal(storb_rs_ctx *ctx, hipStream_t s, int t, uint32_t *) {
  if (!ctx->slice_ev[t]) HIP_TRY(ctx, hipEventCreateWithFlags(&ctx->slice_ev[t], hipEventDisableTiming));
  HIP_TRY(ctx, hipEventRecord(ctx->slice_ev[t], s));
  return STORB_RS_OK;
}
static int slice_wait(storb_rs_ctx *ctx, hipStream_t, int t, uint32_t) {
  HIP_TRY(ctx, hipEventSynchronize(ctx->slice_ev[t]));
  return STORB_RS_OK;
}
#endif

int sliced(storb_rs_ctx *ctx, size_t S, const std::function<void(size_t, size_t)> &pack,
           const std::function<int(size_t, size_t)> &launch,
           const std::function<void(size_t, size_t)> &unpack, const std::function<void()> *during) {
  ctx->n_sliced++;
  int q = static_cast<int>(std::min<size_t>(kMaxSlices, S / (128u << 10)));
  if (q < 2) q = 1;
  const size_t slice = round_up((S + q - 1) / q, kAlign);
  q = static_cast<int>((S + slice - 1) / slice);
  auto range = [&](int t, size_t &off, size_t &cnt) {
    off = static_cast<size_t>(t) * slice;
    cnt = std::min(slice, S - off);
  };
  uint32_t seq[kMaxSlices] = {};
  int rc;
  for (int t = 0; t < q; t++) {
    size_t off, cnt;
    range(t, off, cnt);
    TMARK("pack");
    pack(off, cnt);
    TMARK("launch");
    if ((rc = launch(off, cnt))) return rc;
    TMARK("signal");
    if ((rc = slice_signal(ctx, ctx->stream, t, &seq[t]))) return rc;
    if (t > 0) {
      TMARK("wait");
      if ((rc = slice_wait(ctx, ctx->stream, t - 1, seq[t - 1]))) return rc;
      range(t - 1, off, cnt);
      TMARK("unpack");
      unpack(off, cnt);
    }
  }
  if (during) (*during)();  // host work that overlaps the last slice's kernel
  size_t off, cnt;
  range(q - 1, off, cnt);
  TMARK("wait");
  if ((rc = slice_wait(ctx, ctx->stream, q - 1, seq[q - 1]))) return rc;
  TMARK("unpack");
  unpack(off, cnt);
  TMARK("end");
  return STORB_RS_OK;
}

// The streamed single call (StreamArgs, rs_args.h; rs_apply_stream): one
// launch, issued BEFORE the host packs anything, whose workgroups wait for
// their slice's ready word; the host packs slice after slice and publishes
// each, then unpacks each slice as its done word turns. Per call: one
// launch, no stream synchronisation, the launch latency hidden behind the
// packing of slice 0. For k <= 8 and 1..8 rows on the table kernel (Storb's
// chunks up to 4 MiB, (2,3) (4,6) (8,12)); kNotStreamed = not applicable or
// not completed -- the caller then runs the sliced path, which recomputes
// everything (the caller's buffers are not touched by a failed attempt
// except staging and, for direct outputs, rows the classic path rewrites).
constexpr int kNotStreamed = -1;

int streamed(storb_rs_ctx *ctx, uint32_t k, uint32_t rows, const uint8_t *coef,
             const uint8_t *const *in, uint8_t *const *out, size_t S,
             const std::function<void(size_t, size_t)> &pack,
             const std::function<void(size_t, size_t)> &unpack, uint32_t enc_n = 0,
             const std::function<void()> *during = nullptr) {
  if (ctx->variant != STORB_RS_KERNEL_AUTO || k == 0 || rows == 0 || S % kAlign)
    return kNotStreamed;
  // Encode of (16, 24) / (32, 48): the bit-sliced encoder's streamed form;
  // otherwise the table kernel's, for k <= 8 and <= 8 rows.
  const uint32_t bs_cpt = enc_n ? bitslice_stream_cols_per_tile(k, enc_n) : 0;
  // (The table kernel streams up to k = 32, but measured at k = 32 -- (32, 48)
  // 32 MiB decode 2.32 ms against 0.94 ms on the sliced path, whose
  // compiled bit-sliced kernels read wider -- it stays for k <= 16.) Above
  // k = 16, with STORB_RS_JIT_STREAM=1, the matrix's compiled kernel in its
  // streamed form (rs_jit.cpp try_launch_stream) once it is compiled; off by
  // default, measured slower than the sliced path (rs_jit.cpp stream_enabled).
  const bool jit_st = !bs_cpt && k > 16 && jit::stream_form(k, rows) &&
                      jit::wanted(k, rows, static_cast<uint64_t>(k + rows) * S);
  if (!bs_cpt && !jit_st && (k > 16 || rows > 8)) return kNotStreamed;
  const uint32_t cpt = bs_cpt ? bs_cpt
                              : jit_st ? jit::stream_cols_per_tile(k, rows)
                                       : static_cast<uint32_t>(kThreadsTable);
  const uint32_t cols = static_cast<uint32_t>(S / 16);
  // 64 KiB of every share per slice, at most kMaxStreamSlices slices
  uint32_t slice_cols = 4096;
  if ((cols + slice_cols - 1) / slice_cols > static_cast<uint32_t>(kMaxStreamSlices))
    slice_cols = static_cast<uint32_t>(round_up((cols + kMaxStreamSlices - 1) / kMaxStreamSlices, cpt));
  const uint32_t nsl = (cols + slice_cols - 1) / slice_cols;
  hipStream_t s = ctx->stream;
  if (!ctx->sword_pin.p) {
    HIP_TRY(ctx, ctx->sword_pin.ensure(2 * kMaxStreamSlices * 64));
    std::memset(ctx->sword_pin.p, 0, 2 * kMaxStreamSlices * 64);
    HIP_TRY(ctx, host_dev_ptr(ctx->sword_pin.p, &ctx->sword_dev));
    HIP_TRY(ctx, ctx->scnt.ensure(kMaxStreamSlices * sizeof(uint32_t)));
    HIP_TRY(ctx, hipMemsetAsync(ctx->scnt.p, 0, kMaxStreamSlices * sizeof(uint32_t), s));
    HIP_TRY(ctx, hipStreamSynchronize(s));
    std::memset(ctx->sbase, 0, sizeof(ctx->sbase));
  }
  Tables *t = nullptr;
  int rc;
  if (!bs_cpt && !jit_st && (rc = get_tables(ctx, k, rows, coef, s, &t))) return rc;
  ApplyArgs a{};
  a.k = k;
  a.r = rows;
  for (uint32_t j = 0; j < k; j++) {
    a.in[j] = in[j];
    a.in_stride[j] = S;
  }
  for (uint32_t i = 0; i < rows; i++) {
    a.out[i] = out[i];
    a.out_stride[i] = S;
  }
  if (t) {
    a.ptab = reinterpret_cast<const PermTab *>(t->dev);
    a.tab_rows = static_cast<uint32_t>(rows_bucket(rows));
  }
  a.block = S;
  a.nstripes = 1;
  StreamArgs st{};
  uint32_t *words = reinterpret_cast<uint32_t *>(ctx->sword_dev);
  st.ready = words;
  st.done = words + kMaxStreamSlices * 16;
  st.cnt = reinterpret_cast<uint32_t *>(ctx->scnt.p);
  st.seq = next_seq(ctx->flag_seq);
  st.slice_cols = slice_cols;
  st.nslices = nsl;
  st.timeout_ticks = ctx->stream_timeout_ticks;  // default 1 s of s_memrealtime (100 MHz)
  uint32_t tiles[kMaxStreamSlices] = {};
  for (uint32_t i = 0; i < nsl; i++) {
    const uint32_t len = std::min(slice_cols, cols - i * slice_cols);
    tiles[i] = (len + cpt - 1) / cpt;
    st.target[i] = ctx->sbase[i] + tiles[i];
  }
  if (jit_st) {
    bool launched = false;
    HIP_TRY(ctx, jit::try_launch_stream(ctx->device, a, coef, st, s, &launched));
    if (!launched) return kNotStreamed;  // not compiled yet: nothing was queued
  } else {
    const hipError_t le = bs_cpt ? launch_encode_bitslice_stream(a, enc_n, st, s)
                                : launch_apply_stream(a, st, s);
    if (le == hipErrorInvalidValue) return kNotStreamed;  // nothing was queued
    HIP_TRY(ctx, le);
  }
  if (t && (rc = tables_used(ctx, t, s))) return rc;
  uint32_t *ready_h = reinterpret_cast<uint32_t *>(ctx->sword_pin.p);
  const uint32_t *done_h = ready_h + kMaxStreamSlices * 16;
  auto range = [&](uint32_t i, size_t &off, size_t &cnt) {
    off = static_cast<size_t>(i) * slice_cols * 16;
    cnt = std::min(static_cast<size_t>(slice_cols) * 16, S - off);
  };
  for (uint32_t i = 0; i < nsl; i++) {
    size_t off, cnt;
    range(i, off, cnt);
    TMARK("pack");
    pack(off, cnt);
    if (i == ctx->test_stall_slice && ctx->test_stall_calls > 0) {
      // test knob: the host descheduled past the device's wait
      ctx->test_stall_calls--;
      std::this_thread::sleep_for(std::chrono::microseconds(ctx->test_stall_us));
    }
    __atomic_store_n(ready_h + 16 * i, st.seq, __ATOMIC_RELEASE);
  }
  if (during) (*during)();  // host work that overlaps the kernel
  bool ok = true;
  for (uint32_t i = 0; i < nsl && ok; i++) {
    TMARK("wait");
    const auto t0 = std::chrono::steady_clock::now();
    for (unsigned it = 1; __atomic_load_n(done_h + 16 * i, __ATOMIC_ACQUIRE) != st.seq; it++) {
#if defined(__x86_64__)
      __builtin_ia32_pause();
#endif
      if ((it & 1023) == 0 &&
          std::chrono::steady_clock::now() - t0 >
              std::chrono::milliseconds(ctx->stream_host_wait_ms)) {
        // the GPU may just be busy with other streams' work: drain, look again
        HIP_TRY(ctx, hipStreamSynchronize(s));
        ok = __atomic_load_n(done_h + 16 * i, __ATOMIC_ACQUIRE) == st.seq;
        break;
      }
    }
    if (!ok) break;
    size_t off, cnt;
    range(i, off, cnt);
    TMARK("unpack");
    unpack(off, cnt);
  }
  TMARK("end");
  if (!ok) {  // a workgroup gave up waiting: counters unknown -- reset, redo classically
    HIP_TRY(ctx, hipStreamSynchronize(s));
    HIP_TRY(ctx, hipMemsetAsync(ctx->scnt.p, 0, kMaxStreamSlices * sizeof(uint32_t), s));
    HIP_TRY(ctx, hipStreamSynchronize(s));
    std::memset(ctx->sbase, 0, sizeof(ctx->sbase));
    ctx->n_stream_fallbacks++;
    return kNotStreamed;
  }
  for (uint32_t i = 0; i < nsl; i++) ctx->sbase[i] += tiles[i];
  ctx->n_streamed++;
  return STORB_RS_OK;
}

}  // namespace detail
}  // namespace storb_rs

extern "C" {

// data_out (storb_rs_encode_shares; null for storb_rs_encode): the k data
// shares are written too, B bytes each, the last one zero-padded -- what
// zfec-rs Fec::encode returns beside the parity (piece.rs:329). Those copies
// run on the host pool while the kernel works on the parity.
// Staging for this call on the calling thread's NUMA node (ctx.hpp
// pin_in_node): sched_getcpu is a vDSO read, the buffers are allocated once
// per node and kept.
// A thread that migrates between sockets would otherwise keep a staging pair
// per node at its largest size; on a node switch the other nodes' buffers
// above kStagingKeep are released (a (16, 24) 8 MiB chunk's 12 MiB pair stays).
static constexpr size_t kStagingKeep = 16ull << 20;

static void use_caller_staging(storb_rs_ctx *ctx) {
  int node = staging_node_env();
  if (node == -2) node = cpu_numa_node(sched_getcpu());
  const int slot = node >= 0 && node < storb_rs_ctx::kStagingNodes ? node
                                                                  : storb_rs_ctx::kStagingNodes;
  if (ctx->pin_in != &ctx->pin_in_node[slot]) {
    bool drained = false;
    for (int i = 0; i <= storb_rs_ctx::kStagingNodes; i++) {
      if (i == slot) continue;
      if (ctx->pin_in_node[i].cap <= kStagingKeep && ctx->pin_out_node[i].cap <= kStagingKeep)
        continue;
      // Every path that stages syncs or drains before it returns today; the
      // release still waits for the context's own streams (once, only on a
      // node switch), so a later asynchronous path cannot leave a copy or a
      // zero-copy kernel on unmapped memory.
      if (!drained) {
        (void)hipStreamSynchronize(ctx->stream);
        for (hipStream_t s : ctx->pipe)
          if (s) (void)hipStreamSynchronize(s);
        drained = true;
      }
      if (ctx->pin_in_node[i].cap > kStagingKeep) ctx->pin_in_node[i].release();
      if (ctx->pin_out_node[i].cap > kStagingKeep) ctx->pin_out_node[i].release();
    }
  }
  ctx->pin_in = &ctx->pin_in_node[slot];
  ctx->pin_out = &ctx->pin_out_node[slot];
  ctx->pin_node = slot < storb_rs_ctx::kStagingNodes ? node : -1;
}

static int encode_one(storb_rs_ctx *ctx, uint32_t k, uint32_t n, const uint8_t *data,
                      size_t len, uint8_t *const *parity_out, size_t *block_out,
                      size_t *padlen_out, uint8_t *const *data_out = nullptr) {
  if (!valid_params(k, n)) return fail(ctx, STORB_RS_EINVAL, "invalid (k, n)");
  if (len == 0 || !data) return fail(ctx, STORB_RS_EINVAL, "empty chunk");
  const size_t B = (len + k - 1) / k, pad = B * k - len;
  if (block_out) *block_out = B;
  if (padlen_out) *padlen_out = pad;
  const uint32_t p = n - k;
  if (data_out)
    for (uint32_t j = 0; j < k; j++)
      if (!data_out[j]) return fail(ctx, STORB_RS_EINVAL, "null share output");
  std::vector<CopySeg> dsegs;
  if (data_out)
    for (uint32_t j = 0; j < k; j++) {
      const size_t src = static_cast<size_t>(j) * B;
      const size_t avail = src < len ? std::min(B, len - src) : 0;
      if (avail) dsegs.push_back({data_out[j], data + src, avail});
      if (B > avail) dsegs.push_back({data_out[j] + avail, nullptr, B - avail});
    }
  // Runs once: a streamed call that gives up after its `during` step has
  // copied the data shares retries on the sliced path, which must not copy
  // the k * B bytes again.
  bool data_put = false;
  const std::function<void()> put_data = [&] {
    if (data_put) return;
    data_put = true;
    if (!dsegs.empty()) host_pool(ctx).copy_segs(dsegs.data(), dsegs.size());
  };
  if (p == 0) {
    put_data();
    return STORB_RS_OK;
  }
  if (!parity_out) return fail(ctx, STORB_RS_EINVAL, "null parity_out");
  for (uint32_t i = 0; i < p; i++)
    if (!parity_out[i]) return fail(ctx, STORB_RS_EINVAL, "null parity_out");
  if (k == 1) {
    put_data();
    // Storb sizes every chunk <= 64 KiB (objects < 256 KiB) k = 1, m = 2
    // (piece.rs:307-317). Every generator row is then [1] -- a single data
    // share's Vandermonde column is all ones -- so each parity share IS the
    // data share: a copy with no GF(2^8) work to offload, where a device
    // round trip would only add launch and PCIe latency.
    for (uint32_t i = 0; i < p; i++) std::memcpy(parity_out[i], data, len);
    return STORB_RS_OK;
  }
  const size_t S = round_up(B, kAlign);
  const bool zc = static_cast<size_t>(n) * S <= ctx->zc_max;
  // Page-locked, 16-B aligned caller buffers need no staging at all.
  auto aligned = [](const void *q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; };
  const bool in_direct = zc && pad == 0 && S == B && aligned(data) && range_pinned(data, len);
  bool out_direct = zc && S == B;
  for (uint32_t i = 0; out_direct && i < p; i++)
    out_direct = aligned(parity_out[i]) && range_pinned(parity_out[i], B);
  DeviceGuard g(ctx->device);
  use_caller_staging(ctx);
  if (!in_direct) HIP_TRY(ctx, ctx->pin_in->ensure(static_cast<size_t>(k) * S, ctx->pin_node));
  if (!out_direct) HIP_TRY(ctx, ctx->pin_out->ensure(static_cast<size_t>(p) * S, ctx->pin_node));
  if (!zc) HIP_TRY(ctx, ctx->stage.ensure(static_cast<size_t>(n) * S));
  HostPool &pool = host_pool(ctx);
  hipStream_t s = ctx->stream;
  std::vector<const uint8_t *> in(k);
  std::vector<uint8_t *> out(p);
  std::vector<size_t> ins(k, static_cast<size_t>(k) * S), outs(p, static_cast<size_t>(p) * S);
  // Zero-padded data shares, S-pitched (zfec pads the tail with zeros):
  // columns [off, off + cnt) of every share into pinned staging, the bytes
  // spread evenly over the host pool.
  std::vector<CopySeg> segs;
  auto pack = [&](size_t off, size_t cnt) {
    segs.clear();
    for (uint32_t j = 0; j < k; j++) {
      const size_t src = static_cast<size_t>(j) * B + off;
      size_t avail = off < B ? std::min(cnt, B - off) : 0;
      avail = src < len ? std::min(avail, len - src) : 0;
      uint8_t *dst = ctx->pin_in->p + static_cast<size_t>(j) * S + off;
      if (avail) segs.push_back({dst, data + src, avail});
      if (cnt > avail) segs.push_back({dst + avail, nullptr, cnt - avail});
    }
    pool.copy_segs(segs.data(), segs.size());
  };
  auto unpack = [&](size_t off, size_t cnt) {
    const size_t c = off < B ? std::min(cnt, B - off) : 0;
    if (!c) return;
    segs.clear();
    for (uint32_t i = 0; i < p; i++)
      segs.push_back({parity_out[i] + off, ctx->pin_out->p + static_cast<size_t>(i) * S + off, c});
    pool.copy_segs(segs.data(), segs.size());
  };
  if (zc) {  // the kernel reads and writes page-locked host memory over PCIe
    uint8_t *dd, *dp = nullptr;
    HIP_TRY(ctx, host_dev_ptr(in_direct ? const_cast<uint8_t *>(data) : ctx->pin_in->p, &dd));
    std::vector<uint8_t *> pd(p);
    if (out_direct) {
      for (uint32_t i = 0; i < p; i++) HIP_TRY(ctx, host_dev_ptr(parity_out[i], &pd[i]));
    } else {
      HIP_TRY(ctx, host_dev_ptr(ctx->pin_out->p, &dp));
      for (uint32_t i = 0; i < p; i++) pd[i] = dp + static_cast<size_t>(i) * S;
    }
    auto launch = [&](size_t off, size_t cnt) {
      for (uint32_t j = 0; j < k; j++) in[j] = dd + static_cast<size_t>(j) * S + off;
      for (uint32_t i = 0; i < p; i++) out[i] = pd[i] + off;
      return encode_apply(ctx, k, n, in.data(), ins.data(), out.data(), outs.data(), cnt, 1, s);
    };
    if (in_direct && out_direct) {  // nothing to overlap but the data shares
      const int rc = launch(0, S);
      if (rc) return rc;
      put_data();
      HIP_TRY(ctx, hipStreamSynchronize(s));
      return STORB_RS_OK;
    }
    const std::function<void(size_t, size_t)> pk = [&](size_t off, size_t cnt) {
      if (!in_direct) pack(off, cnt);
    };
    const std::function<void(size_t, size_t)> up = [&](size_t off, size_t cnt) {
      if (!out_direct) unpack(off, cnt);
    };
    {
      const std::vector<uint8_t> &enc = cached_enc(k, n);
      std::vector<const uint8_t *> sin(k);
      for (uint32_t j = 0; j < k; j++) sin[j] = dd + static_cast<size_t>(j) * S;
      const int rs = streamed(ctx, k, p, enc.data() + static_cast<size_t>(k) * k, sin.data(),
                              pd.data(), S, pk, up, n, data_out ? &put_data : nullptr);
      if (rs != kNotStreamed) return rs;
    }
    return sliced(ctx, S, pk, launch, up, data_out ? &put_data : nullptr);
  }
  pack(0, S);
  uint8_t *dd = ctx->stage.p, *dp = ctx->stage.p + static_cast<size_t>(k) * S;
  HIP_TRY(ctx, hipMemcpyAsync(dd, ctx->pin_in->p, static_cast<size_t>(k) * S,
                              hipMemcpyHostToDevice, s));
  for (uint32_t j = 0; j < k; j++) in[j] = dd + static_cast<size_t>(j) * S;
  for (uint32_t i = 0; i < p; i++) out[i] = dp + static_cast<size_t>(i) * S;
  int rc = encode_apply(ctx, k, n, in.data(), ins.data(), out.data(), outs.data(), S, 1, s);
  if (rc) return rc;
  HIP_TRY(ctx, hipMemcpyAsync(ctx->pin_out->p, dp, static_cast<size_t>(p) * S,
                              hipMemcpyDeviceToHost, s));
  put_data();
  HIP_TRY(ctx, hipStreamSynchronize(s));
  unpack(0, S);
  return STORB_RS_OK;
}

static int decode_one(storb_rs_ctx *ctx, uint32_t k, uint32_t n, const uint8_t *const *shares,
                    const uint32_t *share_idx, uint32_t nshares, size_t block,
                    size_t padlen, uint8_t *out) {
  if (!valid_params(k, n)) return fail(ctx, STORB_RS_EINVAL, "invalid (k, n)");
  if (!shares || !share_idx || !out || block == 0 ||
      padlen >= static_cast<size_t>(k) * block)
    return fail(ctx, STORB_RS_EINVAL, "decode: bad arguments");
  std::vector<uint32_t> slot_idx, slot_pos, missing;
  int rc = select_shares(ctx, k, n, share_idx, nshares, slot_idx, slot_pos);
  if (rc) return rc;
  std::vector<uint8_t> coef;
  rc = decode_rows(ctx, k, n, slot_idx, coef, missing);
  if (rc) return rc;
  const size_t outlen = static_cast<size_t>(k) * block - padlen;
  HostPool &pool = host_pool(ctx);
  std::vector<CopySeg> segs;
  auto put_present = [&] {  // surviving data shares: plain copies into out
    segs.clear();
    for (uint32_t s = 0; s < k; s++) {
      const size_t off = static_cast<size_t>(s) * block;
      if (slot_idx[s] < k && off < outlen)
        segs.push_back({out + off, shares[slot_pos[s]], std::min(block, outlen - off)});
    }
    pool.copy_segs(segs.data(), segs.size());
  };
  if (missing.empty()) {  // all data shares present: concatenation, as zfec
    put_present();
    return STORB_RS_OK;
  }
  if (k == 1) {  // any share of a k = 1 code is the data (encode_one)
    std::memcpy(out, shares[slot_pos[0]], outlen);
    return STORB_RS_OK;
  }
  const size_t S = round_up(block, kAlign);
  const uint32_t e = static_cast<uint32_t>(missing.size());
  const bool zc = static_cast<size_t>(k + e) * S <= ctx->zc_max;
  auto aligned = [](const void *q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; };
  // Page-locked, aligned caller shares / output are used in place.
  bool in_direct = zc && S == block;
  for (uint32_t c = 0; in_direct && c < k; c++)
    in_direct = aligned(shares[slot_pos[c]]) && range_pinned(shares[slot_pos[c]], block);
  const bool out_direct = zc && S == block && padlen == 0 && aligned(out) &&
                          range_pinned(out, outlen);
  DeviceGuard g(ctx->device);
  use_caller_staging(ctx);
  if (!in_direct) HIP_TRY(ctx, ctx->pin_in->ensure(static_cast<size_t>(k) * S, ctx->pin_node));
  if (!out_direct) HIP_TRY(ctx, ctx->pin_out->ensure(static_cast<size_t>(e) * S, ctx->pin_node));
  if (!zc) HIP_TRY(ctx, ctx->stage.ensure(static_cast<size_t>(k + e) * S));
  // columns [off, off + cnt) of row `row` of the chunk (truncated at outlen)
  auto put_cols = [&](uint32_t row, size_t off, size_t cnt, const uint8_t *src) {
    const size_t o = static_cast<size_t>(row) * block + off;
    size_t c = off < block ? std::min(cnt, block - off) : 0;
    c = o < outlen ? std::min(c, outlen - o) : 0;
    if (c) segs.push_back({out + o, src, c});
  };
  // slot shares into pinned staging; present data shares also into out
  auto pack = [&](size_t off, size_t cnt) {
    segs.clear();
    for (uint32_t c = 0; c < k; c++) {
      const uint8_t *src = shares[slot_pos[c]] + off;
      const size_t avail = off < block ? std::min(cnt, block - off) : 0;
      if (!in_direct) {
        uint8_t *dst = ctx->pin_in->p + static_cast<size_t>(c) * S + off;
        if (avail) segs.push_back({dst, src, avail});
        if (cnt > avail) segs.push_back({dst + avail, nullptr, cnt - avail});
      }
      if (slot_idx[c] < k) put_cols(c, off, cnt, src);
    }
    pool.copy_segs(segs.data(), segs.size());
  };
  auto unpack = [&](size_t off, size_t cnt) {
    if (out_direct) return;
    segs.clear();
    for (uint32_t r = 0; r < e; r++)
      put_cols(missing[r], off, cnt, ctx->pin_out->p + static_cast<size_t>(r) * S + off);
    pool.copy_segs(segs.data(), segs.size());
  };
  hipStream_t s = ctx->stream;
  std::vector<const uint8_t *> in(k);
  std::vector<uint8_t *> o(e);
  std::vector<size_t> ins(k, static_cast<size_t>(k) * S), outs(e, static_cast<size_t>(e) * S);
  if (zc) {  // zero-copy: the kernel reads / writes page-locked host memory
    std::vector<uint8_t *> id(k), od(e);
    uint8_t *base = nullptr;
    if (in_direct) {
      for (uint32_t c = 0; c < k; c++)
        HIP_TRY(ctx, host_dev_ptr(const_cast<uint8_t *>(shares[slot_pos[c]]), &id[c]));
    } else {
      HIP_TRY(ctx, host_dev_ptr(ctx->pin_in->p, &base));
      for (uint32_t c = 0; c < k; c++) id[c] = base + static_cast<size_t>(c) * S;
    }
    if (out_direct) {
      HIP_TRY(ctx, host_dev_ptr(out, &base));
      for (uint32_t r = 0; r < e; r++) od[r] = base + static_cast<size_t>(missing[r]) * block;
    } else {
      HIP_TRY(ctx, host_dev_ptr(ctx->pin_out->p, &base));
      for (uint32_t r = 0; r < e; r++) od[r] = base + static_cast<size_t>(r) * S;
    }
    auto launch = [&](size_t off, size_t cnt) {
      for (uint32_t c = 0; c < k; c++) in[c] = id[c] + off;
      for (uint32_t r = 0; r < e; r++) o[r] = od[r] + off;
      return apply(ctx, k, e, coef.data(), in.data(), ins.data(), o.data(), outs.data(), cnt, 1,
                   s);
    };
    if (in_direct && out_direct) {
      rc = launch(0, S);
      if (rc) return rc;
      put_present();  // host copies overlap the kernel (disjoint rows of out)
      HIP_TRY(ctx, hipStreamSynchronize(s));
      return STORB_RS_OK;
    }
    {
      std::vector<const uint8_t *> sin(id.begin(), id.end());
      const int rs = streamed(ctx, k, e, coef.data(), sin.data(), od.data(), S, pack, unpack);
      if (rs != kNotStreamed) return rs;
    }
    return sliced(ctx, S, pack, launch, unpack, nullptr);
  }
  pack(0, S);
  uint8_t *din = ctx->stage.p, *dout = ctx->stage.p + static_cast<size_t>(k) * S;
  HIP_TRY(ctx, hipMemcpyAsync(din, ctx->pin_in->p, static_cast<size_t>(k) * S,
                              hipMemcpyHostToDevice, s));
  for (uint32_t c = 0; c < k; c++) in[c] = din + static_cast<size_t>(c) * S;
  for (uint32_t r = 0; r < e; r++) o[r] = dout + static_cast<size_t>(r) * S;
  rc = apply(ctx, k, e, coef.data(), in.data(), ins.data(), o.data(), outs.data(), S, 1, s);
  if (rc) return rc;
  HIP_TRY(ctx, hipMemcpyAsync(ctx->pin_out->p, dout, static_cast<size_t>(e) * S,
                              hipMemcpyDeviceToHost, s));
  HIP_TRY(ctx, hipStreamSynchronize(s));
  unpack(0, S);
  return STORB_RS_OK;
}

static int repair_one(storb_rs_ctx *ctx, uint32_t k, uint32_t n, const uint8_t *const *shares,
                    const uint32_t *share_idx, uint32_t nshares, size_t block,
                    const uint32_t *targets, uint32_t ntargets, uint8_t *const *out) {
  if (!valid_params(k, n)) return fail(ctx, STORB_RS_EINVAL, "invalid (k, n)");
  if (!shares || !share_idx || (ntargets && (!targets || !out)) || block == 0)
    return fail(ctx, STORB_RS_EINVAL, "repair: bad arguments");
  std::vector<uint32_t> slot_idx, slot_pos;
  int rc = select_shares(ctx, k, n, share_idx, nshares, slot_idx, slot_pos);
  if (rc) return rc;
  std::vector<uint8_t> coef;
  rc = repair_rows(ctx, k, n, slot_idx, targets, ntargets, coef);
  if (rc || ntargets == 0) return rc;
  if (k == 1) {  // every share of a k = 1 code is the same bytes (encode_one)
    for (uint32_t r = 0; r < ntargets; r++) std::memcpy(out[r], shares[slot_pos[0]], block);
    return STORB_RS_OK;
  }
  const size_t S = round_up(block, kAlign);
  DeviceGuard g(ctx->device);
  use_caller_staging(ctx);
  HIP_TRY(ctx, ctx->pin_in->ensure(static_cast<size_t>(k) * S, ctx->pin_node));
  HIP_TRY(ctx, ctx->pin_out->ensure(static_cast<size_t>(ntargets) * S, ctx->pin_node));
  HIP_TRY(ctx, ctx->stage.ensure(static_cast<size_t>(k + ntargets) * S));
  for (uint32_t c = 0; c < k; c++) {
    std::memcpy(ctx->pin_in->p + static_cast<size_t>(c) * S, shares[slot_pos[c]], block);
    std::memset(ctx->pin_in->p + static_cast<size_t>(c) * S + block, 0, S - block);
  }
  hipStream_t s = ctx->stream;
  const bool zc = static_cast<size_t>(k + ntargets) * S <= ctx->zc_max;
  uint8_t *din = ctx->stage.p, *dout = ctx->stage.p + static_cast<size_t>(k) * S;
  if (zc) {  // zero-copy: the kernel works on the pinned staging directly
    HIP_TRY(ctx, host_dev_ptr(ctx->pin_in->p, &din));
    HIP_TRY(ctx, host_dev_ptr(ctx->pin_out->p, &dout));
  } else {
    HIP_TRY(ctx, hipMemcpyAsync(din, ctx->pin_in->p, static_cast<size_t>(k) * S,
                                hipMemcpyHostToDevice, s));
  }
  std::vector<const uint8_t *> in(k);
  std::vector<uint8_t *> o(ntargets);
  std::vector<size_t> ins(k, static_cast<size_t>(k) * S),
      outs(ntargets, static_cast<size_t>(ntargets) * S);
  for (uint32_t c = 0; c < k; c++) in[c] = din + static_cast<size_t>(c) * S;
  for (uint32_t r = 0; r < ntargets; r++) o[r] = dout + static_cast<size_t>(r) * S;
  rc = apply(ctx, k, ntargets, coef.data(), in.data(), ins.data(), o.data(), outs.data(), S, 1,
             s);
  if (rc) return rc;
  if (!zc)
    HIP_TRY(ctx, hipMemcpyAsync(ctx->pin_out->p, dout, static_cast<size_t>(ntargets) * S,
                                hipMemcpyDeviceToHost, s));
  HIP_TRY(ctx, hipStreamSynchronize(s));
  for (uint32_t r = 0; r < ntargets; r++)
    std::memcpy(out[r], ctx->pin_out->p + static_cast<size_t>(r) * S, block);
  return STORB_RS_OK;
}

int storb_rs_encode(storb_rs_ctx *ctx, uint32_t k, uint32_t n, const uint8_t *data,
                    size_t len, uint8_t *const *parity_out, size_t *block_out,
                    size_t *padlen_out) {
  if (!ctx) return STORB_RS_EINVAL;
  std::lock_guard<std::mutex> lk(ctx->mu);
  const int rc = encode_one(ctx, k, n, data, len, parity_out, block_out, padlen_out);
  if (rc) drain_streams(ctx);  // queued work may still touch caller buffers
  return rc;
}

int storb_rs_encode_shares(storb_rs_ctx *ctx, uint32_t k, uint32_t n, const uint8_t *data,
                           size_t len, uint8_t *const *shares_out, size_t *block_out,
                           size_t *padlen_out) {
  if (!ctx) return STORB_RS_EINVAL;
  std::lock_guard<std::mutex> lk(ctx->mu);
  if (!shares_out) return fail(ctx, STORB_RS_EINVAL, "null shares_out");
  const int rc = encode_one(ctx, k, n, data, len, valid_params(k, n) ? shares_out + k : nullptr,
                            block_out, padlen_out, valid_params(k, n) ? shares_out : nullptr);
  if (rc) drain_streams(ctx);  // queued work may still touch caller buffers
  return rc;
}

int storb_rs_decode(storb_rs_ctx *ctx, uint32_t k, uint32_t n, const uint8_t *const *shares,
                    const uint32_t *share_idx, uint32_t nshares, size_t block,
                    size_t padlen, uint8_t *out) {
  if (!ctx) return STORB_RS_EINVAL;
  std::lock_guard<std::mutex> lk(ctx->mu);
  const int rc = decode_one(ctx, k, n, shares, share_idx, nshares, block, padlen, out);
  if (rc) drain_streams(ctx);  // queued work may still touch caller buffers
  return rc;
}

int storb_rs_repair(storb_rs_ctx *ctx, uint32_t k, uint32_t n, const uint8_t *const *shares,
                    const uint32_t *share_idx, uint32_t nshares, size_t block,
                    const uint32_t *targets, uint32_t ntargets, uint8_t *const *out) {
  if (!ctx) return STORB_RS_EINVAL;
  std::lock_guard<std::mutex> lk(ctx->mu);
  const int rc = repair_one(ctx, k, n, shares, share_idx, nshares, block, targets, ntargets, out);
  if (rc) drain_streams(ctx);  // queued work may still touch caller buffers
  return rc;
}

}  // extern "C"
