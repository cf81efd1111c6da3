// ctx.hpp -- internals shared by the host-side translation units of the C
// ABI: the context (streams, staging, table cache), error plumbing, and the
// helpers behind every entry point.
//
//   storb_rs.cpp    context lifecycle, parameters, coefficient tables and the
//                   (rows x k) apply, device-resident batched calls, blake3,
//                   page-locked host registry
//   host_calls.cpp  single-chunk host calls (zfec-rs Fec::encode / decode,
//                   repair): zero-copy and column-sliced paths
//   host_batch.cpp  pipelined host batches (encode_chunks[_hashed],
//                   decode_chunks)
//   host_async.cpp  asynchronous single-chunk calls (start / test / finish)
#pragma once

#include <hip/hip_runtime_api.h>

#include <cstdint>
#include <functional>
#include <atomic>
#include <map>
#include <unordered_map>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <vector>

#include "../../include/storb_rs.h"
#include "gf256.hpp"
#include "host_pool.hpp"
#include "rs_kernels.hpp"

namespace storb_rs {
namespace detail {

constexpr size_t kAlign = 16;
constexpr int kMaxSlices = 8;
inline size_t round_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

struct DevBuf {
  uint8_t *p = nullptr;
  size_t cap = 0;
  ~DevBuf() {
    if (p) (void)hipFree(p);
  }
  hipError_t ensure(size_t n) {
    if (n <= cap) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    hipError_t e = hipMalloc(reinterpret_cast<void **>(&p), n);
    if (e == hipSuccess) cap = n;
    return e;
  }
};

// Page-locked memory on NUMA node `node` (mmap + mbind + first touch, then
// hipHostRegister, mapped for zero-copy kernels); unpin_node frees it.
hipError_t pin_alloc_node(size_t n, int node, uint8_t **p);
void pin_free_node(uint8_t *p, size_t n);
// STORB_RS_STAGING_NODE: unset = the single calls stage on the calling
// thread's node, -1 = where hipHostMalloc puts the buffers, N = node N.
int staging_node_env();  // -2 when unset
// NUMA node of logical CPU `cpu` (sysfs, cached; -1 unknown).
int cpu_numa_node(int cpu);

struct PinBuf {
  uint8_t *p = nullptr;
  size_t cap = 0;
  int node = -1;  // >= 0: pin_alloc_node memory on that node
  ~PinBuf() { release(); }
  void release() {
    if (p) {
      if (node >= 0)
        pin_free_node(p, cap);
      else
        (void)hipHostFree(p);
    }
    p = nullptr;
    cap = 0;
    node = -1;
  }
  // want: NUMA node for a new allocation (-1: the runtime's choice).
  hipError_t ensure(size_t n, int want = -1) {
    if (n <= cap && want == node) return hipSuccess;
    release();
    hipError_t e;
    if (want >= 0) {
      e = pin_alloc_node(n, want, &p);
      if (e == hipSuccess) node = want;
    } else {
      e = hipHostMalloc(reinterpret_cast<void **>(&p), n, hipHostMallocDefault);
    }
    if (e == hipSuccess)
      cap = n;
    else
      p = nullptr;
    return e;
  }
};

// Order marks of a stream: the events that tell when the launches reading a
// cached table or a descriptor slot have completed. One event recorded after
// every launch (rounds 1-4) costs ~1.2 us of queue processing per kernel
// boundary (profiles/r5g_ab_use_events.txt: headline step +0.5 %, download
// step +1.0 % without); instead each stream re-records one of kMarks events
// after every kMarkEvery-th use, and a resource keeps the (stream, use index)
// of its last use. A mark recorded at or after that index orders after it
// (stream order); a use no mark covers yet is covered by recording one on
// that stream when it is the caller's current stream (alive), otherwise by a
// device synchronisation (storb_rs.cpp covering_mark).
constexpr int kMarks = 8;
constexpr uint64_t kMarkEvery = 4;
struct StreamMarks {
  hipEvent_t ev[kMarks] = {};
  uint64_t at[kMarks] = {};  // use index ev[i] was last recorded after (0 = never)
  unsigned next = 0;
  uint64_t last = 0;         // newest recorded index
};

// Device-resident coefficient tables for one (rows x k) matrix, tiled in
// kSlotR x kSlotK blocks: for block b, ptab + b_off[b] PermTabs and
// btab + b_off[b]*256 product-table bytes.
//
// Nothing about a table blocks the host: the device copy is allocated
// stream-ordered (hipMallocAsync) and uploaded on the first caller's stream
// (`home`); a call on another stream waits for the `uploaded` event on the
// device. `uses` holds the table's last use index per stream (StreamMarks),
// so eviction (LRU, ctx->table_cap entries) can order the hipFreeAsync after
// the last kernel that reads the table on any stream.
struct Tables {
  uint8_t *dev = nullptr;
  size_t perm_bytes = 0;
  std::vector<size_t> b_off;
  std::vector<uint8_t> host;      // upload source, freed once the upload has completed
  hipStream_t home = nullptr;     // stream the upload was ordered on
  hipEvent_t uploaded = nullptr;  // recorded on `home` after the upload
  bool upload_done = false;
  std::vector<std::pair<hipStream_t, uint64_t>> uses;  // last use index per stream
  uint64_t tick = 0;              // LRU clock
  ~Tables() {
    // dev is pool memory (hipMallocAsync). Eviction and context teardown give
    // it back stream-ordered (storb_rs.cpp release_table, after the upload
    // and the last use on every stream); teardown frees a table whose release
    // failed itself, after a device synchronisation. Nothing is freed here:
    // a destructor has no stream the free could be ordered on.
    if (uploaded) (void)hipEventDestroy(uploaded);
  }
};

// One in-flight asynchronous host call (host_async.cpp): its own stream,
// completion event and page-locked staging, reused once the op is finished.
struct AsyncSlot {
  hipStream_t stream = nullptr;
  hipEvent_t done = nullptr;
  PinBuf in, out;
  bool busy = false;
};

// A decode pattern: which share sits in each of the k slots (zfec's slot
// arrangement of the first k by index, piece.rs:368-381), the rows of the
// inverted survivor matrix that rebuild the missing data shares, and their
// v_perm tables ([input][rows_bucket] PermTabs, padding rows zero) for the
// per-stripe descriptor kernels. Cached per context (LRU by tick).
struct Pattern {
  std::vector<uint32_t> slot_idx;
  std::vector<uint8_t> coef;      // e x k
  std::vector<uint32_t> missing;  // data index (= slot) of output row r
  std::vector<PermTab> tabs;      // k x rows_bucket(max(e, 1))
  uint64_t tick = 0;
};

// Descriptor upload slots per context: a slot is reused kDescRing calls
// later, by when the mark covering its last decode (at most kMarkEvery uses
// after it) has long completed -- the next copy into the slot waits for that
// mark on the descriptor stream, not on the caller's queue.
constexpr int kDescRing = 16;
// Flags of the events recorded after every launch only to ORDER later work
// (a table's last use before its free, a descriptor slot's last use before
// it is rewritten): no system-scope release. A default event's record
// writes back the L2s' dirty lines (up to 4 MiB per XCD of freshly streamed
// shares) before the next kernel on the stream may start; between the
// default bench's encode and decode launches that was most of a ~3.5 us
// boundary.
constexpr unsigned kOrderEvent = hipEventDisableTiming | hipEventDisableSystemFence;
constexpr uint64_t kThreadsTable = 256;  // lanes (16-B columns) per table-kernel tile

struct DeviceGuard {
  int prev = -1;
  bool ok = false;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    ok = hipSetDevice(dev) == hipSuccess;
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

}  // namespace detail
}  // namespace storb_rs

struct storb_rs_op;

struct storb_rs_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  hipStream_t pipe[2] = {nullptr, nullptr};
  int variant = STORB_RS_KERNEL_AUTO;
  std::mutex mu;
  std::string last_error;
  storb_rs::detail::DevBuf stage;
  storb_rs::detail::DevBuf pipe_dev[2];
  // Page-locked staging of the single calls, one pair per NUMA node of the
  // calling thread (host_calls.cpp use_caller_staging): the host copies stay
  // on the caller's socket and the device reaches the buffer over the
  // fabric -- a caller on the other socket than the GPU went 65.3 -> 59.5
  // us per (4, 6) 1 MiB encode, one on the GPU's socket is unchanged at
  // 51.4-51.9 (profiles/r4n_staging_numa.txt). Slot kStagingNodes: placed by the
  // runtime (STORB_RS_STAGING_NODE=-1, or the node is unknown).
  static constexpr int kStagingNodes = 8;
  storb_rs::detail::PinBuf pin_in_node[kStagingNodes + 1], pin_out_node[kStagingNodes + 1];
  storb_rs::detail::PinBuf *pin_in = &pin_in_node[kStagingNodes];
  storb_rs::detail::PinBuf *pin_out = &pin_out_node[kStagingNodes];
  int pin_node = -1;  // NUMA node of *pin_in / *pin_out (-1: runtime placement)
  storb_rs::detail::PinBuf pipe_in[2], pipe_out[2];
  // Events of the staged batch pipelines (host_batch.cpp Staging): per
  // double-buffer slot, H2D done / kernels done / D2H done.
  hipEvent_t stage_ev[3][2] = {};
  std::map<std::vector<uint8_t>, std::unique_ptr<storb_rs::detail::Tables>> tables;
  size_t table_cap = 1024;  // cached matrices (STORB_RS_TABLE_CACHE), LRU-evicted
  uint64_t table_tick = 0;
  std::unique_ptr<storb_rs::HostPool> pool;  // host copy workers, created on first use
  // Single-call paths whose staged bytes (in + out) are at most this size
  // run the kernel straight on the pinned staging buffers (zero-copy over
  // PCIe) instead of DMA in -> kernel -> DMA out: one launch and one sync
  // instead of three operations. STORB_RS_ZC_MAX, bytes; 0 disables.
  size_t zc_max = 0;
  // storb_rs_encode_chunks without piece ids: zero-copy kernels (1) or
  // SDMA H2D -> kernel -> D2H (0). STORB_RS_ZC_BATCH.
  bool zc_batch = true;
  // Encode + blake3 piece ids in one kernel (rs_encode_hash.hip) where the
  // geometry has one; 0 = encode kernel then hash kernel. STORB_RS_FUSED_HASH.
  bool fused_hash = true;
  hipEvent_t slice_ev[storb_rs::detail::kMaxSlices] = {};  // sliced single-call pipeline
  // Slice-completion words the single-call streams write (64 B apart) and
  // the host spins on (host_calls.cpp slice_signal / slice_wait).
  storb_rs::detail::PinBuf flag_pin;
  uint8_t *flag_dev = nullptr;
  uint32_t flag_seq = 0;
  // Streamed single calls (host_calls.cpp streamed): ready / done words
  // (page-locked, 64 B apart), per-slice device counters and their expected
  // base values (the counters only ever count up).
  storb_rs::detail::PinBuf sword_pin;
  uint8_t *sword_dev = nullptr;
  storb_rs::detail::DevBuf scnt;
  uint32_t sbase[storb_rs::kMaxStreamSlices] = {};
  // Decode patterns by (k, n, slot share indices) and the ring the
  // per-stripe descriptors go through: page-locked source, device copy;
  // desc_use[i]: (stream, use index) of that slot's last decode launches;
  // desc_cp[i]: recorded on desc_stream after the slot's last copy.
  std::map<std::vector<uint32_t>, std::unique_ptr<storb_rs::detail::Pattern>> patterns;
  uint64_t pattern_tick = 0;
  storb_rs::detail::PinBuf desc_pin[storb_rs::detail::kDescRing];
  storb_rs::detail::DevBuf desc_dev[storb_rs::detail::kDescRing];
  std::pair<hipStream_t, uint64_t> desc_use[storb_rs::detail::kDescRing] = {};
  hipEvent_t desc_cp[storb_rs::detail::kDescRing] = {};
  // Order marks per stream and the context's use counter (StreamMarks).
  std::unordered_map<hipStream_t, storb_rs::detail::StreamMarks> marks;
  uint64_t use_idx = 0;
  hipStream_t desc_stream = nullptr;  // the descriptor copies
  hipEvent_t desc_copied = nullptr;
  unsigned desc_next = 0;
  // Slots of the asynchronous host calls (host_async.cpp); async_mu guards
  // the busy flags, which finish() clears without holding mu, and the set of
  // ops started and not yet finished, which storb_rs_ctx_destroy invalidates
  // (an op finished after its context is gone must not touch it).
  std::mutex async_mu;
  std::vector<std::unique_ptr<storb_rs::detail::AsyncSlot>> async_slots;
  std::set<storb_rs_op *> live_ops;
  // Single-call path counters (storb_rs_ctx_stats).
  std::atomic<uint64_t> n_streamed{0}, n_stream_fallbacks{0}, n_sliced{0};
  // Device-wide synchronisations the ordering fallbacks took (a table's or a
  // descriptor slot's last use on a stream no mark covers): rare by design,
  // counted so a caller-stream pattern that hits them shows.
  std::atomic<uint64_t> n_device_syncs{0};
  // tables.size(), kept beside the map (updated under mu) so storb_rs_ctx_stats
  // reads it without waiting for a call that holds mu.
  std::atomic<uint64_t> n_tables{0};
  // NUMA node of the thread that created the context (-1 unknown) and of the
  // device it got: storb_rs_ctx_create(-1) picks among the caller's node's GPUs.
  int create_node = -1, device_node = -1;
  // Streamed single calls: how long a workgroup waits for its slice's ready
  // word (s_memrealtime ticks, 100 MHz) and how long the host waits for a
  // done word before it drains the stream and looks again (ms). Test knob
  // (read once, at context creation): STORB_RS_TEST_STREAM_STALL=
  // "<ticks>,<host ms>,<slice>,<us>,<calls>" shortens both and, in the first
  // <calls> streamed calls, makes the host sleep <us> before publishing slice
  // <slice>, so a test can force the give-up path (tests/test_gpu_runtime.py).
  uint64_t stream_timeout_ticks = 100000000ull;
  int stream_host_wait_ms = 500;
  uint32_t test_stall_slice = UINT32_MAX;
  uint32_t test_stall_us = 0;
  uint32_t test_stall_calls = 0;
};

namespace storb_rs {
namespace detail {

inline int fail(storb_rs_ctx *ctx, int code, const std::string &msg) {
  if (ctx) ctx->last_error = msg;
  return code;
}

inline int hip_fail(storb_rs_ctx *ctx, hipError_t e, const char *what) {
  std::string m = std::string(what) + ": " + hipGetErrorString(e);
  return fail(ctx, e == hipErrorOutOfMemory ? STORB_RS_ENOMEM : STORB_RS_EDEVICE, m);
}

#define HIP_TRY(ctx, expr)                              \
  do {                                                  \
    hipError_t e_ = (expr);                             \
    if (e_ != hipSuccess) return hip_fail(ctx, e_, #expr); \
  } while (0)

// Generator rows of (k, n), built once per geometry.
const std::vector<uint8_t> &cached_enc(uint32_t k, uint32_t n);
// Contexts created with device -1 take devices round-robin.
int next_round_robin();
// Host BLAKE3 hash of len bytes (blake3_host.cpp).
void blake3_host(const uint8_t *data, size_t len, uint8_t out[32]);
// [p, p+len) inside one storb_rs_host_alloc / _register range.
bool range_pinned(const void *p, size_t len);
// Base of the registered / allocated page-locked range holding [p, p+len), or null.
const uint8_t *pinned_base(const void *p, size_t len);
Variant pick_variant(const storb_rs_ctx *ctx);
// Device tables of a rows x k coefficient matrix (cached per context), made
// ready for launches on stream s; call tables_used() after those launches.
int get_tables(storb_rs_ctx *ctx, uint32_t k, uint32_t rows, const uint8_t *coef,
               hipStream_t s, Tables **out);
int tables_used(storb_rs_ctx *ctx, Tables *t, hipStream_t s);
// One use of stream s by launches reading a context resource: its index
// (StreamMarks), recording a mark when due.
hipError_t stream_used(storb_rs_ctx *ctx, hipStream_t s, uint64_t *use);
// An event that completes once use `use` on stream s has, or null when none
// can be had without a device synchronisation: a recorded mark at or after
// the use, else a mark recorded now when s is `live` (the stream of the
// current call).
hipError_t covering_mark(storb_rs_ctx *ctx, hipStream_t s, uint64_t use, hipStream_t live,
                         hipEvent_t *ev);
// out_r = sum_j coef[r][j] * in_j for every stripe, tiled onto kernel slots.
// copy[j] != null (decode into a separate buffer): input j is also stored
// to copy[j] (by the kernel where it can, else copied first); rows may be 0.
int apply(storb_rs_ctx *ctx, uint32_t k, uint32_t rows, const uint8_t *coef,
          const uint8_t *const *d_in, const size_t *in_stride, uint8_t *const *d_out,
          const size_t *out_stride, size_t block, uint32_t nstripes, hipStream_t s,
          uint8_t *const *copy = nullptr, const size_t *copy_stride = nullptr);
// Parity rows of (k, n): the bit-sliced encoder where compiled in, else apply.
int encode_apply(storb_rs_ctx *ctx, uint32_t k, uint32_t n, const uint8_t *const *d_in,
                 const size_t *in_stride, uint8_t *const *d_out, const size_t *out_stride,
                 size_t block, uint32_t nstripes, hipStream_t s);
// Encode + blake3 of all n shares in one kernel (rs_encode_hash.hip), digest
// of share t of stripe s at d_hashes + (s*n + t)*32: true if launched (*err
// its launch status), false if the geometry / alignment has no fused kernel
// or ctx->fused_hash is off.
bool try_encode_hash(storb_rs_ctx *ctx, uint32_t k, uint32_t n, size_t block,
                     uint32_t nstripes, const uint8_t *d_data, size_t data_stride,
                     uint8_t *d_parity, size_t parity_stride, uint8_t *d_hashes, hipStream_t s,
                     hipError_t *err);
// decode_chunk's selection (first k by index) and zfec's slot arrangement.
int select_shares(storb_rs_ctx *ctx, uint32_t k, uint32_t n, const uint32_t *share_idx,
                  uint32_t nshares, std::vector<uint32_t> &slot_idx,
                  std::vector<uint32_t> &slot_pos);
// Rows of the inverted survivor matrix that rebuild the missing data shares.
int decode_rows(storb_rs_ctx *ctx, uint32_t k, uint32_t n,
                const std::vector<uint32_t> &slot_idx, std::vector<uint8_t> &coef,
                std::vector<uint32_t> &missing);
// Rows that regenerate arbitrary target shares (data or parity).
int repair_rows(storb_rs_ctx *ctx, uint32_t k, uint32_t n,
                const std::vector<uint32_t> &slot_idx, const uint32_t *targets,
                uint32_t ntargets, std::vector<uint8_t> &coef);
HostPool &host_pool(storb_rs_ctx *ctx);
// The decode pattern of one stripe from its offered shares (select_shares +
// decode_rows, cached on the context); slot_pos[s] = position in share_idx[]
// of the share in slot s.
int get_pattern(storb_rs_ctx *ctx, uint32_t k, uint32_t n, const uint32_t *share_idx,
                uint32_t nshares, const Pattern **out, std::vector<uint32_t> &slot_pos);
// get_pattern for the stripes of one call (k, n fixed): stripes whose offered
// shares are distinct indices < 64 are keyed by the bit set of their first k
// (what the selection depends on) in a small direct-mapped memo, so a batch
// of a download's chunks -- a handful of patterns, each offered in many
// arrival orders -- runs the selection, the key and the cache lookup once per
// pattern instead of once per stripe. Anything else (duplicates, n > 64, the
// error cases) goes to get_pattern itself. Valid within one call only.
class PatternMemo {
 public:
  PatternMemo(storb_rs_ctx *ctx, uint32_t k, uint32_t n) : ctx_(ctx), k_(k), n_(n) {}
  int get(const uint32_t *share_idx, uint32_t nshares, const Pattern **out,
          std::vector<uint32_t> &slot_pos);

 private:
  static constexpr uint32_t kSlots = 256;
  storb_rs_ctx *ctx_;
  uint32_t k_, n_;
  uint64_t key_[kSlots] = {};
  const Pattern *pat_[kSlots] = {};
};
// Per-stripe descriptor launches (rs_apply_desc). Item i rebuilds the rows of
// pattern pats[i] from the k inputs ptr[i*W .. +k) into the outputs
// ptr[i*W + k .. + e) and, with copy, stores input j also to ptr[i*W + k +
// kSlotR + j] (0 = not stored), W = 2k + kSlotR. Items are grouped by row
// count, one launch per group; items with e = 0 only matter with copy.
// Needs desc_ok(). The descriptors are uploaded stream-ordered on s.
int apply_desc(storb_rs_ctx *ctx, uint32_t k, size_t block, bool copy,
               const std::vector<const Pattern *> &pats, const std::vector<uint64_t> &ptr,
               hipStream_t s);
// Drop least recently used patterns once the cache is full (call at the
// start of a call only: Patterns stay valid until the call returns).
void trim_patterns(storb_rs_ctx *ctx);
// One pattern for nstripes stripes of the device layout (storb_rs.h
// decode_batch_dev): rebuild the missing rows into d_out, assembling the
// present data shares too when d_out is a separate buffer.
int decode_pattern_batch(storb_rs_ctx *ctx, uint32_t k, size_t block, uint32_t nstripes,
                         const Pattern &p, const uint8_t *d_data, size_t data_stride,
                         const uint8_t *d_parity, size_t parity_stride, uint8_t *d_out,
                         size_t out_stride, hipStream_t s);
// Whether the descriptor kernel takes this geometry (k <= kSlotK, at most
// kSlotR rows, 16-B shares, the table-kernel variant in use).
bool desc_ok(const storb_rs_ctx *ctx, uint32_t k, uint32_t n, size_t block);
// Wait for everything queued on the context's own streams, ignoring errors
// (the early-error paths of the host calls, whose kernels may still be
// reading / writing the caller's page-locked buffers).
void drain_streams(storb_rs_ctx *ctx);
hipStream_t pick_stream(storb_rs_ctx *ctx, void *s);
// storb_rs_ctx_destroy: every op started on ctx and not finished is
// detached from it (host_async.cpp).
void invalidate_ops(storb_rs_ctx *ctx);
// Device address of page-locked host memory.
hipError_t host_dev_ptr(uint8_t *host, uint8_t **dev);
// Single-call pipeline over column slices of one stripe (host_calls.cpp).
// `during` (optional) runs on the calling thread after the last slice is
// launched, overlapping its kernel.
int sliced(storb_rs_ctx *ctx, size_t S, const std::function<void(size_t, size_t)> &pack,
           const std::function<int(size_t, size_t)> &launch,
           const std::function<void(size_t, size_t)> &unpack,
           const std::function<void()> *during = nullptr);

}  // namespace detail
}  // namespace storb_rs
