// storb_rs.cpp -- implementation of the C ABI in include/storb_rs.h (with
// host_calls.cpp and host_batch.cpp; shared internals in ctx.hpp).
//
// Host side of the MI355X Reed-Solomon path: parameter checks and generator
// matrices (mirroring zfec-rs Fec::new, reached from piece.rs:328,383),
// decode-matrix construction (Fec::decode, piece.rs:384-386), coefficient
// table caches, streams, the tiling of arbitrary (rows x k) matrices onto the
// 16 x 32 slot kernels of rs_kernels.hip, the device-resident batched calls,
// blake3 piece ids and the page-locked host registry.
#include "../../include/storb_rs.h"

#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <chrono>
#include <array>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cctype>
#include <sched.h>
#include <sys/mman.h>
#include <sys/syscall.h>
#include <unistd.h>
#include <cstdio>
#include <cstring>
#include <string>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "blake3.hpp"
#include "ctx.hpp"
#include "rs_jit.hpp"

using namespace storb_rs;
using namespace storb_rs::detail;

namespace storb_rs {
namespace detail {

static std::mutex g_enc_mu;
static std::map<std::pair<uint32_t, uint32_t>, std::vector<uint8_t>> g_enc;

const std::vector<uint8_t> &cached_enc(uint32_t k, uint32_t n) {
  std::lock_guard<std::mutex> lk(g_enc_mu);
  auto key = std::make_pair(k, n);
  auto it = g_enc.find(key);
  if (it == g_enc.end()) it = g_enc.emplace(key, enc_matrix(k, n)).first;
  return it->second;
}

// Round-robin counters of storb_rs_ctx_create(-1): one per NUMA node of the
// calling thread (a node's threads deal out that node's GPUs), the last for
// callers whose node is unknown or has no GPU (they deal out all GPUs).
static constexpr int kRrNodes = 64;
static std::atomic<unsigned long long> g_rr[kRrNodes + 1];

int next_round_robin() { return static_cast<int>(g_rr[kRrNodes].fetch_add(1) & 0x7fffffff); }

// NUMA node of every visible device, read once (sysfs; -1 unknown).
static const std::vector<int> &device_nodes() {
  static const std::vector<int> nodes = [] {
    std::vector<int> v(std::max(0, storb_rs_device_count()));
    for (size_t d = 0; d < v.size(); d++) v[d] = storb_rs_device_numa_node(static_cast<int>(d));
    return v;
  }();
  return nodes;
}

// Page-locked host ranges the caller obtained through storb_rs_host_alloc or
// storb_rs_host_register. The pipelined host path DMAs straight from / into
// such ranges instead of staging through its own pinned buffers.
static std::mutex g_pin_mu;
static std::map<uintptr_t, std::pair<size_t, bool>> g_pinned;  // base -> (len, allocated here)

bool range_pinned(const void *p, size_t len) { return pinned_base(p, len) != nullptr; }

const uint8_t *pinned_base(const void *p, size_t len) {
  if (!p || len == 0) return nullptr;
  const uintptr_t a = reinterpret_cast<uintptr_t>(p);
  std::lock_guard<std::mutex> lk(g_pin_mu);
  auto it = g_pinned.upper_bound(a);
  if (it == g_pinned.begin()) return nullptr;
  --it;
  return a - it->first + len <= it->second.first ? reinterpret_cast<const uint8_t *>(it->first)
                                                  : nullptr;
}


Variant pick_variant(const storb_rs_ctx *ctx) {
  return ctx->variant == STORB_RS_KERNEL_LDS ? Variant::Lds : Variant::Perm;
}

// Evict the least recently used table without blocking the host: the free
// is ordered (on ctx->stream) after the upload and after the last launch
// that read the table on every stream that used it.
// Give a table's device memory back to the stream-ordered pool it came from
// (hipMallocAsync), ordered on ctx->stream after its upload and its last
// use on every stream. Every table free in this file is a hipFreeAsync, the
// pool's own free; a plain hipFree of pool memory (what context teardown did
// until round 3) is legal only after a device-wide synchronisation and is
// not used.
// live: the stream of the current call (a last use on it that no mark
// covers yet gets one now); null at teardown.
static hipError_t release_table(storb_rs_ctx *ctx, Tables *t, hipStream_t live) {
  if (!t->dev) return hipSuccess;
  hipError_t e = hipStreamWaitEvent(ctx->stream, t->uploaded, 0);
  bool sync = false;
  for (auto &u : t->uses) {
    hipEvent_t ev = nullptr;
    if (e == hipSuccess) e = covering_mark(ctx, u.first, u.second, live, &ev);
    if (e == hipSuccess && ev) e = hipStreamWaitEvent(ctx->stream, ev, 0);
    sync = sync || !ev;
  }
  // a last use on a stream this call does not hold, not yet marked (rare:
  // the caller moved to other streams right after it)
  if (e == hipSuccess && sync) {
    ctx->n_device_syncs++;
    e = hipDeviceSynchronize();
  }
  if (e == hipSuccess) e = hipFreeAsync(t->dev, ctx->stream);
  if (e == hipSuccess) t->dev = nullptr;
  return e;
}

static int evict_tables(storb_rs_ctx *ctx, hipStream_t live) {
  auto victim = ctx->tables.begin();
  for (auto it = ctx->tables.begin(); it != ctx->tables.end(); ++it)
    if (it->second->tick < victim->second->tick) victim = it;
  Tables *t = victim->second.get();
  HIP_TRY(ctx, release_table(ctx, t, live));
  // The host source of the upload must outlive the copy; that copy is the
  // oldest work on `home` this table has, long finished in practice.
  HIP_TRY(ctx, hipEventSynchronize(t->uploaded));
  ctx->tables.erase(victim);  // events are released once they complete
  ctx->n_tables = ctx->tables.size();
  return STORB_RS_OK;
}

// Make t usable on stream s: a stream other than the upload's waits for it
// on the device (once the upload is known complete, no wait is issued).
// Once the upload is known complete the host copy is dropped (a k = 64 x
// 32-row matrix is ~130 KiB of tables).
static int tables_ready(storb_rs_ctx *ctx, Tables *t, hipStream_t s) {
  if (t->upload_done) return STORB_RS_OK;
  const hipError_t q = hipEventQuery(t->uploaded);
  if (q == hipSuccess) {
    t->upload_done = true;
    std::vector<uint8_t>().swap(t->host);
    return STORB_RS_OK;
  }
  if (q != hipErrorNotReady) return hip_fail(ctx, q, "hipEventQuery(tables)");
  if (s != t->home) HIP_TRY(ctx, hipStreamWaitEvent(s, t->uploaded, 0));
  return STORB_RS_OK;
}

static hipError_t record_mark(StreamMarks &m, hipStream_t s, uint64_t use) {
  hipEvent_t &e = m.ev[m.next];
  if (!e) {
    const hipError_t r = hipEventCreateWithFlags(&e, kOrderEvent);
    if (r != hipSuccess) return r;
  }
  const hipError_t r = hipEventRecord(e, s);
  if (r != hipSuccess) return r;
  m.at[m.next] = use;
  m.last = use;
  m.next = (m.next + 1) % kMarks;
  return hipSuccess;
}

// Marks of streams the context no longer sees (callers' streams come and
// go): once the map is large, entries whose every mark has completed are
// dropped; a use on a dropped stream then has no covering mark
// (covering_mark's null: device synchronisation).
static void trim_marks(storb_rs_ctx *ctx) {
  if (ctx->marks.size() < 64) return;
  for (auto it = ctx->marks.begin(); it != ctx->marks.end();) {
    bool idle = true;
    for (hipEvent_t e : it->second.ev) idle = idle && (!e || hipEventQuery(e) == hipSuccess);
    if (!idle) {
      ++it;
      continue;
    }
    for (hipEvent_t e : it->second.ev)
      if (e) (void)hipEventDestroy(e);
    it = ctx->marks.erase(it);
  }
}

hipError_t stream_used(storb_rs_ctx *ctx, hipStream_t s, uint64_t *use) {
  const uint64_t u = ++ctx->use_idx;
  *use = u;
  auto it = ctx->marks.find(s);
  if (it == ctx->marks.end()) {
    trim_marks(ctx);
    it = ctx->marks.emplace(s, StreamMarks{}).first;
  }
  StreamMarks &m = it->second;
  if (m.last && u - m.last < kMarkEvery) return hipSuccess;
  return record_mark(m, s, u);
}

hipError_t covering_mark(storb_rs_ctx *ctx, hipStream_t s, uint64_t use, hipStream_t live,
                         hipEvent_t *ev) {
  *ev = nullptr;
  auto it = ctx->marks.find(s);
  if (it == ctx->marks.end()) return hipSuccess;
  StreamMarks &m = it->second;
  if (m.last < use) {  // not marked since that use
    if (s != live) return hipSuccess;
    const hipError_t r = record_mark(m, s, ctx->use_idx);
    if (r != hipSuccess) return r;
  }
  // the oldest mark recorded at or after the use (marks are re-recorded in
  // ring order, so at[] holds the latest index of each)
  uint64_t best = UINT64_MAX;
  for (int i = 0; i < kMarks; i++)
    if (m.ev[i] && m.at[i] >= use && m.at[i] < best) {
      best = m.at[i];
      *ev = m.ev[i];
    }
  return hipSuccess;
}

int tables_used(storb_rs_ctx *ctx, Tables *t, hipStream_t s) {
  uint64_t u = 0;
  HIP_TRY(ctx, stream_used(ctx, s, &u));
  for (auto &x : t->uses)
    if (x.first == s) {
      x.second = u;
      return STORB_RS_OK;
    }
  t->uses.emplace_back(s, u);
  return STORB_RS_OK;
}

// Build (or fetch) the device tables of a rows x k coefficient matrix.
int get_tables(storb_rs_ctx *ctx, uint32_t k, uint32_t rows, const uint8_t *coef,
               hipStream_t s, Tables **out) {
  std::vector<uint8_t> key(8 + static_cast<size_t>(rows) * k);
  std::memcpy(key.data(), &k, 4);
  std::memcpy(key.data() + 4, &rows, 4);
  std::memcpy(key.data() + 8, coef, static_cast<size_t>(rows) * k);
  auto it = ctx->tables.find(key);
  if (it != ctx->tables.end()) {
    Tables *t = it->second.get();
    t->tick = ++ctx->table_tick;
    int rc = tables_ready(ctx, t, s);
    if (rc) return rc;
    *out = t;
    return STORB_RS_OK;
  }
  while (!ctx->tables.empty() && ctx->tables.size() >= std::max<size_t>(ctx->table_cap, 1)) {
    int rc = evict_tables(ctx, s);
    if (rc) return rc;
  }
  auto t = std::make_unique<Tables>();
  // Blocks in the order the launcher walks them; each block's tables are
  // [input][tab_rows] with tab_rows = rows_bucket(rows in block) and the
  // padding rows left as zero tables (the kernels compute them unguarded).
  size_t total = 0;
  for (uint32_t rb = 0; rb < rows; rb += kSlotR)
    for (uint32_t cb = 0; cb < k; cb += kSlotK) {
      t->b_off.push_back(total);
      total += static_cast<size_t>(rows_bucket(std::min<uint32_t>(kSlotR, rows - rb))) *
               std::min<uint32_t>(kSlotK, k - cb);
    }
  t->perm_bytes = round_up(total * sizeof(PermTab), 256);
  std::vector<uint8_t> &host = t->host;
  host.assign(t->perm_bytes + total * 256, 0);
  PermTab *pt = reinterpret_cast<PermTab *>(host.data());
  uint8_t *bt = host.data() + t->perm_bytes;
  const GF256 &g = gf();
  size_t bi = 0;
  for (uint32_t rb = 0; rb < rows; rb += kSlotR)
    for (uint32_t cb = 0; cb < k; cb += kSlotK, bi++) {
      const uint32_t rr = std::min<uint32_t>(kSlotR, rows - rb);
      const uint32_t kk = std::min<uint32_t>(kSlotK, k - cb);
      const uint32_t rp = static_cast<uint32_t>(rows_bucket(rr));
      for (uint32_t i = 0; i < rr; i++)
        for (uint32_t j = 0; j < kk; j++) {
          const uint8_t c = coef[static_cast<size_t>(rb + i) * k + cb + j];
          const size_t o = t->b_off[bi] + static_cast<size_t>(j) * rp + i;  // [col][row]
          pt[o] = perm_tab(c);
          for (int x = 0; x < 256; x++) bt[o * 256 + x] = g.mul(c, static_cast<uint8_t>(x));
        }
    }
  HIP_TRY(ctx, hipEventCreateWithFlags(&t->uploaded, hipEventDisableTiming));
  hipError_t e = hipMallocAsync(reinterpret_cast<void **>(&t->dev), host.size(), s);
  if (e != hipSuccess) return hip_fail(ctx, e, "hipMallocAsync(tables)");
  e = hipMemcpyAsync(t->dev, host.data(), host.size(), hipMemcpyHostToDevice, s);
  if (e == hipSuccess) e = hipEventRecord(t->uploaded, s);
  if (e != hipSuccess) {
    // Nothing may still read or write t's memory; then give it back to its
    // pool (stream-ordered, as every table free) before t goes away.
    (void)hipStreamSynchronize(s);
    (void)hipFreeAsync(t->dev, s);
    (void)hipStreamSynchronize(s);
    t->dev = nullptr;
    return hip_fail(ctx, e, "upload tables");
  }
  t->home = s;
  t->tick = ++ctx->table_tick;
  *out = t.get();
  ctx->tables.emplace(std::move(key), std::move(t));
  ctx->n_tables = ctx->tables.size();
  return STORB_RS_OK;
}

// Whether the table kernel's COPY instantiations can do the assembly: they
// exist for k <= kCopyMaxK in the dwordx4 register-table kernel (not the LDS
// comparison variant), and every share base / stride must be 16-B aligned.
static bool copy_fusable_table(const storb_rs_ctx *ctx, uint32_t k, size_t block,
                               const uint8_t *const *d_in, const size_t *in_stride,
                               uint8_t *const *copy, const size_t *copy_stride) {
  if (k > kCopyMaxK || pick_variant(ctx) != Variant::Perm || block % 16) return false;
  for (uint32_t j = 0; j < k; j++) {
    if ((reinterpret_cast<uintptr_t>(d_in[j]) | in_stride[j]) % 16) return false;
    if (copy[j] && (reinterpret_cast<uintptr_t>(copy[j]) | copy_stride[j]) % 16) return false;
  }
  return true;
}

static int copy_first(storb_rs_ctx *ctx, uint32_t k, const uint8_t *const *d_in,
                      const size_t *in_stride, uint8_t *const *copy, const size_t *copy_stride,
                      size_t block, uint32_t nstripes, hipStream_t s) {
  for (uint32_t j = 0; j < k; j++)
    if (copy[j])
      HIP_TRY(ctx, hipMemcpy2DAsync(copy[j], copy_stride[j], d_in[j], in_stride[j], block, nstripes,
                                    hipMemcpyDeviceToDevice, s));
  return STORB_RS_OK;
}

// out_r = sum_j coef[r][j] * in_j for all stripes. copy (optional, decode
// into a separate chunk buffer): copy[j] != null receives input j as well;
// rows may then be 0 (pure assembly).
//
// Kernel choice: under AUTO a matrix the table kernel is measured slower on
// runs its own compiled bit-sliced kernel once that is built (rs_jit.cpp;
// assembly fused for any k <= 32); otherwise the table kernel, tiled into
// kSlotR x kSlotK blocks, with the assembly fused for k <= kCopyMaxK and
// done by copies first above that.
int apply(storb_rs_ctx *ctx, uint32_t k, uint32_t rows, const uint8_t *coef,
          const uint8_t *const *d_in, const size_t *in_stride, uint8_t *const *d_out,
          const size_t *out_stride, size_t block, uint32_t nstripes, hipStream_t s,
          uint8_t *const *copy, const size_t *copy_stride) {
  if ((rows == 0 && !copy) || block == 0 || nstripes == 0) return STORB_RS_OK;
  int rc;
  if (rows > 0 && ctx->variant == STORB_RS_KERNEL_AUTO && k <= static_cast<uint32_t>(kMaxIn) &&
      rows <= jit::kMaxRows &&
      jit::wanted(k, rows, static_cast<uint64_t>(k + rows) * block * nstripes)) {
    ApplyArgs a{};
    a.k = k;
    a.r = rows;
    for (uint32_t j = 0; j < k; j++) {
      a.in[j] = d_in[j];
      a.in_stride[j] = in_stride[j];
      if (copy && copy[j]) {
        a.copy[j] = copy[j];
        a.copy_stride[j] = copy_stride[j];
        a.ncopy++;
      }
    }
    a.block = block;
    a.nstripes = nstripes;
    bool launched = false;
    HIP_TRY(ctx, jit::try_launch(ctx->device, a, d_out, out_stride, coef, s, &launched));
    if (launched) return STORB_RS_OK;
  }
  if (copy && !copy_fusable_table(ctx, k, block, d_in, in_stride, copy, copy_stride)) {
    if ((rc = copy_first(ctx, k, d_in, in_stride, copy, copy_stride, block, nstripes, s))) return rc;
    copy = nullptr;
    if (rows == 0) return STORB_RS_OK;
  }
  Tables *t = nullptr;
  const std::vector<uint8_t> zero_row(k, 0);
  const uint32_t trows = rows ? rows : 1;  // pure assembly: one zero row of tables
  rc = get_tables(ctx, k, trows, rows ? coef : zero_row.data(), s, &t);
  if (rc) return rc;
  const Variant v = pick_variant(ctx);
  size_t bi = 0;
  for (uint32_t rb = 0; rb < trows; rb += kSlotR)
    for (uint32_t cb = 0; cb < k; cb += kSlotK, bi++) {
      ApplyArgs a{};
      a.r = std::min<uint32_t>(kSlotR, rows - std::min(rows, rb));
      a.k = std::min<uint32_t>(kSlotK, k - cb);
      for (uint32_t j = 0; j < a.k; j++) {
        a.in[j] = d_in[cb + j];
        a.in_stride[j] = in_stride[cb + j];
        if (copy && rb == 0 && copy[cb + j]) {  // each input copied once
          a.copy[j] = copy[cb + j];
          a.copy_stride[j] = copy_stride[cb + j];
          a.ncopy++;
        }
      }
      for (uint32_t i = 0; i < a.r; i++) {
        a.out[i] = d_out[rb + i];
        a.out_stride[i] = out_stride[rb + i];
      }
      a.tab_rows = static_cast<uint32_t>(rows_bucket(a.r ? a.r : 1));
      a.ptab = reinterpret_cast<const PermTab *>(t->dev) + t->b_off[bi];
      a.btab = t->dev + t->perm_bytes + t->b_off[bi] * 256;
      a.block = block;
      a.nstripes = nstripes;
      a.accumulate = cb > 0 ? 1 : 0;
      const hipError_t e = launch_apply(a, v, s);
      if (e != hipSuccess) {
        (void)tables_used(ctx, t, s);  // earlier tiles may be queued
        return hip_fail(ctx, e, "launch_apply");
      }
    }
  return tables_used(ctx, t, s);
}

// Parity of (k, n) = enc[k..n) * data. Under the AUTO variant the geometries
// with a compiled-in bit-sliced encoder take it (rs_bitslice.hpp: 1.5-2.9x
// the v_perm kernel at k = 16 / 32, where that one is VALU-bound); the rest,
// and explicit PERM / LDS requests, go through the table kernels.
int encode_apply(storb_rs_ctx *ctx, uint32_t k, uint32_t n, const uint8_t *const *d_in,
                 const size_t *in_stride, uint8_t *const *d_out, const size_t *out_stride,
                 size_t block, uint32_t nstripes, hipStream_t s) {
  const uint32_t p = n - k;
  if (p == 0 || block == 0 || nstripes == 0) return STORB_RS_OK;
  if (ctx->variant == STORB_RS_KERNEL_AUTO && bitslice_supported(k, n)) {
    ApplyArgs a{};
    a.k = k;
    a.r = p;
    for (uint32_t j = 0; j < k; j++) {
      a.in[j] = d_in[j];
      a.in_stride[j] = in_stride[j];
    }
    for (uint32_t i = 0; i < p; i++) {
      a.out[i] = d_out[i];
      a.out_stride[i] = out_stride[i];
    }
    a.block = block;
    a.nstripes = nstripes;
    if (vector_ok(a)) {
      HIP_TRY(ctx, launch_encode_bitslice(a, n, s));
      return STORB_RS_OK;
    }
  }
  const std::vector<uint8_t> &enc = cached_enc(k, n);
  return apply(ctx, k, p, enc.data() + static_cast<size_t>(k) * k, d_in, in_stride, d_out,
               out_stride, block, nstripes, s);
}

// decode_chunk selection (piece.rs:368-381): sort by index, keep first k,
// then zfec's slot arrangement: primary share s in slot s, parity shares
// fill the holes in index order. Returns the k slot share-indices and the
// position in share_idx[] of each.
int select_shares(storb_rs_ctx *ctx, uint32_t k, uint32_t n, const uint32_t *share_idx,
                  uint32_t nshares, std::vector<uint32_t> &slot_idx,
                  std::vector<uint32_t> &slot_pos) {
  if (nshares < k)
    return fail(ctx, STORB_RS_ENOTENOUGH, "fewer than k shares supplied");
  std::vector<uint32_t> ord(nshares);
  for (uint32_t i = 0; i < nshares; i++) {
    if (share_idx[i] >= n) return fail(ctx, STORB_RS_EINVAL, "share index >= n");
    ord[i] = i;
  }
  std::stable_sort(ord.begin(), ord.end(),
                   [&](uint32_t a, uint32_t b) { return share_idx[a] < share_idx[b]; });
  ord.resize(k);
  for (uint32_t i = 1; i < k; i++)
    if (share_idx[ord[i]] == share_idx[ord[i - 1]])
      return fail(ctx, STORB_RS_ENOTENOUGH, "duplicate share index among the first k");
  slot_idx.assign(k, UINT32_MAX);
  slot_pos.assign(k, UINT32_MAX);
  for (uint32_t i = 0; i < k; i++) {
    const uint32_t id = share_idx[ord[i]];
    if (id < k) {
      slot_idx[id] = id;
      slot_pos[id] = ord[i];
    }
  }
  uint32_t s = 0;
  for (uint32_t i = 0; i < k; i++) {
    const uint32_t id = share_idx[ord[i]];
    if (id < k) continue;
    while (slot_idx[s] != UINT32_MAX) s++;
    slot_idx[s] = id;
    slot_pos[s] = ord[i];
  }
  return STORB_RS_OK;
}

// Rows of D^-1 that rebuild the missing data shares. missing[r] = the data
// index (= slot) of output row r.
int decode_rows(storb_rs_ctx *ctx, uint32_t k, uint32_t n,
                const std::vector<uint32_t> &slot_idx, std::vector<uint8_t> &coef,
                std::vector<uint32_t> &missing) {
  missing.clear();
  for (uint32_t s = 0; s < k; s++)
    if (slot_idx[s] >= k) missing.push_back(s);
  if (missing.empty()) return STORB_RS_OK;
  const std::vector<uint8_t> &enc = cached_enc(k, n);
  std::vector<uint8_t> d(static_cast<size_t>(k) * k, 0);
  for (uint32_t s = 0; s < k; s++)
    std::memcpy(&d[static_cast<size_t>(s) * k], &enc[static_cast<size_t>(slot_idx[s]) * k], k);
  if (!gf_invert(d, k)) return fail(ctx, STORB_RS_EINVAL, "singular decode matrix");
  coef.resize(missing.size() * k);
  for (size_t r = 0; r < missing.size(); r++)
    std::memcpy(&coef[r * k], &d[static_cast<size_t>(missing[r]) * k], k);
  return STORB_RS_OK;
}

// Repair rows (decode-based repair): target share t is
// enc[t] * D^-1 over the k slot shares, where D holds the slot rows of enc.
// For a data target that is exactly decode_rows' row; for a parity target it
// re-encodes the rebuilt data in one pass. Targets must be distinct and must
// not be one of the k shares read (they are written in place).
int repair_rows(storb_rs_ctx *ctx, uint32_t k, uint32_t n,
                const std::vector<uint32_t> &slot_idx, const uint32_t *targets,
                uint32_t ntargets, std::vector<uint8_t> &coef) {
  std::vector<uint8_t> seen(n, 0);
  for (uint32_t s = 0; s < k; s++) seen[slot_idx[s]] = 1;
  for (uint32_t r = 0; r < ntargets; r++) {
    if (targets[r] >= n) return fail(ctx, STORB_RS_EINVAL, "repair target index >= n");
    if (seen[targets[r]] == 1)
      return fail(ctx, STORB_RS_EINVAL, "repair target is one of the k shares read");
    if (seen[targets[r]] == 2) return fail(ctx, STORB_RS_EINVAL, "duplicate repair target");
    seen[targets[r]] = 2;
  }
  const std::vector<uint8_t> &enc = cached_enc(k, n);
  std::vector<uint8_t> d(static_cast<size_t>(k) * k, 0);
  for (uint32_t s = 0; s < k; s++)
    std::memcpy(&d[static_cast<size_t>(s) * k], &enc[static_cast<size_t>(slot_idx[s]) * k], k);
  if (!gf_invert(d, k)) return fail(ctx, STORB_RS_EINVAL, "singular decode matrix");
  const GF256 &g = gf();
  coef.assign(static_cast<size_t>(ntargets) * k, 0);
  for (uint32_t r = 0; r < ntargets; r++) {
    const uint8_t *e = &enc[static_cast<size_t>(targets[r]) * k];
    for (uint32_t s = 0; s < k; s++) {
      if (!e[s]) continue;
      const uint8_t *row = &d[static_cast<size_t>(s) * k];
      for (uint32_t c = 0; c < k; c++) coef[static_cast<size_t>(r) * k + c] ^= g.mul(e[s], row[c]);
    }
  }
  return STORB_RS_OK;
}

// Host copy threads: STORB_RS_HOST_THREADS, default 8 (capped by the
// machine). The pageable <-> pinned copies of the pipelined path use them.
HostPool &host_pool(storb_rs_ctx *ctx) {
  if (!ctx->pool) {
    int n = 8;
    if (const char *e = std::getenv("STORB_RS_HOST_THREADS")) n = std::atoi(e);
    const int hw = static_cast<int>(std::thread::hardware_concurrency());
    if (hw > 0) n = std::min(n, hw);
    ctx->pool = std::make_unique<HostPool>(std::max(1, std::min(n, 64)));
  }
  return *ctx->pool;
}

void drain_streams(storb_rs_ctx *ctx) {
  DeviceGuard g(ctx->device);
  if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
  for (auto &p : ctx->pipe)
    if (p) (void)hipStreamSynchronize(p);
}

// NULL is the HIP null stream (ordered with the device's legacy default
// stream, which is also PyTorch's default stream), not the context's own.
hipStream_t pick_stream(storb_rs_ctx *, void *s) {
  return reinterpret_cast<hipStream_t>(s);
}

// Device address of page-locked host memory (the kernels read / write it
// over PCIe directly on the zero-copy path).
hipError_t host_dev_ptr(uint8_t *host, uint8_t **dev) {
  void *d = nullptr;
  const hipError_t e = hipHostGetDevicePointer(&d, host, 0);
  *dev = static_cast<uint8_t *>(d);
  return e;
}

}  // namespace detail
}  // namespace storb_rs



// ======================================================================
extern "C" {

const char *storb_rs_version(void) { return "storb-rs-mi355x 0.1.0 (gfx950)"; }

const char *storb_rs_strerror(int code) {
  switch (code) {
    case STORB_RS_OK: return "ok";
    case STORB_RS_EINVAL: return "invalid argument";
    case STORB_RS_ENOTENOUGH: return "not enough distinct shares to decode";
    case STORB_RS_EDEVICE: return "HIP device error";
    case STORB_RS_ENOMEM: return "out of memory";
    case STORB_RS_ENODEV: return "no usable gfx950 device";
    case STORB_RS_EAGAIN: return "async op still running";
    case STORB_RS_EBUSY: return "too many unfinished async ops on the context";
    case STORB_RS_ECLOSED: return "the async op's context was destroyed before the op was finished";
    default: return "unknown error";
  }
}

int storb_rs_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

}  // extern "C"

namespace storb_rs {
namespace detail {

int staging_node_env() {
  static const int v = [] {
    const char *e = std::getenv("STORB_RS_STAGING_NODE");
    return e && *e ? std::max(-1, std::atoi(e)) : -2;
  }();
  return v;
}

int cpu_numa_node(int cpu) {
  static const std::vector<int> map = [] {
    std::vector<int> m;
    for (int c = 0; c < 4096; c++) {
      const std::string dir = "/sys/devices/system/cpu/cpu" + std::to_string(c);
      if (access(dir.c_str(), F_OK) != 0) break;
      int node = -1;
      for (int n = 0; n < 64 && node < 0; n++)
        if (access((dir + "/node" + std::to_string(n)).c_str(), F_OK) == 0) node = n;
      m.push_back(node);
    }
    return m;
  }();
  return cpu >= 0 && cpu < static_cast<int>(map.size()) ? map[cpu] : -1;
}

hipError_t pin_alloc_node(size_t n, int node, uint8_t **out) {
  *out = nullptr;
  if (node < 0 || node >= 64) return hipErrorInvalidValue;
  void *m = mmap(nullptr, n, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
  if (m == MAP_FAILED) return hipErrorOutOfMemory;
  const unsigned long mask = 1ul << node;
  // MPOL_PREFERRED (1): pages from `node` while it has free memory, else
  // from the nearest node that does (BIND would fault on an exhausted node)
  if (syscall(SYS_mbind, m, n, 1, &mask, sizeof(mask) * 8 + 1, 0) != 0) {
    munmap(m, n);
    return hipErrorInvalidValue;
  }
  std::memset(m, 0, n);  // first touch places the pages
  const hipError_t e = hipHostRegister(m, n, hipHostRegisterPortable | hipHostRegisterMapped);
  if (e != hipSuccess) {
    munmap(m, n);
    return e;
  }
  *out = static_cast<uint8_t *>(m);
  return hipSuccess;
}

void pin_free_node(uint8_t *p, size_t n) {
  (void)hipHostUnregister(p);
  munmap(p, n);
}

}  // namespace detail
}  // namespace storb_rs

extern "C" {

int storb_rs_device_numa_node(int device) {
  char bus[32] = {};
  if (hipDeviceGetPCIBusId(bus, sizeof(bus), device) != hipSuccess) return -1;
  for (char *c = bus; *c; c++) *c = static_cast<char>(std::tolower(*c));
  const std::string path = std::string("/sys/bus/pci/devices/") + bus + "/numa_node";
  FILE *f = std::fopen(path.c_str(), "r");
  if (!f) return -1;
  int node = -1;
  if (std::fscanf(f, "%d", &node) != 1) node = -1;
  std::fclose(f);
  return node;
}

int storb_rs_select_device(int caller_node, const int *device_nodes, int ndev,
                           uint64_t ticket) {
  if (ndev <= 0 || !device_nodes) return -1;
  int local = 0;
  if (caller_node >= 0)
    for (int d = 0; d < ndev; d++) local += device_nodes[d] == caller_node;
  if (local == 0) return static_cast<int>(ticket % static_cast<unsigned long long>(ndev));
  unsigned long long want = ticket % static_cast<unsigned long long>(local);
  for (int d = 0; d < ndev; d++)
    if (device_nodes[d] == caller_node && want-- == 0) return d;
  return -1;  // unreachable
}

int storb_rs_ctx_create(int device_ordinal, storb_rs_ctx **out) {
  if (!out) return STORB_RS_EINVAL;
  *out = nullptr;
  const int ndev = storb_rs_device_count();
  if (ndev <= 0) return STORB_RS_ENODEV;
  int dev = device_ordinal;
  if (dev < 0) {
    // Round-robin over the GPUs on the calling thread's socket (upload.rs:
    // 418-420's task reaches the context through the shim's thread-local,
    // lib.rs:97-114): a context on the other socket's GPU pays the socket
    // link on every staged call (58.4 vs 53.3 us per (4, 6) 1 MiB encode,
    // BENCH_r04 shim_path.numa). STORB_RS_NUMA_PICK=0: plain round-robin.
    const char *e = std::getenv("STORB_RS_NUMA_PICK");
    const bool numa = !(e && std::atoi(e) == 0);
    const std::vector<int> &nodes = device_nodes();
    int node = numa ? cpu_numa_node(sched_getcpu()) : -1;
    int local = 0;
    if (node >= 0 && node < kRrNodes)
      for (int x : nodes) local += x == node;
    const int ctr = local ? node : kRrNodes;
    dev = storb_rs_select_device(local ? node : -1, nodes.data(), ndev, g_rr[ctr].fetch_add(1));
    if (dev < 0) return STORB_RS_ENODEV;
  }
  if (dev >= ndev) return STORB_RS_EINVAL;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return STORB_RS_ENODEV;
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) return STORB_RS_ENODEV;
  DeviceGuard g(dev);
  if (!g.ok) return STORB_RS_ENODEV;
  auto *c = new storb_rs_ctx();
  c->device = dev;
  c->create_node = cpu_numa_node(sched_getcpu());
  c->device_node = storb_rs_device_numa_node(dev);
  c->zc_max = 64ull << 20;
  if (const char *e = std::getenv("STORB_RS_ZC_MAX")) c->zc_max = std::strtoull(e, nullptr, 10);
  if (const char *e = std::getenv("STORB_RS_ZC_BATCH")) c->zc_batch = std::atoi(e) != 0;
  if (const char *e = std::getenv("STORB_RS_FUSED_HASH")) c->fused_hash = std::atoi(e) != 0;
  if (const char *e = std::getenv("STORB_RS_TABLE_CACHE"))
    c->table_cap = std::max<size_t>(1, std::strtoull(e, nullptr, 10));
  if (const char *e = std::getenv("STORB_RS_TEST_STREAM_STALL")) {
    unsigned long long ticks = 0, us = 0;
    unsigned host_ms = 0, slice = 0, calls = 1;
    if (std::sscanf(e, "%llu,%u,%u,%llu,%u", &ticks, &host_ms, &slice, &us, &calls) >= 4 &&
        ticks > 0) {
      c->stream_timeout_ticks = ticks;
      c->stream_host_wait_ms = static_cast<int>(std::max(1u, host_ms));
      c->test_stall_slice = slice;
      c->test_stall_us = static_cast<uint32_t>(std::min<unsigned long long>(us, 5000000ull));
      c->test_stall_calls = calls;
    }
  }
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
      hipStreamCreateWithFlags(&c->pipe[0], hipStreamNonBlocking) != hipSuccess ||
      hipStreamCreateWithFlags(&c->pipe[1], hipStreamNonBlocking) != hipSuccess) {
    storb_rs_ctx_destroy(c);
    return STORB_RS_EDEVICE;
  }
  *out = c;
  return STORB_RS_OK;
}

void storb_rs_ctx_destroy(storb_rs_ctx *ctx) {
  if (!ctx) return;
  DeviceGuard g(ctx->device);
  if (ctx->stream) {
    // tables back to their pool, after every use on any stream
    for (auto &kv : ctx->tables) (void)release_table(ctx, kv.second.get(), nullptr);
    (void)hipStreamSynchronize(ctx->stream);
  }
  // A table whose stream-ordered release failed: once nothing on the device
  // can still read it, free it on the null stream (still the pool's own
  // free, hipFreeAsync) and wait for that.
  bool leftover = false;
  for (auto &kv : ctx->tables) leftover = leftover || kv.second->dev;
  if (leftover) {
    (void)hipDeviceSynchronize();
    for (auto &kv : ctx->tables)
      if (kv.second->dev) {
        (void)hipFreeAsync(kv.second->dev, nullptr);
        kv.second->dev = nullptr;
      }
    (void)hipDeviceSynchronize();
  }
  for (auto &p : ctx->pipe)
    if (p) (void)hipStreamSynchronize(p);
  if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
  for (auto &p : ctx->pipe)
    if (p) (void)hipStreamDestroy(p);
  for (auto &e : ctx->slice_ev)
    if (e) (void)hipEventDestroy(e);
  for (auto &row : ctx->stage_ev)
    for (auto &e : row)
      if (e) (void)hipEventDestroy(e);
  if (ctx->desc_stream) {
    (void)hipStreamSynchronize(ctx->desc_stream);
    (void)hipStreamDestroy(ctx->desc_stream);
    (void)hipEventDestroy(ctx->desc_copied);
  }
  // a descriptor slot's last decode no mark covers (on a caller's stream)
  bool desc_sync = false;
  for (auto &u : ctx->desc_use) {
    hipEvent_t ev = nullptr;
    if (u.second && covering_mark(ctx, u.first, u.second, nullptr, &ev) == hipSuccess && !ev)
      desc_sync = true;
  }
  if (desc_sync) (void)hipDeviceSynchronize();
  for (auto &e : ctx->desc_cp)
    if (e) (void)hipEventDestroy(e);
  // descriptor launches may run on callers' streams: their last marks
  for (auto &kv : ctx->marks)
    for (hipEvent_t e : kv.second.ev)
      if (e) {
        (void)hipEventSynchronize(e);
        (void)hipEventDestroy(e);
      }
  // Unfinished async ops: their device work ends here (the slot streams are
  // drained below) and they are cut loose from the context, so a later
  // storb_rs_op_test / _finish returns STORB_RS_ECLOSED without touching it.
  invalidate_ops(ctx);
  for (auto &sl : ctx->async_slots) {
    (void)hipStreamSynchronize(sl->stream);
    (void)hipStreamDestroy(sl->stream);
    (void)hipEventDestroy(sl->done);
  }
  delete ctx;  // frees tables, staging and pinned buffers on ctx->device
}

int storb_rs_device_pool_stats(int device, uint64_t *used, uint64_t *reserved) {
  if (device < 0 || device >= storb_rs_device_count()) return STORB_RS_EINVAL;
  DeviceGuard g(device);
  hipMemPool_t pool = nullptr;
  if (hipDeviceGetDefaultMemPool(&pool, device) != hipSuccess) return STORB_RS_EDEVICE;
  uint64_t u = 0, r = 0;
  if (hipMemPoolGetAttribute(pool, hipMemPoolAttrUsedMemCurrent, &u) != hipSuccess ||
      hipMemPoolGetAttribute(pool, hipMemPoolAttrReservedMemCurrent, &r) != hipSuccess)
    return STORB_RS_EDEVICE;
  if (used) *used = u;
  if (reserved) *reserved = r;
  return STORB_RS_OK;
}

int storb_rs_ctx_stats(const storb_rs_ctx *ctx, storb_rs_ctx_stats_t *out) {
  if (!ctx || !out) return STORB_RS_EINVAL;
  out->streamed_calls = ctx->n_streamed.load();
  out->stream_fallbacks = ctx->n_stream_fallbacks.load();
  out->sliced_calls = ctx->n_sliced.load();
  storb_rs_ctx *c = const_cast<storb_rs_ctx *>(ctx);
  {
    std::lock_guard<std::mutex> lk(c->async_mu);
    out->live_ops = c->live_ops.size();
  }
  out->tables = ctx->n_tables.load();  // no lock: a monitor must not wait on a batch call
  out->device_syncs = ctx->n_device_syncs.load();
  out->caller_node = ctx->create_node;
  out->device_node = ctx->device_node;
  return STORB_RS_OK;
}

int storb_rs_ctx_device(const storb_rs_ctx *ctx) { return ctx ? ctx->device : -1; }

const char *storb_rs_last_error(const storb_rs_ctx *ctx) {
  return ctx ? ctx->last_error.c_str() : "";
}

int storb_rs_check_params(uint32_t k, uint32_t n) {
  return valid_params(k, n) ? STORB_RS_OK : STORB_RS_EINVAL;
}

int storb_rs_enc_matrix(uint32_t k, uint32_t n, uint8_t *out_nk) {
  if (!valid_params(k, n) || !out_nk) return STORB_RS_EINVAL;
  const std::vector<uint8_t> &e = cached_enc(k, n);
  std::memcpy(out_nk, e.data(), e.size());
  return STORB_RS_OK;
}

size_t storb_rs_block_size(uint32_t k, size_t len) {
  return k ? (len + k - 1) / k : 0;
}

// piece.rs:292-303. `f64 as i32` saturates (NaN -> 0, -inf -> i32::MIN);
// release-mode `1u64 << e` masks the shift to e & 63.
uint64_t storb_piece_length(uint64_t content_length, uint64_t min_size,
                            uint64_t max_size) {
  if (min_size == 0) min_size = 16ull * 1024;           // constants.rs:5
  if (max_size == 0) max_size = 256ull * 1024 * 1024;   // constants.rs:6
  const double e = std::log2(static_cast<double>(content_length)) * 0.5 + 8.39;
  int32_t ei;
  if (std::isnan(e)) ei = 0;
  else if (e <= -2147483648.0) ei = INT32_MIN;
  else if (e >= 2147483647.0) ei = INT32_MAX;
  else ei = static_cast<int32_t>(e);
  uint64_t len = 1ull << (static_cast<uint32_t>(ei) & 63u);
  return std::min(std::max(len, min_size), max_size);
}

void storb_get_k_and_m(uint64_t chunk_size, uint64_t *k, uint64_t *m) {
  const uint64_t ps = storb_piece_length(chunk_size, 0, 0);
  const uint64_t kk = static_cast<uint64_t>(
      std::ceil(static_cast<double>(chunk_size) / static_cast<double>(ps)));
  const uint64_t pp = static_cast<uint64_t>(std::ceil(static_cast<double>(kk) / 2.0));
  if (k) *k = kk;
  if (m) *m = kk + pp;
}

int storb_rs_set_kernel(storb_rs_ctx *ctx, int variant) {
  if (!ctx || variant < 0 || variant > 2) return STORB_RS_EINVAL;
  std::lock_guard<std::mutex> lk(ctx->mu);
  ctx->variant = variant;
  return STORB_RS_OK;
}

int storb_rs_host_alloc(size_t len, void **out) {
  if (!out || len == 0) return STORB_RS_EINVAL;
  *out = nullptr;
  void *p = nullptr;
  const hipError_t e = hipHostMalloc(&p, len, hipHostMallocPortable);
  if (e != hipSuccess) return e == hipErrorOutOfMemory ? STORB_RS_ENOMEM : STORB_RS_EDEVICE;
  std::lock_guard<std::mutex> lk(g_pin_mu);
  g_pinned[reinterpret_cast<uintptr_t>(p)] = {len, true};
  *out = p;
  return STORB_RS_OK;
}

// hipHostFree / hipHostUnregister wait only for the null stream of each
// device; the zero-copy kernels run on non-blocking streams (the contexts'
// own, async slots, callers'), so a range could be unmapped under a kernel
// still reading or writing it -- a GPU page fault reported later, against
// whatever HIP call comes next. Every device is synchronised first. These
// calls are rare (buffer teardown); the cost is one device-wide wait.
static void sync_all_devices() {
  int n = 0, prev = -1;
  if (hipGetDeviceCount(&n) != hipSuccess) return;
  (void)hipGetDevice(&prev);
  for (int d = 0; d < n; d++)
    if (hipSetDevice(d) == hipSuccess) (void)hipDeviceSynchronize();
  if (prev >= 0) (void)hipSetDevice(prev);
}

int storb_rs_host_free(void *p) {
  if (!p) return STORB_RS_OK;
  {
    std::lock_guard<std::mutex> lk(g_pin_mu);
    auto it = g_pinned.find(reinterpret_cast<uintptr_t>(p));
    if (it == g_pinned.end() || !it->second.second) return STORB_RS_EINVAL;
    g_pinned.erase(it);
  }
  sync_all_devices();
  return hipHostFree(p) == hipSuccess ? STORB_RS_OK : STORB_RS_EDEVICE;
}

int storb_rs_host_register(void *p, size_t len) {
  if (!p || len == 0) return STORB_RS_EINVAL;
  // Mapped: the zero-copy kernels address registered ranges through
  // hipHostGetDevicePointer, which needs a device mapping of the range.
  const hipError_t e = hipHostRegister(p, len, hipHostRegisterPortable | hipHostRegisterMapped);
  if (e != hipSuccess) return e == hipErrorOutOfMemory ? STORB_RS_ENOMEM : STORB_RS_EDEVICE;
  std::lock_guard<std::mutex> lk(g_pin_mu);
  g_pinned[reinterpret_cast<uintptr_t>(p)] = {len, false};
  return STORB_RS_OK;
}

int storb_rs_host_unregister(void *p) {
  if (!p) return STORB_RS_EINVAL;
  {
    std::lock_guard<std::mutex> lk(g_pin_mu);
    auto it = g_pinned.find(reinterpret_cast<uintptr_t>(p));
    if (it == g_pinned.end() || it->second.second) return STORB_RS_EINVAL;
    g_pinned.erase(it);
  }
  sync_all_devices();
  return hipHostUnregister(p) == hipSuccess ? STORB_RS_OK : STORB_RS_EDEVICE;
}

int storb_rs_host_is_pinned(const void *p, size_t len) { return range_pinned(p, len) ? 1 : 0; }

int storb_rs_sync(storb_rs_ctx *ctx) {
  if (!ctx) return STORB_RS_EINVAL;
  std::lock_guard<std::mutex> lk(ctx->mu);
  DeviceGuard g(ctx->device);
  HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
  for (auto &p : ctx->pipe) HIP_TRY(ctx, hipStreamSynchronize(p));
  // Device calls given hip_stream = NULL run on the HIP null stream, which
  // the (non-blocking) context streams do not order with: wait for it too.
  HIP_TRY(ctx, hipStreamSynchronize(nullptr));
  return STORB_RS_OK;
}

// ---------------------------------------------------------------- device
int storb_rs_apply_dev(storb_rs_ctx *ctx, uint32_t k, uint32_t rows, const uint8_t *coef,
                       const uint8_t *const *d_in, const size_t *in_stride,
                       uint8_t *const *d_out, const size_t *out_stride, size_t block,
                       uint32_t nstripes, void *hip_stream) {
  if (!ctx) return STORB_RS_EINVAL;
  std::lock_guard<std::mutex> lk(ctx->mu);
  if (k < 1 || k > STORB_RS_MAX_SHARES || rows > STORB_RS_MAX_SHARES || !coef ||
      !d_in || !in_stride || !d_out || !out_stride)
    return fail(ctx, STORB_RS_EINVAL, "apply: bad arguments");
  DeviceGuard g(ctx->device);
  return apply(ctx, k, rows, coef, d_in, in_stride, d_out, out_stride, block, nstripes,
               pick_stream(ctx, hip_stream));
}

int storb_rs_encode_batch_dev(storb_rs_ctx *ctx, uint32_t k, uint32_t n, size_t block,
                              uint32_t nstripes, const uint8_t *d_data,
                              size_t data_stride, uint8_t *d_parity,
                              size_t parity_stride, void *hip_stream) {
  if (!ctx) return STORB_RS_EINVAL;
  std::lock_guard<std::mutex> lk(ctx->mu);
  if (!valid_params(k, n)) return fail(ctx, STORB_RS_EINVAL, "invalid (k, n)");
  if (n == k || block == 0 || nstripes == 0) return STORB_RS_OK;
  if (!d_data || !d_parity) return fail(ctx, STORB_RS_EINVAL, "null device pointer");
  if (data_stride == 0) data_stride = static_cast<size_t>(k) * block;
  if (parity_stride == 0) parity_stride = static_cast<size_t>(n - k) * block;
  DeviceGuard g(ctx->device);
  const uint32_t p = n - k;
  std::vector<const uint8_t *> in(k);
  std::vector<size_t> ins(k, data_stride), outs(p, parity_stride);
  std::vector<uint8_t *> out(p);
  for (uint32_t j = 0; j < k; j++) in[j] = d_data + static_cast<size_t>(j) * block;
  for (uint32_t i = 0; i < p; i++) out[i] = d_parity + static_cast<size_t>(i) * block;
  return encode_apply(ctx, k, n, in.data(), ins.data(), out.data(), outs.data(), block,
                      nstripes, pick_stream(ctx, hip_stream));
}

int storb_rs_decode_batch_dev(storb_rs_ctx *ctx, uint32_t k, uint32_t n, size_t block,
                              uint32_t nstripes, const uint32_t *share_idx,
                              uint32_t nshares, const uint8_t *d_data,
                              size_t data_stride, const uint8_t *d_parity,
                              size_t parity_stride, uint8_t *d_out, size_t out_stride,
                              void *hip_stream) {
  if (!ctx) return STORB_RS_EINVAL;
  std::lock_guard<std::mutex> lk(ctx->mu);
  if (!valid_params(k, n)) return fail(ctx, STORB_RS_EINVAL, "invalid (k, n)");
  if (!share_idx || !d_out) return fail(ctx, STORB_RS_EINVAL, "null argument");
  if (data_stride == 0) data_stride = static_cast<size_t>(k) * block;
  if (parity_stride == 0) parity_stride = static_cast<size_t>(n - k) * block;
  if (out_stride == 0) out_stride = static_cast<size_t>(k) * block;
  trim_patterns(ctx);
  const Pattern *p = nullptr;
  std::vector<uint32_t> slot_pos;
  const int rc = get_pattern(ctx, k, n, share_idx, nshares, &p, slot_pos);
  if (rc) return rc;
  if (block == 0 || nstripes == 0) return STORB_RS_OK;
  DeviceGuard g(ctx->device);
  return decode_pattern_batch(ctx, k, block, nstripes, *p, d_data, data_stride, d_parity,
                              parity_stride, d_out, out_stride, pick_stream(ctx, hip_stream));
}

int storb_rs_repair_batch_dev(storb_rs_ctx *ctx, uint32_t k, uint32_t n, size_t block,
                              uint32_t nstripes, const uint32_t *share_idx,
                              uint32_t nshares, const uint32_t *targets, uint32_t ntargets,
                              uint8_t *d_data, size_t data_stride, uint8_t *d_parity,
                              size_t parity_stride, void *hip_stream) {
  if (!ctx) return STORB_RS_EINVAL;
  std::lock_guard<std::mutex> lk(ctx->mu);
  if (!valid_params(k, n)) return fail(ctx, STORB_RS_EINVAL, "invalid (k, n)");
  if (!share_idx || (ntargets && !targets)) return fail(ctx, STORB_RS_EINVAL, "null argument");
  if (data_stride == 0) data_stride = static_cast<size_t>(k) * block;
  if (parity_stride == 0) parity_stride = static_cast<size_t>(n - k) * block;
  std::vector<uint32_t> slot_idx, slot_pos;
  int rc = select_shares(ctx, k, n, share_idx, nshares, slot_idx, slot_pos);
  if (rc) return rc;
  std::vector<uint8_t> coef;
  rc = repair_rows(ctx, k, n, slot_idx, targets, ntargets, coef);
  if (rc) return rc;
  if (ntargets == 0 || block == 0 || nstripes == 0) return STORB_RS_OK;
  auto where = [&](uint32_t id, uint8_t *&p, size_t &stride) -> bool {
    if (id < k) {
      p = d_data ? d_data + static_cast<size_t>(id) * block : nullptr;
      stride = data_stride;
    } else {
      p = d_parity ? d_parity + static_cast<size_t>(id - k) * block : nullptr;
      stride = parity_stride;
    }
    return p != nullptr;
  };
  std::vector<const uint8_t *> in(k);
  std::vector<size_t> ins(k), outs(ntargets);
  std::vector<uint8_t *> out(ntargets);
  for (uint32_t c = 0; c < k; c++) {
    uint8_t *p;
    if (!where(slot_idx[c], p, ins[c])) return fail(ctx, STORB_RS_EINVAL, "share in null region");
    in[c] = p;
  }
  for (uint32_t r = 0; r < ntargets; r++)
    if (!where(targets[r], out[r], outs[r]))
      return fail(ctx, STORB_RS_EINVAL, "target in null region");
  DeviceGuard g(ctx->device);
  return apply(ctx, k, ntargets, coef.data(), in.data(), ins.data(), out.data(), outs.data(),
               block, nstripes, pick_stream(ctx, hip_stream));
}

int storb_rs_jit_prepare_decode(uint32_t k, uint32_t n, const uint32_t *share_idx,
                                uint32_t nshares, int assemble, int wait) {
  if (!valid_params(k, n) || !share_idx) return STORB_RS_EINVAL;
  std::vector<uint32_t> slot_idx, slot_pos, missing;
  int rc = select_shares(nullptr, k, n, share_idx, nshares, slot_idx, slot_pos);
  if (rc) return rc;
  std::vector<uint8_t> coef;
  rc = decode_rows(nullptr, k, n, slot_idx, coef, missing);
  if (rc || missing.empty()) return rc;
  uint64_t mask = 0;
  for (uint32_t c = 0; assemble && c < k && c < 64; c++)
    if (slot_idx[c] < k) mask |= 1ull << c;
  return jit::prepare(k, static_cast<uint32_t>(missing.size()), coef.data(), mask, wait != 0) < 0
             ? STORB_RS_EDEVICE
             : STORB_RS_OK;
}

// Host BLAKE3 (blake3_host.cpp: 16 chunks per AVX-512 compression where
// the CPU has it, else the scalar compression of blake3.hpp).
void storb_blake3(const uint8_t *data, size_t len, uint8_t out[32]) {
  blake3_host(data, len, out);
}

int storb_rs_blake3_batch_dev(storb_rs_ctx *ctx, const uint8_t *d_in, size_t len,
                              uint32_t count, size_t stride, uint8_t *d_out,
                              void *hip_stream) {
  if (!ctx) return STORB_RS_EINVAL;
  std::lock_guard<std::mutex> lk(ctx->mu);
  if (count && (!d_out || (!d_in && len)))
    return fail(ctx, STORB_RS_EINVAL, "blake3: null device pointer");
  if (len > 16ull * 1024 * 1024)
    return fail(ctx, STORB_RS_EINVAL, "blake3: message larger than 16 MiB");
  if (stride == 0) stride = len;
  DeviceGuard g(ctx->device);
  HIP_TRY(ctx, launch_blake3_batch(d_in, len, count, stride, d_out,
                                   pick_stream(ctx, hip_stream)));
  return STORB_RS_OK;
}

}  // extern "C"

namespace storb_rs {
namespace detail {

// The one-kernel encode + piece ids when the geometry has one and the
// pointers are dwordx4-aligned (false: nothing launched).
bool try_encode_hash(storb_rs_ctx *ctx, uint32_t k, uint32_t n, size_t block,
                     uint32_t nstripes, const uint8_t *d_data, size_t data_stride,
                     uint8_t *d_parity, size_t parity_stride, uint8_t *d_hashes, hipStream_t s,
                     hipError_t *err) {
  *err = hipSuccess;
  if (!ctx->fused_hash || !encode_hash_supported(k, n, block)) return false;
  const uintptr_t al = reinterpret_cast<uintptr_t>(d_data) | reinterpret_cast<uintptr_t>(d_parity) |
                       reinterpret_cast<uintptr_t>(d_hashes) | data_stride | parity_stride;
  if (al & 15) return false;
  const uint32_t p = n - k;
  const std::vector<uint8_t> &enc = cached_enc(k, n);
  EncHashArgs a{};
  a.data = d_data;
  a.data_stride = data_stride;
  a.parity = d_parity;
  a.parity_stride = parity_stride;
  a.hashes = d_hashes;
  a.block = block;
  a.share_stride = block;
  a.nstripes = nstripes;
  a.nchunks = static_cast<uint32_t>(block / 1024);
  while ((1u << a.seg_log2) < a.nchunks) a.seg_log2++;
  for (uint32_t j = 0; j < k; j++)
    for (uint32_t i = 0; i < p; i++) {
      const PermTab t = perm_tab(enc[static_cast<size_t>(k + i) * k + j]);
      uint32_t *w = a.tab[j * p + i];
      w[0] = t.t0lo;
      w[1] = t.t0hi;
      w[2] = t.t1lo;
      w[3] = t.t1hi;
      w[4] = t.t2;
    }
  *err = launch_encode_hash(a, k, n, s);
  return true;
}

}  // namespace detail
}  // namespace storb_rs

extern "C" {

int storb_rs_encode_hashed_dev(storb_rs_ctx *ctx, uint32_t k, uint32_t n, size_t block,
                               uint32_t nstripes, const uint8_t *d_data, size_t data_stride,
                               uint8_t *d_parity, size_t parity_stride, uint8_t *d_hashes,
                               void *hip_stream) {
  if (!ctx) return STORB_RS_EINVAL;
  std::lock_guard<std::mutex> lk(ctx->mu);
  if (!valid_params(k, n)) return fail(ctx, STORB_RS_EINVAL, "invalid (k, n)");
  if (block == 0 || nstripes == 0) return STORB_RS_OK;
  if (!d_data || !d_hashes || (n > k && !d_parity))
    return fail(ctx, STORB_RS_EINVAL, "null device pointer");
  if (block > 16ull * 1024 * 1024)
    return fail(ctx, STORB_RS_EINVAL, "blake3: share larger than 16 MiB");
  if (data_stride == 0) data_stride = static_cast<size_t>(k) * block;
  if (parity_stride == 0) parity_stride = static_cast<size_t>(n - k) * block;
  DeviceGuard g(ctx->device);
  hipStream_t s = pick_stream(ctx, hip_stream);
  hipError_t e;
  if (n > k && try_encode_hash(ctx, k, n, block, nstripes, d_data, data_stride, d_parity,
                               parity_stride, d_hashes, s, &e)) {
    HIP_TRY(ctx, e);
    return STORB_RS_OK;
  }
  // Two kernels: encode, then one hash launch over all n shares of every
  // stripe (digests written at (s*n + t)*32 directly). Sub-batches pipelined
  // over two streams (the hash of batch i beside the encode of i + 1) and
  // interleaved on one stream both measured slower at every size, e.g.
  // (16, 24) x 128 stripes 0.895 ms sequential vs 0.90-1.46 ms
  // (profiles/r5d_widehash_pipelining.jsonl): a sub-batch's hash launch has
  // too few shards to fill the chip, and the encoder's LDS reservation keeps
  // the two kernels off each other's CUs. Hashing the data shares on a second
  // stream beside the whole encode (parity after it) measured 0.886 ms, and
  // 0.858 with the encoder uncapped so the two share CUs (1.06x at (16, 24),
  // none or a loss at (32, 48) / (8, 12); profiles/r5i_widehash.jsonl): not
  // kept. DESIGN.md §5 has the VALU arithmetic that bounds any overlap.
  const uint32_t p = n - k;
  if (p > 0) {
    std::vector<const uint8_t *> in(k);
    std::vector<size_t> ins(k, data_stride), outs(p, parity_stride);
    std::vector<uint8_t *> out(p);
    for (uint32_t j = 0; j < k; j++) in[j] = d_data + static_cast<size_t>(j) * block;
    for (uint32_t i = 0; i < p; i++) out[i] = d_parity + static_cast<size_t>(i) * block;
    const int rc = encode_apply(ctx, k, n, in.data(), ins.data(), out.data(), outs.data(), block,
                                nstripes, s);
    if (rc) return rc;
  }
  // every share of every stripe in one hash launch, digests in place
  HIP_TRY(ctx, launch_blake3_stripes(d_data, data_stride, d_parity, parity_stride, block, k, n,
                                     block, nstripes, d_hashes, s));
  return STORB_RS_OK;
}

int storb_rs_fill_splitmix_dev(storb_rs_ctx *ctx, uint8_t *d, size_t obj_len,
                               uint32_t nobj, size_t obj_stride, uint64_t seed_base,
                               void *hip_stream) {
  if (!ctx) return STORB_RS_EINVAL;
  std::lock_guard<std::mutex> lk(ctx->mu);
  if (!d && obj_len && nobj) return fail(ctx, STORB_RS_EINVAL, "null device pointer");
  if (obj_stride == 0) obj_stride = obj_len;
  DeviceGuard g(ctx->device);
  HIP_TRY(ctx, launch_fill_splitmix(d, obj_len, nobj, obj_stride, seed_base,
                                    pick_stream(ctx, hip_stream)));
  return STORB_RS_OK;
}

}  // extern "C"
