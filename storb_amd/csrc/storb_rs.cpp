// storb_rs.cpp -- implementation of the C ABI in include/storb_rs.h.
//
// Host side of the MI355X Reed-Solomon path: parameter checks and generator
// matrices (mirroring zfec-rs Fec::new, reached from piece.rs:328,383),
// decode-matrix construction (Fec::decode, piece.rs:384-386), coefficient
// table caches, pinned staging, streams, and the tiling of arbitrary
// (rows x k) matrices onto the 16 x 32 slot kernels of rs_kernels.hip.
#include "../../include/storb_rs.h"

#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "blake3.hpp"
#include "gf256.hpp"
#include "host_pool.hpp"
#include "rs_kernels.hpp"

using namespace storb_rs;

namespace {

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

struct PinBuf {
  uint8_t *p = nullptr;
  size_t cap = 0;
  ~PinBuf() {
    if (p) (void)hipHostFree(p);
  }
  hipError_t ensure(size_t n) {
    if (n <= cap) return hipSuccess;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
    hipError_t e = hipHostMalloc(reinterpret_cast<void **>(&p), n, hipHostMallocDefault);
    if (e == hipSuccess) cap = n;
    return e;
  }
};

// Device-resident coefficient tables for one (rows x k) matrix, tiled in
// kSlotR x kSlotK blocks: for block b, ptab + b_off[b] PermTabs and
// btab + b_off[b]*256 product-table bytes.
struct Tables {
  uint8_t *dev = nullptr;
  size_t perm_bytes = 0;
  std::vector<size_t> b_off;
  ~Tables() {
    if (dev) (void)hipFree(dev);
  }
};

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

std::mutex g_enc_mu;
std::map<std::pair<uint32_t, uint32_t>, std::vector<uint8_t>> g_enc;

const std::vector<uint8_t> &cached_enc(uint32_t k, uint32_t n) {
  std::lock_guard<std::mutex> lk(g_enc_mu);
  auto key = std::make_pair(k, n);
  auto it = g_enc.find(key);
  if (it == g_enc.end()) it = g_enc.emplace(key, enc_matrix(k, n)).first;
  return it->second;
}

std::atomic<int> g_rr{0};

// Page-locked host ranges the caller obtained through storb_rs_host_alloc or
// storb_rs_host_register. The pipelined host path DMAs straight from / into
// such ranges instead of staging through its own pinned buffers.
std::mutex g_pin_mu;
std::map<uintptr_t, std::pair<size_t, bool>> g_pinned;  // base -> (len, allocated here)

bool range_pinned(const void *p, size_t len) {
  if (!p || len == 0) return false;
  const uintptr_t a = reinterpret_cast<uintptr_t>(p);
  std::lock_guard<std::mutex> lk(g_pin_mu);
  auto it = g_pinned.upper_bound(a);
  if (it == g_pinned.begin()) return false;
  --it;
  return a - it->first + len <= it->second.first;
}

}  // namespace

struct storb_rs_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  hipStream_t pipe[2] = {nullptr, nullptr};
  int variant = STORB_RS_KERNEL_AUTO;
  std::mutex mu;
  std::string last_error;
  DevBuf stage;
  DevBuf pipe_dev[2];
  PinBuf pin_in, pin_out;
  PinBuf pipe_in[2], pipe_out[2];
  std::map<std::vector<uint8_t>, std::unique_ptr<Tables>> tables;
  std::unique_ptr<HostPool> pool;  // host copy workers, created on first use
  // Single-call paths whose staged bytes (in + out) are at most this size
  // run the kernel straight on the pinned staging buffers (zero-copy over
  // PCIe) instead of DMA in -> kernel -> DMA out: one launch and one sync
  // instead of three operations. STORB_RS_ZC_MAX, bytes; 0 disables.
  size_t zc_max = 0;
  // storb_rs_encode_chunks without piece ids: zero-copy kernels (1) or
  // SDMA H2D -> kernel -> D2H (0). STORB_RS_ZC_BATCH.
  bool zc_batch = true;
  hipEvent_t slice_ev[kMaxSlices] = {};  // sliced single-call pipeline
};

namespace {

int fail(storb_rs_ctx *ctx, int code, const std::string &msg) {
  if (ctx) ctx->last_error = msg;
  return code;
}

int hip_fail(storb_rs_ctx *ctx, hipError_t e, const char *what) {
  std::string m = std::string(what) + ": " + hipGetErrorString(e);
  return fail(ctx, e == hipErrorOutOfMemory ? STORB_RS_ENOMEM : STORB_RS_EDEVICE, m);
}

#define HIP_TRY(ctx, expr)                              \
  do {                                                  \
    hipError_t e_ = (expr);                             \
    if (e_ != hipSuccess) return hip_fail(ctx, e_, #expr); \
  } while (0)

Variant pick_variant(const storb_rs_ctx *ctx) {
  return ctx->variant == STORB_RS_KERNEL_LDS ? Variant::Lds : Variant::Perm;
}

// Build (or fetch) the device tables of a rows x k coefficient matrix.
int get_tables(storb_rs_ctx *ctx, uint32_t k, uint32_t rows, const uint8_t *coef,
               hipStream_t s, const Tables **out) {
  std::vector<uint8_t> key(8 + static_cast<size_t>(rows) * k);
  std::memcpy(key.data(), &k, 4);
  std::memcpy(key.data() + 4, &rows, 4);
  std::memcpy(key.data() + 8, coef, static_cast<size_t>(rows) * k);
  auto it = ctx->tables.find(key);
  if (it != ctx->tables.end()) {
    *out = it->second.get();
    return STORB_RS_OK;
  }
  if (ctx->tables.size() > 4096) ctx->tables.clear();
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
  std::vector<uint8_t> host(t->perm_bytes + total * 256, 0);
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
  hipError_t e = hipMalloc(reinterpret_cast<void **>(&t->dev), host.size());
  if (e != hipSuccess) return hip_fail(ctx, e, "hipMalloc(tables)");
  e = hipMemcpyAsync(t->dev, host.data(), host.size(), hipMemcpyHostToDevice, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e != hipSuccess) return hip_fail(ctx, e, "upload tables");
  *out = t.get();
  ctx->tables.emplace(std::move(key), std::move(t));
  return STORB_RS_OK;
}

// out_r = sum_j coef[r][j] * in_j for all stripes, tiled into slot blocks.
int apply(storb_rs_ctx *ctx, uint32_t k, uint32_t rows, const uint8_t *coef,
          const uint8_t *const *d_in, const size_t *in_stride, uint8_t *const *d_out,
          const size_t *out_stride, size_t block, uint32_t nstripes, hipStream_t s) {
  if (rows == 0 || block == 0 || nstripes == 0) return STORB_RS_OK;
  const Tables *t = nullptr;
  int rc = get_tables(ctx, k, rows, coef, s, &t);
  if (rc) return rc;
  const Variant v = pick_variant(ctx);
  size_t bi = 0;
  for (uint32_t rb = 0; rb < rows; rb += kSlotR)
    for (uint32_t cb = 0; cb < k; cb += kSlotK, bi++) {
      ApplyArgs a{};
      a.r = std::min<uint32_t>(kSlotR, rows - rb);
      a.k = std::min<uint32_t>(kSlotK, k - cb);
      for (uint32_t j = 0; j < a.k; j++) {
        a.in[j] = d_in[cb + j];
        a.in_stride[j] = in_stride[cb + j];
      }
      for (uint32_t i = 0; i < a.r; i++) {
        a.out[i] = d_out[rb + i];
        a.out_stride[i] = out_stride[rb + i];
      }
      a.tab_rows = static_cast<uint32_t>(rows_bucket(a.r));
      a.ptab = reinterpret_cast<const PermTab *>(t->dev) + t->b_off[bi];
      a.btab = t->dev + t->perm_bytes + t->b_off[bi] * 256;
      a.block = block;
      a.nstripes = nstripes;
      a.accumulate = cb > 0 ? 1 : 0;
      HIP_TRY(ctx, launch_apply(a, v, s));
    }
  return STORB_RS_OK;
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

// Single-call pipeline over column slices of one stripe. A chunk's shares
// are split into q column ranges [off, off+cnt) (16-B multiples); while the
// kernel works on slice t (zero-copy, over PCIe), the host packs slice t+1
// into pinned staging and unpacks slice t-1's outputs, so the staging copies
// of pageable caller buffers overlap the kernel instead of adding to it.
// q = 1 (small chunks) degenerates to pack -> launch -> sync -> unpack.
int sliced(storb_rs_ctx *ctx, size_t S, const std::function<void(size_t, size_t)> &pack,
           const std::function<int(size_t, size_t)> &launch,
           const std::function<void(size_t, size_t)> &unpack) {
  int q = static_cast<int>(std::min<size_t>(kMaxSlices, S / (128u << 10)));
  if (q < 2) q = 1;
  const size_t slice = round_up((S + q - 1) / q, kAlign);
  q = static_cast<int>((S + slice - 1) / slice);
  for (int t = 0; t < q; t++)
    if (!ctx->slice_ev[t])
      HIP_TRY(ctx, hipEventCreateWithFlags(&ctx->slice_ev[t], hipEventDisableTiming));
  auto range = [&](int t, size_t &off, size_t &cnt) {
    off = static_cast<size_t>(t) * slice;
    cnt = std::min(slice, S - off);
  };
  for (int t = 0; t < q; t++) {
    size_t off, cnt;
    range(t, off, cnt);
    pack(off, cnt);
    const int rc = launch(off, cnt);
    if (rc) return rc;
    HIP_TRY(ctx, hipEventRecord(ctx->slice_ev[t], ctx->stream));
    if (t > 0) {
      HIP_TRY(ctx, hipEventSynchronize(ctx->slice_ev[t - 1]));
      range(t - 1, off, cnt);
      unpack(off, cnt);
    }
  }
  size_t off, cnt;
  range(q - 1, off, cnt);
  HIP_TRY(ctx, hipEventSynchronize(ctx->slice_ev[q - 1]));
  unpack(off, cnt);
  return STORB_RS_OK;
}

}  // namespace

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
    default: return "unknown error";
  }
}

int storb_rs_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int storb_rs_ctx_create(int device_ordinal, storb_rs_ctx **out) {
  if (!out) return STORB_RS_EINVAL;
  *out = nullptr;
  const int ndev = storb_rs_device_count();
  if (ndev <= 0) return STORB_RS_ENODEV;
  int dev = device_ordinal;
  if (dev < 0) dev = g_rr.fetch_add(1) % ndev;
  if (dev >= ndev) return STORB_RS_EINVAL;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return STORB_RS_ENODEV;
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) return STORB_RS_ENODEV;
  DeviceGuard g(dev);
  if (!g.ok) return STORB_RS_ENODEV;
  auto *c = new storb_rs_ctx();
  c->device = dev;
  c->zc_max = 64ull << 20;
  if (const char *e = std::getenv("STORB_RS_ZC_MAX")) c->zc_max = std::strtoull(e, nullptr, 10);
  if (const char *e = std::getenv("STORB_RS_ZC_BATCH")) c->zc_batch = std::atoi(e) != 0;
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
  if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
  for (auto &p : ctx->pipe)
    if (p) (void)hipStreamSynchronize(p);
  if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
  for (auto &p : ctx->pipe)
    if (p) (void)hipStreamDestroy(p);
  for (auto &e : ctx->slice_ev)
    if (e) (void)hipEventDestroy(e);
  delete ctx;  // frees tables, staging and pinned buffers on ctx->device
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

int storb_rs_host_free(void *p) {
  if (!p) return STORB_RS_OK;
  {
    std::lock_guard<std::mutex> lk(g_pin_mu);
    auto it = g_pinned.find(reinterpret_cast<uintptr_t>(p));
    if (it == g_pinned.end() || !it->second.second) return STORB_RS_EINVAL;
    g_pinned.erase(it);
  }
  return hipHostFree(p) == hipSuccess ? STORB_RS_OK : STORB_RS_EDEVICE;
}

int storb_rs_host_register(void *p, size_t len) {
  if (!p || len == 0) return STORB_RS_EINVAL;
  const hipError_t e = hipHostRegister(p, len, hipHostRegisterPortable);
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
  return hipHostUnregister(p) == hipSuccess ? STORB_RS_OK : STORB_RS_EDEVICE;
}

int storb_rs_host_is_pinned(const void *p, size_t len) { return range_pinned(p, len) ? 1 : 0; }

int storb_rs_sync(storb_rs_ctx *ctx) {
  if (!ctx) return STORB_RS_EINVAL;
  std::lock_guard<std::mutex> lk(ctx->mu);
  DeviceGuard g(ctx->device);
  HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
  for (auto &p : ctx->pipe) HIP_TRY(ctx, hipStreamSynchronize(p));
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
  std::vector<uint32_t> slot_idx, slot_pos, missing;
  int rc = select_shares(ctx, k, n, share_idx, nshares, slot_idx, slot_pos);
  if (rc) return rc;
  std::vector<uint8_t> coef;
  rc = decode_rows(ctx, k, n, slot_idx, coef, missing);
  if (rc) return rc;
  if (block == 0 || nstripes == 0) return STORB_RS_OK;
  DeviceGuard g(ctx->device);
  hipStream_t s = pick_stream(ctx, hip_stream);
  std::vector<const uint8_t *> in(k);
  std::vector<size_t> ins(k);
  for (uint32_t c = 0; c < k; c++) {
    const uint32_t id = slot_idx[c];
    if (id < k) {
      if (!d_data) return fail(ctx, STORB_RS_EINVAL, "survivor in null data region");
      in[c] = d_data + static_cast<size_t>(id) * block;
      ins[c] = data_stride;
    } else {
      if (!d_parity) return fail(ctx, STORB_RS_EINVAL, "survivor in null parity region");
      in[c] = d_parity + static_cast<size_t>(id - k) * block;
      ins[c] = parity_stride;
    }
  }
  // Surviving data shares: in place when d_out aliases d_data, else copied.
  if (d_out != d_data || out_stride != data_stride) {
    for (uint32_t c = 0; c < k; c++)
      if (slot_idx[c] < k)
        HIP_TRY(ctx, hipMemcpy2DAsync(d_out + static_cast<size_t>(c) * block, out_stride,
                                      in[c], ins[c], block, nstripes,
                                      hipMemcpyDeviceToDevice, s));
  }
  if (missing.empty()) return STORB_RS_OK;
  std::vector<uint8_t *> out(missing.size());
  std::vector<size_t> outs(missing.size(), out_stride);
  for (size_t r = 0; r < missing.size(); r++)
    out[r] = d_out + static_cast<size_t>(missing[r]) * block;
  return apply(ctx, k, static_cast<uint32_t>(missing.size()), coef.data(), in.data(),
               ins.data(), out.data(), outs.data(), block, nstripes, s);
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

// Host BLAKE3: chunks in order with a stack of complete subtrees; the last
// chunk is folded right to left so the final parent carries ROOT.
void storb_blake3(const uint8_t *data, size_t len, uint8_t out[32]) {
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
  std::vector<std::array<uint32_t, 8>> stack;
  for (uint64_t c = 0; c + 1 < n; c++) {
    b3::chunk_cv(cv, data + c * b3::kChunkLen, b3::kChunkLen, c, 0);
    for (uint64_t t = c + 1; (t & 1) == 0; t >>= 1) {
      b3::parent_cv(cv, stack.back().data(), cv, 0);
      stack.pop_back();
    }
    std::array<uint32_t, 8> a;
    std::memcpy(a.data(), cv, 32);
    stack.push_back(a);
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

// ------------------------------------------------------------------ host
int storb_rs_encode(storb_rs_ctx *ctx, uint32_t k, uint32_t n, const uint8_t *data,
                    size_t len, uint8_t *const *parity_out, size_t *block_out,
                    size_t *padlen_out) {
  if (!ctx) return STORB_RS_EINVAL;
  std::lock_guard<std::mutex> lk(ctx->mu);
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
  const size_t S = round_up(B, kAlign);
  const bool zc = static_cast<size_t>(n) * S <= ctx->zc_max;
  // Page-locked, 16-B aligned caller buffers need no staging at all.
  auto aligned = [](const void *q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; };
  const bool in_direct = zc && pad == 0 && S == B && aligned(data) && range_pinned(data, len);
  bool out_direct = zc && S == B;
  for (uint32_t i = 0; out_direct && i < p; i++)
    out_direct = aligned(parity_out[i]) && range_pinned(parity_out[i], B);
  DeviceGuard g(ctx->device);
  if (!in_direct) HIP_TRY(ctx, ctx->pin_in.ensure(static_cast<size_t>(k) * S));
  if (!out_direct) HIP_TRY(ctx, ctx->pin_out.ensure(static_cast<size_t>(p) * S));
  if (!zc) HIP_TRY(ctx, ctx->stage.ensure(static_cast<size_t>(n) * S));
  HostPool &pool = host_pool(ctx);
  hipStream_t s = ctx->stream;
  std::vector<const uint8_t *> in(k);
  std::vector<uint8_t *> out(p);
  std::vector<size_t> ins(k, static_cast<size_t>(k) * S), outs(p, static_cast<size_t>(p) * S);
  // Zero-padded data shares, S-pitched (zfec pads the tail with zeros):
  // columns [off, off + cnt) of every share into pinned staging.
  auto pack = [&](size_t off, size_t cnt) {
    const int parts = static_cast<size_t>(k) * cnt >= (2u << 20) ? static_cast<int>(k) : 1;
    pool.run(parts, [&](int part) {
      for (uint32_t j = static_cast<uint32_t>(part); j < k; j += parts) {
        const size_t src = static_cast<size_t>(j) * B + off;
        size_t avail = off < B ? std::min(cnt, B - off) : 0;
        avail = src < len ? std::min(avail, len - src) : 0;
        uint8_t *dst = ctx->pin_in.p + static_cast<size_t>(j) * S + off;
        if (avail) std::memcpy(dst, data + src, avail);
        if (cnt > avail) std::memset(dst + avail, 0, cnt - avail);
      }
    });
  };
  auto unpack = [&](size_t off, size_t cnt) {
    const size_t c = off < B ? std::min(cnt, B - off) : 0;
    if (!c) return;
    const int parts = static_cast<size_t>(p) * c >= (2u << 20) ? static_cast<int>(p) : 1;
    pool.run(parts, [&](int part) {
      for (uint32_t i = static_cast<uint32_t>(part); i < p; i += parts)
        std::memcpy(parity_out[i] + off, ctx->pin_out.p + static_cast<size_t>(i) * S + off, c);
    });
  };
  if (zc) {  // the kernel reads and writes page-locked host memory over PCIe
    uint8_t *dd, *dp = nullptr;
    HIP_TRY(ctx, host_dev_ptr(in_direct ? const_cast<uint8_t *>(data) : ctx->pin_in.p, &dd));
    std::vector<uint8_t *> pd(p);
    if (out_direct) {
      for (uint32_t i = 0; i < p; i++) HIP_TRY(ctx, host_dev_ptr(parity_out[i], &pd[i]));
    } else {
      HIP_TRY(ctx, host_dev_ptr(ctx->pin_out.p, &dp));
      for (uint32_t i = 0; i < p; i++) pd[i] = dp + static_cast<size_t>(i) * S;
    }
    auto launch = [&](size_t off, size_t cnt) {
      for (uint32_t j = 0; j < k; j++) in[j] = dd + static_cast<size_t>(j) * S + off;
      for (uint32_t i = 0; i < p; i++) out[i] = pd[i] + off;
      return encode_apply(ctx, k, n, in.data(), ins.data(), out.data(), outs.data(), cnt, 1, s);
    };
    if (in_direct && out_direct) {  // nothing to overlap
      const int rc = launch(0, S);
      if (rc) return rc;
      HIP_TRY(ctx, hipStreamSynchronize(s));
      return STORB_RS_OK;
    }
    return sliced(
        ctx, S, [&](size_t off, size_t cnt) { if (!in_direct) pack(off, cnt); }, launch,
        [&](size_t off, size_t cnt) { if (!out_direct) unpack(off, cnt); });
  }
  pack(0, S);
  uint8_t *dd = ctx->stage.p, *dp = ctx->stage.p + static_cast<size_t>(k) * S;
  HIP_TRY(ctx, hipMemcpyAsync(dd, ctx->pin_in.p, static_cast<size_t>(k) * S,
                              hipMemcpyHostToDevice, s));
  for (uint32_t j = 0; j < k; j++) in[j] = dd + static_cast<size_t>(j) * S;
  for (uint32_t i = 0; i < p; i++) out[i] = dp + static_cast<size_t>(i) * S;
  int rc = encode_apply(ctx, k, n, in.data(), ins.data(), out.data(), outs.data(), S, 1, s);
  if (rc) return rc;
  HIP_TRY(ctx, hipMemcpyAsync(ctx->pin_out.p, dp, static_cast<size_t>(p) * S,
                              hipMemcpyDeviceToHost, s));
  HIP_TRY(ctx, hipStreamSynchronize(s));
  unpack(0, S);
  return STORB_RS_OK;
}

int storb_rs_decode(storb_rs_ctx *ctx, uint32_t k, uint32_t n, const uint8_t *const *shares,
                    const uint32_t *share_idx, uint32_t nshares, size_t block,
                    size_t padlen, uint8_t *out) {
  if (!ctx) return STORB_RS_EINVAL;
  std::lock_guard<std::mutex> lk(ctx->mu);
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
  auto put = [&](uint32_t row, const uint8_t *src) {
    const size_t off = static_cast<size_t>(row) * block;
    if (off < outlen) std::memcpy(out + off, src, std::min(block, outlen - off));
  };
  HostPool &pool = host_pool(ctx);
  const int parts = static_cast<size_t>(k) * block >= (1u << 20) ? static_cast<int>(k) : 1;
  auto put_present = [&] {  // surviving data shares: plain copies into out
    pool.run(parts, [&](int part) {
      for (uint32_t s = static_cast<uint32_t>(part); s < k; s += parts)
        if (slot_idx[s] < k) put(s, shares[slot_pos[s]]);
    });
  };
  if (missing.empty()) {  // all data shares present: concatenation, as zfec
    put_present();
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
  if (!in_direct) HIP_TRY(ctx, ctx->pin_in.ensure(static_cast<size_t>(k) * S));
  if (!out_direct) HIP_TRY(ctx, ctx->pin_out.ensure(static_cast<size_t>(e) * S));
  if (!zc) HIP_TRY(ctx, ctx->stage.ensure(static_cast<size_t>(k + e) * S));
  // columns [off, off + cnt) of row `row` of the chunk (truncated at outlen)
  auto put_cols = [&](uint32_t row, size_t off, size_t cnt, const uint8_t *src) {
    const size_t o = static_cast<size_t>(row) * block + off;
    size_t c = off < block ? std::min(cnt, block - off) : 0;
    c = o < outlen ? std::min(c, outlen - o) : 0;
    if (c) std::memcpy(out + o, src, c);
  };
  // slot shares into pinned staging; present data shares also into out
  auto pack = [&](size_t off, size_t cnt) {
    const int pp = static_cast<size_t>(k) * cnt >= (2u << 20) ? static_cast<int>(k) : 1;
    pool.run(pp, [&](int part) {
      for (uint32_t c = static_cast<uint32_t>(part); c < k; c += pp) {
        const uint8_t *src = shares[slot_pos[c]] + off;
        const size_t avail = off < block ? std::min(cnt, block - off) : 0;
        if (!in_direct) {
          uint8_t *dst = ctx->pin_in.p + static_cast<size_t>(c) * S + off;
          if (avail) std::memcpy(dst, src, avail);
          if (cnt > avail) std::memset(dst + avail, 0, cnt - avail);
        }
        if (slot_idx[c] < k) put_cols(c, off, cnt, src);
      }
    });
  };
  auto unpack = [&](size_t off, size_t cnt) {
    if (out_direct) return;
    for (uint32_t r = 0; r < e; r++)
      put_cols(missing[r], off, cnt, ctx->pin_out.p + static_cast<size_t>(r) * S + off);
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
      HIP_TRY(ctx, host_dev_ptr(ctx->pin_in.p, &base));
      for (uint32_t c = 0; c < k; c++) id[c] = base + static_cast<size_t>(c) * S;
    }
    if (out_direct) {
      HIP_TRY(ctx, host_dev_ptr(out, &base));
      for (uint32_t r = 0; r < e; r++) od[r] = base + static_cast<size_t>(missing[r]) * block;
    } else {
      HIP_TRY(ctx, host_dev_ptr(ctx->pin_out.p, &base));
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
    return sliced(ctx, S, pack, launch, unpack);
  }
  pack(0, S);
  uint8_t *din = ctx->stage.p, *dout = ctx->stage.p + static_cast<size_t>(k) * S;
  HIP_TRY(ctx, hipMemcpyAsync(din, ctx->pin_in.p, static_cast<size_t>(k) * S,
                              hipMemcpyHostToDevice, s));
  for (uint32_t c = 0; c < k; c++) in[c] = din + static_cast<size_t>(c) * S;
  for (uint32_t r = 0; r < e; r++) o[r] = dout + static_cast<size_t>(r) * S;
  rc = apply(ctx, k, e, coef.data(), in.data(), ins.data(), o.data(), outs.data(), S, 1, s);
  if (rc) return rc;
  HIP_TRY(ctx, hipMemcpyAsync(ctx->pin_out.p, dout, static_cast<size_t>(e) * S,
                              hipMemcpyDeviceToHost, s));
  HIP_TRY(ctx, hipStreamSynchronize(s));
  unpack(0, S);
  return STORB_RS_OK;
}

int storb_rs_repair(storb_rs_ctx *ctx, uint32_t k, uint32_t n, const uint8_t *const *shares,
                    const uint32_t *share_idx, uint32_t nshares, size_t block,
                    const uint32_t *targets, uint32_t ntargets, uint8_t *const *out) {
  if (!ctx) return STORB_RS_EINVAL;
  std::lock_guard<std::mutex> lk(ctx->mu);
  if (!valid_params(k, n)) return fail(ctx, STORB_RS_EINVAL, "invalid (k, n)");
  if (!shares || !share_idx || (ntargets && (!targets || !out)) || block == 0)
    return fail(ctx, STORB_RS_EINVAL, "repair: bad arguments");
  std::vector<uint32_t> slot_idx, slot_pos;
  int rc = select_shares(ctx, k, n, share_idx, nshares, slot_idx, slot_pos);
  if (rc) return rc;
  std::vector<uint8_t> coef;
  rc = repair_rows(ctx, k, n, slot_idx, targets, ntargets, coef);
  if (rc || ntargets == 0) return rc;
  const size_t S = round_up(block, kAlign);
  DeviceGuard g(ctx->device);
  HIP_TRY(ctx, ctx->pin_in.ensure(static_cast<size_t>(k) * S));
  HIP_TRY(ctx, ctx->pin_out.ensure(static_cast<size_t>(ntargets) * S));
  HIP_TRY(ctx, ctx->stage.ensure(static_cast<size_t>(k + ntargets) * S));
  for (uint32_t c = 0; c < k; c++) {
    std::memcpy(ctx->pin_in.p + static_cast<size_t>(c) * S, shares[slot_pos[c]], block);
    std::memset(ctx->pin_in.p + static_cast<size_t>(c) * S + block, 0, S - block);
  }
  hipStream_t s = ctx->stream;
  const bool zc = static_cast<size_t>(k + ntargets) * S <= ctx->zc_max;
  uint8_t *din = ctx->stage.p, *dout = ctx->stage.p + static_cast<size_t>(k) * S;
  if (zc) {  // zero-copy: the kernel works on the pinned staging directly
    HIP_TRY(ctx, host_dev_ptr(ctx->pin_in.p, &din));
    HIP_TRY(ctx, host_dev_ptr(ctx->pin_out.p, &dout));
  } else {
    HIP_TRY(ctx, hipMemcpyAsync(din, ctx->pin_in.p, static_cast<size_t>(k) * S,
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
    HIP_TRY(ctx, hipMemcpyAsync(ctx->pin_out.p, dout, static_cast<size_t>(ntargets) * S,
                                hipMemcpyDeviceToHost, s));
  HIP_TRY(ctx, hipStreamSynchronize(s));
  for (uint32_t r = 0; r < ntargets; r++)
    std::memcpy(out[r], ctx->pin_out.p + static_cast<size_t>(r) * S, block);
  return STORB_RS_OK;
}

// Pipelined batch encode: two pinned in/out buffer pairs and two streams.
// While the GPU copies and encodes batch i, the host packs batch i+1 and
// unpacks batch i-1 (hipMemcpyAsync from pinned memory is a true DMA).
// With hashes_out, the blake3 of every share is computed on the device
// right after the encode kernel and only the digests come back.
static int encode_chunks_impl(storb_rs_ctx *ctx, uint32_t k, uint32_t n,
                              const uint8_t *data, size_t chunk_len, uint32_t nchunks,
                              uint8_t *parity_out, uint8_t *hashes_out) {
  if (!ctx) return STORB_RS_EINVAL;
  std::lock_guard<std::mutex> lk(ctx->mu);
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
  // share one ceiling (57 GB/s total, tools/pcie_probe.py): 47 vs 35 GiB/s
  // measured. From pageable chunks the SDMA pipeline stays ahead (34 vs
  // 20 GiB/s: the host's packing competes with the kernel's reads of the
  // same staging), and the hashed path keeps the shares on the device.
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
  auto unpack = [&](uint32_t bi) {
    const int b = bi & 1;
    const uint32_t c0 = bi * batch, cn = std::min(batch, nchunks - c0);
    if (p > 0 && !out_direct) {
      if (S == B) {
        pool.copy(parity_out + static_cast<size_t>(c0) * p * B, ctx->pipe_out[b].p,
                  static_cast<size_t>(cn) * p * B);
      } else {
        pool.run(static_cast<int>(cn), [&](int c) {
          for (uint32_t i = 0; i < p; i++)
            std::memcpy(parity_out + ((static_cast<size_t>(c0) + c) * p + i) * B,
                        ctx->pipe_out[b].p + (static_cast<size_t>(c) * p + i) * S, B);
        });
      }
    }
    if (hashes_out) {
      // device order: [c][j] data digests, then [c][i] parity digests
      const uint8_t *hd = ctx->pipe_out[b].p + static_cast<size_t>(p) * S * batch;
      const uint8_t *hp = hd + static_cast<size_t>(cn) * k * 32;
      for (uint32_t c = 0; c < cn; c++) {
        uint8_t *o = hashes_out + (static_cast<size_t>(c0) + c) * n * 32;
        std::memcpy(o, hd + static_cast<size_t>(c) * k * 32, static_cast<size_t>(k) * 32);
        std::memcpy(o + static_cast<size_t>(k) * 32, hp + static_cast<size_t>(c) * p * 32,
                    static_cast<size_t>(p) * 32);
      }
    }
  };
  for (uint32_t bi = 0; bi < nb; bi++) {
    const int b = bi & 1;
    hipStream_t s = ctx->pipe[b];
    // Pinned buffer pair b is free once batch bi-2 has landed (device
    // buffers are reused in stream order and need no host wait).
    if (bi >= 2 && !(in_direct && (out_direct || p == 0) && !hashes_out)) {
      HIP_TRY(ctx, hipStreamSynchronize(s));
      unpack(bi - 2);
    }
    const uint32_t c0 = bi * batch, cn = std::min(batch, nchunks - c0);
    const uint8_t *hin = in_direct ? data + static_cast<size_t>(c0) * chunk_len
                                   : ctx->pipe_in[b].p;
    if (in_direct) {
      // the H2D below reads the caller's page-locked chunks in place
    } else if (packed) {
      pool.copy(ctx->pipe_in[b].p, data + static_cast<size_t>(c0) * chunk_len, per * cn);
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
    HIP_TRY(ctx, hipMemcpyAsync(dd, hin, per * cn, hipMemcpyHostToDevice, s));
    if (p > 0) {
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
    if (hashes_out) {
      // shares are pitched S apart across the whole batch: one launch each
      HIP_TRY(ctx, launch_blake3_batch(dd, B, cn * k, S, dh, s));
      if (p > 0)
        HIP_TRY(ctx, launch_blake3_batch(dp, B, cn * p, S, dh + static_cast<size_t>(cn) * k * 32,
                                         s));
    }
    if (back)
      HIP_TRY(ctx, hipMemcpyAsync(out_direct ? parity_out + static_cast<size_t>(c0) * p * B
                                             : ctx->pipe_out[b].p,
                                  dp, back, hipMemcpyDeviceToHost, s));
    if (hashes_out)
      HIP_TRY(ctx, hipMemcpyAsync(ctx->pipe_out[b].p + static_cast<size_t>(p) * S * batch, dh,
                                  static_cast<size_t>(cn) * n * 32, hipMemcpyDeviceToHost, s));
  }
  for (uint32_t bi = nb >= 2 ? nb - 2 : 0; bi < nb; bi++) {
    HIP_TRY(ctx, hipStreamSynchronize(ctx->pipe[bi & 1]));
    unpack(bi);
  }
  return STORB_RS_OK;
}

// Pipelined batch decode (the download path, download.rs:453-465, one
// chunk after another today). Every chunk selects its first k shares by
// index (decode_chunk, piece.rs:368-381). Chunks whose k data shares are all
// present are pure host copies; the rest are grouped by erasure pattern, so
// each batch is one launch of one decode matrix, and stream through the same
// double-buffered pinned pipeline as encode: pack the k survivors into
// pinned staging (present data shares also go straight to `out`), H2D,
// rebuild only the missing rows, D2H them, unpack into `out`.
int storb_rs_decode_chunks(storb_rs_ctx *ctx, uint32_t k, uint32_t n, size_t block,
                           size_t padlen, uint32_t nchunks, const uint8_t *const *shares,
                           const uint32_t *share_idx, const uint32_t *nshares, uint8_t *out,
                           size_t out_stride) {
  if (!ctx) return STORB_RS_EINVAL;
  std::lock_guard<std::mutex> lk(ctx->mu);
  if (!valid_params(k, n)) return fail(ctx, STORB_RS_EINVAL, "invalid (k, n)");
  if (nchunks == 0) return STORB_RS_OK;
  if (!shares || !share_idx || !nshares || !out || block == 0 ||
      padlen >= static_cast<size_t>(k) * block)
    return fail(ctx, STORB_RS_EINVAL, "decode_chunks: bad arguments");
  const size_t outlen = static_cast<size_t>(k) * block - padlen;
  if (out_stride == 0) out_stride = outlen;
  if (out_stride < outlen) return fail(ctx, STORB_RS_EINVAL, "decode_chunks: out_stride < chunk");
  // per chunk: its k slot shares (pointers) and erasure pattern
  std::vector<const uint8_t *> slot_ptr(static_cast<size_t>(nchunks) * k);
  std::map<std::vector<uint32_t>, std::vector<uint32_t>> groups;
  std::vector<uint32_t> plain;
  size_t off = 0;
  for (uint32_t c = 0; c < nchunks; c++) {
    std::vector<uint32_t> slot_idx, slot_pos;
    const int rc = select_shares(ctx, k, n, share_idx + off, nshares[c], slot_idx, slot_pos);
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
    bool all_data = true;
    for (uint32_t s = 0; s < k; s++) all_data &= slot_idx[s] == s;
    if (all_data)
      plain.push_back(c);
    else
      groups[slot_idx].push_back(c);
  }
  HostPool &pool = host_pool(ctx);
  auto put_row = [&](uint32_t c, uint32_t row, const uint8_t *src) {
    const size_t o = static_cast<size_t>(row) * block;
    if (o < outlen)
      std::memcpy(out + static_cast<size_t>(c) * out_stride + o, src, std::min(block, outlen - o));
  };
  if (!plain.empty())  // all data shares present: concatenation (zfec does the same)
    pool.run(static_cast<int>(plain.size()), [&](int i) {
      for (uint32_t s = 0; s < k; s++)
        put_row(plain[i], s, slot_ptr[static_cast<size_t>(plain[i]) * k + s]);
    });
  if (groups.empty()) return STORB_RS_OK;

  struct Item {
    const std::vector<uint32_t> *slots;
    const uint32_t *chunks;
    uint32_t cn;
    std::vector<uint8_t> coef;
    std::vector<uint32_t> missing;
  };
  const size_t S = round_up(block, kAlign);
  const size_t per = static_cast<size_t>(k) * S;
  uint32_t batch = static_cast<uint32_t>(std::max<size_t>(1, (64ull << 20) / per));
  std::vector<Item> items;
  uint32_t emax = 0;
  for (auto &g : groups) {
    std::vector<uint8_t> coef;
    std::vector<uint32_t> missing;
    const int rc = decode_rows(ctx, k, n, g.first, coef, missing);
    if (rc) return rc;
    emax = std::max<uint32_t>(emax, static_cast<uint32_t>(missing.size()));
    for (size_t i = 0; i < g.second.size(); i += batch)
      items.push_back(Item{&g.first, g.second.data() + i,
                           static_cast<uint32_t>(std::min<size_t>(batch, g.second.size() - i)),
                           coef, missing});
  }
  batch = 0;
  for (auto &it : items) batch = std::max(batch, it.cn);
  DeviceGuard dg(ctx->device);
  for (int b = 0; b < 2; b++) {
    HIP_TRY(ctx, ctx->pipe_in[b].ensure(per * batch));
    HIP_TRY(ctx, ctx->pipe_out[b].ensure(static_cast<size_t>(emax) * S * batch));
    HIP_TRY(ctx, ctx->pipe_dev[b].ensure(static_cast<size_t>(k + emax) * S * batch));
  }
  auto unpack = [&](size_t ii) {
    const Item &it = items[ii];
    const uint8_t *src = ctx->pipe_out[ii & 1].p;
    const uint32_t e = static_cast<uint32_t>(it.missing.size());
    pool.run(static_cast<int>(it.cn), [&](int c) {
      for (uint32_t r = 0; r < e; r++)
        put_row(it.chunks[c], it.missing[r], src + (static_cast<size_t>(c) * e + r) * S);
    });
  };
  for (size_t ii = 0; ii < items.size(); ii++) {
    const int b = ii & 1;
    hipStream_t s = ctx->pipe[b];
    if (ii >= 2) {  // pinned pair b is free once item ii-2 has landed
      HIP_TRY(ctx, hipStreamSynchronize(s));
      unpack(ii - 2);
    }
    const Item &it = items[ii];
    const uint32_t e = static_cast<uint32_t>(it.missing.size());
    uint8_t *hin = ctx->pipe_in[b].p;
    pool.run(static_cast<int>(it.cn), [&](int c) {
      const uint32_t ch = it.chunks[c];
      for (uint32_t sl = 0; sl < k; sl++) {
        const uint8_t *src = slot_ptr[static_cast<size_t>(ch) * k + sl];
        uint8_t *dst = hin + static_cast<size_t>(c) * per + static_cast<size_t>(sl) * S;
        std::memcpy(dst, src, block);
        if (S > block) std::memset(dst + block, 0, S - block);
        if ((*it.slots)[sl] == sl) put_row(ch, sl, src);  // present data share
      }
    });
    uint8_t *dd = ctx->pipe_dev[b].p;
    uint8_t *dm = dd + per * it.cn;
    HIP_TRY(ctx, hipMemcpyAsync(dd, hin, per * it.cn, hipMemcpyHostToDevice, s));
    std::vector<const uint8_t *> in(k);
    std::vector<uint8_t *> o(e);
    std::vector<size_t> ins(k, per), outs(e, static_cast<size_t>(e) * S);
    for (uint32_t j = 0; j < k; j++) in[j] = dd + static_cast<size_t>(j) * S;
    for (uint32_t r = 0; r < e; r++) o[r] = dm + static_cast<size_t>(r) * S;
    const int rc = apply(ctx, k, e, it.coef.data(), in.data(), ins.data(), o.data(), outs.data(),
                         S, it.cn, s);
    if (rc) return rc;
    HIP_TRY(ctx, hipMemcpyAsync(ctx->pipe_out[b].p, dm, static_cast<size_t>(e) * S * it.cn,
                                hipMemcpyDeviceToHost, s));
  }
  for (size_t ii = items.size() >= 2 ? items.size() - 2 : 0; ii < items.size(); ii++) {
    HIP_TRY(ctx, hipStreamSynchronize(ctx->pipe[ii & 1]));
    unpack(ii);
  }
  return STORB_RS_OK;
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
