// decode_stripes.cpp -- decode where every stripe lost different shares.
//
// Storb's download keeps whichever k + 1 pieces of a chunk arrive first from
// its 10 fetch threads (crates/storb_validator/src/download.rs:363-451), then
// decode_chunk sorts them and takes the first k (piece.rs:368-381). So the
// survivor set, and with it the decode matrix, varies from chunk to chunk. A
// launch per erasure pattern would be one small launch per chunk (and, with
// the run-time-compiled kernels, one compile per pattern). Here a batch of
// chunks is one launch (rows 0-4, the common case) plus one per larger
// missing-row count: every workgroup reads its own stripe's descriptor --
// the k input pointers, the rebuilt rows' pointers, the assembly targets --
// and its own pattern's v_perm tables (rs_device.hpp rs_apply_desc; the
// table kernel's tile, unchanged).
//
// Patterns (slot arrangement, inverted rows, tables) are cached per context.
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <cstring>
#include <mutex>
#include <unordered_map>
#include <vector>

#include "ctx.hpp"

using namespace storb_rs;
using namespace storb_rs::detail;

namespace storb_rs {
namespace detail {

constexpr size_t kPatternCap = 4096;  // cached decode patterns per context

// Called at the start of a call (never inside one, so every Pattern a call
// holds stays valid until it returns): drop the least recently used quarter
// once the cache is full.
void trim_patterns(storb_rs_ctx *ctx) {
  if (ctx->patterns.size() < kPatternCap) return;
  std::vector<uint64_t> ticks;
  ticks.reserve(ctx->patterns.size());
  for (auto &p : ctx->patterns) ticks.push_back(p.second->tick);
  std::nth_element(ticks.begin(), ticks.begin() + ticks.size() / 4, ticks.end());
  const uint64_t cut = ticks[ticks.size() / 4];
  for (auto it = ctx->patterns.begin(); it != ctx->patterns.end();)
    it = it->second->tick < cut ? ctx->patterns.erase(it) : std::next(it);
}

int get_pattern(storb_rs_ctx *ctx, uint32_t k, uint32_t n, const uint32_t *share_idx,
                uint32_t nshares, const Pattern **out, std::vector<uint32_t> &slot_pos) {
  std::vector<uint32_t> slot_idx;
  int rc = select_shares(ctx, k, n, share_idx, nshares, slot_idx, slot_pos);
  if (rc) return rc;
  std::vector<uint32_t> key;
  key.reserve(k + 2);
  key.push_back(k);
  key.push_back(n);
  key.insert(key.end(), slot_idx.begin(), slot_idx.end());
  auto it = ctx->patterns.find(key);
  if (it == ctx->patterns.end()) {
    auto p = std::make_unique<Pattern>();
    rc = decode_rows(ctx, k, n, slot_idx, p->coef, p->missing);
    if (rc) return rc;
    p->slot_idx = std::move(slot_idx);
    const uint32_t e = static_cast<uint32_t>(p->missing.size());
    const uint32_t rb = static_cast<uint32_t>(rows_bucket(e ? e : 1));
    if (e <= static_cast<uint32_t>(kSlotR)) {  // tables only for what rs_apply_desc takes
      p->tabs.assign(static_cast<size_t>(k) * rb, PermTab{});
      for (uint32_t r = 0; r < e; r++)
        for (uint32_t j = 0; j < k; j++)
          p->tabs[static_cast<size_t>(j) * rb + r] = perm_tab(p->coef[static_cast<size_t>(r) * k + j]);
    }
    it = ctx->patterns.emplace(std::move(key), std::move(p)).first;
  }
  it->second->tick = ++ctx->pattern_tick;
  *out = it->second.get();
  return STORB_RS_OK;
}

int PatternMemo::get(const uint32_t *share_idx, uint32_t nshares, const Pattern **out,
                     std::vector<uint32_t> &slot_pos) {
  if (n_ > 64 || nshares < k_) return get_pattern(ctx_, k_, n_, share_idx, nshares, out, slot_pos);
  uint64_t mask = 0;
  uint8_t pos[64];
  for (uint32_t i = 0; i < nshares; i++) {
    const uint32_t id = share_idx[i];
    if (id >= n_ || (mask >> id & 1)) return get_pattern(ctx_, k_, n_, share_idx, nshares, out, slot_pos);
    mask |= 1ull << id;
    pos[id] = static_cast<uint8_t>(i);
  }
  // no duplicates: the first k by index are the k lowest set bits
  uint64_t key = 0, m = mask;
  for (uint32_t i = 0; i < k_; i++) {
    const uint64_t low = m & (~m + 1);
    key |= low;
    m ^= low;
  }
  const uint32_t h = static_cast<uint32_t>((key * 0x9E3779B97F4A7C15ull) >> 56) % kSlots;
  if (pat_[h] && key_[h] == key) {
    const Pattern *p = pat_[h];
    slot_pos.resize(k_);
    for (uint32_t s = 0; s < k_; s++) slot_pos[s] = pos[p->slot_idx[s]];
    *out = p;
    return STORB_RS_OK;
  }
  const int rc = get_pattern(ctx_, k_, n_, share_idx, nshares, out, slot_pos);
  if (rc == STORB_RS_OK) {
    key_[h] = key;
    pat_[h] = *out;
  }
  return rc;
}

bool desc_ok(const storb_rs_ctx *ctx, uint32_t k, uint32_t n, size_t block) {
  return ctx->variant != STORB_RS_KERNEL_LDS && k >= 1 && k <= static_cast<uint32_t>(kSlotK) &&
         std::min(k, n - k) <= static_cast<uint32_t>(kSlotR) && block % kAlign == 0;
}

// Tiles per workgroup of a descriptor launch set covering `tiles` tiles in
// all. One: two or more per workgroup measured slower at every size once the
// records are scalar loads (k = 16 download mix: tpw 1 / 2 / 4 / 8 = 66.8 /
// 63.3 / 55.0 / 54.0 % per-row-count, 72.4 / 65.2 % mixed, descbench); more
// only when the grid would exceed the launch limit.
uint32_t desc_tpw(uint64_t tiles) {
  return static_cast<uint32_t>(std::max<uint64_t>(1, (tiles + 0x3FFFFFFFull) / 0x40000000ull));
}

int apply_desc(storb_rs_ctx *ctx, uint32_t k, size_t block, bool copy,
               const std::vector<const Pattern *> &pats, const std::vector<uint64_t> &ptr,
               hipStream_t s) {
  const size_t W = 2 * static_cast<size_t>(k) + kSlotR;
  // Items of up to kMixR rebuilt rows (a download's chunks: most lost 0-3
  // data shares, each chunk a different set) go to ONE mixed-row launch; each
  // row count above that gets a launch of its own. Everything on the
  // caller's stream, in order: after the address-space fix the launches are
  // HBM-bound, and sequential launches measured faster than the same ones
  // fanned out over three streams (67.7 vs 62.0 % of peak, descbench).
  struct Group {
    uint32_t r = 0, rec_q = 0;
    bool mix = false;
    std::vector<uint32_t> items;
    size_t tab_off = 0, rec_off = 0, ntab = 0;
    std::unordered_map<const Pattern *, size_t> tab_at;  // pattern -> its tables (PermTabs)
  };
  std::vector<Group> by_r(kSlotR + 1);
  Group mixg;
  mixg.mix = true;
  mixg.r = kMixR;
  for (uint32_t i = 0; i < pats.size(); i++) {
    const uint32_t e = static_cast<uint32_t>(pats[i]->missing.size());
    if (e > static_cast<uint32_t>(kSlotR)) return fail(ctx, STORB_RS_EINVAL, "apply_desc: > 16 rows");
    if (!e && !copy) continue;
    (e <= kMixR ? mixg : by_r[e]).items.push_back(i);
  }
  // The mixed launch's items heaviest first (most rebuilt rows): the
  // workgroups with the longest folds start first, and the launch's tail is
  // its lightest tiles (tools/mixbench.hip "heaviest items first": k = 32
  // download mix 73.9-74.3 -> 74.7-75.7 % of 8 TB/s, profiles/r6i_mixbench32.txt,
  // r6j_*; with k = 16's input-split tiles 77.2-77.4 -> 77.8-77.9 %).
  std::stable_sort(mixg.items.begin(), mixg.items.end(), [&](uint32_t x, uint32_t y) {
    return pats[x]->missing.size() > pats[y]->missing.size();
  });
  std::vector<Group *> groups;
  if (!mixg.items.empty()) groups.push_back(&mixg);
  for (uint32_t e = kMixR + 1; e <= static_cast<uint32_t>(kSlotR); e++)
    if (!by_r[e].items.empty()) {
      by_r[e].r = e;
      groups.push_back(&by_r[e]);
    }
  if (groups.empty()) return STORB_RS_OK;
  size_t total = 0;
  uint64_t tiles = 0;
  const uint64_t tps = (block / 16 + kThreadsTable - 1) / kThreadsTable;
  // item i's tables within its group's table block (the same pattern in
  // consecutive items -- the common case -- skips the hash lookup)
  std::vector<size_t> item_tab(pats.size());
  for (Group *g : groups) {
    g->rec_q = 1 + k + g->r + (copy ? k : 0);
    g->tab_off = total;
    const Pattern *last = nullptr;
    size_t last_at = 0;
    for (uint32_t i : g->items) {
      if (pats[i] != last) {
        auto ins = g->tab_at.emplace(pats[i], g->ntab);
        if (ins.second) g->ntab += pats[i]->tabs.size();
        last = pats[i];
        last_at = ins.first->second;
      }
      item_tab[i] = last_at;
    }
    total = round_up(total + g->ntab * sizeof(PermTab), 256);
    g->rec_off = total;
    total = round_up(total + g->items.size() * g->rec_q * 8, 256);
    tiles += tps * g->items.size();
  }
  const uint32_t tpw = desc_tpw(tiles);
  // Upload slot (page-locked source + device copy). The page-locked source
  // is rewritten once the slot's previous copy has completed (host wait, on
  // the descriptor stream's own event); the device copy is overwritten once
  // the previous decode launches have (the copy waits for their mark on the
  // descriptor stream). A slot that must grow is reallocated, and hipFree /
  // hipHostFree synchronise the device first.
  const unsigned slot = ctx->desc_next++ % kDescRing;
  if (ctx->desc_cp[slot]) HIP_TRY(ctx, hipEventSynchronize(ctx->desc_cp[slot]));
  else HIP_TRY(ctx, hipEventCreateWithFlags(&ctx->desc_cp[slot], kOrderEvent));
  hipEvent_t prev = nullptr;  // the mark after the slot's previous decode
  if (ctx->desc_use[slot].second) {
    HIP_TRY(ctx, covering_mark(ctx, ctx->desc_use[slot].first, ctx->desc_use[slot].second, s, &prev));
    if (!prev) {  // its stream is not this call's: rare (counted, storb_rs_ctx_stats)
      ctx->n_device_syncs++;
      HIP_TRY(ctx, hipDeviceSynchronize());
    }
  }
  HIP_TRY(ctx, ctx->desc_pin[slot].ensure(total));
  HIP_TRY(ctx, ctx->desc_dev[slot].ensure(total));
  uint8_t *h = ctx->desc_pin[slot].p;
  for (Group *g : groups) {
    PermTab *t = reinterpret_cast<PermTab *>(h + g->tab_off);
    for (auto &pt : g->tab_at)
      std::memcpy(t + pt.second, pt.first->tabs.data(), pt.first->tabs.size() * sizeof(PermTab));
    uint64_t *rec = reinterpret_cast<uint64_t *>(h + g->rec_off);
    for (uint32_t i : g->items) {
      const uint64_t *src = &ptr[i * W];
      const uint64_t e = pats[i]->missing.size();
      rec[0] = static_cast<uint64_t>(item_tab[i]) | (e << 32);
      std::memcpy(rec + 1, src, static_cast<size_t>(k) * 8);
      std::memset(rec + 1 + k, 0, static_cast<size_t>(g->r) * 8);
      std::memcpy(rec + 1 + k, src + k, static_cast<size_t>(e) * 8);
      if (copy) std::memcpy(rec + 1 + k + g->r, src + k + kSlotR, static_cast<size_t>(k) * 8);
      rec += g->rec_q;
    }
  }
  uint8_t *dev = ctx->desc_dev[slot].p, *hd = nullptr;
  HIP_TRY(ctx, host_dev_ptr(h, &hd));
  // The copy runs on the context's descriptor stream, so it overlaps whatever
  // the caller's stream is still running (the slot is free: its last use has
  // completed); the decode launches wait for it on the device.
  if (!ctx->desc_stream) {
    // Highest priority: a stream of its own priority class gets a hardware
    // queue of its own, so the copy can run under the caller's previous
    // kernel instead of queueing behind it (a default-priority stream can
    // share the caller's queue: profiles/r5j_download_timeline.txt).
    int lo = 0, hi = 0;
    if (hipDeviceGetStreamPriorityRange(&lo, &hi) != hipSuccess) hi = 0;
    HIP_TRY(ctx, hipStreamCreateWithPriority(&ctx->desc_stream, hipStreamNonBlocking, hi));
    HIP_TRY(ctx, hipEventCreateWithFlags(&ctx->desc_copied, hipEventDisableTiming));
  }
  hipError_t e = prev ? hipStreamWaitEvent(ctx->desc_stream, prev, 0) : hipSuccess;
  if (e == hipSuccess) e = launch_copy16(dev, hd, total, ctx->desc_stream);
  if (e == hipSuccess) e = hipEventRecord(ctx->desc_cp[slot], ctx->desc_stream);
  if (e == hipSuccess) e = hipEventRecord(ctx->desc_copied, ctx->desc_stream);
  if (e == hipSuccess) e = hipStreamWaitEvent(s, ctx->desc_copied, 0);
  for (size_t gi = 0; e == hipSuccess && gi < groups.size(); gi++) {
    const Group &g = *groups[gi];
    DescArgs a{};
    a.desc = reinterpret_cast<const uint64_t *>(dev + g.rec_off);
    a.ptab = reinterpret_cast<const PermTab *>(dev + g.tab_off);
    a.block = block;
    a.k = k;
    a.r = g.r;
    a.tpw = tpw;
    a.nitems = static_cast<uint32_t>(g.items.size());
    a.copy = copy ? 1u : 0u;
    a.rec_qwords = g.rec_q;
    a.mix = g.mix ? 1u : 0u;
    e = launch_apply_desc(a, s);
  }
  // the slot's last use (also after a failed launch: earlier ones may be queued)
  uint64_t use = 0;
  const hipError_t er = stream_used(ctx, s, &use);
  ctx->desc_use[slot] = {s, use};
  if (e != hipSuccess) return hip_fail(ctx, e, "apply_desc");
  if (er != hipSuccess) return hip_fail(ctx, er, "hipEventRecord(descriptors)");
  return STORB_RS_OK;
}

// One pattern for nstripes stripes of the device layout (storb_rs.h): the
// uniform batch decode. Compiled bit-sliced kernels where the policy wants
// them (apply); fused assembly when d_out is a separate buffer.
int decode_pattern_batch(storb_rs_ctx *ctx, uint32_t k, size_t block, uint32_t nstripes,
                         const Pattern &p, const uint8_t *d_data, size_t data_stride,
                         const uint8_t *d_parity, size_t parity_stride, uint8_t *d_out,
                         size_t out_stride, hipStream_t s) {
  std::vector<const uint8_t *> in(k);
  std::vector<size_t> ins(k);
  for (uint32_t c = 0; c < k; c++) {
    const uint32_t id = p.slot_idx[c];
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
  const size_t e = p.missing.size();
  std::vector<uint8_t *> out(e);
  std::vector<size_t> outs(e, out_stride);
  for (size_t r = 0; r < e; r++) out[r] = d_out + static_cast<size_t>(p.missing[r]) * block;
  // Surviving data shares: in place when d_out aliases d_data; else stored
  // to their slots of d_out by the decode kernel itself as it reads them
  // (fused assembly), or, where no such kernel applies, copied first (apply).
  const bool assemble = d_out != d_data || out_stride != data_stride;
  std::vector<uint8_t *> copy(k, nullptr);
  std::vector<size_t> copys(k, out_stride);
  if (assemble)
    for (uint32_t c = 0; c < k; c++)
      if (p.slot_idx[c] < k) copy[c] = d_out + static_cast<size_t>(c) * block;
  return apply(ctx, k, static_cast<uint32_t>(e), p.coef.data(), in.data(), ins.data(), out.data(),
               outs.data(), block, nstripes, s, assemble ? copy.data() : nullptr,
               assemble ? copys.data() : nullptr);
}

}  // namespace detail
}  // namespace storb_rs

extern "C" {

int storb_rs_decode_stripes_dev(storb_rs_ctx *ctx, uint32_t k, uint32_t n, size_t block,
                                uint32_t nstripes, const uint32_t *share_idx,
                                const uint32_t *nshares, const uint8_t *d_data,
                                size_t data_stride, const uint8_t *d_parity,
                                size_t parity_stride, uint8_t *d_out, size_t out_stride,
                                void *hip_stream) {
  if (!ctx) return STORB_RS_EINVAL;
  std::lock_guard<std::mutex> lk(ctx->mu);
  if (!valid_params(k, n)) return fail(ctx, STORB_RS_EINVAL, "invalid (k, n)");
  if (nstripes && (!share_idx || !nshares || !d_out))
    return fail(ctx, STORB_RS_EINVAL, "null argument");
  if (data_stride == 0) data_stride = static_cast<size_t>(k) * block;
  if (parity_stride == 0) parity_stride = static_cast<size_t>(n - k) * block;
  if (out_stride == 0) out_stride = static_cast<size_t>(k) * block;
  trim_patterns(ctx);
  std::vector<const Pattern *> pats(nstripes);
  std::vector<uint32_t> slot_pos;
  size_t off = 0;
  bool uniform = true;
  PatternMemo memo(ctx, k, n);
  for (uint32_t st = 0; st < nstripes; st++) {
    const int rc = memo.get(share_idx + off, nshares[st], &pats[st], slot_pos);
    if (rc) {
      ctx->last_error += " (stripe " + std::to_string(st) + ")";
      return rc;
    }
    off += nshares[st];
    uniform = uniform && pats[st] == pats[0];
  }
  if (block == 0 || nstripes == 0) return STORB_RS_OK;
  DeviceGuard g(ctx->device);
  hipStream_t s = pick_stream(ctx, hip_stream);
  const bool assemble = d_out != d_data || out_stride != data_stride;
  if (uniform)  // one pattern: the uniform path (compiled kernels, where wanted)
    return decode_pattern_batch(ctx, k, block, nstripes, *pats[0], d_data, data_stride, d_parity,
                                parity_stride, d_out, out_stride, s);
  auto al = [](const void *p, size_t st) { return ((reinterpret_cast<uintptr_t>(p) | st) % kAlign) == 0; };
  bool need_data = false, need_par = false;
  for (const Pattern *p : pats)
    for (uint32_t c = 0; c < k; c++) (p->slot_idx[c] < k ? need_data : need_par) = true;
  if (need_data && !d_data) return fail(ctx, STORB_RS_EINVAL, "survivor in null data region");
  if (need_par && !d_parity) return fail(ctx, STORB_RS_EINVAL, "survivor in null parity region");
  if (!desc_ok(ctx, k, n, block) || !al(d_data, data_stride) || !al(d_parity, parity_stride) ||
      !al(d_out, out_stride)) {
    // Geometries the descriptor kernel does not take: one launch per run of
    // consecutive stripes with the same pattern.
    for (uint32_t a = 0; a < nstripes;) {
      uint32_t b = a + 1;
      while (b < nstripes && pats[b] == pats[a]) b++;
      const int rc = decode_pattern_batch(
          ctx, k, block, b - a, *pats[a], d_data ? d_data + a * data_stride : nullptr, data_stride,
          d_parity ? d_parity + a * parity_stride : nullptr, parity_stride,
          d_out + a * out_stride, out_stride, s);
      if (rc) return rc;
      a = b;
    }
    return STORB_RS_OK;
  }
  // Assembly into a separate buffer: stored by the kernel from its own loads
  // for k <= kCopyMaxK; wider codes copy all data slots first (one 2-D copy)
  // and rebuild the missing rows over them.
  // (With no surviving data share in any stripe -- possible when n >= 2k --
  // every data row is rebuilt and d_data may be null: nothing to copy.)
  const bool fused = assemble && k <= kCopyMaxK;
  if (assemble && !fused && need_data)
    HIP_TRY(ctx, hipMemcpy2DAsync(d_out, out_stride, d_data, data_stride,
                                  static_cast<size_t>(k) * block, nstripes,
                                  hipMemcpyDeviceToDevice, s));
  const size_t W = 2 * static_cast<size_t>(k) + kSlotR;
  std::vector<uint64_t> ptr(static_cast<size_t>(nstripes) * W, 0);
  for (uint32_t st = 0; st < nstripes; st++) {
    const Pattern &p = *pats[st];
    uint64_t *q = &ptr[st * W];
    for (uint32_t c = 0; c < k; c++) {
      const uint32_t id = p.slot_idx[c];
      q[c] = id < k ? reinterpret_cast<uint64_t>(d_data + st * data_stride + id * block)
                    : reinterpret_cast<uint64_t>(d_parity + st * parity_stride + (id - k) * block);
      if (fused && id < k)
        q[k + kSlotR + c] = reinterpret_cast<uint64_t>(d_out + st * out_stride + id * block);
    }
    for (size_t r = 0; r < p.missing.size(); r++)
      q[k + r] = reinterpret_cast<uint64_t>(d_out + st * out_stride + p.missing[r] * block);
  }
  return apply_desc(ctx, k, block, fused, pats, ptr, s);
}

}  // extern "C"
