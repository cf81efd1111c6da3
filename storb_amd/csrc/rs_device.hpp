// rs_device.hpp -- device-side templates of the GF(2^8) shard kernels.
//
// What the reference computes here: zfec's addmul loop (fec.c, ported by
// zfec-rs @3f3a3720 and called from crates/storb_base/src/piece.rs:329 for
// encode and :384-386 for decode): out_r[b] = XOR_j M[r][j] * in_j[b] over
// GF(2^8), byte-wise. Encode uses M = the parity rows of the systematic
// generator, decode uses the rows of the inverted survivor matrix that
// rebuild the missing data shares. Both are this one streaming kernel.
//
// Design (DESIGN.md "Kernels"):
//  * HBM-bound byte work, no MFMA. Every lane streams 16 B (dwordx4) of each
//    of the k input shares at the same column, so each wave-instruction
//    moves one contiguous, fully coalesced 1 KiB per share.
//  * Multiplication by a constant c is GF(2)-linear in the data byte x, so
//    c*x = T0[x & 7] ^ T1[(x >> 3) & 7] ^ T2[x >> 6]. T0/T1 are 8-entry and
//    T2 4-entry byte tables that fit one v_perm_b32 each: 3 v_perm_b32 +
//    ~1.5 v_xor per dword per coefficient, with the per-dword selectors
//    (two masks, two shifts) shared by every output row. The tables are
//    wave-uniform and live in SGPRs (s_load from the coefficient buffer),
//    so the kernel touches no LDS at all and has no bank conflicts.
//  * Variant LDS (rs_apply_lds) stages classic 256-byte product tables in
//    LDS and looks each byte up with ds_read_u8 -- the textbook GPU layout,
//    kept as the measured comparison point for the register-table variant.
//  * The grid is nstripes x tiles; a tile is 256 lanes x U dwordx4 columns.
//    Full tiles (the common case) run without per-lane bounds checks.
#pragma once

#include <hip/hip_runtime.h>

#include "rs_kernels.hpp"
#include "rs_stream.hpp"

namespace storb_rs {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

static constexpr int kThreads = 256;

// Launch shape per (k, r) bucket: T threads per block, U dwordx4 columns
// per lane, BAR = sched_barrier between coefficients (needed only where the
// compiler would otherwise hoist tables/selectors past the register file).
// Chosen by measurement (tools/kbench_tune.hip, DESIGN.md "Tuning").
// G = input shares per load group (double-buffered); TL = stage the
// k*RM nibble tables in LDS at block start and read them as broadcast
// ds_reads instead of s_loads.
// Resident workgroups per CU (rs_kernels.hpp wg_cap; 0 = uncapped), from
// the product-level sweep (a removed script) (profiles/r1_occupancy.txt):
// RS(4,2) encode / decode 6.40 -> 6.65 TB/s at 4, its one-row repair +5-7 %,
// RS(16,2) decode (config 5) +13 % at 2, RS(16,1) repair +9 % at 4; RS(8,4)
// encode, config 3's <8,3> decode and the 8-row k = 16 decode +1-4 % at 4
// (tools/kbench_tune.hip occ). RS(2,1) (Storb's own 256 KiB chunks) and the
// k = 1 copy measured best uncapped. For 256-lane workgroups caps 2 and 3
// measure the same, as do 4 and 5: the reservation resolves to even counts.
// (Round 5: the download-decode probe's finding that one-wave workgroups
// capped at 16 per CU stream RS(4,2)'s own access shape faster -- 0.852 vs
// 0.807 of peak with no GF work, tools/dlprobe.hip -- did not carry over to
// the product kernel: config 2 0.4830 -> 0.4882-0.4913 ms per step at caps 12
// / 16, config 4 within 0.3 %, profiles/r5m_ab_headline_t64.txt.)
constexpr int occ_for(int KM, int RM, bool copy) {
  if (copy) {  // fused assembly: config 3's into-a-fresh-buffer decode, pure copy
    if (KM == 8 && RM == 3) return 4;
    if (KM == 8 && RM == 1) return 2;
  }
  if (KM == 4 && RM <= 2) return 4;
  if (KM == 8 && (RM == 3 || RM == 4)) return 4;
  if (KM == 16 && RM == 1) return 4;
  if (KM == 16 && RM == 2) return 2;
  if (KM == 16 && RM == 8) return 4;
  return 0;
}

constexpr int g32(int RM) {
  return RM <= 2 ? 16 : (RM == 3 || RM == 5 || RM == 6 || RM == 7) ? 2 : RM == 16 ? 8 : 4;
}

template <int KM, int RM>
struct Tune {
  static constexpr int OCC = occ_for(KM, RM, false);
  static constexpr int OCC_COPY = occ_for(KM, RM, true);
  static constexpr int T = 256;
  static constexpr int U = 1;
  static constexpr bool BAR = false;
  // k = 32: shares per load group by row count (tools/k32_tune.hip, config 6
  // geometry, every variant bit-exact against the round-3 shape G = 8;
  // profiles/r3zb_k32_tune.txt for R = 1, 2, 4, profiles/r4a_k32_tune.txt for
  // the rest): R = 1 G16 78.7 % (G8 74.0), R = 2 G16 75.6 (63.9), R = 3 G2
  // 62.9 (55.0), R = 4 G4 59.6 (54.3), R = 5 G2 53.3 (46.5), R = 6 G2 48.6
  // (40.4), R = 8 G4 43.2 (36.0); R = 16 keeps G8 (27.8; G4 26.0).
  static constexpr int G = KM < 8 ? KM : KM == 32 ? g32(RM) : 8;
  static constexpr bool TL = KM >= 8;
  static constexpr bool PAIR = KM == 8 && RM <= 4;  // measured +2.5 % (W2)
};

template <int KM>
struct Unroll {  // LDS comparison kernel
  static constexpr int U = KM <= 4 ? 2 : 1;
};

// a ^ b ^ c in one v_bitop3_b32 (gfx950; truth table 0x96).
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

__device__ __forceinline__ uint32_t gf_mul_perm(const PermTab &t, uint32_t s0,
                                                uint32_t s1, uint32_t s2) {
  return xor3(__builtin_amdgcn_perm(t.t0hi, t.t0lo, s0),
              __builtin_amdgcn_perm(t.t1hi, t.t1lo, s1),
              __builtin_amdgcn_perm(0u, t.t2, s2));
}

// acc ^ c*x with the three lookups folded in two XOR instructions.
__device__ __forceinline__ uint32_t gf_madd_perm(uint32_t acc, const PermTab &t,
                                                 uint32_t s0, uint32_t s1, uint32_t s2) {
  acc = xor3(acc, __builtin_amdgcn_perm(t.t0hi, t.t0lo, s0),
             __builtin_amdgcn_perm(t.t1hi, t.t1lo, s1));
  return acc ^ __builtin_amdgcn_perm(0u, t.t2, s2);
}

// Shards are streamed exactly once: non-temporal loads and stores keep them
// from churning L2/MALL. Measured back to back (tools/kbench_tune.hip built
// with STORB_RS_NT_STORES=0/1, profiles/r1_store_policy.txt): nt stores
// 6.51 vs 6.19 TB/s on RS(4,2) encode, 6.60 vs 6.12 on RS(8,4) decode, 5.87
// vs 5.38 for the bit-sliced RS(16,8) encoder. (A single-launch timing
// favours default stores, tools/hbm_probe.hip, because dirty lines left in
// L2/MALL at kernel end are written back after the end event.)
// (P: a generic or a global-address-space pointer to u32x4.)
template <class P>
__device__ __forceinline__ u32x4 ld_stream(P p) {
  return __builtin_nontemporal_load(p);
}
template <class P>
__device__ __forceinline__ void st_stream(P p, u32x4 v) {
#if STORB_RS_NT_STORES
  __builtin_nontemporal_store(v, p);
#else
  *p = v;
#endif
}

// Where a tile's shares are: the pointers of input j, output row i and the
// assembly target of input j for the stripe a workgroup works on.
// ArgsView: one matrix and one stride per slot for every stripe of the
// launch (ApplyArgs); DescView: the stripe's own record (DescArgs), for
// launches whose stripes each lost different shares.
struct ArgsView {
  const ApplyArgs &a;
  uint32_t stripe;
  // (Pointers read from the kernel arguments: the compiler already knows
  // they are global, and emits global_load / global_store.)
  __device__ __forceinline__ const u32x4 *in(int j) const {
    return reinterpret_cast<const u32x4 *>(a.in[j] + static_cast<uint64_t>(stripe) * a.in_stride[j]);
  }
  __device__ __forceinline__ u32x4 *out(int i) const {
    return reinterpret_cast<u32x4 *>(a.out[i] + static_cast<uint64_t>(stripe) * a.out_stride[i]);
  }
  __device__ __forceinline__ bool has_copy(int j) const { return a.copy[j] != nullptr; }
  __device__ __forceinline__ u32x4 *copy(int j) const {
    return reinterpret_cast<u32x4 *>(a.copy[j] + static_cast<uint64_t>(stripe) * a.copy_stride[j]);
  }
  __device__ __forceinline__ bool accumulate() const { return a.accumulate != 0; }
};

// Global (address space 1) and constant (address space 4) pointers. The
// descriptor kernel reads its shares' addresses from memory, where the
// compiler cannot tell they are global: as generic pointers every share load
// and store became flat_load / flat_store, which count against lgkmcnt too,
// so each LDS table read waited for the in-flight share loads (no double
// buffering: 41 % of HBM peak against 77 % for the same tile on kernel
// arguments, tools/descbench.cpp). And the record, read through a generic
// pointer, came in as per-lane global_load_dwordx2 instead of s_load.
typedef u32x4 __attribute__((address_space(1))) gu32x4;
typedef const uint64_t __attribute__((address_space(4))) cu64;

struct DescView {
  cu64 *rec;        // this item's record (wave-uniform: scalar loads)
  uint32_t k, ro;   // ro = output slots per record
  __device__ __forceinline__ const gu32x4 *in(int j) const {
    return (const gu32x4 *)(rec[1 + j]);
  }
  __device__ __forceinline__ gu32x4 *out(int i) const {
    return (gu32x4 *)(rec[1 + k + i]);
  }
  __device__ __forceinline__ bool has_copy(int j) const { return rec[1 + k + ro + j] != 0; }
  __device__ __forceinline__ gu32x4 *copy(int j) const {
    return (gu32x4 *)(rec[1 + k + ro + j]);
  }
  __device__ __forceinline__ bool accumulate() const { return false; }
};

// A coefficient's table from LDS / a generic pointer, or field by field
// from a constant-address-space one (wave-uniform: s_load).
__device__ __forceinline__ PermTab get_tab(const PermTab *p) { return *p; }
template <class P>
__device__ __forceinline__ PermTab get_tab(P p) {
  PermTab t{};
  t.t0lo = p->t0lo;
  t.t0hi = p->t0hi;
  t.t1lo = p->t1lo;
  t.t1hi = p->t1hi;
  t.t2 = p->t2;
  return t;
}

// Inputs are consumed in groups of up to 8 shares; the next group's
// dwordx4 loads are issued before the current group is multiplied (double
// buffer), so a k = 32 tile needs 2 x 8 input registers per column instead
// of 32.
template <int KM, int G, int T, int U, bool GUARD, class V>
__device__ __forceinline__ void load_group(const V &v, uint32_t k, uint32_t cols, uint32_t c0,
                                           int g, u32x4 (&dst)[G][U]) {
#pragma unroll
  for (int jj = 0; jj < G; jj++) {
    const int j = g * G + jj;
    if (j >= static_cast<int>(k)) continue;
    const auto p = v.in(j);
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint32_t c = c0 + u * T;
      if (GUARD)
        dst[jj][u] = c < cols ? ld_stream(p + c) : u32x4{0, 0, 0, 0};
      else
        dst[jj][u] = ld_stream(p + c);
    }
  }
}

// Register budget: the compiler would otherwise hoist every coefficient's
// five table dwords and every input's selectors into VGPRs up front (254+
// VGPRs and scratch spills at k = 8, r = 4). Per input the selectors are
// computed once; per (row, input) the table is read from SGPRs right
// before its v_perm_b32s, and a sched_barrier stops the hoisting.
// Fused assembly (COPY): a decode into a separate chunk buffer stores each
// surviving data share straight from the registers it was loaded into, so
// the chunk is assembled in the same pass (k*B read + k*B written instead of
// a separate copy pass re-reading the k - e present shares).
template <int G, int T, int U, bool GUARD, class V>
__device__ __forceinline__ void copy_group(const V &v, uint32_t k, uint32_t cols, uint32_t c0,
                                           int g, const u32x4 (&src)[G][U]) {
#pragma unroll
  for (int jj = 0; jj < G; jj++) {
    const int j = g * G + jj;
    if (j >= static_cast<int>(k) || !v.has_copy(j)) continue;
    const auto q = v.copy(j);
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint32_t c = c0 + u * T;
      if (!GUARD || c < cols) st_stream(q + c, src[jj][u]);
    }
  }
}

// The folds of one tile: acc[i] = XOR_j M[i][j] * in_j over the tile's
// column(s), for the k <= KM inputs of view v (perm_tile stores them; the
// input-split descriptor tiles reduce several waves' acc first).
template <int KM, int RM, int T, int U, bool BAR, int G, bool PAIR, bool GUARD,
          bool COPY = false, class V, class TP>
__device__ __forceinline__ void perm_acc(const V &v, TP tabs, uint32_t k, uint32_t r,
                                         uint32_t cols, uint32_t c0, u32x4 (&acc)[RM][U]) {
  // the groups cover the bucket's KM input slots (inputs >= k skipped): a G
  // that does not divide KM would drop the last KM % G inputs (a G = 12 A/B
  // build at k = 32 failed the bench's round-trip check, round 5)
  static_assert(KM % G == 0, "load group size must divide the k bucket");
  constexpr int NG = KM / G;
  u32x4 buf[2][G][U];
#pragma unroll
  for (int i = 0; i < RM; i++)
#pragma unroll
    for (int u = 0; u < U; u++) acc[i][u] = u32x4{0, 0, 0, 0};

  load_group<KM, G, T, U, GUARD>(v, k, cols, c0, 0, buf[0]);
#pragma unroll
  for (int g = 0; g < NG; g++) {
    if (g + 1 < NG)
      load_group<KM, G, T, U, GUARD>(v, k, cols, c0, g + 1, buf[(g + 1) & 1]);
    if constexpr (COPY) {
      copy_group<G, T, U, GUARD>(v, k, cols, c0, g, buf[g & 1]);
      if (r == 0) continue;  // pure assembly: nothing missing
    }
    if constexpr (PAIR) {
      // Inputs two at a time: per (row, dword) the six v_perm_b32 lookups
      // of inputs j and j+1 fold into acc with three 3-input XORs (instead
      // of four XOR instructions); tables are read per row (LDS / SGPR)
      // just before use so their registers do not scale with RM.
#pragma unroll
      for (int jj = 0; jj < G; jj += 2) {
        const int j = g * G + jj;
        if (j >= static_cast<int>(k)) continue;
        const bool two = jj + 1 < G && j + 1 < static_cast<int>(k);
        uint32_t s0[2][U][4], s1[2][U][4], s2[2][U][4];
#pragma unroll
        for (int h = 0; h < 2; h++)
#pragma unroll
          for (int u = 0; u < U; u++)
#pragma unroll
            for (int w = 0; w < 4; w++) {
              const uint32_t d = (h == 0 || two) ? buf[g & 1][jj + h][u][w] : 0u;
              s0[h][u][w] = d & 0x07070707u;
              s1[h][u][w] = (d >> 3) & 0x07070707u;
              s2[h][u][w] = (d >> 6) & 0x03030303u;
            }
#pragma unroll
        for (int i = 0; i < RM; i++) {
          const PermTab ta = get_tab(tabs + (j * RM + i));
          const PermTab tb = two ? get_tab(tabs + ((j + 1) * RM + i)) : PermTab{};
#pragma unroll
          for (int u = 0; u < U; u++)
#pragma unroll
            for (int w = 0; w < 4; w++) {
              uint32_t x = acc[i][u][w];
              x = xor3(x, __builtin_amdgcn_perm(ta.t0hi, ta.t0lo, s0[0][u][w]),
                       __builtin_amdgcn_perm(ta.t1hi, ta.t1lo, s1[0][u][w]));
              x = xor3(x, __builtin_amdgcn_perm(0u, ta.t2, s2[0][u][w]),
                       __builtin_amdgcn_perm(tb.t0hi, tb.t0lo, s0[1][u][w]));
              x = xor3(x, __builtin_amdgcn_perm(tb.t1hi, tb.t1lo, s1[1][u][w]),
                       __builtin_amdgcn_perm(0u, tb.t2, s2[1][u][w]));
              acc[i][u][w] = x;
            }
          if constexpr (BAR) __builtin_amdgcn_sched_barrier(0);  // per-row tables
        }
      }
    } else {
#pragma unroll
      for (int jj = 0; jj < G; jj++) {
        const int j = g * G + jj;
        if (j >= static_cast<int>(k)) continue;
        uint32_t s0[U][4], s1[U][4], s2[U][4];
#pragma unroll
        for (int u = 0; u < U; u++)
#pragma unroll
          for (int w = 0; w < 4; w++) {
            const uint32_t d = buf[g & 1][jj][u][w];
            s0[u][w] = d & 0x07070707u;
            s1[u][w] = (d >> 3) & 0x07070707u;
            s2[u][w] = (d >> 6) & 0x03030303u;
          }
        // Tables are stored [input][RM rows], rows >= r zero-padded by the
        // host: no per-row guard, so input j is one basic block in which all
        // RM table loads issue together and overlap the v_perm work (per-row
        // guards made every coefficient wait out a full load latency).
        PermTab t[RM];
#pragma unroll
        for (int i = 0; i < RM; i++) t[i] = get_tab(tabs + (j * RM + i));
#pragma unroll
        for (int i = 0; i < RM; i++)
#pragma unroll
          for (int u = 0; u < U; u++)
#pragma unroll
            for (int w = 0; w < 4; w++)
              acc[i][u][w] = gf_madd_perm(acc[i][u][w], t[i], s0[u][w], s1[u][w], s2[u][w]);
        if constexpr (BAR) __builtin_amdgcn_sched_barrier(0);
      }
    }
  }
}

template <int KM, int RM, int T, int U, bool BAR, int G, bool PAIR, bool GUARD,
          bool COPY = false, class V, class TP>
__device__ __forceinline__ void perm_tile(const V &v, TP tabs, uint32_t k,
                                          uint32_t r, uint32_t cols, uint32_t c0) {
  u32x4 acc[RM][U];
  perm_acc<KM, RM, T, U, BAR, G, PAIR, GUARD, COPY>(v, tabs, k, r, cols, c0, acc);
#pragma unroll
  for (int i = 0; i < RM; i++) {
    if (i >= static_cast<int>(r)) continue;
    const auto q = v.out(i);
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint32_t c = c0 + u * T;
      if (!GUARD || c < cols) {
        u32x4 x = acc[i][u];
        if (v.accumulate()) x ^= q[c];
        st_stream(q + c, x);
      }
    }
  }
}

// k <= KM and r <= RM at run time. The j < k / i < r guards are uniform
// scalar branches; they also split the body into basic blocks, which keeps
// the scheduler from hoisting every table load and selector (a guard-free
// "exact" specialisation measured 181-256 VGPRs and scratch spills).
template <int KM, int RM, int T, int U, bool BAR, int G, bool TL, bool PAIR = false,
          bool COPY = false>
__global__ __launch_bounds__(T) void rs_apply_perm(const ApplyArgs a) {
  constexpr uint32_t TILE = T * U;
  const uint32_t cols = static_cast<uint32_t>(a.block >> 4);
  const uint32_t tps = (cols + TILE - 1) / TILE;
  const uint32_t stripe = blockIdx.x / tps;
  const uint32_t base = (blockIdx.x - stripe * tps) * TILE;
  const PermTab *tabs = a.ptab;
  if constexpr (TL) {
    __shared__ __attribute__((aligned(16))) PermTab lds_ptab[KM * RM];
    const uint32_t n16 = (COPY && a.r == 0) ? 0u : a.k * RM * (sizeof(PermTab) / 16);
    for (uint32_t t = threadIdx.x; t < n16; t += T)
      reinterpret_cast<u32x4 *>(lds_ptab)[t] = reinterpret_cast<const u32x4 *>(a.ptab)[t];
    __syncthreads();
    tabs = lds_ptab;
  }
  const ArgsView v{a, stripe};
  if (base + TILE <= cols)
    perm_tile<KM, RM, T, U, BAR, G, PAIR, false, COPY>(v, tabs, a.k, a.r, cols,
                                                      base + threadIdx.x);
  else
    perm_tile<KM, RM, T, U, BAR, G, PAIR, true, COPY>(v, tabs, a.k, a.r, cols,
                                                     base + threadIdx.x);
}

// The same tile for a launch of per-stripe descriptors (DescArgs). A
// workgroup reads its item's record -- the inputs, outputs and assembly
// targets of its own stripe, the offset of its own matrix's tables -- with
// scalar loads, stages the tables in LDS, then runs perm_tile exactly as
// rs_apply_perm does over `tpw` consecutive tiles of the stripe: the record
// -> tables -> first loads chain (~1-2 us of dependent latency a workgroup
// of one tile pays before its first byte streams) is paid once per tpw tiles.
// ONE (the mixed launch): exactly one tile per workgroup, the launcher
// refuses tpw != 1, and without COPY the row count is the branch's own
// compile-time RM -- no tile loop or run-time row guards in the code, which
// held the mixed kernel 1-2 % below the same tile without them
// (tools/mixbench.hip "same shape here").
template <int KM, int RM, int T, int U, bool BAR, int G, bool TL, bool PAIR, bool COPY,
          int RL = RM, bool ONE = false>
__device__ __forceinline__ void desc_body(const DescArgs &a, cu64 *rec, uint32_t r,
                                          PermTab *lds_ptab) {
  constexpr uint32_t TILE = T * U;
  const uint32_t cols = static_cast<uint32_t>(a.block >> 4);
  const uint32_t tps = (cols + TILE - 1) / TILE;
  if constexpr (ONE) {
    typedef const PermTab __attribute__((address_space(4))) cPermTab;
    cPermTab *gt = (cPermTab *)(a.ptab) + (rec[0] & 0xFFFFFFFFu);
    // (Round 5 A/B, not kept: reading the k input pointers in one scalar
    // load with k a compile-time constant issued the share loads back to back
    // but measured equal at k = 4 and 32 % slower at k = 16, which then held
    // 16 pointers in SGPRs; tools/gpu/ab_multi.sh, profiles/r5h_ab_download.txt.)
    const uint32_t kk = a.k;
    const DescView v{rec, kk, a.r};
    const uint32_t base = (blockIdx.x % tps) * TILE;
    const uint32_t rr = COPY ? r : static_cast<uint32_t>(RM);
    auto go = [&](auto tabs) __attribute__((always_inline)) {
      if (base + TILE <= cols)
        perm_tile<KM, RM, T, U, BAR, G, PAIR, false, COPY>(v, tabs, kk, rr, cols,
                                                          base + threadIdx.x);
      else
        perm_tile<KM, RM, T, U, BAR, G, PAIR, true, COPY>(v, tabs, kk, rr, cols,
                                                         base + threadIdx.x);
    };
    if constexpr (TL) {
      const uint32_t n16 = (COPY && r == 0) ? 0u : kk * RM * (sizeof(PermTab) / 16);
      typedef const u32x4 __attribute__((address_space(1))) gcu32x4;
      for (uint32_t t = threadIdx.x; t < n16; t += T)
        reinterpret_cast<u32x4 *>(lds_ptab)[t] = ((gcu32x4 *)(gt))[t];
      __syncthreads();
      go(static_cast<const PermTab *>(lds_ptab));
    } else {
      go(gt);
    }
    return;
  }
  const uint32_t wps = (tps + a.tpw - 1) / a.tpw;  // workgroups per stripe
  const uint32_t item = blockIdx.x / wps;
  const uint32_t t0 = (blockIdx.x - item * wps) * a.tpw;
  const uint32_t t1 = t0 + a.tpw < tps ? t0 + a.tpw : tps;
  typedef const PermTab __attribute__((address_space(4))) cPermTab;
  cPermTab *gtabs = (cPermTab *)(a.ptab) + (rec[0] & 0xFFFFFFFFu);
  const DescView v{rec, a.k, a.r};
  auto run = [&](auto tabs0) __attribute__((always_inline)) {
    if constexpr (RM > 8) {
      // 9-16 rebuilt rows: one guarded tile shape for every case. With the
      // four shapes below (one tile / loop, guarded / not) the body was too
      // large to inline at k = 32, and the out-of-line copy the compiler
      // made instead (every uniform value in VGPRs, flat loads of the
      // captures) never finished on a 16-byte share (tools/fuzz.py seed
      // 4242; tests/test_gpu_patterns.py::test_decode_chunks_tiny_shares_many_lost).
      for (uint32_t t = t0; t < t1; t++) {
        uint32_t zero = 0;
        asm volatile("" : "+s"(zero));
        perm_tile<KM, RM, T, U, BAR, G, PAIR, true, COPY>(v, tabs0 + zero, a.k, r, cols,
                                                         t * TILE + threadIdx.x);
      }
      return;
    }
    if (a.tpw == 1) {  // one tile (desc_tpw's choice unless the grid is huge): no loop
      const uint32_t base = t0 * TILE;
      if (base + TILE <= cols)
        perm_tile<KM, RM, T, U, BAR, G, PAIR, false, COPY>(v, tabs0, a.k, r, cols,
                                                          base + threadIdx.x);
      else
        perm_tile<KM, RM, T, U, BAR, G, PAIR, true, COPY>(v, tabs0, a.k, r, cols,
                                                         base + threadIdx.x);
      return;
    }
    for (uint32_t t = t0; t < t1; t++) {
      // The tables are the same for every tile: without this opaque zero,
      // loop-invariant code motion hoists all k x RM of them out of the tile
      // loop into VGPRs (256 VGPRs and scratch from 3 rows at k = 16).
      uint32_t zero = 0;
      asm volatile("" : "+s"(zero));
      const auto tabs = tabs0 + zero;
      const uint32_t base = t * TILE;
      if (base + TILE <= cols)
        perm_tile<KM, RM, T, U, BAR, G, PAIR, false, COPY>(v, tabs, a.k, r, cols,
                                                          base + threadIdx.x);
      else
        perm_tile<KM, RM, T, U, BAR, G, PAIR, true, COPY>(v, tabs, a.k, r, cols,
                                                         base + threadIdx.x);
    }
  };
  if constexpr (TL) {
    const uint32_t n16 = (COPY && r == 0) ? 0u : a.k * RM * (sizeof(PermTab) / 16);
    typedef const u32x4 __attribute__((address_space(1))) gcu32x4;
    for (uint32_t t = threadIdx.x; t < n16; t += T)
      reinterpret_cast<u32x4 *>(lds_ptab)[t] = ((gcu32x4 *)(gtabs))[t];
    __syncthreads();
    run(static_cast<const PermTab *>(lds_ptab));
  } else {
    run(gtabs);  // wave-uniform table reads: s_load
  }
}

template <int KM, int RM, int T, int U, bool BAR, int G, bool TL, bool PAIR = false,
          bool COPY = false>
__global__ __launch_bounds__(T) void rs_apply_desc(const DescArgs a) {
  __shared__ __attribute__((aligned(16))) PermTab lds_ptab[TL ? KM * RM : 1];
  const uint32_t tps = (static_cast<uint32_t>(a.block >> 4) + T * U - 1) / (T * U);
  const uint32_t item = blockIdx.x / ((tps + a.tpw - 1) / a.tpw);
  cu64 *rec = (cu64 *)(a.desc) + static_cast<uint64_t>(item) * a.rec_qwords;
  desc_body<KM, RM, T, U, BAR, G, TL, PAIR, COPY>(a, rec, a.r, lds_ptab);
}

// Shares per load group of the mixed launch's branch with R rows: the table
// kernel's, except at k = 32, where 16 for every branch measured best in the
// mixed launch (tools/mixbench.hip on config 6's download shape,
// profiles/r4b_mixbench32.txt: 74.3 % against 72.8 with the per-R uniform
// choice and 70.3 with G = 4).
template <int KM, int R>
constexpr int mix_g() { return KM == 32 ? 16 : Tune<KM, R>::G; }
// Inputs two at a time (PAIR: 4.5 instead of 5 VALU per row and dword) in the
// mixed launch at k = 16 too: 73.1 -> 75.7 % on config 5's download shape,
// interleaved on one box (profiles/r4c_mixbench16.txt); at k = 32 it lost
// (75.1 -> 73.1 %). (The uniform k = 16 kernels keep PAIR off: it raised
// their VGPRs past an occupancy step; the mixed kernel's registers are its
// largest branch's anyway.)
template <int KM, int R>
constexpr bool mix_pair() { return KM == 16 || Tune<KM, R>::PAIR; }

// Mixed row counts in one launch (DescArgs::mix): each workgroup reads its
// item's count and runs that count's tile (the Tune of that bucket), so a
// download's chunks -- most lost 1-3 data shares, each a different set --
// are one launch: no per-count launch gaps and tails, and no 3-row VALU
// spent on a 1-row item. Registers: the largest branch's.
// Workgroup size of the mixed launch. k <= 4 (the default line's download
// leg): one-wave workgroups, capped at 16 per CU -- the access shape's own
// ceiling without GF work (tools/dlprobe.hip, profiles/r5e_dlprobe.txt) is
// 0.799 of 8 TB/s that way against 0.784 for 256-lane workgroups at their
// best cap (4) and 0.806 for a uniform launch over contiguous stripes.
template <int KM>
// k = 16 (config 5's download mix): one-wave workgroups as well, left to
// their register limit (152 VGPRs: 12 per CU); decode leg 0.1852 -> 0.1829 ms
// against 256 lanes, where 64 lanes capped at 8 and 128 lanes capped at 4
// lost 6-8 % (profiles/r5q_ab_k16_mixed_shape.txt, three interleaved rounds).
// k = 32 keeps 256 lanes capped at 3: one-wave workgroups uncapped or
// capped at 12 lost 2-3 % on config 6's download leg (0.1736 -> 0.1776-0.1784
// ms, profiles/r5s_ab_k32_mixed_shape.txt).
constexpr int mix_threads() { return KM <= 4 || KM == 16 ? 64 : kThreads; }
// Tables staged in LDS (Tune::TL) in the mixed launch, one-wave workgroups
// included: read with s_load straight from the constant pool instead, the
// k = 16 decode leg went 0.1826 -> 0.1878 ms (profiles/r5r_ab_k16_sload_tables.txt).
template <int KM>
constexpr bool mix_tl() { return Tune<KM, 1>::TL; }

template <int KM, bool COPY>
__global__ __launch_bounds__(mix_threads<KM>()) void rs_apply_desc_mix(const DescArgs a) {
  constexpr int MT = mix_threads<KM>();
  __shared__ __attribute__((aligned(16))) PermTab lds_ptab[mix_tl<KM>() ? KM * kMixR : 1];
  const uint32_t tps = (static_cast<uint32_t>(a.block >> 4) + MT - 1) / MT;
  const uint32_t item = blockIdx.x / tps;  // one tile per workgroup (launch_desc_mix)
  cu64 *rec = (cu64 *)(a.desc) + static_cast<uint64_t>(item) * a.rec_qwords;
  const uint32_t r = static_cast<uint32_t>(rec[0] >> 32);
#define STORB_MIX_CASE(R)                                                                   \
  {                                                                                         \
    using C = Tune<KM, R>;                                                                  \
    static_assert(C::U == 1, "mixed launch: one column per lane");                          \
    desc_body<KM, R, MT, C::U, C::BAR, mix_g<KM, R>(), mix_tl<KM>(), mix_pair<KM, R>(), COPY, R, \
              true>(a, rec, r, lds_ptab);                                                   \
    return;                                                                                 \
  }
  if (r <= 1) STORB_MIX_CASE(1)
  if (r == 2) STORB_MIX_CASE(2)
  if (r == 3) STORB_MIX_CASE(3)
  STORB_MIX_CASE(4)
#undef STORB_MIX_CASE
}

// ------------------------------------------- input-split descriptor tiles
// Inputs j0 .. of a view (one wave's part of an input-split tile).
template <class V>
struct OffsetView {
  const V &v;
  uint32_t j0;
  __device__ __forceinline__ auto in(int j) const { return v.in(static_cast<int>(j0) + j); }
  __device__ __forceinline__ auto out(int i) const { return v.out(i); }
  __device__ __forceinline__ bool has_copy(int j) const { return v.has_copy(static_cast<int>(j0) + j); }
  __device__ __forceinline__ auto copy(int j) const { return v.copy(static_cast<int>(j0) + j); }
  __device__ __forceinline__ bool accumulate() const { return v.accumulate(); }
};

// The mixed-row descriptor launch with W waves per 64-column tile
// (rs_apply_desc_mix_ks): the waves of a workgroup cover the SAME 1 KiB of
// every share and split the k inputs (KM / W each); their partial rows meet
// in LDS and wave w stores rows w, w + W, ... So a tile keeps the one-wave
// tile's footprint (1 KiB of each share) with W waves to hide the v_perm
// folds' latency: the access shape that streams best for k = 16 -- one-wave
// tiles capped at 8 per CU, 0.794 of 8 TB/s with no GF work
// (tools/dlprobe.hip, profiles/r5e_dlprobe.txt) -- needed more waves than
// that cap leaves for the GF work (the uncapped product held 0.769).
template <int KM, int W>
struct MixKs {
  static constexpr int T = 64 * W, KW = KM / W;
  static_assert(KM % W == 0, "W must divide the k bucket");
};

// One wave's part of an input-split tile: its KW inputs' loads are issued
// FIRST, then the workgroup stages the item's tables in LDS (their global
// loads overlap the share loads' latency instead of preceding it: the
// record -> tables -> barrier -> share loads chain is what a short-lived
// workgroup otherwise waits through twice), then the folds (inputs two at a
// time, as perm_acc's PAIR), then the partial rows meet in LDS.
template <int KM, int W, int R, bool GUARD>
__device__ __forceinline__ void mix_ks_tile(const DescArgs &a, cu64 *rec, PermTab *lds_ptab,
                                            uint32_t cols, uint32_t c0, u32x4 *red) {
  using S = MixKs<KM, W>;
  constexpr int KW = S::KW;
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t j0 = w * KW;
  const uint32_t kw = a.k > j0 ? (a.k - j0 < KW ? a.k - j0 : KW) : 0u;
  const DescView v{rec, a.k, a.r};
  u32x4 buf[KW];
#pragma unroll
  for (int jj = 0; jj < KW; jj++) {
    if (jj >= static_cast<int>(kw)) {
      buf[jj] = u32x4{0, 0, 0, 0};
      continue;
    }
    const auto p = v.in(static_cast<int>(j0) + jj);
    buf[jj] = (!GUARD || c0 < cols) ? ld_stream(p + c0) : u32x4{0, 0, 0, 0};
  }
  {
    typedef const PermTab __attribute__((address_space(4))) cPermTab;
    typedef const u32x4 __attribute__((address_space(1))) gcu32x4;
    cPermTab *gt = (cPermTab *)(a.ptab) + (rec[0] & 0xFFFFFFFFu);
    const uint32_t n16 = a.k * R * (sizeof(PermTab) / 16);
    for (uint32_t t = threadIdx.x; t < n16; t += S::T)
      reinterpret_cast<u32x4 *>(lds_ptab)[t] = ((gcu32x4 *)(gt))[t];
    // LDS writes done, then the workgroup barrier; no vmcnt wait for the
    // share loads beyond what the table writes needed (__syncthreads' fences
    // would wait for every outstanding load)
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  }
  const PermTab *tabs = lds_ptab + j0 * R;
  u32x4 acc[R];
#pragma unroll
  for (int i = 0; i < R; i++) acc[i] = u32x4{0, 0, 0, 0};
#pragma unroll
  for (int jj = 0; jj < KW; jj += 2) {
    if (jj >= static_cast<int>(kw)) continue;
    const bool two = jj + 1 < static_cast<int>(kw);
    uint32_t s0[2][4], s1[2][4], s2[2][4];
#pragma unroll
    for (int h = 0; h < 2; h++)
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const uint32_t d = (h == 0 || two) ? buf[jj + h][q] : 0u;
        s0[h][q] = d & 0x07070707u;
        s1[h][q] = (d >> 3) & 0x07070707u;
        s2[h][q] = (d >> 6) & 0x03030303u;
      }
#pragma unroll
    for (int i = 0; i < R; i++) {
      const PermTab ta = tabs[jj * R + i];
      const PermTab tb = two ? tabs[(jj + 1) * R + i] : PermTab{};
#pragma unroll
      for (int q = 0; q < 4; q++) {
        uint32_t x = acc[i][q];
        x = xor3(x, __builtin_amdgcn_perm(ta.t0hi, ta.t0lo, s0[0][q]),
                 __builtin_amdgcn_perm(ta.t1hi, ta.t1lo, s1[0][q]));
        x = xor3(x, __builtin_amdgcn_perm(0u, ta.t2, s2[0][q]),
                 __builtin_amdgcn_perm(tb.t0hi, tb.t0lo, s0[1][q]));
        x = xor3(x, __builtin_amdgcn_perm(tb.t1hi, tb.t1lo, s1[1][q]),
                 __builtin_amdgcn_perm(0u, tb.t2, s2[1][q]));
        acc[i][q] = x;
      }
    }
  }
#pragma unroll
  for (int i = 0; i < R; i++) red[(w * R + i) * 64 + lane] = acc[i];
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
#pragma unroll
  for (int i = 0; i < R; i++) {
    if (i % W != static_cast<int>(w)) continue;  // wave-uniform
    u32x4 x = acc[i];
#pragma unroll
    for (int q = 0; q < W; q++)
      if (q != static_cast<int>(w)) x ^= red[(q * R + i) * 64 + lane];
    if (!GUARD || c0 < cols) st_stream(v.out(i) + c0, x);
  }
}

template <int KM, int W>
__global__ __launch_bounds__((MixKs<KM, W>::T)) void rs_apply_desc_mix_ks(const DescArgs a) {
  __shared__ __attribute__((aligned(16))) PermTab lds_ptab[KM * kMixR];
  __shared__ u32x4 red[W * kMixR * 64];
  const uint32_t cols = static_cast<uint32_t>(a.block >> 4);
  const uint32_t tps = (cols + 63) / 64;
  const uint32_t item = blockIdx.x / tps;
  const uint32_t base = (blockIdx.x - item * tps) * 64;
  cu64 *rec = (cu64 *)(a.desc) + static_cast<uint64_t>(item) * a.rec_qwords;
  const uint32_t r = static_cast<uint32_t>(rec[0] >> 32);
  const uint32_t c0 = base + (threadIdx.x & 63);
  const bool full = base + 64 <= cols;
#define STORB_MIXKS_CASE(R)                                                          \
  {                                                                                  \
    if (full)                                                                        \
      mix_ks_tile<KM, W, R, false>(a, rec, lds_ptab, cols, c0, red);                 \
    else                                                                             \
      mix_ks_tile<KM, W, R, true>(a, rec, lds_ptab, cols, c0, red);                  \
    return;                                                                          \
  }
  if (r <= 1) STORB_MIXKS_CASE(1)
  if (r == 2) STORB_MIXKS_CASE(2)
  if (r == 3) STORB_MIXKS_CASE(3)
  STORB_MIXKS_CASE(4)
#undef STORB_MIXKS_CASE
}

template <int KM, int W>
hipError_t launch_desc_mix_ks(const DescArgs &a, hipStream_t s, int cap) {
  const uint64_t tps = ((a.block >> 4) + 63) / 64;
  if (a.tpw != 1 || a.copy) return hipErrorInvalidConfiguration;
  const uint64_t blocks = tps * a.nitems;
  if (blocks == 0) return hipSuccess;
  if (blocks > 0x7FFFFFFFull) return hipErrorInvalidConfiguration;
  constexpr size_t stat = sizeof(PermTab) * KM * kMixR + sizeof(u32x4) * W * kMixR * 64;
  return launch_lds<rs_apply_desc_mix_ks<KM, W>>(blocks, MixKs<KM, W>::T, cap_lds(cap, stat), s,
                                                 a);
}

// The streamed single call's kernel (StreamArgs, rs_args.h): the table
// kernel's tile over one stripe, gated per slice on a host-written word and
// reporting per slice through a device counter and a host-visible word. The
// waits are bounded, so the grid always drains.
template <int KM, int RM, int T, int U, bool BAR, int G, bool TL, bool PAIR>
__global__ __launch_bounds__(T) void rs_apply_stream(const ApplyArgs a, const StreamArgs st) {
  constexpr uint32_t TILE = T * U;
  const uint32_t cols = static_cast<uint32_t>(a.block >> 4);
  const uint32_t base = blockIdx.x * TILE;
  const uint32_t slice = base / st.slice_cols;
  if (!stream_gate(st, slice)) return;
  const PermTab *tabs = a.ptab;
  if constexpr (TL) {
    __shared__ __attribute__((aligned(16))) PermTab lds_ptab[KM * RM];
    const uint32_t n16 = a.k * RM * (sizeof(PermTab) / 16);
    for (uint32_t t = threadIdx.x; t < n16; t += T)
      reinterpret_cast<u32x4 *>(lds_ptab)[t] = reinterpret_cast<const u32x4 *>(a.ptab)[t];
    __syncthreads();
    tabs = lds_ptab;
  }
  const ArgsView v{a, 0};
  if (base + TILE <= cols)
    perm_tile<KM, RM, T, U, BAR, G, PAIR, false>(v, tabs, a.k, a.r, cols, base + threadIdx.x);
  else
    perm_tile<KM, RM, T, U, BAR, G, PAIR, true>(v, tabs, a.k, a.r, cols, base + threadIdx.x);
  stream_report(st, slice);
}

template <int KM, int RM>
hipError_t launch_stream_t(const ApplyArgs &a, const StreamArgs &st, hipStream_t s) {
  using C = Tune<KM, RM>;
  static_assert(C::T == kThreads && C::U == 1, "streamed calls: one tile shape");
  const uint64_t blocks = ((a.block >> 4) + kThreads - 1) / kThreads;
  if (blocks == 0) return hipSuccess;
  hipLaunchKernelGGL((rs_apply_stream<KM, RM, C::T, C::U, C::BAR, C::G, C::TL, C::PAIR>),
                     dim3(blocks), dim3(kThreads), 0, s, a, st);
  return hipGetLastError();
}

template <int KM>
hipError_t go_stream_r(const ApplyArgs &a, const StreamArgs &st, hipStream_t s) {
  switch (rows_bucket(a.r)) {
    case 1: return launch_stream_t<KM, 1>(a, st, s);
    case 2: return launch_stream_t<KM, 2>(a, st, s);
    case 3: return launch_stream_t<KM, 3>(a, st, s);
    case 4: return launch_stream_t<KM, 4>(a, st, s);
    case 5: return launch_stream_t<KM, 5>(a, st, s);
    case 6: return launch_stream_t<KM, 6>(a, st, s);
    case 7: return launch_stream_t<KM, 7>(a, st, s);
    case 8: return launch_stream_t<KM, 8>(a, st, s);
    default: return hipErrorInvalidValue;
  }
}

template <int KM, int RM, int T, int U, bool BAR, int G, bool TL, bool PAIR = false>
hipError_t launch_perm(const ApplyArgs &a, hipStream_t s, int occ = 0, int occ_copy = 0) {
  const uint64_t cols = a.block >> 4;
  const uint64_t blocks = ((cols + T * U - 1) / (T * U)) * a.nstripes;
  if (blocks == 0) return hipSuccess;
  if (blocks > 0x7FFFFFFFull) return hipErrorInvalidConfiguration;
  const size_t dyn = cap_lds(wg_cap(a.ncopy ? occ_copy : occ),
                             TL ? sizeof(PermTab) * KM * RM : 0);
  if (a.ncopy) {
    if constexpr (KM <= static_cast<int>(kCopyMaxK))
      return launch_lds<rs_apply_perm<KM, RM, T, U, BAR, G, TL, PAIR, true>>(blocks, T, dyn, s,
                                                                             a);
    else
      return hipErrorInvalidValue;
  }
  return launch_lds<rs_apply_perm<KM, RM, T, U, BAR, G, TL, PAIR>>(blocks, T, dyn, s, a);
}

template <int KM, int RM, int T, int U, bool BAR, int G, bool TL, bool PAIR = false>
hipError_t launch_desc(const DescArgs &a, hipStream_t s, int occ = 0, int occ_copy = 0) {
  const uint64_t cols = a.block >> 4;
  const uint64_t tps = (cols + T * U - 1) / (T * U);
  if (a.tpw == 0) return hipErrorInvalidValue;
  const uint64_t blocks = ((tps + a.tpw - 1) / a.tpw) * a.nitems;
  if (blocks == 0) return hipSuccess;
  if (blocks > 0x7FFFFFFFull) return hipErrorInvalidConfiguration;
  const size_t dyn = cap_lds(a.cap ? static_cast<int>(a.cap) : wg_cap(a.copy ? occ_copy : occ),
                             TL ? sizeof(PermTab) * KM * RM : 0);
  if (a.copy) {
    if constexpr (KM <= static_cast<int>(kCopyMaxK))
      return launch_lds<rs_apply_desc<KM, RM, T, U, BAR, G, TL, PAIR, true>>(blocks, T, dyn, s,
                                                                             a);
    else
      return hipErrorInvalidValue;
  }
  return launch_lds<rs_apply_desc<KM, RM, T, U, BAR, G, TL, PAIR>>(blocks, T, dyn, s, a);
}

// Default resident-workgroup cap of a mixed-row launch (DescArgs::cap = 0).
// k = 16 download mix (tools/descbench.cpp, profiles/r3j_descbench.txt):
// capped at 2 or 3 per CU 61.5 %, at 4 72.1 %, uncapped 72.4 % of 8 TB/s.
// k <= 4 keeps the RS(4,2) table kernel's measured cap of 4.
// k = 32 (16 shares per group): 3 per CU, +0.5-0.7 % over uncapped in three
// interleaved runs (profiles/r4{b,c,d}_mixbench32.txt "G16 cap3").
// k <= 4 with one-wave workgroups (mix_threads): 16 per CU -- unlike the
// uniform <4,2> launch (PermShape, 14 per CU), lower caps lose here: config 2
// download step 0.377 ms at 16 against 0.379 / 0.386 / 0.392 at 14 / 13 / 12
// (tools/gpu/r6s_abmix.sh, profiles/r6s_abmix.jsonl).
#ifndef STORB_MIX4_OCC  // experiment builds only
#define STORB_MIX4_OCC 16
#endif
constexpr int mix_occ(int KM) { return KM <= 4 ? STORB_MIX4_OCC : KM == 32 ? 3 : 0; }

// k = 16 (config 5's download mix) runs the input-split tiles, two waves per
// 1 KiB tile (rs_apply_desc_mix_ks<16, 2>), uncapped: tools/mixbench.hip on
// config 5's download shape, records heaviest first as apply_desc orders
// them, 76.0-76.9 -> 77.4-77.9 % of 8 TB/s (profiles/r6i_mixbench16.txt,
// r6j_*, r6l_*); four waves per tile 70-77 %. k = 32 (config 6's): four waves
// per tile (8 inputs each), 4 per CU, 72.8 -> 74.1 % against the one-tile
// 256-lane kernel with the same heaviest-first records on one box
// (profiles/r6t_mixbench32.txt; two waves 72.9-73.2, eight 57-63). Fused
// assembly (copy) keeps rs_apply_desc_mix.
template <int KM>
constexpr int mix_ks_waves() { return KM == 16 ? 2 : KM == 32 ? 4 : 0; }
template <int KM>
constexpr int mix_ks_cap() { return KM == 32 ? 4 : 0; }

template <int KM>
hipError_t launch_desc_mix(const DescArgs &a, hipStream_t s) {
  if constexpr (mix_ks_waves<KM>() > 0)
    if (!a.copy && a.tpw == 1)
      return launch_desc_mix_ks<KM, mix_ks_waves<KM>()>(
          a, s, a.cap ? static_cast<int>(a.cap) : mix_ks_cap<KM>());
  constexpr uint64_t TILE = mix_threads<KM>();
  const uint64_t tps = ((a.block >> 4) + TILE - 1) / TILE;
  if (a.tpw != 1) return hipErrorInvalidConfiguration;  // one tile per workgroup
  const uint64_t blocks = ((tps + a.tpw - 1) / a.tpw) * a.nitems;
  if (blocks == 0) return hipSuccess;
  if (blocks > 0x7FFFFFFFull) return hipErrorInvalidConfiguration;
  const size_t dyn = cap_lds(a.cap ? static_cast<int>(a.cap) : mix_occ(KM),
                             mix_tl<KM>() ? sizeof(PermTab) * KM * kMixR : 0);
  const int T = static_cast<int>(TILE);
  if (a.copy) {
    if constexpr (KM <= static_cast<int>(kCopyMaxK))
      return launch_lds<rs_apply_desc_mix<KM, true>>(blocks, T, dyn, s, a);
    else
      return hipErrorInvalidValue;
  }
  return launch_lds<rs_apply_desc_mix<KM, false>>(blocks, T, dyn, s, a);
}

template <int KM>
hipError_t go_desc_r(const DescArgs &a, hipStream_t s) {
  if (a.mix) return launch_desc_mix<KM>(a, s);
  switch (rows_bucket(a.r)) {
#define STORB_DESC_CASE(R)                                                                 \
  case R: {                                                                                \
    using C = Tune<KM, R>;                                                                 \
    return launch_desc<KM, R, C::T, C::U, C::BAR, C::G, C::TL, C::PAIR>(a, s, C::OCC,      \
                                                                        C::OCC_COPY);      \
  }
    case 0:  // pure assembly (COPY, nothing missing): one zero row of tables
      STORB_DESC_CASE(1)
      STORB_DESC_CASE(2)
      STORB_DESC_CASE(3)
      STORB_DESC_CASE(4)
      STORB_DESC_CASE(5)
      STORB_DESC_CASE(6)
      STORB_DESC_CASE(7)
      STORB_DESC_CASE(8)
#undef STORB_DESC_CASE
    default: {
      using C = Tune<KM, 16>;
      return launch_desc<KM, 16, C::T, C::U, C::BAR, C::G, C::TL, C::PAIR>(a, s, C::OCC,
                                                                           C::OCC_COPY);
    }
  }
}

template <int KM, int RM>
__global__ __launch_bounds__(kThreads) void rs_apply_lds(const ApplyArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds_tab[];
  constexpr int U = Unroll<KM>::U;
  constexpr uint32_t TILE = kThreads * U;
  const uint32_t k = a.k, r = a.r;
  const uint32_t cols = static_cast<uint32_t>(a.block >> 4);
  const uint32_t tps = (cols + TILE - 1) / TILE;
  const uint32_t stripe = blockIdx.x / tps;
  const uint32_t c0 = (blockIdx.x - stripe * tps) * TILE + threadIdx.x;

  // Stage the r*k product tables (256 B each) into LDS, 16 B per lane.
  const uint32_t tab16 = a.tab_rows * k * 16;
  for (uint32_t t = threadIdx.x; t < tab16; t += kThreads)
    reinterpret_cast<u32x4 *>(lds_tab)[t] =
        reinterpret_cast<const u32x4 *>(a.btab)[t];

  u32x4 x[KM][U];
#pragma unroll
  for (int j = 0; j < KM; j++) {
    if (j < static_cast<int>(k)) {
      const u32x4 *p = reinterpret_cast<const u32x4 *>(
          a.in[j] + static_cast<uint64_t>(stripe) * a.in_stride[j]);
#pragma unroll
      for (int u = 0; u < U; u++) {
        const uint32_t c = c0 + u * kThreads;
        x[j][u] = c < cols ? ld_stream(p + c) : u32x4{0, 0, 0, 0};
      }
    }
  }
  __syncthreads();

  u32x4 acc[RM][U];
#pragma unroll
  for (int i = 0; i < RM; i++)
#pragma unroll
    for (int u = 0; u < U; u++) acc[i][u] = u32x4{0, 0, 0, 0};

#pragma unroll
  for (int j = 0; j < KM; j++) {
    if (j >= static_cast<int>(k)) continue;
#pragma unroll
    for (int u = 0; u < U; u++) {
#pragma unroll
      for (int w = 0; w < 4; w++) {
        const uint32_t d = x[j][u][w];
#pragma unroll
        for (int i = 0; i < RM; i++) {
          if (i >= static_cast<int>(r)) continue;
          const uint8_t *row = lds_tab + (j * a.tab_rows + i) * 256u;
          acc[i][u][w] ^= static_cast<uint32_t>(row[d & 0xFF]) |
                          static_cast<uint32_t>(row[(d >> 8) & 0xFF]) << 8 |
                          static_cast<uint32_t>(row[(d >> 16) & 0xFF]) << 16 |
                          static_cast<uint32_t>(row[d >> 24]) << 24;
        }
      }
    }
  }

#pragma unroll
  for (int i = 0; i < RM; i++) {
    if (i >= static_cast<int>(r)) continue;
    u32x4 *q = reinterpret_cast<u32x4 *>(
        a.out[i] + static_cast<uint64_t>(stripe) * a.out_stride[i]);
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint32_t c = c0 + u * kThreads;
      if (c < cols) {
        u32x4 v = acc[i][u];
        if (a.accumulate) v ^= q[c];
        st_stream(q + c, v);
      }
    }
  }
}

template <int KM>
inline uint64_t tile_blocks(const ApplyArgs &a) {
  constexpr uint32_t TILE = kThreads * Unroll<KM>::U;
  const uint64_t cols = a.block >> 4;
  return ((cols + TILE - 1) / TILE) * a.nstripes;
}

// Launch shape of a uniform table-kernel launch without fused assembly, where
// it differs from Tune (whose T / G the streamed and descriptor launches
// share). <8,3> (config 3's decode of 3 lost shares; k = 5..8 encodes with
// 3 parity rows): one-wave workgroups, load groups of 4, 16 resident per CU
// -- 82.4 -> 83.3 % of 8 TB/s at config 3's in-place layout
// (tools/kbench_tune.hip occ, profiles/r6s_occ_c3.txt; 64-lane caps 14-20
// within 0.5 points, 10-12 fall to 69-78 %). The shape's no-GF ceiling:
// 0.814 for 256-lane workgroups at 4 per CU against 0.851 for one-wave
// workgroups at 12 (tools/dlprobe.hip c3, profiles/r6s_dlprobe_c3.txt).
template <int KM, int RM>
struct PermShape {
  static constexpr int T = Tune<KM, RM>::T, G = Tune<KM, RM>::G, OCC = Tune<KM, RM>::OCC;
};
template <>
struct PermShape<8, 3> {
  static constexpr int T = 64, G = 4, OCC = 16;
};
// Not taken: <4,1> (single-row rebuilds at k = 3-4) streams faster one-wave
// in tools/kbench_tune.hip's compact layout (at 14 per CU 81.8 -> 86.6 %,
// profiles/r6s_occ_41.txt), but on the product's in-place repair of a data
// share it lost 10 % (0.2014 -> 0.2215 ms; a parity share +1 %;
// tools/gpu/r6s_ab41.sh, profiles/r6s_ab41.jsonl), so it keeps Tune's shape.
// <2,1> (Storb's (2, 3) geometry, 256 KiB chunks): one-wave workgroups,
// uncapped -- on the device batch calls (tools/ab21.py, tools/gpu/r6s_ab21.sh,
// profiles/r6s_ab21.jsonl, builds interleaved) encode 245.6 -> 240.9 us and
// the in-place decode of a data share 246.8 -> 240.5 us per 4096 chunks
// (0.82 -> 0.84 of 8 TB/s); kbench W7: 28-32 per CU the same, 24 and below
// lose (profiles/r6s_occ_21*.txt).
template <>
struct PermShape<2, 1> {
  static constexpr int T = 64, G = 2, OCC = 0;
};
// <8,1> / <8,2> (Storb's (8, 12) geometry, 2 MiB chunks: 1-2 data shares
// rebuilt in place): one-wave workgroups, load groups of 4, 16 per CU --
// 196.8 -> 187.5 us and 216.6 -> 212.4 us per 1024 x 1 MiB of shares
// (tools/ab21.py AB_K=8, tools/gpu/r6s_ab8r.sh, profiles/r6s_ab8r.jsonl,
// builds interleaved; 14 per CU the same for one row, noisy for two).
template <>
struct PermShape<8, 1> {
  static constexpr int T = 64, G = 4, OCC = 16;
};
template <>
struct PermShape<8, 2> {
  static constexpr int T = 64, G = 4, OCC = 16;
};
// <4,2>: the headline RS(4,2) encode and decode of 2 lost shares, one-wave
// workgroups at 14 per CU. The default bench line, interleaved A/B of
// library builds on two boxes (tools/build_variant.sh, tools/gpu/r6s_ab42.sh,
// profiles/r6s_ab42_round1/2.jsonl): 4,136-4,160 -> 4,201-4,224 GiB/s
// (+1.5 %), config 4 4,120-4,126 -> 4,244-4,247 (+3 %). The cap is sharp:
// 13 per CU +0.7 %, 16 (which 15 also resolves to: 10 KiB each) -1 %, 12 or
// 22 -1.7 %; 128-lane workgroups at 7 or 8 per CU -0.5 / +0.7 %. Round 5's
// one-wave A/B (profiles/r5m_ab_headline_t64.txt) had tried caps 12 and 16.
// STORB_PERM42_T / _OCC: experiment builds only.
#ifndef STORB_PERM42_T
#define STORB_PERM42_T 64
#endif
#ifndef STORB_PERM42_OCC
#define STORB_PERM42_OCC 14
#endif
template <>
struct PermShape<4, 2> {
  static constexpr int T = STORB_PERM42_T, G = 4, OCC = STORB_PERM42_OCC;
};

template <int KM, int RM>
hipError_t go_perm(const ApplyArgs &a, hipStream_t s) {
  using C = Tune<KM, RM>;
  using P = PermShape<KM, RM>;
  if (a.ncopy || (P::T == C::T && P::G == C::G && P::OCC == C::OCC))
    return launch_perm<KM, RM, C::T, C::U, C::BAR, C::G, C::TL, C::PAIR>(a, s, C::OCC,
                                                                         C::OCC_COPY);
  return launch_perm<KM, RM, P::T, C::U, C::BAR, P::G, C::TL, C::PAIR>(a, s, P::OCC, 0);
}

template <int KM>
hipError_t go_perm_r(const ApplyArgs &a, hipStream_t s) {
  switch (rows_bucket(a.r)) {
    case 0:  // pure assembly (COPY with nothing missing); tables of one zero row
    case 1: return go_perm<KM, 1>(a, s);
    case 2: return go_perm<KM, 2>(a, s);
    case 3: return go_perm<KM, 3>(a, s);
    case 4: return go_perm<KM, 4>(a, s);
    case 5: return go_perm<KM, 5>(a, s);
    case 6: return go_perm<KM, 6>(a, s);
    case 7: return go_perm<KM, 7>(a, s);
    case 8: return go_perm<KM, 8>(a, s);
    default: return go_perm<KM, 16>(a, s);
  }
}

// One translation unit per KM bucket (rs_perm_k*.hip) so hipcc can build
// the instantiations in parallel.
hipError_t dispatch_perm_k1(const ApplyArgs &a, hipStream_t s);
hipError_t dispatch_perm_k2(const ApplyArgs &a, hipStream_t s);
hipError_t dispatch_perm_k4(const ApplyArgs &a, hipStream_t s);
hipError_t dispatch_perm_k8(const ApplyArgs &a, hipStream_t s);
hipError_t dispatch_perm_k16(const ApplyArgs &a, hipStream_t s);
hipError_t dispatch_perm_k32(const ApplyArgs &a, hipStream_t s);
hipError_t dispatch_lds(const ApplyArgs &a, hipStream_t s);
hipError_t dispatch_desc_k1(const DescArgs &a, hipStream_t s);
hipError_t dispatch_desc_k2(const DescArgs &a, hipStream_t s);
hipError_t dispatch_desc_k4(const DescArgs &a, hipStream_t s);
hipError_t dispatch_desc_k8(const DescArgs &a, hipStream_t s);
hipError_t dispatch_desc_k16(const DescArgs &a, hipStream_t s);
hipError_t dispatch_desc_k32(const DescArgs &a, hipStream_t s);

}  // namespace storb_rs
