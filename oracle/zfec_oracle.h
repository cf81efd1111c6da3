/*
 * zfec_oracle.h -- CPU ORACLE (test infrastructure only).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this code, and only as the checker / the timed CPU baseline. The
 * product path (storb_amd/, include/storb_rs.h) never links or calls it.
 *
 * What it restates
 *   Storb's chunk->shard Reed-Solomon stage calls the external crate
 *   zfec-rs @ git rev 3f3a3720def2294dc62e65f614862f1a7ddd3187
 *   (reference Cargo.toml:81, Cargo.lock:9508-9511), which is NOT vendored
 *   in /root/reference and cannot be fetched (no network, no cargo). zfec-rs
 *   is a port of zfec's fec.c (L. Rizzo, 1997; Z. Wilcox-O'Hearn): a
 *   systematic Vandermonde RS code over GF(2^8). This file restates that
 *   published algorithm in plain scalar C, mirroring
 *   zfec's table-driven addmul with 8 KiB STRIDE blocking, and Storb's own
 *   sizing from crates/storb_base/src/piece.rs:292-317.
 *
 * Parity status: PARITY UNPINNED for the encode parity bytes. The reference
 *   repo holds no parity golden vectors (its tests, piece.rs:506-689, only
 *   round-trip), and zfec-rs cannot be built or run here. Reconstructed data
 *   IS pinned: decode(encode(x)) == x is exactly what the reference tests
 *   assert, and MDS decoding of any k valid shares is unique.
 */
#ifndef STORB_ZFEC_ORACLE_H
#define STORB_ZFEC_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* GF(2^8) tables (fec.c generate_gf / init_mul_table). Idempotent. */
void zo_init(void);
uint8_t zo_gf_mul(uint8_t a, uint8_t b);
uint8_t zo_gf_inv(uint8_t a);
uint8_t zo_gf_exp(unsigned i);

/* Fec::new(k, n): n*k systematic encoding matrix, row-major.
 * Returns 0, or -1 for invalid (k<1, n<1, n>256, k>n). */
int zo_fec_new(unsigned k, unsigned n, uint8_t *enc_matrix);

/* Generic Gauss-Jordan inversion of a k*k matrix over GF(2^8) (fec.c
 * _invert_mat restated). Returns 0, -1 if singular. */
int zo_invert_mat(uint8_t *m, unsigned k);

/* Fec::encode: B = ceil(len/k), zero-pad to k*B, write all n shares
 * (shares[i*B .. (i+1)*B)) in index order. Returns 0 / -1. */
int zo_encode(unsigned k, unsigned n, const uint8_t *data, size_t len,
              uint8_t *shares, size_t *block_out, size_t *padlen_out);

/* Parity-only encode into (n-k) caller buffers of B bytes each. */
int zo_encode_parity(unsigned k, unsigned n, const uint8_t *data, size_t len,
                     uint8_t *const *parity, size_t *block_out,
                     size_t *padlen_out);

/* decode_chunk + Fec::decode: given nshares >= k shares of B bytes with
 * indices idx[], sort by index, keep the first k (piece.rs:368-381), rebuild
 * the data and write k*B - padlen bytes to out. Returns 0, -1 invalid,
 * -2 not enough / duplicate shares. */
int zo_decode(unsigned k, unsigned n, const uint8_t *const *shares,
              const unsigned *idx, unsigned nshares, size_t block,
              size_t padlen, uint8_t *out);
/* The same with caller-provided scratch (NULL = allocate per call, the
 * reference's behaviour): encode's zero-padded data copy (k*B) and
 * generator (n*k), decode's rebuilt row (B). */
int zo_encode_impl(unsigned k, unsigned n, const uint8_t *data, size_t len,
                   uint8_t *const *out_rows, int parity_only, size_t *block_out,
                   size_t *padlen_out, uint8_t *scratch, uint8_t *enc);
int zo_decode_impl(unsigned k, unsigned n, const uint8_t *const *shares,
                   const unsigned *idx, unsigned nshares, size_t block, size_t padlen,
                   uint8_t *out, uint8_t *row_scratch);

/* CPU baseline loop (cpu_bench.c), timed and accounted on the calling
 * thread: encode and/or decode round trips over nsample chunks of len bytes
 * (chunk i at chunks + i*len), survivor set (i mod nsets) of surv (k each),
 * until `seconds` of wall time. fresh = 1: every call allocates its outputs
 * as zfec-rs does (Vec per share, Vec out; the oracle's own per-call
 * buffers); fresh = 0: all buffers allocated once (arithmetic only). */
typedef struct {
  double wall_s, user_s, sys_s;
  long minflt, majflt, nvcsw, nivcsw;
  unsigned long long calls;
  int cpu_start, cpu_end;
  int bad;
  /* the thread's own hardware counters over the loop (perf_event_open, user
   * mode; -1 when the kernel refuses them) and a clock probe before / after:
   * a dependent 64-bit multiply-add chain, iterations per ns */
  long long cycles, instructions;
  double probe_before, probe_after;
  /* memory-side probes after the loop, GB/s: the oracle's addmul on an
   * L1-resident 4 KiB block, a 512 KiB (L2) and a 256 MiB (DRAM) sequential
   * read by this thread */
  double l1_addmul_gbs, l2_read_gbs, dram_read_gbs;
} zo_bench_t;
/* fec.c's addmul (dst ^= c * src) as the oracle runs it (cpu_bench.c probe) */
void zo_addmul(uint8_t *dst, const uint8_t *src, uint8_t c, size_t sz);
int zo_bench_roundtrip(unsigned k, unsigned n, const uint8_t *chunks, size_t len,
                       unsigned nsample, const unsigned *surv, unsigned nsets, int do_encode,
                       int do_decode, int fresh, double seconds, zo_bench_t *out);

/* Storb sizing: piece_length (piece.rs:292-303; 0 = default bounds) and
 * get_k_and_m (piece.rs:307-317; m = TOTAL share count). */
uint64_t zo_piece_length(uint64_t content_length, uint64_t min_size,
                         uint64_t max_size);
void zo_get_k_and_m(uint64_t chunk_size, uint64_t *k, uint64_t *m);

/* Synthetic input generator shared with the device fill kernel:
 * little-endian splitmix64 stream, word i = mix(seed + (i+1)*golden). */
void zo_splitmix_fill(uint64_t seed, uint8_t *out, size_t len);

/* Multi-threaded parity encode of nchunks independent chunks of len bytes
 * (CPU baseline "nproc threads" figure). threads<=0 -> 1. */
int zo_encode_many(unsigned k, unsigned n, const uint8_t *data, size_t len,
                   unsigned nchunks, uint8_t *parity, int threads);

/* Multi-threaded batch decode (test checker for whole device batches):
 * chunk c's data share i < k at data + (c*k + i)*block, parity share i >= k
 * at parity + (c*(n-k) + i-k)*block; the k survivors surv[] (sorted) rebuild
 * chunk c (padlen 0) into out + c*k*block. Returns the number of chunks
 * that failed (0 = all rebuilt), -1 on bad input. */
int zo_decode_many(unsigned k, unsigned n, const uint8_t *data, const uint8_t *parity,
                   size_t block, unsigned nchunks, const unsigned *surv, uint8_t *out,
                   int threads);

/* Multi-threaded encode + decode round trips of nchunks independent chunks
 * of len bytes (data back to back), losing the `nerased` shares listed in
 * erased[] (first k survivors by index decode). Returns the number of
 * chunks whose round trip failed (0 = all bit-exact), -1 on bad input.
 * CPU baseline "nproc threads" figure. */
int zo_roundtrip_many(unsigned k, unsigned n, const uint8_t *data, size_t len,
                      unsigned nchunks, const unsigned *erased, unsigned nerased,
                      int threads);

#ifdef __cplusplus
}
#endif
#endif
