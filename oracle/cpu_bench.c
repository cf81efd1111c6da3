/* cpu_bench.c -- the CPU baseline loop of bench.py (TEST INFRASTRUCTURE:
 * the timed reference CPU path, never the product).
 *
 * The reference encodes an object's chunks one after another in one task
 * (crates/storb_validator/src/upload.rs:418-420) and decodes them one after
 * another (download.rs:505-529), each chunk through zfec-rs Fec::new + encode
 * / decode (crates/storb_base/src/piece.rs:328-329,383-386), whose results
 * are freshly allocated Vecs. This runs that loop over the oracle's scalar
 * restatement (zfec_oracle.c) inside C, on the calling thread, and accounts
 * for the thread itself: getrusage(RUSAGE_THREAD) user / system time, minor
 * and major page faults, context switches, and the CPU it started / ended
 * on -- so a baseline that moves between boxes can be told apart into
 * arithmetic and memory-management (page-fault) cost.
 *
 * fresh = 1: each call allocates what zfec-rs allocates (n share buffers of
 *            B bytes, the decode output, the oracle's own scratch) and frees
 *            it: the reported baseline.
 * fresh = 0: every buffer allocated once: the arithmetic alone. */
#include <linux/perf_event.h>
#include <sched.h>
#include <stdlib.h>
#include <string.h>
#include <sys/ioctl.h>
#include <sys/resource.h>
#include <sys/syscall.h>
#include <time.h>
#include <unistd.h>

#include "zfec_oracle.h"

static double now_s(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + ts.tv_nsec * 1e-9;
}

static double tv_s(struct timeval t) { return t.tv_sec + t.tv_usec * 1e-6; }

/* A hardware counter of the calling thread, user mode only; -1 if refused
 * (containers often forbid perf_event_open). */
static int perf_open(unsigned long long config) {
  struct perf_event_attr a;
  memset(&a, 0, sizeof(a));
  a.type = PERF_TYPE_HARDWARE;
  a.size = sizeof(a);
  a.config = config;
  a.disabled = 1;
  a.exclude_kernel = 1;
  a.exclude_hv = 1;
  return (int)syscall(__NR_perf_event_open, &a, 0, -1, -1, 0);
}

static long long perf_read(int fd) {
  long long v = -1;
  if (fd < 0 || read(fd, &v, sizeof(v)) != (ssize_t)sizeof(v)) return -1;
  return v;
}

/* Clock probe: a dependent multiply-add chain for ~0.1 s; iterations per ns
 * scale with the core's clock and with nothing else it shares. */
static double clock_probe(void) {
  volatile unsigned long long sink;
  unsigned long long x = 1, it = 0;
  const double t0 = now_s();
  double t = t0;
  while (t - t0 < 0.1) {
    for (int i = 0; i < 100000; i++) x = x * 6364136223846793005ull + 1442695040888963407ull;
    it += 100000;
    t = now_s();
  }
  sink = x;
  (void)sink;
  return it / ((t - t0) * 1e9);
}

/* Sequential read of `bytes` by this thread, GB/s (best of 3 passes). */
static double read_probe(size_t bytes) {
  uint64_t *b = malloc(bytes);
  if (!b) return -1;
  const size_t n = bytes / 8;
  for (size_t i = 0; i < n; i++) b[i] = i * 0x9E3779B97F4A7C15ull;
  volatile uint64_t sink;
  double best = 0;
  for (int pass = 0; pass < 3; pass++) {
    uint64_t acc0 = 0, acc1 = 0, acc2 = 0, acc3 = 0;
    const int reps = bytes <= (1u << 20) ? 200 : 1;
    const double t0 = now_s();
    for (int r = 0; r < reps; r++)
      for (size_t i = 0; i + 4 <= n; i += 4) {
        acc0 += b[i];
        acc1 += b[i + 1];
        acc2 += b[i + 2];
        acc3 += b[i + 3];
      }
    const double el = now_s() - t0;
    sink = acc0 ^ acc1 ^ acc2 ^ acc3;
    const double gbs = (double)bytes * reps / el / 1e9;
    if (gbs > best) best = gbs;
  }
  (void)sink;
  free(b);
  return best;
}

/* The oracle's own addmul over an L1-resident 4 KiB block, GB/s of src. */
static double l1_addmul_probe(void) {
  static uint8_t src[4096], dst[4096];
  for (int i = 0; i < 4096; i++) src[i] = (uint8_t)(i * 31 + 7);
  zo_addmul(dst, src, 0x53, sizeof(src));
  const double t0 = now_s();
  int it = 0;
  double t = t0;
  while (t - t0 < 0.05) {
    for (int r = 0; r < 256; r++) zo_addmul(dst, src, (uint8_t)(0x53 + r), sizeof(src));
    it += 256;
    t = now_s();
  }
  return (double)it * sizeof(src) / (t - t0) / 1e9;
}

int zo_bench_roundtrip(unsigned k, unsigned n, const uint8_t *chunks, size_t len,
                       unsigned nsample, const unsigned *surv, unsigned nsets, int do_encode,
                       int do_decode, int fresh, double seconds, zo_bench_t *out) {
  if (k < 1 || n < k || n > 256 || !len || !nsample || !nsets || !out) return -1;
  memset(out, 0, sizeof(*out));
  const size_t B = (len + k - 1) / k;
  /* pre-encoded shares for decode-only runs, and the buffers of fresh = 0 */
  uint8_t *pre = malloc((size_t)nsample * n * B);
  uint8_t *shares_keep = malloc((size_t)n * B), *out_keep = malloc(len);
  uint8_t *scratch = malloc((size_t)k * B), *enc = malloc((size_t)n * k), *row = malloc(B);
  uint8_t **rows = malloc(sizeof(uint8_t *) * n);
  const uint8_t **sv = malloc(sizeof(uint8_t *) * k);
  if (!pre || !shares_keep || !out_keep || !scratch || !enc || !row || !rows || !sv) return -1;
  size_t b, pad = 0;
  for (unsigned i = 0; i < nsample; i++) {
    for (unsigned r = 0; r < n; r++) rows[r] = pre + ((size_t)i * n + r) * B;
    if (zo_encode_impl(k, n, chunks + (size_t)i * len, len, rows, 0, &b, &pad, NULL, NULL))
      return -1;
  }
  memset(shares_keep, 0, (size_t)n * B); /* first touch outside the timed loop */
  memset(out_keep, 0, len);
  memset(scratch, 0, (size_t)k * B);
  memset(row, 0, B);
  out->probe_before = clock_probe();
  const int fcyc = perf_open(PERF_COUNT_HW_CPU_CYCLES);
  const int fins = perf_open(PERF_COUNT_HW_INSTRUCTIONS);
  if (fcyc >= 0) ioctl(fcyc, PERF_EVENT_IOC_ENABLE, 0);
  if (fins >= 0) ioctl(fins, PERF_EVENT_IOC_ENABLE, 0);
  struct rusage r0, r1;
  getrusage(RUSAGE_THREAD, &r0);
  out->cpu_start = sched_getcpu();
  const double t0 = now_s();
  unsigned long long calls = 0;
  for (;;) {
    const unsigned i = (unsigned)(calls % nsample);
    const uint8_t *src = chunks + (size_t)i * len;
    uint8_t *shares = pre + (size_t)i * n * B;
    uint8_t *fresh_shares = NULL, *o;
    if (do_encode) {
      fresh_shares = fresh ? malloc((size_t)n * B) : shares_keep;
      for (unsigned r = 0; r < n; r++) rows[r] = fresh_shares + (size_t)r * B;
      if (zo_encode_impl(k, n, src, len, rows, 0, &b, &pad, fresh ? NULL : scratch,
                         fresh ? NULL : enc))
        out->bad++;
      shares = fresh_shares;
    }
    if (do_decode) {
      const unsigned *s = surv + (size_t)(calls % nsets) * k;
      for (unsigned c = 0; c < k; c++) sv[c] = shares + (size_t)s[c] * B;
      o = fresh ? malloc(len) : out_keep;
      if (zo_decode_impl(k, n, sv, s, k, B, pad, o, fresh ? NULL : row)) out->bad++;
      if (calls < nsample && memcmp(o, src, len)) out->bad++;
      if (fresh) free(o);
    }
    if (fresh && fresh_shares) free(fresh_shares);
    calls++;
    if (now_s() - t0 >= seconds) break;
  }
  out->wall_s = now_s() - t0;
  out->cpu_end = sched_getcpu();
  getrusage(RUSAGE_THREAD, &r1);
  out->cycles = perf_read(fcyc);
  out->instructions = perf_read(fins);
  if (fcyc >= 0) close(fcyc);
  if (fins >= 0) close(fins);
  out->probe_after = clock_probe();
  out->l1_addmul_gbs = l1_addmul_probe();
  out->l2_read_gbs = read_probe(512u << 10);
  out->dram_read_gbs = read_probe(256u << 20);
  out->user_s = tv_s(r1.ru_utime) - tv_s(r0.ru_utime);
  out->sys_s = tv_s(r1.ru_stime) - tv_s(r0.ru_stime);
  out->minflt = r1.ru_minflt - r0.ru_minflt;
  out->majflt = r1.ru_majflt - r0.ru_majflt;
  out->nvcsw = r1.ru_nvcsw - r0.ru_nvcsw;
  out->nivcsw = r1.ru_nivcsw - r0.ru_nivcsw;
  out->calls = calls;
  free(pre);
  free(shares_keep);
  free(out_keep);
  free(scratch);
  free(enc);
  free(row);
  free(rows);
  free(sv);
  return 0;
}
