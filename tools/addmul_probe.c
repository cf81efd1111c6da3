/* addmul_probe.c -- is the slow scalar CPU baseline on some GPU boxes the
 * byte read-modify-write loop of fec.c's addmul (oracle/zfec_oracle.c), or
 * the machine? Times dst ^= c*src over 1 MiB rows three ways: (a) fec.c's
 * byte loop (16-way unrolled, restrict), (b) the same lookups packed into one
 * 64-bit load/xor/store per 8 bytes, (c) a plain memcpy of the same bytes.
 * build: gcc -O2 -o _build/addmul_probe addmul_probe.c */
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <stdlib.h>
#include <time.h>

static uint8_t mul[256][256];

static void addmul_a(uint8_t *restrict d, const uint8_t *restrict s, uint8_t c, size_t n) {
  const uint8_t *row = mul[c];
  size_t i = 0;
  for (; i + 16 <= n; i += 16)
    for (int u = 0; u < 16; u++) d[i + u] ^= row[s[i + u]];
  for (; i < n; i++) d[i] ^= row[s[i]];
}

static void addmul_b(uint8_t *restrict d, const uint8_t *restrict s, uint8_t c, size_t n) {
  const uint8_t *row = mul[c];
  for (size_t i = 0; i + 8 <= n; i += 8) {
    uint64_t v = 0;
    for (int u = 0; u < 8; u++) v |= (uint64_t)row[s[i + u]] << (8 * u);
    uint64_t x;
    memcpy(&x, d + i, 8);
    x ^= v;
    memcpy(d + i, &x, 8);
  }
}

static double now(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec + t.tv_nsec * 1e-9;
}

int main(void) {
  for (int a = 0; a < 256; a++)
    for (int b = 0; b < 256; b++) {
      unsigned x = a, y = b, p = 0;
      while (y) {
        if (y & 1) p ^= x;
        x <<= 1;
        if (x & 0x100) x ^= 0x11D;
        y >>= 1;
      }
      mul[a][b] = (uint8_t)p;
    }
  const size_t n = 1 << 20;
  uint8_t *s = malloc(n), *d = calloc(n, 1);
  for (size_t i = 0; i < n; i++) s[i] = (uint8_t)(i * 2654435761u >> 13);
  const int reps = 200;
  double t0 = now();
  for (int r = 0; r < reps; r++) addmul_a(d, s, (uint8_t)(r | 2), n);
  double ta = now() - t0;
  t0 = now();
  for (int r = 0; r < reps; r++) addmul_b(d, s, (uint8_t)(r | 2), n);
  double tb = now() - t0;
  t0 = now();
  for (int r = 0; r < reps; r++) memcpy(d, s + (r & 1), n - 1);
  double tc = now() - t0;
  printf("{\"byte_loop_MBps\": %.0f, \"packed64_MBps\": %.0f, \"memcpy_MBps\": %.0f, \"chk\": %u}\n",
         reps * n / ta / 1e6, reps * n / tb / 1e6, reps * n / tc / 1e6, d[12345]);
  return 0;
}
