/* addmul_probe3.c -- which memory layout makes fec.c's byte addmul loop slow
 * on the GPU boxes' host CPUs (AMD EPYC 9575F)? dst ^= c*src over 8 KiB
 * blocks (fec.c's STRIDE), RS(4,2)-shaped (2 parity rows x 4 data rows of
 * 256 KiB), with the 64 KiB product table at a chosen offset inside a page
 * and the source / destination rows at chosen page offsets. MB/s of parity
 * work (bytes of src consumed per second).
 * build: gcc -O2 -o _build/addmul_probe3 addmul_probe3.c */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

static uint8_t *mul;  /* 256 x 256, placed by the caller */

static void addmul(uint8_t *restrict d, const uint8_t *restrict s, uint8_t c, size_t n) {
  const uint8_t *row = mul + 256 * c;
  size_t i = 0;
  for (; i + 16 <= n; i += 16)
    for (int u = 0; u < 16; u++) d[i + u] ^= row[s[i + u]];
  for (; i < n; i++) d[i] ^= row[s[i]];
}

static double now(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec + t.tv_nsec * 1e-9;
}

int main(void) {
  uint8_t *tbase = aligned_alloc(4096, 65536 + 8192);
  uint8_t *sbase = aligned_alloc(4096, (4 << 18) + 8192);
  uint8_t *dbase = aligned_alloc(4096, (2 << 18) + 8192);
  const size_t toffs[] = {0, 0x100, 0x810}, soffs[] = {0x10, 0x810}, doffs[] = {0x10, 0x410};
  printf("[");
  int first = 1;
  for (int ti = 0; ti < 3; ti++)
    for (int si = 0; si < 2; si++)
      for (int di = 0; di < 2; di++) {
        mul = tbase + toffs[ti];
        for (int a = 0; a < 256; a++)
          for (int b = 0; b < 256; b++) {
            unsigned x = a, y = b, p = 0;
            while (y) {
              if (y & 1) p ^= x;
              x <<= 1;
              if (x & 0x100) x ^= 0x11D;
              y >>= 1;
            }
            mul[256 * a + b] = (uint8_t)p;
          }
        uint8_t *src = sbase + soffs[si], *dst = dbase + doffs[di];
        const size_t B = 1 << 18;
        for (size_t i = 0; i < 4 * B; i++) src[i] = (uint8_t)(i * 2654435761u >> 13);
        memset(dst, 0, 2 * B);
        int reps = 0;
        double t0 = now();
        while (now() - t0 < 0.3) {
          for (size_t off = 0; off < B; off += 8192)
            for (int p = 0; p < 2; p++)
              for (int j = 0; j < 4; j++)
                addmul(dst + p * B + off, src + j * B + off, (uint8_t)(3 + 5 * p + j), 8192);
          reps++;
        }
        const double el = now() - t0;
        printf("%s{\"table_off\": %zu, \"src_off\": %zu, \"dst_off\": %zu, \"MBps\": %.0f}",
               first ? "" : ", ", toffs[ti], soffs[si], doffs[di], reps * 8.0 * B / el / 1e6);
        first = 0;
      }
  printf("]\n");
  return 0;
}
