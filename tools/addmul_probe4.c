/* addmul_probe4.c -- where zo_encode's time goes on a GPU-box host: the
 * generator build (zo_fec_new), the zero-padded copy (calloc + memcpy +
 * free of 1 MiB), and the whole zo_encode, per RS(4,2) call on 1 MiB.
 * build: gcc -O2 -D_GNU_SOURCE -I../oracle -o _build/addmul_probe4 addmul_probe4.c \
 *        -L../oracle/_build -lzfec_oracle -Wl,-rpath,'$ORIGIN/../../oracle/_build' */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "zfec_oracle.h"

static double now(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec + t.tv_nsec * 1e-9;
}

int main(void) {
  const size_t n = 1 << 20;
  uint8_t *d = malloc(n), *sh = malloc(6 * (n / 4)), enc[64];
  for (size_t i = 0; i < n; i++) d[i] = (uint8_t)(i * 2654435761u >> 13);
  zo_init();
  const int R = 50;
  double t0 = now();
  for (int r = 0; r < R; r++) zo_fec_new(4, 6, enc);
  const double t_fec = (now() - t0) / R;
  t0 = now();
  for (int r = 0; r < R; r++) {
    uint8_t *s = calloc(n, 1);
    memcpy(s, d, n);
    __asm__ volatile("" ::"r"(s) : "memory");
    free(s);
  }
  const double t_copy = (now() - t0) / R;
  size_t b, p;
  t0 = now();
  for (int r = 0; r < R; r++) zo_encode(4, 6, d, n, sh, &b, &p);
  const double t_enc = (now() - t0) / R;
  printf("{\"fec_new_us\": %.1f, \"calloc_copy_free_us\": %.1f, \"zo_encode_us\": %.1f}\n",
         t_fec * 1e6, t_copy * 1e6, t_enc * 1e6);
  return 0;
}
