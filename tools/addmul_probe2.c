/* addmul_probe2.c -- follow-up to addmul_probe.c: the oracle's own zo_encode
 * (oracle/zfec_oracle.c compiled in statically, and the shared library via
 * dlopen) on malloc'd buffers, RS(4,2) of 1 MiB chunks, MiB/s of user data.
 * build: gcc -O2 -D_GNU_SOURCE -I../oracle -o _build/addmul_probe2 addmul_probe2.c \
 *        ../oracle/zfec_oracle.c -ldl -lpthread -lm */
#include <dlfcn.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <time.h>

#include "zfec_oracle.h"

typedef int (*enc_fn)(unsigned, unsigned, const uint8_t *, size_t, uint8_t *, size_t *, size_t *);

static double now(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec + t.tv_nsec * 1e-9;
}

static double rate(enc_fn f, const uint8_t *d, uint8_t *sh, size_t n) {
  size_t b, p;
  int reps = 0;
  double t0 = now();
  while (now() - t0 < 1.0) {
    f(4, 6, d, n, sh, &b, &p);
    reps++;
  }
  return reps / (now() - t0) * (n / 1048576.0);
}

int main(int argc, char **argv) {
  const size_t n = 1 << 20;
  uint8_t *d = malloc(n), *sh = malloc(6 * (n / 4));
  for (size_t i = 0; i < n; i++) d[i] = (uint8_t)(i * 2654435761u >> 13);
  printf("{\"static_zo_encode_MiBps\": %.0f", rate(zo_encode, d, sh, n));
  void *h = dlopen(argc > 1 ? argv[1] : "oracle/_build/libzfec_oracle.so", RTLD_NOW);
  if (h) {
    enc_fn f = (enc_fn)dlsym(h, "zo_encode");
    void (*init)(void) = (void (*)(void))dlsym(h, "zo_init");
    init();
    printf(", \"dlopen_zo_encode_MiBps\": %.0f", rate(f, d, sh, n));
  }
  printf("}\n");
  return 0;
}
