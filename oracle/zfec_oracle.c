/*
 * zfec_oracle.c -- CPU ORACLE (test infrastructure only; see zfec_oracle.h).
 *
 * Plain scalar restatement of zfec's fec.c as ported by zfec-rs
 * @3f3a3720 (Cargo.toml:81), driven the way Storb drives it in
 * crates/storb_base/src/piece.rs:320-387. Nothing here is SIMD or threaded
 * except zo_encode_many, which only fans independent chunks out to threads
 * for the "nproc" CPU figure. Compiled with -O2 to mirror the reference's
 * release profile (Cargo.toml:87-89: opt-level = 2, codegen-units = 1).
 *
 * PARITY UNPINNED (encode parity bytes): no zfec-rs binary or golden vector
 * exists offline. Pinned: reconstructed data (round-trip, the reference's
 * own assertion in piece.rs:513-519, 543-550, 597-618).
 */
#include "zfec_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ---------------------------------------------------------------- GF(2^8)
 * fec.c generate_gf(): primitive polynomial Pp = "101110001" read LSB
 * first = x^8+x^4+x^3+x^2+1 (0x11D), generator alpha = 2. */
static uint8_t g_exp[510];
static int g_log[256];
static uint8_t g_inv[256];
static uint8_t g_mul[256][256];
static pthread_once_t g_once = PTHREAD_ONCE_INIT;

static void build_tables(void) {
  const char *pp = "101110001";
  unsigned mask = 1;
  g_exp[8] = 0;
  for (int i = 0; i < 8; i++, mask <<= 1) {
    g_exp[i] = (uint8_t)mask;
    g_log[g_exp[i]] = i;
    if (pp[i] == '1') g_exp[8] ^= (uint8_t)mask;
  }
  g_log[g_exp[8]] = 8;
  /* alpha^i = alpha * alpha^(i-1): shift, reduce when bit 7 was set. */
  for (int i = 9; i < 255; i++) {
    unsigned prev = g_exp[i - 1];
    unsigned v = (prev << 1) & 0xFF;
    if (prev & 0x80) v ^= g_exp[8];
    g_exp[i] = (uint8_t)v;
    g_log[g_exp[i]] = i;
  }
  g_log[0] = 255; /* sentinel, as in fec.c */
  for (int i = 0; i < 255; i++) g_exp[i + 255] = g_exp[i];
  g_inv[0] = 0;
  g_inv[1] = 1;
  for (int i = 2; i < 256; i++) g_inv[i] = g_exp[255 - g_log[i]];
  for (int a = 0; a < 256; a++)
    for (int b = 0; b < 256; b++)
      g_mul[a][b] = (a == 0 || b == 0)
                        ? 0
                        : g_exp[(g_log[a] + g_log[b]) % 255];
}

void zo_init(void) { pthread_once(&g_once, build_tables); }

uint8_t zo_gf_mul(uint8_t a, uint8_t b) {
  zo_init();
  return g_mul[a][b];
}
uint8_t zo_gf_inv(uint8_t a) {
  zo_init();
  return g_inv[a];
}
uint8_t zo_gf_exp(unsigned i) {
  zo_init();
  return g_exp[i % 255];
}

/* fec.c addmul() / _addmul1(): dst ^= c * src, table driven, with fec.c's
 * restrict-qualified, 16-way unrolled main loop (UNROLL = 16). Rust's &mut /
 * & borrows give zfec-rs the same no-alias guarantee, so this is the fair
 * scalar speed for the CPU baseline (1.4x the naive byte loop at -O2). */
#define ZO_UNROLL 16
static void addmul(uint8_t *restrict dst, const uint8_t *restrict src, uint8_t c, size_t sz) {
  if (c == 0) return;
  const uint8_t *row = g_mul[c];
  size_t i = 0;
  for (; i + ZO_UNROLL <= sz; i += ZO_UNROLL) {
    dst[i + 0] ^= row[src[i + 0]];
    dst[i + 1] ^= row[src[i + 1]];
    dst[i + 2] ^= row[src[i + 2]];
    dst[i + 3] ^= row[src[i + 3]];
    dst[i + 4] ^= row[src[i + 4]];
    dst[i + 5] ^= row[src[i + 5]];
    dst[i + 6] ^= row[src[i + 6]];
    dst[i + 7] ^= row[src[i + 7]];
    dst[i + 8] ^= row[src[i + 8]];
    dst[i + 9] ^= row[src[i + 9]];
    dst[i + 10] ^= row[src[i + 10]];
    dst[i + 11] ^= row[src[i + 11]];
    dst[i + 12] ^= row[src[i + 12]];
    dst[i + 13] ^= row[src[i + 13]];
    dst[i + 14] ^= row[src[i + 14]];
    dst[i + 15] ^= row[src[i + 15]];
  }
  for (; i < sz; i++) dst[i] ^= row[src[i]];
}

/* ------------------------------------------------------------ matrices */

/* fec.c _invert_vdm(): invert the k*k Vandermonde whose row i is the powers
 * of p_i = src[i*k+1] (p_0 = 0 for the x=0 row), by building the
 * coefficients of P(x) = prod (x - p_i) and synthetic division per row. */
static void invert_vdm(uint8_t *src, unsigned k) {
  if (k == 1) return; /* [1] is its own inverse */
  uint8_t *c = calloc(k, 1), *b = calloc(k, 1), *p = calloc(k, 1);
  for (unsigned i = 0; i < k; i++) p[i] = src[i * k + 1];
  /* P_0 = x + p_0; P_i = x*P_{i-1} + p_i*P_{i-1} (char 2: - == +).
   * c[] holds the non-leading coefficients, c[k] = 1 implicit. */
  c[k - 1] = p[0];
  for (unsigned i = 1; i < k; i++) {
    uint8_t pi = p[i];
    for (unsigned j = k - i; j < k - 1; j++) c[j] ^= g_mul[pi][c[j + 1]];
    c[k - 1] ^= pi;
  }
  for (unsigned row = 0; row < k; row++) {
    uint8_t xx = p[row], t = 1;
    b[k - 1] = 1;
    for (unsigned i = k - 1; i > 0; i--) {
      b[i - 1] = c[i] ^ g_mul[xx][b[i]];
      t = g_mul[xx][t] ^ b[i - 1];
    }
    for (unsigned col = 0; col < k; col++)
      src[col * k + row] = g_mul[g_inv[t]][b[col]];
  }
  free(c);
  free(b);
  free(p);
}

int zo_invert_mat(uint8_t *m, unsigned k) {
  zo_init();
  /* Gauss-Jordan over GF(2^8) with an augmented identity. */
  uint8_t *a = malloc((size_t)k * 2 * k);
  for (unsigned r = 0; r < k; r++) {
    memcpy(a + (size_t)r * 2 * k, m + (size_t)r * k, k);
    memset(a + (size_t)r * 2 * k + k, 0, k);
    a[(size_t)r * 2 * k + k + r] = 1;
  }
  for (unsigned col = 0; col < k; col++) {
    unsigned piv = col;
    while (piv < k && a[(size_t)piv * 2 * k + col] == 0) piv++;
    if (piv == k) {
      free(a);
      return -1;
    }
    if (piv != col)
      for (unsigned x = 0; x < 2 * k; x++) {
        uint8_t t = a[(size_t)piv * 2 * k + x];
        a[(size_t)piv * 2 * k + x] = a[(size_t)col * 2 * k + x];
        a[(size_t)col * 2 * k + x] = t;
      }
    uint8_t *pr = a + (size_t)col * 2 * k;
    uint8_t ip = g_inv[pr[col]];
    for (unsigned x = 0; x < 2 * k; x++) pr[x] = g_mul[ip][pr[x]];
    for (unsigned r = 0; r < k; r++) {
      if (r == col) continue;
      uint8_t *rr = a + (size_t)r * 2 * k;
      uint8_t f = rr[col];
      if (f)
        for (unsigned x = 0; x < 2 * k; x++) rr[x] ^= g_mul[f][pr[x]];
    }
  }
  for (unsigned r = 0; r < k; r++)
    memcpy(m + (size_t)r * k, a + (size_t)r * 2 * k + k, k);
  free(a);
  return 0;
}

/* fec.c fec_new(): V (n*k) with row 0 = point 0 and row r>=1 = point
 * alpha^(r-1); enc = [I ; V[k..n) * V[0..k)^-1]. zfec-rs
 * Fec::new rejects k<1, m<1, m>256, k>m. */
int zo_fec_new(unsigned k, unsigned n, uint8_t *enc) {
  zo_init();
  if (k < 1 || n < 1 || n > 256 || k > n) return -1;
  uint8_t *v = calloc((size_t)n * k, 1);
  v[0] = 1;
  for (unsigned row = 0; row + 1 < n; row++)
    for (unsigned col = 0; col < k; col++)
      v[(size_t)(row + 1) * k + col] = g_exp[(row * col) % 255];
  invert_vdm(v, k); /* top k*k block now holds V_top^-1 */
  memset(enc, 0, (size_t)k * k);
  for (unsigned i = 0; i < k; i++) enc[(size_t)i * k + i] = 1;
  for (unsigned row = k; row < n; row++)
    for (unsigned col = 0; col < k; col++) {
      uint8_t acc = 0;
      for (unsigned i = 0; i < k; i++)
        acc ^= g_mul[v[(size_t)row * k + i]][v[(size_t)i * k + col]];
      enc[(size_t)row * k + col] = acc;
    }
  free(v);
  return 0;
}

/* ------------------------------------------------------------- encode */
#define ZO_STRIDE 8192 /* fec.c STRIDE blocking of the addmul loop */

void zo_addmul(uint8_t *dst, const uint8_t *src, uint8_t c, size_t sz) {
  zo_init();
  addmul(dst, src, c, sz);
}

/* scratch (k*B bytes) / enc (n*k): caller-provided buffers for the
 * allocation-free CPU baseline (cpu_bench.c); NULL = allocate per call, as
 * zfec-rs does (a Fec per chunk, piece.rs:328; Vecs per share). */
int zo_encode_impl(unsigned k, unsigned n, const uint8_t *data, size_t len,
                   uint8_t *const *out_rows, int parity_only, size_t *block_out,
                   size_t *padlen_out, uint8_t *scratch, uint8_t *enc_in) {
  zo_init();
  if (k < 1 || n < 1 || n > 256 || k > n || len == 0) return -1;
  uint8_t *enc = enc_in ? enc_in : malloc((size_t)n * k);
  zo_fec_new(k, n, enc);
  size_t B = (len + k - 1) / k; /* piece.rs:331-332 div_ceil(len, k) */
  size_t pad = B * k - len;
  /* zero-padded copies of the k data shards (zfec-rs splits into Vecs). */
  uint8_t *shards = scratch ? scratch : calloc((size_t)k * B, 1);
  memcpy(shards, data, len);
  if (scratch && pad) memset(shards + len, 0, pad);
  unsigned first = parity_only ? k : 0;
  for (unsigned i = first; i < n; i++) {
    uint8_t *dst = out_rows[i - first];
    if (i < k) {
      memcpy(dst, shards + (size_t)i * B, B);
      continue;
    }
    memset(dst, 0, B);
  }
  for (size_t off = 0; off < B; off += ZO_STRIDE) {
    size_t sz = B - off < ZO_STRIDE ? B - off : ZO_STRIDE;
    for (unsigned i = k; i < n; i++) {
      uint8_t *dst = out_rows[i - first] + off;
      for (unsigned j = 0; j < k; j++)
        addmul(dst, shards + (size_t)j * B + off, enc[(size_t)i * k + j], sz);
    }
  }
  if (!scratch) free(shards);
  if (!enc_in) free(enc);
  if (block_out) *block_out = B;
  if (padlen_out) *padlen_out = pad;
  return 0;
}

int zo_encode(unsigned k, unsigned n, const uint8_t *data, size_t len,
              uint8_t *shares, size_t *block_out, size_t *padlen_out) {
  if (k < 1 || n < 1 || n > 256 || k > n || len == 0) return -1;
  size_t B = (len + k - 1) / k;
  uint8_t **rows = malloc(sizeof(uint8_t *) * n);
  for (unsigned i = 0; i < n; i++) rows[i] = shares + (size_t)i * B;
  int rc = zo_encode_impl(k, n, data, len, rows, 0, block_out, padlen_out, NULL, NULL);
  free(rows);
  return rc;
}

int zo_encode_parity(unsigned k, unsigned n, const uint8_t *data, size_t len,
                     uint8_t *const *parity, size_t *block_out,
                     size_t *padlen_out) {
  return zo_encode_impl(k, n, data, len, parity, 1, block_out, padlen_out, NULL, NULL);
}

/* ------------------------------------------------------------- decode */
int zo_decode(unsigned k, unsigned n, const uint8_t *const *shares,
              const unsigned *idx, unsigned nshares, size_t B, size_t padlen,
              uint8_t *out) {
  return zo_decode_impl(k, n, shares, idx, nshares, B, padlen, out, NULL);
}

/* row_scratch (B bytes): the allocation-free baseline's buffer for the
 * rebuilt row; NULL = allocate per call. */
int zo_decode_impl(unsigned k, unsigned n, const uint8_t *const *shares,
                   const unsigned *idx, unsigned nshares, size_t B, size_t padlen,
                   uint8_t *out, uint8_t *row_scratch) {
  zo_init();
  if (k < 1 || n < 1 || n > 256 || k > n || B == 0 || padlen >= (size_t)k * B + 1)
    return -1;
  if (nshares < k) return -2;
  for (unsigned i = 0; i < nshares; i++)
    if (idx[i] >= n) return -1;
  /* piece.rs:368-381: sort by piece index, keep the first k. */
  unsigned *ord = malloc(sizeof(unsigned) * nshares);
  for (unsigned i = 0; i < nshares; i++) ord[i] = i;
  for (unsigned i = 1; i < nshares; i++) { /* stable insertion sort */
    unsigned t = ord[i], j = i;
    while (j > 0 && idx[ord[j - 1]] > idx[t]) {
      ord[j] = ord[j - 1];
      j--;
    }
    ord[j] = t;
  }
  for (unsigned i = 1; i < k; i++)
    if (idx[ord[i]] == idx[ord[i - 1]]) {
      free(ord);
      return -2;
    }
  /* Slot s holds primary share s when present; parity shares fill the
   * remaining slots in index order (zfec's decoder arrangement). */
  const uint8_t **slot = calloc(k, sizeof(uint8_t *));
  unsigned *slot_idx = malloc(sizeof(unsigned) * k);
  unsigned char *have = calloc(k, 1);
  for (unsigned i = 0; i < k; i++) {
    unsigned id = idx[ord[i]];
    if (id < k) {
      slot[id] = shares[ord[i]];
      slot_idx[id] = id;
      have[id] = 1;
    }
  }
  unsigned s = 0;
  for (unsigned i = 0; i < k; i++) {
    unsigned id = idx[ord[i]];
    if (id >= k) {
      while (have[s]) s++;
      slot[s] = shares[ord[i]];
      slot_idx[s] = id;
      s++;
    }
  }
  uint8_t *enc = malloc((size_t)n * k);
  zo_fec_new(k, n, enc);
  uint8_t *dm = malloc((size_t)k * k);
  for (unsigned r = 0; r < k; r++) {
    if (slot_idx[r] < k) {
      memset(dm + (size_t)r * k, 0, k);
      dm[(size_t)r * k + r] = 1;
    } else {
      memcpy(dm + (size_t)r * k, enc + (size_t)slot_idx[r] * k, k);
    }
  }
  int rc = zo_invert_mat(dm, k);
  if (rc == 0) {
    size_t outlen = (size_t)k * B - padlen;
    uint8_t *row = row_scratch ? row_scratch : malloc(B);
    for (unsigned r = 0; r < k; r++) {
      const uint8_t *src = slot[r];
      if (slot_idx[r] >= k) {
        memset(row, 0, B);
        for (unsigned c = 0; c < k; c++)
          addmul(row, slot[c], dm[(size_t)r * k + c], B);
        src = row;
      }
      size_t off = (size_t)r * B;
      if (off < outlen) {
        size_t cnt = outlen - off < B ? outlen - off : B;
        memcpy(out + off, src, cnt);
      }
    }
    if (!row_scratch) free(row);
  } else {
    rc = -2;
  }
  free(dm);
  free(enc);
  free(have);
  free(slot_idx);
  free(slot);
  free(ord);
  return rc;
}

/* -------------------------------------------------------------- sizing
 * piece.rs:292-303 with constants.rs:5-8. Rust `f64 as i32` saturates
 * (NaN -> 0, -inf -> i32::MIN) and release-mode `1u64 << e` masks e & 63,
 * so piece_length(0) = 1 << 0 = 1 -> clamped to the 16 KiB minimum. */
uint64_t zo_piece_length(uint64_t content_length, uint64_t min_size,
                         uint64_t max_size) {
  if (min_size == 0) min_size = 16ull * 1024;
  if (max_size == 0) max_size = 256ull * 1024 * 1024;
  double e = log2((double)content_length) * 0.5 + 8.39;
  int32_t ei;
  if (isnan(e)) ei = 0;
  else if (e <= -2147483648.0) ei = INT32_MIN;
  else if (e >= 2147483647.0) ei = INT32_MAX;
  else ei = (int32_t)e; /* truncation toward zero */
  uint64_t length = 1ull << ((uint32_t)ei & 63u);
  if (length < min_size) length = min_size;
  if (length > max_size) length = max_size;
  return length;
}

/* piece.rs:307-317: k = ceil(chunk / piece_length(chunk)), m = k +
 * ceil(k / 2); both via f64 like the reference. */
void zo_get_k_and_m(uint64_t chunk_size, uint64_t *k, uint64_t *m) {
  uint64_t ps = zo_piece_length(chunk_size, 0, 0);
  uint64_t kk = (uint64_t)ceil((double)chunk_size / (double)ps);
  uint64_t pp = (uint64_t)ceil((double)kk / 2.0);
  *k = kk;
  *m = kk + pp;
}

/* ------------------------------------------------------------ synthetic */
void zo_splitmix_fill(uint64_t seed, uint8_t *out, size_t len) {
  size_t words = len / 8, i;
  for (i = 0; i < words; i++) {
    uint64_t z = seed + (uint64_t)(i + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    memcpy(out + i * 8, &z, 8); /* little-endian host */
  }
  if (len % 8) {
    uint64_t z = seed + (uint64_t)(words + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    memcpy(out + words * 8, &z, len % 8);
  }
}

/* ------------------------------------------------------- threaded fanout */
typedef struct {
  unsigned k, n, first, last;
  const uint8_t *data;
  size_t len;
  uint8_t *parity;
} many_job;

static void *many_worker(void *arg) {
  many_job *j = (many_job *)arg;
  size_t B = (j->len + j->k - 1) / j->k;
  unsigned p = j->n - j->k;
  uint8_t **rows = malloc(sizeof(uint8_t *) * (p ? p : 1));
  for (unsigned c = j->first; c < j->last; c++) {
    for (unsigned r = 0; r < p; r++)
      rows[r] = j->parity + ((size_t)c * p + r) * B;
    zo_encode_impl(j->k, j->n, j->data + (size_t)c * j->len, j->len, rows, 1,
                   NULL, NULL, NULL, NULL);
  }
  free(rows);
  return NULL;
}

int zo_encode_many(unsigned k, unsigned n, const uint8_t *data, size_t len,
                   unsigned nchunks, uint8_t *parity, int threads) {
  zo_init();
  if (k < 1 || n < 1 || n > 256 || k > n || len == 0) return -1;
  if (threads <= 0) threads = 1;
  if ((unsigned)threads > nchunks) threads = (int)nchunks;
  pthread_t *tid = malloc(sizeof(pthread_t) * threads);
  many_job *jobs = malloc(sizeof(many_job) * threads);
  unsigned per = (nchunks + threads - 1) / threads;
  for (int t = 0; t < threads; t++) {
    jobs[t].k = k;
    jobs[t].n = n;
    jobs[t].data = data;
    jobs[t].len = len;
    jobs[t].parity = parity;
    jobs[t].first = t * per < nchunks ? t * per : nchunks;
    jobs[t].last = (t + 1) * per < nchunks ? (t + 1) * per : nchunks;
    pthread_create(&tid[t], NULL, many_worker, &jobs[t]);
  }
  for (int t = 0; t < threads; t++) pthread_join(tid[t], NULL);
  free(tid);
  free(jobs);
  return 0;
}

/* ------------------------------------------------- threaded batch decode */
typedef struct {
  unsigned k, n, first, last;
  const uint8_t *data, *parity;
  size_t block;
  const unsigned *surv;
  uint8_t *out;
  int bad;
} dec_job;

static void *dec_worker(void *arg) {
  dec_job *j = (dec_job *)arg;
  const size_t B = j->block, p = j->n - j->k;
  const uint8_t **sv = malloc(sizeof(uint8_t *) * j->k);
  for (unsigned c = j->first; c < j->last; c++) {
    for (unsigned i = 0; i < j->k; i++) {
      const unsigned s = j->surv[i];
      sv[i] = s < j->k ? j->data + ((size_t)c * j->k + s) * B
                       : j->parity + ((size_t)c * p + (s - j->k)) * B;
    }
    if (zo_decode_impl(j->k, j->n, sv, j->surv, j->k, B, 0, j->out + (size_t)c * j->k * B,
                       NULL) != 0)
      j->bad++;
  }
  free(sv);
  return NULL;
}

int zo_decode_many(unsigned k, unsigned n, const uint8_t *data, const uint8_t *parity,
                   size_t block, unsigned nchunks, const unsigned *surv, uint8_t *out,
                   int threads) {
  zo_init();
  if (k < 1 || n > 256 || k > n || block == 0 || nchunks == 0) return -1;
  if (threads <= 0) threads = 1;
  if ((unsigned)threads > nchunks) threads = (int)nchunks;
  pthread_t *tid = malloc(sizeof(pthread_t) * threads);
  dec_job *jobs = malloc(sizeof(dec_job) * threads);
  const unsigned per = (nchunks + threads - 1) / threads;
  for (int t = 0; t < threads; t++) {
    dec_job jb = {k, n, t * per < nchunks ? t * per : nchunks,
                  (t + 1) * per < nchunks ? (t + 1) * per : nchunks,
                  data, parity, block, surv, out, 0};
    jobs[t] = jb;
    pthread_create(&tid[t], NULL, dec_worker, &jobs[t]);
  }
  int bad = 0;
  for (int t = 0; t < threads; t++) {
    pthread_join(tid[t], NULL);
    bad += jobs[t].bad;
  }
  free(tid);
  free(jobs);
  return bad;
}

/* ----------------------------------------------- threaded round trips */
typedef struct {
  unsigned k, n, first, last, nerased;
  const unsigned *erased;
  const uint8_t *data;
  size_t len;
  int bad;
} rt_job;

static void *rt_worker(void *arg) {
  rt_job *j = (rt_job *)arg;
  size_t B = (j->len + j->k - 1) / j->k;
  uint8_t *shares = malloc((size_t)j->n * B);
  uint8_t *out = malloc(j->len);
  const uint8_t **sv = malloc(sizeof(uint8_t *) * j->n);
  unsigned *idx = malloc(sizeof(unsigned) * j->n);
  for (unsigned c = j->first; c < j->last; c++) {
    const uint8_t *src = j->data + (size_t)c * j->len;
    size_t b, pad;
    if (zo_encode(j->k, j->n, src, j->len, shares, &b, &pad) != 0) {
      j->bad++;
      continue;
    }
    unsigned m = 0;
    for (unsigned i = 0; i < j->n; i++) {
      int lost = 0;
      for (unsigned e = 0; e < j->nerased; e++) lost |= j->erased[e] == i;
      if (!lost) {
        sv[m] = shares + (size_t)i * B;
        idx[m++] = i;
      }
    }
    if (zo_decode(j->k, j->n, sv, idx, m, B, pad, out) != 0 || memcmp(out, src, j->len))
      j->bad++;
  }
  free(shares);
  free(out);
  free(sv);
  free(idx);
  return NULL;
}

int zo_roundtrip_many(unsigned k, unsigned n, const uint8_t *data, size_t len,
                      unsigned nchunks, const unsigned *erased, unsigned nerased,
                      int threads) {
  zo_init();
  if (k < 1 || n < 1 || n > 256 || k > n || len == 0) return -1;
  if (threads <= 0) threads = 1;
  if ((unsigned)threads > nchunks) threads = (int)nchunks;
  pthread_t *tid = malloc(sizeof(pthread_t) * threads);
  rt_job *jobs = calloc(threads, sizeof(rt_job));
  unsigned per = (nchunks + threads - 1) / threads;
  for (int t = 0; t < threads; t++) {
    jobs[t] = (rt_job){k, n, t * per < nchunks ? t * per : nchunks,
                       (t + 1) * per < nchunks ? (t + 1) * per : nchunks, nerased, erased,
                       data, len, 0};
    pthread_create(&tid[t], NULL, rt_worker, &jobs[t]);
  }
  int bad = 0;
  for (int t = 0; t < threads; t++) {
    pthread_join(tid[t], NULL);
    bad += jobs[t].bad;
  }
  free(tid);
  free(jobs);
  return bad;
}
