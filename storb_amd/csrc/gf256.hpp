// gf256.hpp -- GF(2^8) arithmetic and zfec's systematic generator, host side.
//
// Product code (does not use oracle/). The field and the generator are the
// ones zfec-rs @3f3a3720 (reference Cargo.toml:81) inherits from zfec's
// fec.c: x^8+x^4+x^3+x^2+1, alpha = 2, Vandermonde on the points
// {0, alpha^0, ..., alpha^(n-2)}, enc = [I ; V[k..n) * V[0..k)^-1]
// (SURVEY.md Appendix A). The matrices are tiny (n <= 256) and built once
// per (k, n) / erasure pattern, so this stays plain host C++; the byte
// streams go through the HIP kernels in rs_kernels.hip.
#pragma once

#include <cstdint>
#include <cstring>
#include <vector>

namespace storb_rs {

struct GF256 {
  uint8_t exp[512];
  uint8_t log[256];
  uint8_t inv[256];

  GF256() {
    unsigned x = 1;
    for (int i = 0; i < 255; i++) {
      exp[i] = static_cast<uint8_t>(x);
      log[x] = static_cast<uint8_t>(i);
      x <<= 1;
      if (x & 0x100) x ^= 0x11D;
    }
    for (int i = 255; i < 512; i++) exp[i] = exp[i - 255];
    log[0] = 0;  // never read: mul() short-circuits zero operands
    inv[0] = 0;
    for (int a = 1; a < 256; a++) inv[a] = exp[255 - log[a]];
  }

  uint8_t mul(uint8_t a, uint8_t b) const {
    if (a == 0 || b == 0) return 0;
    return exp[log[a] + log[b]];
  }
};

inline const GF256 &gf() {
  static const GF256 g;
  return g;
}

// Gauss-Jordan inverse of a k*k row-major matrix; false if singular.
inline bool gf_invert(std::vector<uint8_t> &m, unsigned k) {
  const GF256 &g = gf();
  std::vector<uint8_t> a(static_cast<size_t>(k) * 2 * k, 0);
  const size_t w = 2 * k;
  for (unsigned r = 0; r < k; r++) {
    std::memcpy(&a[r * w], &m[static_cast<size_t>(r) * k], k);
    a[r * w + k + r] = 1;
  }
  for (unsigned c = 0; c < k; c++) {
    unsigned p = c;
    while (p < k && a[p * w + c] == 0) p++;
    if (p == k) return false;
    if (p != c)
      for (size_t x = 0; x < w; x++) std::swap(a[p * w + x], a[c * w + x]);
    const uint8_t ip = g.inv[a[c * w + c]];
    for (size_t x = 0; x < w; x++) a[c * w + x] = g.mul(ip, a[c * w + x]);
    for (unsigned r = 0; r < k; r++) {
      const uint8_t f = a[r * w + c];
      if (r == c || f == 0) continue;
      for (size_t x = 0; x < w; x++) a[r * w + x] ^= g.mul(f, a[c * w + x]);
    }
  }
  for (unsigned r = 0; r < k; r++)
    std::memcpy(&m[static_cast<size_t>(r) * k], &a[r * w + k], k);
  return true;
}

inline bool valid_params(uint32_t k, uint32_t n) {
  return k >= 1 && n >= 1 && n <= 256 && k <= n;
}

// n*k systematic generator, row-major.
inline std::vector<uint8_t> enc_matrix(unsigned k, unsigned n) {
  const GF256 &g = gf();
  std::vector<uint8_t> v(static_cast<size_t>(n) * k, 0);
  v[0] = 1;  // row 0: evaluation point 0
  for (unsigned r = 1; r < n; r++)
    for (unsigned c = 0; c < k; c++)
      v[static_cast<size_t>(r) * k + c] = g.exp[((r - 1) * c) % 255];
  std::vector<uint8_t> top(v.begin(), v.begin() + static_cast<size_t>(k) * k);
  gf_invert(top, k);  // Vandermonde on distinct points: never singular
  std::vector<uint8_t> enc(static_cast<size_t>(n) * k, 0);
  for (unsigned i = 0; i < k; i++) enc[static_cast<size_t>(i) * k + i] = 1;
  for (unsigned r = k; r < n; r++)
    for (unsigned c = 0; c < k; c++) {
      uint8_t acc = 0;
      for (unsigned t = 0; t < k; t++)
        acc ^= g.mul(v[static_cast<size_t>(r) * k + t],
                     top[static_cast<size_t>(t) * k + c]);
      enc[static_cast<size_t>(r) * k + c] = acc;
    }
  return enc;
}

// Nibble-split product tables for v_perm_b32: c*x = T0[x&7] ^ T1[(x>>3)&7]
// ^ T2[x>>6] (multiplication by c is GF(2)-linear in x). T0/T1 hold 8
// entries (two dwords, selector 0..3 -> low dword, 4..7 -> high dword),
// T2 holds 4 entries (one dword).
struct alignas(32) PermTab {
  uint32_t t0lo, t0hi, t1lo, t1hi, t2, pad0, pad1, pad2;
};

inline PermTab perm_tab(uint8_t c) {
  const GF256 &g = gf();
  auto pack = [&](unsigned step, unsigned first) {
    uint32_t w = 0;
    for (unsigned b = 0; b < 4; b++)
      w |= static_cast<uint32_t>(g.mul(c, static_cast<uint8_t>((first + b) * step)))
           << (8 * b);
    return w;
  };
  PermTab t{};
  t.t0lo = pack(1, 0);
  t.t0hi = pack(1, 4);
  t.t1lo = pack(8, 0);
  t.t1hi = pack(8, 4);
  t.t2 = pack(64, 0);
  return t;
}

}  // namespace storb_rs
