// PatternMemo (decode_stripes.cpp) against get_pattern, host only: random
// offered-share lists in arrival order -- with and without duplicates, short
// lists, out-of-range indices, n above the memo's 64 -- must give the same
// pattern, slot positions and error code. Links libstorb_rs.so; needs no GPU
// (the pattern cache and the selection are host code).
#include "../../storb_amd/csrc/ctx.hpp"

#include <algorithm>
#include <cstdio>
#include <random>

using namespace storb_rs::detail;

int main() {
  auto *ctx = new storb_rs_ctx;  // host fields only; never destroyed (no HIP here)
  std::mt19937 rng(20261018);
  const uint32_t geos[][2] = {{1, 1}, {1, 3}, {2, 3}, {4, 6}, {8, 12}, {16, 24}, {32, 48},
                              {10, 64}, {40, 64}, {5, 80}, {64, 96}};
  size_t checked = 0, errors = 0;
  for (auto &g : geos) {
    const uint32_t k = g[0], n = g[1];
    for (int call = 0; call < 20; call++) {
      PatternMemo memo(ctx, k, n);
      for (int st = 0; st < 200; st++) {
        std::vector<uint32_t> ids(n);
        for (uint32_t i = 0; i < n; i++) ids[i] = i;
        std::shuffle(ids.begin(), ids.end(), rng);
        uint32_t m = k + rng() % (n - k + 1);
        const int kind = rng() % 10;
        if (kind == 0 && m > 1) ids[m - 1] = ids[rng() % (m - 1)];  // a duplicate
        if (kind == 1) m = k ? rng() % k : 0;                         // too few
        if (kind == 2 && m) ids[rng() % m] = n + rng() % 3;         // out of range
        ids.resize(m);
        const Pattern *a = nullptr, *b = nullptr;
        std::vector<uint32_t> pa, pb;
        const int ra = memo.get(ids.data(), m, &a, pa);
        const int rb = get_pattern(ctx, k, n, ids.data(), m, &b, pb);
        if (ra != rb || (ra == 0 && (a != b || pa != pb))) {
          std::printf("MISMATCH k=%u n=%u call=%d stripe=%d rc %d/%d\n", k, n, call, st, ra, rb);
          return 1;
        }
        checked++;
        errors += ra != 0;
      }
    }
  }
  std::printf("pattern memo ok: %zu stripes, %zu error cases\n", checked, errors);
  return 0;
}
