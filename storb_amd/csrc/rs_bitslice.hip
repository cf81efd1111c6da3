// rs_bitslice.hip -- instantiations of the bit-sliced encoders
// (rs_bitslice.hpp) for Storb's wide full-chunk geometries.
#include <cstdlib>

#include "rs_bitslice.hpp"

namespace storb_rs {

hipError_t launch_encode_bitslice_64_96(const ApplyArgs &a, hipStream_t s);  // rs_bitslice64.hip

bool bitslice_supported(uint32_t k, uint32_t n) {
  return (k == 16 && n == 24) || (k == 32 && n == 48) || (k == 64 && n == 96);
}

hipError_t launch_encode_bitslice(const ApplyArgs &a, uint32_t n, hipStream_t s) {
  if (a.r != n - a.k || !vector_ok(a)) return hipErrorInvalidValue;
  // STORB_RS_BS_SPLIT=1: the row-split form for (16, 24) / (32, 48) too (A/B
  // only: two waves of 4 / 8 rows sharing planes, 6 per CU).
  static const bool split = [] {
    const char *e = std::getenv("STORB_RS_BS_SPLIT");
    return e && e[0] == '1';
  }();
  if (split && a.k == 16 && n == 24) return bs::launch_bitslice_split<16, 24, 6>(a, s);
  if (split && a.k == 32 && n == 48) return bs::launch_bitslice_split<32, 48, 6>(a, s);
  if (a.k == 16 && n == 24) return bs::launch_bitslice<16, 24>(a, s);
  if (a.k == 32 && n == 48) return bs::launch_bitslice<32, 48>(a, s);
  if (a.k == 64 && n == 96) return launch_encode_bitslice_64_96(a, s);
  return hipErrorInvalidValue;
}

}  // namespace storb_rs
