// rs_bitslice.hip -- instantiations of the bit-sliced encoders
// (rs_bitslice.hpp) for Storb's wide full-chunk geometries.
#include "rs_bitslice.hpp"

namespace storb_rs {

hipError_t launch_encode_bitslice_64_96(const ApplyArgs &a, hipStream_t s);  // rs_bitslice64.hip

bool bitslice_supported(uint32_t k, uint32_t n) {
  return (k == 16 && n == 24) || (k == 32 && n == 48) || (k == 64 && n == 96);
}

hipError_t launch_encode_bitslice(const ApplyArgs &a, uint32_t n, hipStream_t s) {
  if (a.r != n - a.k || !vector_ok(a)) return hipErrorInvalidValue;
  // (The row-split form measured equal for (16, 24) and within noise for
  // (32, 48) in the product, profiles/r2_k64/split_aot_k16_k32_ab.txt: one
  // wave per tile stays.)
  if (a.k == 16 && n == 24) return bs::launch_bitslice<16, 24>(a, s);
  if (a.k == 32 && n == 48) return bs::launch_bitslice<32, 48>(a, s);
  if (a.k == 64 && n == 96) return launch_encode_bitslice_64_96(a, s);
  return hipErrorInvalidValue;
}

uint32_t bitslice_stream_cols_per_tile(uint32_t k, uint32_t n) {
  if (k == 16 && n == 24) return static_cast<uint32_t>(bs::BsTune<16, 24>::CPT);
  if (k == 32 && n == 48) return static_cast<uint32_t>(bs::BsTune<32, 48>::CPT);
  return 0;
}

hipError_t launch_encode_bitslice_stream(const ApplyArgs &a, uint32_t n, const StreamArgs &st,
                                         hipStream_t s) {
  const uint32_t cpt = bitslice_stream_cols_per_tile(a.k, n);
  if (!cpt || a.r != n - a.k || a.nstripes != 1 || !vector_ok(a) || st.slice_cols == 0 ||
      st.slice_cols % cpt || st.nslices == 0 || st.nslices > kMaxStreamSlices ||
      static_cast<uint64_t>(st.slice_cols) * st.nslices < (a.block >> 4))
    return hipErrorInvalidValue;
  if (a.k == 16) return bs::launch_bitslice_stream<16, 24>(a, st, s);
  return bs::launch_bitslice_stream<32, 48>(a, st, s);
}

}  // namespace storb_rs
