// rs_lds.hip -- LDS product-table kernels (k <= 16, r <= 8), the measured
// comparison point for the register-table kernels.
#include "rs_device.hpp"

namespace storb_rs {
namespace {

template <int KM, int RM>
hipError_t go_lds(const ApplyArgs &a, hipStream_t s) {
  const uint64_t blocks = tile_blocks<KM>(a);
  if (blocks == 0) return hipSuccess;
  if (blocks > 0x7FFFFFFFull) return hipErrorInvalidConfiguration;
  const size_t lds = static_cast<size_t>(a.tab_rows) * a.k * 256;
  hipLaunchKernelGGL((rs_apply_lds<KM, RM>), dim3(blocks), dim3(kThreads), lds, s,
                     a);
  return hipGetLastError();
}

template <int KM>
hipError_t go_lds_r(const ApplyArgs &a, hipStream_t s) {
  switch (rows_bucket(a.r)) {
    case 1: return go_lds<KM, 1>(a, s);
    case 2: return go_lds<KM, 2>(a, s);
    case 3:
    case 4: return go_lds<KM, 4>(a, s);
    default: return go_lds<KM, 8>(a, s);
  }
}

}  // namespace

hipError_t dispatch_lds(const ApplyArgs &a, hipStream_t s) {
  switch (pow2_bucket(a.k)) {
    case 1: return go_lds_r<1>(a, s);
    case 2: return go_lds_r<2>(a, s);
    case 4: return go_lds_r<4>(a, s);
    case 8: return go_lds_r<8>(a, s);
    default: return go_lds_r<16>(a, s);
  }
}

}  // namespace storb_rs
