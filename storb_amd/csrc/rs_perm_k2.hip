// rs_perm_k2.hip -- register-table kernels for k <= 2 input slots
// (one translation unit per k bucket so they compile in parallel).
#include "rs_device.hpp"

namespace storb_rs {
hipError_t dispatch_perm_k2(const ApplyArgs &a, hipStream_t s) {
  return go_perm_r<2>(a, s);
}
hipError_t dispatch_desc_k2(const DescArgs &a, hipStream_t s) {
  return go_desc_r<2>(a, s);
}
}  // namespace storb_rs
