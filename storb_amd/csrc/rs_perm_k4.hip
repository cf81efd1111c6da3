// rs_perm_k4.hip -- register-table kernels for k <= 4 input slots
// (one translation unit per k bucket so they compile in parallel).
#include "rs_device.hpp"

namespace storb_rs {
hipError_t dispatch_perm_k4(const ApplyArgs &a, hipStream_t s) {
  return go_perm_r<4>(a, s);
}
hipError_t dispatch_desc_k4(const DescArgs &a, hipStream_t s) {
  return go_desc_r<4>(a, s);
}
}  // namespace storb_rs
