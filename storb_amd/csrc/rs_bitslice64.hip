// rs_bitslice64.hip -- the bit-sliced encoder for Storb's widest geometry,
// (k, n) = (64, 96): chunks of 128-256 MiB, objects from ~160 GiB
// (piece.rs:292-317). Its 32 parity rows run as one row-split launch
// (rs_bitslice_core.h bs_split_body). Built ahead of time so the first
// encode of a process does not wait for (or fall back during) a ~5-10 s
// run-time compile. Its own translation unit: the constexpr generator needs
// a raised -fconstexpr-steps (Makefile) and the build runs in parallel.
#include "rs_bitslice.hpp"

namespace storb_rs {

hipError_t launch_encode_bitslice_64_96(const ApplyArgs &a, hipStream_t s) {
  return bs::launch_bitslice<64, 96>(a, s);
}

}  // namespace storb_rs
