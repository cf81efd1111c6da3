// seq.hpp -- sequence numbers of the host-written / device-written words the
// single calls synchronise on (host_calls.cpp slice_signal / streamed).
//
// The words are zero-filled when created and compared for equality with the
// call's sequence number. A counter that wrapped to 0 would hand out the one
// value a never-written word already holds: a slice gate would open before
// the host had packed the slice, and the host would unpack before the kernel
// had written it. So 0 is never handed out.
#pragma once

#include <cstdint>

namespace storb_rs {

inline uint32_t next_seq(uint32_t &counter) {
  if (++counter == 0) ++counter;
  return counter;
}

}  // namespace storb_rs
