// rs_stream.hip -- the streamed single-call kernels (rs_device.hpp
// rs_apply_stream; StreamArgs in rs_args.h): k <= 32 inputs, <= 8 rows, one
// stripe -- Storb's per-chunk calls through the zfec-rs shim: encode of the
// (2, 3), (4, 6), (8, 12) chunks of objects up to ~256 MiB and decode of
// every geometry up to k = 32 with up to 8 lost data shares
// (piece.rs:307-317); over PCIe the table kernel is nowhere near VALU-bound.
#include "rs_device.hpp"

namespace storb_rs {

hipError_t launch_apply_stream(const ApplyArgs &a, const StreamArgs &st, hipStream_t s) {
  if (a.k == 0 || a.k > kSlotK || a.r == 0 || a.r > 8 || a.nstripes != 1 || a.ncopy ||
      a.accumulate || !vector_ok(a) || st.slice_cols == 0 || st.slice_cols % kThreads ||
      st.nslices == 0 || st.nslices > kMaxStreamSlices ||
      static_cast<uint64_t>(st.slice_cols) * st.nslices < (a.block >> 4) ||
      a.tab_rows != static_cast<uint32_t>(rows_bucket(a.r)))
    return hipErrorInvalidValue;
  switch (pow2_bucket(a.k)) {
    case 1:
    case 2: return go_stream_r<2>(a, st, s);
    case 4: return go_stream_r<4>(a, st, s);
    case 8: return go_stream_r<8>(a, st, s);
    case 16: return go_stream_r<16>(a, st, s);
    default: return go_stream_r<32>(a, st, s);
  }
}

}  // namespace storb_rs
