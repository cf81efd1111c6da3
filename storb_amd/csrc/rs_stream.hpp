// rs_stream.hpp -- the device half of the streamed single calls (StreamArgs,
// rs_args.h; host half: host_calls.cpp streamed): a workgroup waits for its
// slice's host-written ready word, and reports its slice's completion.
// Self-contained under hipRTC too: the run-time-compiled decode kernels'
// streamed form (rs_jit.cpp) includes it as an in-memory header.
#pragma once

#ifndef __HIPCC_RTC__
#include <hip/hip_runtime.h>
#endif

#include "rs_args.h"

namespace storb_rs {

// Lane 0 polls ready[16 * slice] (system scope, over PCIe) until it equals
// seq or timeout_ticks of s_memrealtime (100 MHz) have passed; the verdict
// is shared through LDS. True: the slice is packed, and the acquire makes
// the host's writes before the word visible to this workgroup's loads.
// False: give up (the workgroup must exit without writing).
__device__ __forceinline__ bool stream_gate(const StreamArgs &st, uint32_t slice) {
  __shared__ uint32_t go;
  if (threadIdx.x == 0) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    uint32_t ok = 1;
    while (__hip_atomic_load(st.ready + 16 * slice, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) !=
           st.seq) {
      __builtin_amdgcn_s_sleep(2);
      if (__builtin_amdgcn_s_memrealtime() - t0 > st.timeout_ticks) {
        ok = 0;
        break;
      }
    }
    go = ok;
  }
  __syncthreads();
  const bool ok = go != 0;
  if (ok) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  return ok;
}

// After the workgroup's stores: make every lane's stores complete and
// visible to the host, count the workgroup on its slice, and let the slice's
// last workgroup publish done[16 * slice] = seq.
__device__ __forceinline__ void stream_report(const StreamArgs &st, uint32_t slice) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t n = __hip_atomic_fetch_add(st.cnt + slice, 1u, __ATOMIC_ACQ_REL,
                                              __HIP_MEMORY_SCOPE_AGENT) + 1u;
    if (n == st.target[slice])
      __hip_atomic_store(st.done + 16 * slice, st.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

}  // namespace storb_rs
