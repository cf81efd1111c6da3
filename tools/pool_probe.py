#!/usr/bin/env python3
"""Stream-ordered pool accounting around a context's table cache.

The table cache allocates each coefficient matrix's device tables with
hipMallocAsync (the device's default memory pool). Until round 3 context
teardown released them with a plain hipFree, which is not the pool's free.
This creates tables (distinct decode patterns on the table kernel), destroys
the context and reads the default pool's used / reserved bytes
(hipMemPoolGetAttribute) -- no kernel touches freed memory, so a pool that
still counts the tables as used shows up as a number, not as a fault.

usage (GPU box): python tools/pool_probe.py [path/to/libstorb_rs.so]
"""
import ctypes as C
import json
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

from storb_amd import _lib  # noqa: E402


def hip_runtime():
    for line in open("/proc/self/maps"):
        if "libamdhip64" in line:
            return C.CDLL(line.split()[-1])
    raise SystemExit("libamdhip64 not loaded")


def main():
    if len(sys.argv) > 1:
        _lib.LIB_PATH = os.path.abspath(sys.argv[1])
    torch.zeros(1, device="cuda:0")
    hip = hip_runtime()
    pool = C.c_void_p()
    assert hip.hipDeviceGetDefaultMemPool(C.byref(pool), 0) == 0

    def attrs():
        out = {}
        for name, a in (("reserved", 0x5), ("used", 0x7)):
            v = C.c_uint64()
            rc = hip.hipMemPoolGetAttribute(pool, a, C.byref(v))
            out[name] = v.value if rc == 0 else f"rc {rc}"
        hip.hipGetLastError()
        return out

    rows = {"lib": _lib.LIB_PATH, "start": attrs()}
    k, n, B, ns = 8, 12, 4096, 4
    data = torch.zeros(ns * k * B, dtype=torch.uint8, device="cuda:0")
    par = torch.zeros(ns * (n - k) * B, dtype=torch.uint8, device="cuda:0")
    for round_ in range(3):
        ctx = _lib.Context(0)
        ctx.set_kernel(_lib.KERNEL_PERM)
        ctx.default_stream = torch.cuda.current_stream(0).cuda_stream
        pats = 0
        for a in range(n):
            for b in range(a + 1, n):
                surv = [i for i in range(n) if i not in (a, b)][:k]
                ctx.decode_batch_dev(k, n, B, ns, surv, data.data_ptr(), par.data_ptr(),
                                     data.data_ptr())
                pats += 1
        torch.cuda.synchronize()
        rows[f"round{round_}_with_{pats}_tables"] = attrs()
        ctx.close()
        torch.cuda.synchronize()
        rows[f"round{round_}_after_close"] = attrs()
    print(json.dumps(rows, indent=1))


if __name__ == "__main__":
    main()
