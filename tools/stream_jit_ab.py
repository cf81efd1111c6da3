#!/usr/bin/env python3
"""A/B of the per-chunk decode with k > 16 (piece.rs:384-386 through the
shim's storb_rs_decode, pageable buffers, one thread pinned to the GPU's
NUMA node, output buffer reused): the matrix's compiled kernel in its
streamed form (one launch gated per slice, rs_jit.cpp try_launch_stream)
against the sliced path (the default: a launch and a stream-written flag
per slice). One JSON line per run.

usage: STORB_RS_JIT_STREAM=1|0 python tools/stream_jit_ab.py
"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from benchkit import cpu as bcpu  # noqa: E402
from oracle import coracle  # noqa: E402  (inputs and the check only)
from storb_amd import _lib  # noqa: E402

pin = bcpu.pin_rank(0, "numa")
pin.pop("allowed")
res = {"stream": os.environ.get("STORB_RS_JIT_STREAM", "0"), "pin": pin}
ctx = _lib.Context(0)
L = _lib.lib()
for (k, n, B, lost) in ((32, 48, 1 << 20, [0, 1]), (32, 48, 1 << 20, [3, 17, 30]),
                        (24, 36, 256 << 10, [0, 1])):
    data = np.frombuffer(np.random.default_rng(k).bytes(k * B), np.uint8).copy()
    shares, b, pad = coracle.encode(k, n, data)
    surv = [i for i in range(n) if i not in lost][:k]
    _lib.jit_prepare_decode(k, n, surv, False, True)
    sh = [np.ascontiguousarray(shares[i]) for i in surv]
    ptrs = (_lib.vp * k)(*[x.ctypes.data for x in sh])
    ids = (_lib.C.c_uint32 * k)(*surv)
    out = np.zeros(k * B, np.uint8)

    def call():
        rc = L.storb_rs_decode(ctx.handle, k, n, ptrs, ids, k, b, pad, out.ctypes.data)
        if rc:
            raise SystemExit(f"storb_rs_decode rc {rc}")

    call()
    assert np.array_equal(out, data)
    lat = []
    for _ in range(60):
        t = time.perf_counter_ns()
        call()
        lat.append(time.perf_counter_ns() - t)
    lat.sort()
    res[f"k{k}_n{n}_lost{len(lost)}_B{B >> 10}K"] = {
        "median_us": round(lat[30] / 1e3, 1), "p10_us": round(lat[6] / 1e3, 1),
        "GiBps": round(k * B / 2**30 / (lat[30] * 1e-9), 2)}
res["stats"] = ctx.stats()
print(json.dumps(res))
