#!/usr/bin/env python3
"""Host-side latency of device-resident decode calls, new vs cached erasure
patterns (a new pattern used to hipMalloc + upload its
tables and then hipStreamSynchronize, blocking the caller until everything
already queued on the stream had finished).

For each geometry: queue ~2 ms of encodes on the stream, then issue decode
calls (storb_rs_decode_batch_dev) with never-seen survivor sets and time how
long each call takes to RETURN (host µs; the kernels run later). Then the same
with one cached pattern. A blocking call would take ~the queued GPU time.
Output: one JSON line per geometry.

usage: python tools/pattern_latency.py  (on a GPU box)
"""
import itertools
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from storb_amd import _lib  # noqa: E402


def main():
    dev = "cuda:0"
    ctx = _lib.Context(0)
    st = torch.cuda.Stream(device=dev)
    sp = st.cuda_stream
    for k, n, B, ns in [(4, 6, 1 << 20, 64), (8, 12, 256 << 10, 256), (16, 24, 512 << 10, 16)]:
        d = torch.empty(ns * k * B, dtype=torch.uint8, device=dev)
        p = torch.empty(ns * (n - k) * B, dtype=torch.uint8, device=dev)
        o = torch.empty_like(d)
        ctx.fill_splitmix_dev(d.data_ptr(), k * B, ns, k * B, 1, stream=sp)
        ctx.encode_batch_dev(k, n, B, ns, d.data_ptr(), p.data_ptr(), stream=sp)
        st.synchronize()
        pats = [list(c) for c in itertools.combinations(range(n), k) if list(c) != list(range(k))]
        res = {"k": k, "n": n, "block": B, "stripes": ns}
        for name, seq in (("new_pattern", pats[:40]), ("cached_pattern", [pats[0]] * 40)):
            times = []
            for surv in seq:
                big = torch.empty(256 << 20, dtype=torch.uint8, device=dev)
                with torch.cuda.stream(st):
                    big.fill_(1)  # ~0.1 ms of queued work ahead of the call
                    for _ in range(4):
                        big.add_(1)
                t0 = time.perf_counter()
                ctx.decode_batch_dev(k, n, B, ns, surv, d.data_ptr(), p.data_ptr(), o.data_ptr(),
                                     stream=sp)
                times.append((time.perf_counter() - t0) * 1e6)
                busy = not st.query()
                st.synchronize()
                if not torch.equal(o, d):
                    raise SystemExit(f"decode mismatch {k},{n} {surv}")
                times[-1] = (times[-1], busy)
            us = [t for t, _ in times]
            res[name] = {"calls": len(us), "median_us": round(statistics.median(us), 1),
                         "max_us": round(max(us), 1),
                         "stream_still_busy_after_return": sum(b for _, b in times)}
        print(json.dumps(res), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
