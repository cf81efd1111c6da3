#!/usr/bin/env python3
"""Host-in/host-out batch decode (storb_rs_decode_chunks) and encode rates vs
host copy threads (STORB_RS_HOST_THREADS is read when a context creates its
copy pool, so each setting runs in its own process). One JSON line per run.

usage: python tools/hostpath_decode.py THREADS
"""
import json
import os
import sys
import time

import numpy as np
import torch  # noqa: F401  (HIP runtime order, see storb_amd/_lib.py)

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from storb_amd import _lib  # noqa: E402

GIB = float(1 << 30)


def main():
    threads = int(sys.argv[1])
    os.environ["STORB_RS_HOST_THREADS"] = str(threads)
    ctx = _lib.Context(0)
    out = {"threads": threads}
    for k, n, L, nch in [(4, 6, 1 << 20, 256), (16, 24, 8 << 20, 32)]:
        B = L // k
        host = np.frombuffer(np.random.default_rng(k).bytes(nch * L), np.uint8).copy()
        par = ctx.encode_chunks(k, n, host, L, nch)
        t0 = time.perf_counter()
        for _ in range(3):
            ctx.encode_chunks(k, n, host, L, nch, out=par)
        enc = 3 * nch * L / GIB / (time.perf_counter() - t0)
        surv = [i for i in range(n) if i not in (0, 1)][:k]
        dat, pv = host.reshape(nch, k, B), par.reshape(nch, n - k, B)
        chunks = [([dat[c, i] if i < k else pv[c, i - k] for i in surv], surv) for c in range(nch)]
        rec = np.empty((nch, L), np.uint8)
        ctx.decode_chunks(k, n, B, 0, chunks, out=rec)
        assert np.array_equal(rec.reshape(-1), host)
        t0 = time.perf_counter()
        for _ in range(3):
            ctx.decode_chunks(k, n, B, 0, chunks, out=rec)
        dec = 3 * nch * L / GIB / (time.perf_counter() - t0)
        out[f"k{k}"] = {"encode_GiBps": round(enc, 2), "decode_GiBps": round(dec, 2)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
