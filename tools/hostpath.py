"""Host-in/host-out encode rate (storb_rs_encode_chunks) vs host copy threads.

Pageable host chunks -> pinned staging -> H2D -> encode -> D2H -> caller's
parity buffer; the number DESIGN.md reports as "PCIe-inclusive". Each
setting gets a fresh context (the copy pool reads STORB_RS_HOST_THREADS when
it is created). Output: one JSON line per (geometry, threads).
"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from storb_amd import _lib  # noqa: E402

GIB = 1 << 30


def rate(k, n, chunk, nchunks, threads, reps=4):
    os.environ["STORB_RS_HOST_THREADS"] = str(threads)
    ctx = _lib.Context(0)
    host = np.frombuffer(np.random.default_rng(7).bytes(nchunks * chunk), dtype=np.uint8).copy()
    out = np.zeros(nchunks * (n - k) * (-(-chunk // k)), np.uint8)  # touched before timing
    ctx.encode_chunks(k, n, host, chunk, nchunks, out=out)  # warm: staging, pool, tables
    t0 = time.perf_counter()
    for _ in range(reps):
        ctx.encode_chunks(k, n, host, chunk, nchunks, out=out)
    el = time.perf_counter() - t0
    ctx.close()
    return reps * nchunks * chunk / GIB / el


def main():
    for k, n, chunk in [(4, 6, 1 << 20), (16, 24, 8 << 20)]:
        nchunks = max(8, (512 << 20) // chunk)
        for t in (1, 2, 4, 8, 16):
            r = rate(k, n, chunk, nchunks, t)
            print(json.dumps({"k": k, "n": n, "chunk": chunk, "nchunks": nchunks,
                              "host_threads": t, "GiB_per_s_input": round(r, 2)}), flush=True)


if __name__ == "__main__":
    main()
