#!/usr/bin/env python3
"""Host-inclusive batch decode (storb_rs_decode_chunks) with a fixed survivor
set vs Storb's download survivor sets (first k + 1 pieces to arrive), from
pageable and page-locked shares: per-call time, the context's device-sync
and table counters and the JIT counters around the timed calls -- to find
where the download-pattern calls lose time. One JSON line per (geometry, mode,
pattern).
usage: python tools/dl_decode_probe.py [--k 16 --n 24 --chunk 8388608 --chunks 32]"""
import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

import torch  # noqa: E402,F401  (HIP runtime before the library)
import numpy as np  # noqa: E402

from benchkit import GIB, SEED_BASE, cpu as bcpu, device as bdev  # noqa: E402
from storb_amd import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=16)
    ap.add_argument("--n", type=int, default=24)
    ap.add_argument("--chunk", type=int, default=8 << 20)
    ap.add_argument("--chunks", type=int, default=32)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    pin = bcpu.pin_rank(0)
    pin.pop("allowed")
    ctx = _lib.Context(0)
    k, n, L, N = a.k, a.n, a.chunk, a.chunks
    B = -(-L // k)
    fixed = [i for i in range(n) if i not in (0, 1)][:k]
    sets = bdev.download_sets(k, n, 64, SEED_BASE + 4343)
    for mode in ("pageable", "pinned"):
        bufs = []
        if mode == "pinned":
            bufs = [_lib.PinnedBuffer(N * L), _lib.PinnedBuffer(N * (n - k) * B), _lib.PinnedBuffer(N * L)]
            host, par, rec = (b.array for b in bufs)
            rec = rec.reshape(N, L)
        else:
            host, par, rec = np.empty(N * L, np.uint8), np.empty(N * (n - k) * B, np.uint8), np.empty((N, L), np.uint8)
        host[:] = np.frombuffer(np.random.default_rng(7).bytes(host.size), dtype=np.uint8)
        par[:] = 0
        rec[:] = 0
        ctx.encode_chunks(k, n, host, L, N, out=par)
        dat, pv = host.reshape(N, k, B), par.reshape(N, n - k, B)
        for pname in ("fixed", "download"):
            ids_of = (lambda c: fixed) if pname == "fixed" else (lambda c: sets[c % len(sets)])
            chunks = [([dat[c, i] if i < k else pv[c, i - k] for i in ids_of(c)], ids_of(c)) for c in range(N)]
            ctx.decode_chunks(k, n, B, 0, chunks, out=rec)
            assert np.array_equal(rec.reshape(-1), host), (mode, pname)
            mp, mi, mc, keep = _lib.marshal_chunks(chunks, B)
            s0, j0 = ctx.stats(), _lib.jit_stats()
            ts = []
            for _ in range(a.reps):
                t0 = time.perf_counter()
                ctx.decode_chunks_raw(k, n, B, 0, mp, mi, mc, rec)
                ts.append(time.perf_counter() - t0)
            s1, j1 = ctx.stats(), _lib.jit_stats()
            lost = [len([j for j in range(k) if j not in sorted(ids_of(c))[:k]]) for c in range(N)]
            print(json.dumps({"k": k, "n": n, "chunk": L, "chunks": N, "mode": mode, "pattern": pname,
                              "ms": [round(t * 1e3, 3) for t in ts],
                              "GiBps_best": round(N * L / GIB / min(ts), 2),
                              "GiBps_median": round(N * L / GIB / sorted(ts)[len(ts) // 2], 2),
                              "lost_hist": {x: lost.count(x) for x in sorted(set(lost))},
                              "device_syncs": s1["device_syncs"] - s0["device_syncs"],
                              "tables": s1["tables"],
                              "jit": {x: j1[x] - j0[x] for x in ("compiled", "launches", "fallbacks", "pending")}}),
                  flush=True)
            del keep
        for b in bufs:
            b.free()
    ctx.close()


if __name__ == "__main__":
    main()
