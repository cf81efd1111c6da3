#!/usr/bin/env python3
"""JIT churn fuzz (VERDICT r2 'next' 7): many decode calls whose erasure
patterns follow a skewed (Zipf) draw from a large pool at k = 16, as a
download of many objects from a node with a few flaky miners sees them.

Every call decodes in place on the GPU (storb_rs_decode_batch_dev) and is
checked against the original bytes (the oracle's decode: MDS decoding of
k valid shares is unique; parity from the oracle's encode). Reports the JIT
counters: kernels compiled / loaded / evicted (loaded must stay <= the
STORB_RS_JIT_MAX this is run with), fallbacks and launches, and the
host-path decode rate (storb_rs_decode_chunks, one pattern) measured before
and while compiles run.

usage (GPU box): STORB_RS_JIT_MAX=32 python tools/jit_fuzz.py [calls] [pool]
"""
import json
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

from oracle import coracle  # noqa: E402  (checker: the parity the decodes start from)
from storb_amd import _lib  # noqa: E402


def host_rate(ctx, k, n, B, nch, shares, data):
    chunks = [([shares[c][i] for i in range(2, k + 2)], list(range(2, k + 2))) for c in range(nch)]
    out = np.empty((nch, k * B), np.uint8)
    ctx.decode_chunks(k, n, B, 0, chunks, out=out)
    t0 = time.perf_counter()
    ctx.decode_chunks(k, n, B, 0, chunks, out=out)
    el = time.perf_counter() - t0
    assert np.array_equal(out.reshape(-1), data[:nch * k * B])
    return nch * k * B / el / 2**30


def main():
    calls = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
    pool = int(sys.argv[2]) if len(sys.argv) > 2 else 2000
    k, n, B, ns = 16, 24, 64 << 10, 4          # 4.5 MiB per call: the JIT policy's batch floor
    rng = np.random.default_rng(2024)
    data_h = np.frombuffer(rng.bytes(ns * k * B), np.uint8).copy()
    par_h = coracle.encode_parity_many(k, n, data_h, k * B, ns, threads=8)
    ctx = _lib.Context(0)
    ref = torch.from_numpy(data_h).to("cuda:0")
    par = torch.from_numpy(par_h).to("cuda:0")
    data = torch.empty_like(ref)
    # pattern pool: 2..5 data shares lost, survivors the first k of the rest
    pats = []
    for _ in range(pool):
        e = int(rng.integers(2, 6))
        lost = sorted(rng.choice(k, size=e, replace=False).tolist())
        pats.append(([i for i in range(n) if i not in lost][:k], lost))
    w = 1.0 / np.arange(1, pool + 1) ** 1.1
    w /= w.sum()
    draws = rng.choice(pool, size=calls, p=w)
    # host path probe: 64 chunks of 1 MiB (k = 16), pageable shares, 2 lost
    hn = 64
    hdata = np.frombuffer(rng.bytes(hn * k * B), np.uint8).copy()
    hs = []
    for c in range(hn):
        sh = coracle.encode(k, n, hdata[c * k * B:(c + 1) * k * B])[0]
        hs.append([np.ascontiguousarray(sh[i]) for i in range(n)])
    before = host_rate(ctx, k, n, B, hn, hs, hdata)
    bad = 0
    during = []
    t0 = time.perf_counter()
    st0 = _lib.jit_stats()
    max_loaded = 0
    for ci, pi in enumerate(draws):
        surv, lost = pats[pi]
        data.copy_(ref)
        view = data.view(ns, k, B)
        for e in lost:
            view[:, e].zero_()
        ctx.decode_batch_dev(k, n, B, ns, surv, data.data_ptr(), par.data_ptr(), data.data_ptr(),
                             stream=torch.cuda.current_stream().cuda_stream)
        if not torch.equal(data, ref):
            bad += 1
        st = _lib.jit_stats()
        max_loaded = max(max_loaded, st["loaded"])
        if ci % 2000 == 1000 and st["pending"]:
            during.append(host_rate(ctx, k, n, B, hn, hs, hdata))
        if ci % 1000 == 0:
            print(json.dumps({"call": ci, "t": round(time.perf_counter() - t0, 2), "bad": bad, **st}),
                  flush=True)
    torch.cuda.synchronize()
    _lib.jit_wait()
    st = _lib.jit_stats()
    out = {"calls": calls, "pattern_pool": pool, "distinct_drawn": int(len(set(draws.tolist()))),
           "mismatches": bad, "seconds": round(time.perf_counter() - t0, 1),
           "jit_max": int(os.environ.get("STORB_RS_JIT_MAX", "256")), "max_loaded": max_loaded,
           "jit": {x: st[x] - st0[x] if x in ("compiled", "failed", "launches", "fallbacks",
                                              "evicted") else st[x] for x in st},
           "host_decode_GiBps_before": round(before, 2),
           "host_decode_GiBps_while_compiling": [round(x, 2) for x in during]}
    print(json.dumps(out), flush=True)
    ctx.close()
    return 1 if bad or max_loaded > out["jit_max"] else 0


if __name__ == "__main__":
    sys.exit(main())
