#!/usr/bin/env python3
"""Storb's (2, 3) geometry on the device-resident batch calls (the <2,1>
table-kernel bucket): encode of 4096 x 256 KiB chunks and the in-place decode
of data share 0 from shares {1, 2}, timed with HIP events over back-to-back
calls. With AB_K / AB_LOST (env): (k, 1.5 k) chunks of k x 128 KiB... with the
first AB_LOST data shares rebuilt in place (e.g. AB_K=8 AB_LOST=2: the <8,2>
bucket, Storb's (8, 12) geometry). usage: python tools/ab21.py
[path/to/libstorb_rs.so]  (one JSON line; A/B of library builds with
tools/build_variant.sh)"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from storb_amd import _lib  # noqa: E402

if len(sys.argv) > 1:
    _lib.LIB_PATH = os.path.abspath(sys.argv[1])
import torch  # noqa: E402

k = int(os.environ.get("AB_K", "2"))
lost = int(os.environ.get("AB_LOST", "1"))
n, B, reps = k + (k + 1) // 2, 128 << 10, 50
ns = 4096 * 2 // k
dev = torch.device("cuda:0")
data = torch.randint(0, 256, (ns * k * B,), dtype=torch.uint8, device=dev)
par = torch.empty(ns * (n - k) * B, dtype=torch.uint8, device=dev)
ctx = _lib.Context(0)
s = torch.cuda.current_stream(dev)
ctx.default_stream = s.cuda_stream
ref = data.clone()


def enc():
    ctx.encode_batch_dev(k, n, B, ns, data.data_ptr(), par.data_ptr())


surv = list(range(lost, k + lost))  # the first k by index with data shares 0..lost-1 gone


def dec():  # data shares 0..lost-1 rebuilt in place from the next k shares
    ctx.decode_batch_dev(k, n, B, ns, surv, data.data_ptr(), par.data_ptr(), data.data_ptr())


out = {"geometry": f"({k}, {n})", "lost": lost, "chunks": ns, "chunk_bytes": k * B}
for name, fn, alg in (("encode", enc, ns * n * B), ("decode_in_place", dec, ns * (k + lost) * B)):
    for _ in range(10):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        fn()
    e1.record(s)
    e1.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / reps
    out[name] = {"us": round(us, 2), "frac_of_8TBps": round(alg / (us * 1e-6) / 8e12, 4)}
torch.cuda.synchronize()
out["decode_bit_exact"] = bool(torch.equal(data, ref))
print(json.dumps(out))
