#!/usr/bin/env python3
"""Throughput of the batched BLAKE3 shard-hashing kernel (storb piece ids).

Shapes: the shards of BASELINE config 2 (6144 x 256 KiB: 1024 RS(4,2)
chunks) and config 5 (3072 x 512 KiB: 128 RS(16,8) chunks of 8 MiB), plus
small shards. Reports GB/s of hashed bytes (HIP events, launch stream)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from storb_amd import _lib  # noqa: E402

ctx = _lib.Context(0)
s = torch.cuda.Stream()
res = []
for count, length in [(6144, 256 << 10), (3072, 512 << 10), (65536, 16 << 10), (1536, 1 << 20)]:
    buf = torch.empty(count * length, dtype=torch.uint8, device="cuda")
    out = torch.empty(count * 32, dtype=torch.uint8, device="cuda")
    ctx.fill_splitmix_dev(buf.data_ptr(), length, count, length, 1, stream=s.cuda_stream)
    go = lambda: ctx.blake3_batch_dev(buf.data_ptr(), length, count, length, out.data_ptr(),
                                      stream=s.cuda_stream)
    go()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(5):
        go()
    e1.record(s)
    e1.synchronize()
    ms = e0.elapsed_time(e1) / 5
    res.append({"shards": count, "shard_bytes": length, "ms": round(ms, 4),
                "GBps": round(count * length / ms / 1e6, 1)})
    print(json.dumps(res[-1]), flush=True)
