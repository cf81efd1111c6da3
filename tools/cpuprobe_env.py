#!/usr/bin/env python3
"""Why the bench's single-thread CPU baseline reads 0.11 GiB/s on some GPU
boxes and 1.9 GiB/s on others: time the oracle's encode+decode of a 1 MiB
RS(4,2) chunk (bench.cpu_baseline's loop) in this process at stages --
before torch, after torch + CUDA init, after our context and a GPU bench
leg -- and print the rate with the process's thread count and CPU affinity.
Test infrastructure only (the oracle is the checker/baseline)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import coracle  # noqa: E402


def rate(tag, seconds=3.0):
    k, n, L = 4, 6, 1 << 20
    d = coracle.splitmix_bytes(0x5709B, L)
    surv = [2, 3, 4, 5]
    done, t0 = 0, time.perf_counter()
    c0 = time.process_time()
    while time.perf_counter() - t0 < seconds:
        sh, B, pad = coracle.encode(k, n, d)
        coracle.decode(k, n, [sh[s] for s in surv], surv, B, pad)
        done += 1
    el = time.perf_counter() - t0
    cpu = time.process_time() - c0
    print(json.dumps({"stage": tag, "GiBps": round(2 * done * L / 2**30 / el, 3),
                      "iters": done, "wall_s": round(el, 2), "process_cpu_s": round(cpu, 2),
                      "threads": len(os.listdir("/proc/self/task")),
                      "affinity": len(os.sched_getaffinity(0))}), flush=True)


rate("fresh")
import torch  # noqa: E402
rate("torch imported")
torch.cuda.init()
x = torch.ones(1 << 20, device="cuda")
torch.cuda.synchronize()
rate("cuda initialised")
from storb_amd import _lib  # noqa: E402
ctx = _lib.Context(0)
data = torch.zeros(1024 * (1 << 20), dtype=torch.uint8, device="cuda")
par = torch.zeros(512 * (1 << 20), dtype=torch.uint8, device="cuda")
for _ in range(20):
    ctx.encode_batch_dev(4, 6, 256 << 10, 1024, data.data_ptr(), par.data_ptr())
ctx.sync()
rate("after storb ctx + 20 encodes")
torch.set_num_threads(1)
rate("torch threads = 1")
