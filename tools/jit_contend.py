#!/usr/bin/env python3
"""JIT compile progress inside a torch process (tools/jit_contend.cpp's
question, from Python): queue 16 k = 16 decode patterns
(jit_prepare_decode, no wait), then for 10 s either sleep, run torch ops
(copy_, zero_, torch.equal -- what tools/jit_fuzz.py's loop does around its
decodes), or call decode_batch_dev back to back, printing the compile count
every 2 s. usage (GPU box): python tools/jit_contend.py idle|torch|decode [seed]"""
import os
import sys
import time

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

from storb_amd import _lib  # noqa: E402


def main():
    mode = sys.argv[1]
    seed = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    k, n, B, ns = 16, 24, 64 << 10, 4
    ctx = _lib.Context(0)
    ref = torch.randint(0, 255, (ns * k * B,), dtype=torch.uint8, device="cuda:0")
    par = torch.zeros(ns * (n - k) * B, dtype=torch.uint8, device="cuda:0")
    data = torch.empty_like(ref)
    for q in range(16):
        lost = {(q + seed) % 16, (q * 5 + 3 + seed) % 16, (q * 11 + 7 + seed) % 16}
        surv = [i for i in range(n) if i not in lost][:k]
        _lib.jit_prepare_decode(k, n, surv, assemble=False, wait=False)
    t0 = time.perf_counter()
    last, calls = -2.0, 0
    surv = list(range(2, 18))
    while True:
        if mode == "torch":
            data.copy_(ref)
            data[:B].zero_()
            torch.equal(data, ref)
        elif mode == "decode":
            ctx.decode_batch_dev(k, n, B, ns, surv, data.data_ptr(), par.data_ptr(), data.data_ptr(),
                                 stream=torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()
        else:
            time.sleep(0.001)
        calls += 1
        el = time.perf_counter() - t0
        if el - last >= 2.0:
            last = el
            st = _lib.jit_stats()
            print(f"{mode} t={el:.1f} calls={calls} compiled={st['compiled']} pending={st['pending']}",
                  flush=True)
        if el > 10:
            break
    ctx.close()


if __name__ == "__main__":
    main()
