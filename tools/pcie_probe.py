"""PCIe ceiling for the host path: pinned H2D alone, D2H alone, and both
directions at once (the shape storb_rs_encode_chunks drives: 1 byte in and
(n-k)/k bytes out per user byte). Prints one JSON line.

    python tools/pcie_probe.py [--mib 256] [--reps 5]
"""
import argparse
import json
import time

import torch

GIB = float(1 << 30)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--mib", type=int, default=256)
    p.add_argument("--reps", type=int, default=5)
    a = p.parse_args()
    n = a.mib << 20
    h_in = torch.empty(n, dtype=torch.uint8).pin_memory()
    h_out = torch.empty(n // 2, dtype=torch.uint8).pin_memory()
    d_in = torch.empty(n, dtype=torch.uint8, device="cuda")
    d_out = torch.empty(n // 2, dtype=torch.uint8, device="cuda")
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    res = {}

    def timed(name, fn, nbytes):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.reps):
            fn()
        torch.cuda.synchronize()
        res[name] = round(nbytes * a.reps / (time.perf_counter() - t0) / 1e9, 2)

    def h2d():
        with torch.cuda.stream(s1):
            d_in.copy_(h_in, non_blocking=True)

    def d2h():
        with torch.cuda.stream(s2):
            h_out.copy_(d_out, non_blocking=True)

    def both():
        h2d()
        d2h()

    timed("h2d_GBps", h2d, n)
    timed("d2h_GBps", d2h, n // 2)
    timed("duplex_GBps_total", both, n + n // 2)
    # the same chopped into 64 MiB pieces on two streams, like the pipeline
    piece = 64 << 20

    def chopped():
        for i in range(0, n, piece):
            s = s1 if (i // piece) % 2 == 0 else s2
            with torch.cuda.stream(s):
                d_in[i:i + piece].copy_(h_in[i:i + piece], non_blocking=True)
                o = i // 2
                h_out[o:o + piece // 2].copy_(d_out[o:o + piece // 2], non_blocking=True)

    timed("chopped_duplex_GBps_total", chopped, n + n // 2)
    res["user_GiBps_if_h2d_bound"] = round(res["duplex_GBps_total"] * 1e9 / 1.5 / GIB, 2)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
