#!/usr/bin/env python3
"""Encode + piece ids at Storb's wide geometries: the
device-resident storb_rs_encode_hashed_dev against encode alone, digests
checked against the host blake3 of a few shares. (Round 5 also timed
pipelining and concurrency settings here, knobs since removed:
profiles/r5d_widehash_pipelining.jsonl, profiles/r5i_widehash.jsonl.)

usage: python tools/widehash.py [--reps 10]
prints one JSON line per geometry.
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from storb_amd import _lib  # noqa: E402

GEOMS = [  # (k, n, B, stripes): Storb's sizing of 8 MiB / 32 MiB / 4 MiB chunks
    (16, 24, 512 << 10, 128),
    (32, 48, 1 << 20, 32),
    (8, 12, 512 << 10, 256),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    st = torch.cuda.Stream(device=dev)
    sp = st.cuda_stream
    settings = [None]
    for k, n, B, ns in GEOMS:
        data = torch.empty(ns * k * B, dtype=torch.uint8, device=dev)
        par = torch.empty(ns * (n - k) * B, dtype=torch.uint8, device=dev)
        hashes = torch.empty(ns * n * 32, dtype=torch.uint8, device=dev)
        ref = None
        for sset in settings:
            ctx = _lib.Context(0)
            ctx.fill_splitmix_dev(data.data_ptr(), k * B, ns, k * B, 0x5709B, stream=sp)

            def enc():
                ctx.encode_batch_dev(k, n, B, ns, data.data_ptr(), par.data_ptr(), stream=sp)

            def eh():
                ctx.encode_hashed_dev(k, n, B, ns, data.data_ptr(), par.data_ptr(),
                                      hashes.data_ptr(), stream=sp)

            res = {"k": k, "n": n, "B": B, "stripes": ns, "setting": sset or "sequential"}
            for name, f in (("encode", enc), ("encode_hashed", eh)):
                for _ in range(3):
                    f()
                st.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                for _ in range(a.reps):
                    f()
                e1.record(st)
                st.synchronize()
                res[name + "_ms"] = round(e0.elapsed_time(e1) / a.reps, 4)
            h = hashes.cpu().numpy().reshape(ns, n, 32)
            if ref is None:
                ref = h.copy()
                d = data.cpu().numpy().reshape(ns, k, B)
                p = par.cpu().numpy().reshape(ns, n - k, B)
                for s_, t in ((0, 0), (ns - 1, k - 1), (ns // 2, k), (ns - 1, n - 1)):
                    src = d[s_, t] if t < k else p[s_, t - k]
                    assert _lib.blake3(src.tobytes()) == h[s_, t].tobytes(), (s_, t)
                res["host_blake3_check"] = "ok"
            else:
                res["same_digests"] = bool(np.array_equal(h, ref))
            res["ratio_vs_sequential"] = None
            ctx.close()
            print(json.dumps(res), flush=True)
        del data, par, hashes
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
