#!/usr/bin/env python3
"""Host-in / host-out batch encode and decode rates (storb_rs_encode_chunks,
storb_rs_decode_chunks) for one library setting per process: the settings
are environment variables the library reads at context creation
(STORB_RS_ZC_BATCH, STORB_RS_HOST_THREADS), so run one process per setting.
Also the box's PCIe copy rates (bench.py pcie_ceiling) for reference.

usage: STORB_RS_ZC_BATCH=0 python tools/hostpath.py [--k 4 --n 6 --chunk 1048576 --chunks 256]
       [--lib path/to/libstorb_rs.so]   (another build, for an A/B in one session)
prints one JSON line.
"""
import argparse
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

import torch  # noqa: E402,F401  (HIP runtime before the library, storb_amd/_lib.py)

from benchkit import SEED_BASE, cpu as bcpu, device as bdev, host as bhost  # noqa: E402
from storb_amd import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=4)
    ap.add_argument("--n", type=int, default=6)
    ap.add_argument("--chunk", type=int, default=1 << 20)
    ap.add_argument("--chunks", type=int, default=256)
    ap.add_argument("--lib", default=None)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    if a.lib:
        _lib.LIB_PATH = os.path.abspath(a.lib)
    pin = bcpu.pin_rank(0)  # as bench.py: onto the GPU's NUMA node first
    pin.pop("allowed")
    ctx = _lib.Context(0)
    erased = [0] if a.n > a.k else []
    r = bhost.host_path_rate(ctx, a.k, a.n, a.chunk, nchunks=a.chunks, reps=a.reps, erased=erased,
                             sets=bdev.download_sets(a.k, a.n, 64, SEED_BASE + 4343))
    r.pop("what", None)
    out = {"lib": a.lib, "reps": a.reps, "k": a.k, "n": a.n, "chunk": a.chunk, "chunks": a.chunks,
           "env": {x: os.environ.get(x) for x in ("STORB_RS_ZC_BATCH", "STORB_RS_HOST_THREADS")},
           "pin": pin,
           **r, "pcie": bhost.pcie_ceiling(torch.device("cuda", 0))}
    print(json.dumps(out), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
