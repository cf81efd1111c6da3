#!/usr/bin/env python3
"""The per-chunk drop-in calls (benchkit/host.py shim_path_rate) for one library
setting per process -- STORB_RS_HOST_THREADS is read at context creation:
  STORB_RS_HOST_THREADS=16 python tools/shimpath.py
  python tools/shimpath.py --lib path/to/libstorb_rs.so   (another build, for an A/B)
prints one JSON line: median us per call for each geometry."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

import torch  # noqa: E402,F401  (HIP runtime before the library)

from benchkit import host as bhost  # noqa: E402
from storb_amd import _lib  # noqa: E402


def main():
    if len(sys.argv) > 2 and sys.argv[1] == "--lib":
        _lib.LIB_PATH = os.path.abspath(sys.argv[2])
    ctx = _lib.Context(0)
    r = bhost.shim_path_rate(ctx, seconds=0.6)
    out = {"lib": _lib.LIB_PATH, "threads": os.environ.get("STORB_RS_HOST_THREADS"),
           "rows": [{"k": g["k"], "m": g["m_total"],
                     **{x: g[x]["median_us"] for x in ("encode_call", "encode_shim", "decode_call",
                                                       "decode_shim")}}
                    for g in r["geometries"]]}
    print(json.dumps(out), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
