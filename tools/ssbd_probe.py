#!/usr/bin/env python3
"""Is the slow CPU baseline Speculative Store Bypass Disable? Runs the CPU
baseline loop (oracle/cpu_bench.c, RS(4,2) encode + decode of 1 MiB chunks)
on this thread as it is, then again after turning SSBD on for this thread
only (prctl PR_SET_SPECULATION_CTRL / PR_SPEC_STORE_BYPASS / PR_SPEC_DISABLE:
the mitigation, i.e. stricter, never looser; it cannot be undone for the
thread, so this runs in its own process). Prints one JSON line per state:
GiB/s, IPC, effective clock, the L1-resident addmul probe and the thread's
/proc status line. (Test infrastructure: the oracle is the workload here.)

    python tools/ssbd_probe.py [--seconds 3]
"""
import argparse
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from oracle import coracle  # noqa: E402

PR_GET_SPECULATION_CTRL, PR_SET_SPECULATION_CTRL = 52, 53
PR_SPEC_STORE_BYPASS, PR_SPEC_DISABLE = 0, 4


def status():
    for line in open("/proc/thread-self/status"):
        if line.startswith("Speculation_Store_Bypass"):
            return line.split(":", 1)[1].strip()
    return None


def measure(seconds):
    k, n, L, ns = 4, 6, 1 << 20, 8
    data = np.frombuffer(np.random.default_rng(1).bytes(ns * L), dtype=np.uint8)
    r = coracle.bench_roundtrip(k, n, data, L, ns, [[2, 3, 4, 5]], True, True, True, seconds)
    return {"GiBps": round(2 * r["calls"] * L / (1 << 30) / r["wall_s"], 4),
            "ipc": round(r["instructions"] / r["cycles"], 3) if r["cycles"] > 0 else None,
            "effective_ghz": round(r["cycles"] / r["wall_s"] / 1e9, 3) if r["cycles"] > 0 else None,
            "l1_addmul_GBps": round(r["l1_addmul_gbs"], 2),
            "dram_read_GBps": round(r["dram_read_gbs"], 2),
            "ssb": status()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=3.0)
    a = ap.parse_args()
    libc = ctypes.CDLL(None, use_errno=True)
    host = {}
    for line in open("/proc/cpuinfo"):
        if line.startswith(("model name", "microcode")):
            host[line.split(":")[0].strip()] = line.split(":", 1)[1].strip()
        if len(host) == 2:
            break
    print(json.dumps({"host": host}), flush=True)
    print(json.dumps({"state": "as started", **measure(a.seconds)}), flush=True)
    rc = libc.prctl(PR_SET_SPECULATION_CTRL, PR_SPEC_STORE_BYPASS, PR_SPEC_DISABLE, 0, 0)
    err = ctypes.get_errno()
    print(json.dumps({"state": "SSBD on for this thread", "prctl_rc": rc, "errno": err,
                      **measure(a.seconds)}), flush=True)


if __name__ == "__main__":
    main()
