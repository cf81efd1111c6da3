#!/usr/bin/env python3
"""Turn rocprofv3 CSV output into the committed per-round summaries.

usage: summarize.py ROUND TRACE_DIR FETCH_DIR WRITE_DIR [--kernel SUBSTR]

* copies the --kernel-trace --stats summary to profiles/ROUND_kernel_stats.csv
* reduces the two PMC passes (FETCH_SIZE, WRITE_SIZE -- separate passes, the
  TCC block cannot hold both) to per-launch HBM bytes for the hot kernel and
  writes profiles/ROUND_pmc.json and profiles/pmc_traffic.json (read by
  bench.py for roofline.traffic).

gfx950 correction (MI355X_MICROARCH.md, HBM section): FETCH_SIZE reports
exactly half the bytes of a wide coalesced streaming read (16 B/lane
dwordx4), so read bytes = 2 * FETCH_SIZE KiB; WRITE_SIZE is exact for
16-B-per-lane streaming stores. Both counters are in KiB.
"""
import csv
import glob
import json
import os
import shutil
import statistics
import sys

HERE = os.path.dirname(os.path.abspath(__file__))


def one(d, pat):
    m = glob.glob(os.path.join(d, "**", pat), recursive=True)
    if not m:
        raise SystemExit(f"no {pat} under {d}")
    return m[0]


def counter(d, name, ksub):
    rows = [r for r in csv.DictReader(open(one(d, "*counter_collection.csv")))
            if ksub in r["Kernel_Name"] and r["Counter_Name"] == name]
    return [float(r["Counter_Value"]) for r in rows], rows


def main():
    rnd, tdir, fdir, wdir = sys.argv[1:5]
    ksub = "rs_apply_perm<4, 2, true>"
    if "--kernel" in sys.argv:
        ksub = sys.argv[sys.argv.index("--kernel") + 1]
    stats = one(tdir, "*kernel_stats.csv")
    shutil.copy(stats, os.path.join(HERE, f"{rnd}_kernel_stats.csv"))
    avg_ns = None
    for r in csv.DictReader(open(stats)):
        if ksub in r["Name"]:
            avg_ns = float(r["AverageNs"])
    fetch, frows = counter(fdir, "FETCH_SIZE", ksub)
    write, _ = counter(wdir, "WRITE_SIZE", ksub)
    f_kib, w_kib = statistics.median(fetch), statistics.median(write)
    read_b = 2 * f_kib * 1024
    write_b = w_kib * 1024
    out = {
        "round": rnd,
        "kernel": "perm",
        "kernel_name": ksub,
        "chunks": 1024,
        "chunk_bytes": 1 << 20,
        "launches_counted": len(fetch),
        "FETCH_SIZE_KiB_median": f_kib,
        "WRITE_SIZE_KiB_median": w_kib,
        "read_bytes_per_launch": read_b,
        "write_bytes_per_launch": write_b,
        "bytes_per_launch": read_b + write_b,
        "correction": "read = 2 x FETCH_SIZE (gfx950 half-count on dwordx4 streams)",
        "avg_kernel_ns_from_trace": avg_ns,
        "vgpr": frows[0]["VGPR_Count"] if frows else None,
        "sgpr": frows[0]["SGPR_Count"] if frows else None,
    }
    if avg_ns:
        out["achieved_GBps_from_trace"] = round((read_b + write_b) / avg_ns, 1)
    json.dump(out, open(os.path.join(HERE, f"{rnd}_pmc.json"), "w"), indent=1)
    json.dump(out, open(os.path.join(HERE, "pmc_traffic.json"), "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
