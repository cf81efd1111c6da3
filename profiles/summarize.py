#!/usr/bin/env python3
"""Turn a round's GPU-box profile directory (tools/profile_round.sh) into the
committed summaries under profiles/.

usage: summarize.py ROUND PROF_DIR

For every PROF_DIR/trace_<name>/ (rocprofv3 --kernel-trace --stats of one
bench.py run):
  * profiles/<ROUND>_<name>_kernel_stats.csv  -- the --stats summary as is
  * profiles/<ROUND>_bench_<name>.json       -- that run's bench line
and a check that each leg's kernel average duration from the trace agrees
with the bench line's per-leg time (roofline.leg_ms, HIP events).
PROF_DIR/bench_default.log (the untraced default run, whose
roofline.traffic is measured live by its own FETCH_SIZE / WRITE_SIZE passes)
becomes profiles/<ROUND>_bench.json. Prints a JSON summary.
"""
import csv
import glob
import json
import os
import shutil
import sys

HERE = os.path.dirname(os.path.abspath(__file__))


def last_json(path):
    for line in reversed(open(path).read().strip().splitlines()):
        if line.startswith("{"):
            return json.loads(line)
    raise SystemExit(f"no JSON line in {path}")


def kernel_match(line, leg):
    """The rocprof name substring of the kernel a bench leg launched."""
    byleg = line["roofline"].get("traffic_by_leg") or {}
    if leg in byleg:
        return byleg[leg]["kernel"]
    name = line["roofline"]["kernel"][leg]
    if name.startswith("storb_bs_jit"):
        return "storb_bs_jit"
    base, args = name.split("<", 1)
    return f"{base}<{args.rstrip('>').replace(',', ', ')}"


def main():
    rnd, pdir = sys.argv[1:3]
    summary = {}
    for tdir in sorted(glob.glob(os.path.join(pdir, "trace_*"))):
        name = os.path.basename(tdir)[len("trace_"):]
        stats = glob.glob(os.path.join(tdir, "**", "*kernel_stats.csv"), recursive=True)
        if not stats:
            continue
        dst = os.path.join(HERE, f"{rnd}_{name}_kernel_stats.csv")
        shutil.copy(stats[0], dst)
        line = last_json(os.path.join(pdir, f"bench_{name}.log"))
        json.dump(line, open(os.path.join(HERE, f"{rnd}_bench_{name}.json"), "w"))
        rows = list(csv.DictReader(open(stats[0])))
        legs = {}
        for leg, ms in line["roofline"]["leg_ms"].items():
            sub = (line["roofline"].get("kernel_match") or {}).get(leg) or kernel_match(line, leg)
            per_leg = (line["roofline"].get("launches_per_leg") or {}).get(leg, 1)
            hit = [r for r in rows if sub in r["Name"]]
            if not hit:
                legs[leg] = {"kernel": sub, "trace": None}
                continue
            r = max(hit, key=lambda x: int(x["Calls"]))
            # a leg of several launches (row blocks of a compiled matrix)
            avg_ms = float(r["AverageNs"]) / 1e6 * per_leg
            alg = line["roofline"]["alg_bytes_per_launch"][leg]
            legs[leg] = {"kernel": r["Name"], "calls": int(r["Calls"]),
                         "trace_avg_ms": round(avg_ms, 4), "bench_leg_ms": ms,
                         "trace_GBps": round(alg / (avg_ms * 1e-3) / 1e9, 1),
                         "trace_frac_of_8TBps": round(alg / (avg_ms * 1e-3) / 8e12, 4)}
        summary[name] = {"value": line["value"], "frac": line["roofline"]["frac"], "legs": legs}
    dflt = os.path.join(pdir, "bench_default.log")
    if os.path.exists(dflt):
        line = last_json(dflt)
        json.dump(line, open(os.path.join(HERE, f"{rnd}_bench.json"), "w"))
        summary["default"] = {"value": line["value"], "frac": line["roofline"]["frac"],
                              "traffic": line["roofline"].get("traffic"),
                              "traffic_source": line["roofline"].get("traffic_source")}
    json.dump(summary, open(os.path.join(HERE, f"{rnd}_summary.json"), "w"), indent=1)
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
