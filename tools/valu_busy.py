#!/usr/bin/env python3
"""Is an RS kernel VALU- or LDS-bound? ("confirm the kernel is
not VALU- or LDS-bound in rocprof".) Summarises a rocprofv3 --pmc run of

  GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU
  SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_LDS   (one pass: 6 SQ + 1 GRBM)

per kernel (median over its dispatches):
  clock_GHz   = GRBM_GUI_ACTIVE / 8 XCDs / duration  (the clock the chip held)
  valu_busy   = SQ_INSTS_VALU x 4 cycles / (duration x clock x 1024 SIMDs):
                the fraction of SIMD issue cycles the kernel's VALU
                instructions need (1.0 = VALU-issue-bound)
  lds_per_valu = SQ_INSTS_LDS / SQ_INSTS_VALU
  wait_inst   = SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES (waves stalled on issue)
  hbm_GBps    = algorithmic bytes / duration, when the bench line names them

usage: python tools/valu_busy.py <rocprof dir with run_counter_collection.csv> [...]
"""
from __future__ import annotations

import csv
import json
import os
import statistics
import sys
from collections import defaultdict

SIMDS = 256 * 4
XCDS = 8


def short(name: str) -> str:
    head = name.replace("(anonymous namespace)::", "").split("(")[0].strip()
    if head.startswith("void "):
        head = head[5:]
    base, lt, targs = head.partition("<")
    return base.split("::")[-1] + lt + targs


def summarise(d: str):
    rows = defaultdict(lambda: defaultdict(dict))  # kernel -> dispatch -> counter
    meta = {}
    with open(os.path.join(d, "run_counter_collection.csv")) as f:
        for r in csv.DictReader(f):
            k = short(r["Kernel_Name"])
            disp = int(r["Dispatch_Id"])
            rows[k][disp][r["Counter_Name"]] = float(r["Counter_Value"])
            rows[k][disp]["dur_ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            meta[k] = {"vgpr": int(r["VGPR_Count"]), "wg": int(r["Workgroup_Size"]),
                       "grid": int(r["Grid_Size"])}
    out = {}
    for k, disps in rows.items():
        vals = defaultdict(list)
        for c in disps.values():
            if "SQ_INSTS_VALU" not in c or c["dur_ns"] <= 0:
                continue
            dur = c["dur_ns"] * 1e-9
            clk = c["GRBM_GUI_ACTIVE"] / XCDS / dur
            vals["dur_us"].append(c["dur_ns"] / 1e3)
            vals["clock_GHz"].append(clk / 1e9)
            vals["valu_busy"].append(c["SQ_INSTS_VALU"] * 4 / (dur * clk * SIMDS))
            vals["lds_per_valu"].append(c.get("SQ_INSTS_LDS", 0) / max(c["SQ_INSTS_VALU"], 1))
            vals["wait_inst"].append(c["SQ_WAIT_INST_ANY"] / max(c["SQ_WAVE_CYCLES"], 1))
        if not vals:
            continue
        out[k] = {"dispatches": len(vals["dur_us"]), **meta[k],
                  **{n: round(statistics.median(v), 4) for n, v in vals.items()}}
    return out


def main():
    res = {}
    for d in sys.argv[1:]:
        s = summarise(d)
        log = d.rstrip("/") + ".log"
        if os.path.exists(log):
            for line in open(log):
                if line.startswith("{") and "roofline" in json.loads(line):
                    b = json.loads(line)["roofline"]
                    for leg, kname in b["kernel"].items():
                        for k in s:
                            # the timed leg's kernel: rs_apply_perm<KM,RM,...> without
                            # the fused-assembly (COPY = last template flag) variant
                            kk = k.replace(" ", "")
                            if kk.startswith(kname.replace(" ", "")[:-1] + ",") and \
                                    not kk.endswith(",true>") or kk == kname.replace(" ", ""):
                                s[k]["hbm_GBps"] = round(b["alg_bytes_per_launch"][leg] /
                                                         (s[k]["dur_us"] * 1e-6) / 1e9, 1)
                                s[k]["leg"] = leg
        res[os.path.basename(d.rstrip("/"))] = s
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
