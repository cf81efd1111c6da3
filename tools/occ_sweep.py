#!/usr/bin/env python3
"""Resident-workgroup cap sweep at the product level: bench.py configs 2-5
(+ their repair / assembly / Storb-faithful legs) under STORB_RS_WG_PER_CU =
each cap, one child process per (config, cap), interleaved over rounds.
Prints one line per run; used to pick Tune<KM,RM>::OCC / BsTune::OCC
(profiles/r1_occupancy.txt).

usage: python tools/occ_sweep.py [rounds] [caps...]   (cap "t" = the tuned table)
"""
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def run(cfg, cap):
    env = dict(os.environ, STORB_RS_WG_PER_CU=str(cap))
    if cap == "t":  # the tuned per-kernel caps (no override)
        env.pop("STORB_RS_WG_PER_CU")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--config", str(cfg),
                        "--steps", "100", "--cpu-seconds", "0", "--no-host-path"],
                       env=env, capture_output=True, text=True, timeout=180)
    line = [x for x in p.stdout.splitlines() if x.startswith("{")]
    if p.returncode or not line:
        raise SystemExit(f"config {cfg} cap {cap} failed:\n{p.stderr[-2000:]}")
    d = json.loads(line[-1])
    r = d["roofline"]
    extra = {}
    for key in ("repair", "assembly", "storb_faithful"):
        if key in d:
            v = d[key]
            if key == "repair":
                extra["repair_data_GBps"] = v["data"]["GBps"]
                extra["repair_parity_GBps"] = v["parity"]["GBps"]
            elif key == "assembly":
                extra["assembly_GBps"] = v["erased_data"]["fused"]["GBps"]
                extra["control_GBps"] = v["control"]["fused"]["GBps"]
            else:
                extra["faithful_GBps"] = v["GBps"]
    return {"config": cfg, "cap": cap, "value": d["value"], "achieved": r["achieved"],
            "leg_ms": r["leg_ms"], **extra}


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    caps = [x if x == "t" else int(x) for x in sys.argv[2:]] or [0, 3, 4, 5, 6]
    for rd in range(rounds):
        for cfg in (2, 3, 4, 5):
            for cap in caps:
                print(json.dumps({"round": rd, **run(cfg, cap)}), flush=True)


if __name__ == "__main__":
    main()
