"""Rank 0's bounded side legs of the bench line (bench.py line_extras),
all run after the timed region: the kernel trace and live HBM traffic of
the timed workload, the copy ceiling, PCIe-inclusive and per-call host
rates, piece-id hashing, decode-based repair, Storb's download decode, and
configs 3 / 4's extra figures. (The CPU baselines stay in bench.py: they are
its only oracle/ users.)"""
from __future__ import annotations

from . import SEED_BASE, device as bdev, host as bhost, prof


def side_legs(out, a, ctx, dev, stream, w, ex):
    if "kernel_trace" in ex and not a.no_traffic:
        kt = prof.kernel_trace(a, w, a.settle_ms)
        if "legs" in kt:
            # without the pre-roll: what a short region right after idle measures
            kt0 = prof.kernel_trace(a, w, 0.0)
            kt["without_settle"] = ({k: kt0[k] for k in ("window_ms_per_step",
                                                         "busy_ms_per_step", "median_gap_us")}
                                    | {"legs": {leg: {x: v[x] for x in (
                                        "avg_us", "first_half_avg_us", "second_half_avg_us",
                                        "durations_us")} for leg, v in kt0["legs"].items()}}
                                    if "legs" in kt0 else kt0)
        out["roofline"]["kernel_trace"] = kt
    if "traffic" in ex and not a.no_traffic:
        if any(v > 1 for leg, v in out["roofline"]["launches_per_leg"].items()
               if not (leg == "decode" and w.sets is not None)):
            out["roofline"]["traffic_source"] = (
                "not measured: a leg is several compiled launches (row blocks)")
        else:
            out["roofline"].update(prof.pmc_traffic(a, w))
    if "copy_ceiling" in ex:
        out["roofline"]["copy_ceiling_gbs"] = bdev.copy_ceiling(ctx, dev, stream)
    if "host_path" in ex and not a.no_host_path:
        pc = bhost.pcie_ceiling(dev)
        out["pcie_inclusive"] = bhost.host_path_rate(
            ctx, w.k, w.n, w.chunk, nchunks=max(8, (256 << 20) // w.chunk),
            erased=[e for e in w.fixed_erased if e < w.k],
            sets=w.sets or bdev.download_sets(w.k, w.n, 64, SEED_BASE + 4343))
        out["pcie_inclusive"]["pcie_ceiling"] = pc
    if "shim_path" in ex:
        out["shim_path"] = bhost.shim_path_rate(ctx)
    if "hashing" in ex:
        out["shard_hashing"] = bdev.shard_hash_rate(ctx, w, stream)
    if "repair" in ex:
        out["repair"] = bdev.repair_rate(ctx, w, stream)
    if "download" in ex and w.sets is None and "decode" in w.legs:
        out["download_decode"] = bdev.download_leg(ctx, w, stream, a)
    if "assembly" in ex:
        out["assembly"] = bdev.config3_assembly(ctx, w, stream)
    if "storb_faithful" in ex:
        out["storb_faithful"] = bdev.config4_storb_faithful(ctx, w, stream)
