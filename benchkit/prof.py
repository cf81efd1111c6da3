"""rocprofv3 child passes of the bench line (kernel trace of the timed
region, live FETCH_SIZE / WRITE_SIZE traffic), the GPU's clock levels, and
the mirror of the JIT launch policy (kernel names, launches per leg)."""
from __future__ import annotations

import os
import sys
import time

from . import BENCH, HBM_PEAK_GBS


def leg_rows(w, leg):
    """Rows of the matrix a leg applies: parity rows (encode) or lost data
    shares (decode; the most any stripe lost with per-chunk patterns)."""
    if leg == "encode":
        return w.n - w.k
    return max(len(x) for x in w.lost_rows())


def jit_blocks(k, rows):
    """Compiled launches of a rows-row matrix and the first launch's rows
    (rs_jit.cpp): 17-32 rows at even k are one row-split launch, otherwise
    row blocks of <= 16, balanced."""
    if 16 < rows <= 32 and k % 2 == 0:
        return 1, rows
    nb = -(-rows // 16)
    return nb, rows // nb


def leg_kernel_match(a, w, leg):
    """Substring of the rocprofv3 kernel name each leg launches (compiled
    kernels are named storb_bs_jit_k<k>_r<rows>_{ip,asm}, rs_jit.cpp)."""
    if leg == "decode" and w.sets is not None:
        return "rs_apply_desc_mix"
    if leg in w.jit_legs:
        return f"storb_bs_jit_k{w.k}_r{jit_blocks(w.k, leg_rows(w, leg))[1]}_"
    if leg == "encode":
        if a.kernel == "auto" and (w.k, w.n) in ((16, 24), (32, 48), (64, 96)):
            # (16, 24) / (32, 48): the input-split form (rs_bitslice.hpp KsTune)
            ks = "_ks" if (w.k, w.n) in ((16, 24), (32, 48)) else ""
            return f"rs_encode_bitslice{ks}<{w.k}, {w.n}>"
        k, r = w.k, w.n - w.k
    else:
        k, r = w.k, sum(1 for x in w.erased if x < w.k)
    kb = 1
    while kb < min(k, 32):
        kb <<= 1
    return f"rs_apply_{'lds' if a.kernel == 'lds' else 'perm'}<{kb}, {r if r <= 8 else 16},"


def child_cmd(a, erase_pattern, steps=3, warmup=1, settle_ms=0.0):
    """This workload as a short child run (the program rocprofv3 starts)."""
    child = [sys.executable, BENCH, "--config", str(a.config),
             "--steps", str(steps), "--warmup", str(warmup), "--settle-ms", str(settle_ms),
             "--minimal", "--no-check", "--kernel", a.kernel,
             "--objects", str(a.objects), "--erase-pattern", erase_pattern,
             "--fail", str(a.fail)]
    if a.chunks:
        child += ["--chunks", str(a.chunks)]
    if a.erase is not None:
        child += ["--erase", str(a.erase)]
    return child


def kernel_trace(a, w, settle_ms, erase_pattern=None, subs=None):
    """One rocprofv3 --kernel-trace --stats child run of exactly this line's
    sequence (same steps, warm-up and settle pre-roll): the launches of the
    timed region, identified from the end of the trace (after it come only
    the min(K, 50) steps of the per-leg event pass), their durations, and the
    idle time between consecutive dispatches. Says whether a step's GPU time
    is kernel time or launch gaps."""
    import csv
    import glob
    import shutil
    import statistics
    import subprocess
    import tempfile

    prof = shutil.which("rocprofv3")
    if not prof:
        return {"error": "rocprofv3 not found"}
    t0 = time.perf_counter()
    d = tempfile.mkdtemp(prefix="storb_kt_", dir="/tmp")
    try:
        cmd = ["timeout", "-s", "KILL", "150", prof, "--kernel-trace", "--stats",
               "--output-format", "csv", "-d", d, "-o", "run", "--",
               *child_cmd(a, erase_pattern or a.erase_pattern, a.steps, a.warmup, settle_ms)]
        r = subprocess.run(cmd, cwd="/tmp", env=dict(os.environ, TMPDIR="/tmp"),
                           stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True)
        files = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
        if r.returncode != 0 or not files:
            return {"error": f"rocprofv3 --kernel-trace failed (rc {r.returncode}): "
                             f"{r.stderr.strip()[-300:]}"}
        rows = sorted(csv.DictReader(open(files[0])), key=lambda x: int(x["Start_Timestamp"]))
    finally:
        shutil.rmtree(d, ignore_errors=True)
    K, probe = a.steps, min(a.steps, 50)
    legs, lo, hi = {}, None, None
    subs = subs or [leg_kernel_match(a, w, leg) for leg in w.legs]
    for li, leg in enumerate(w.legs):
        sub = subs[li]
        # legs that launch the same kernel (config 2: encode and decode are
        # both rs_apply_perm<4,2>) alternate in launch order
        same = [i for i, x in enumerate(subs) if x == sub]
        g, pos = len(same), same.index(li)
        mine = [x for x in rows if sub in x["Kernel_Name"]]
        if len(mine) < (K + probe) * g:
            return {"error": f"{len(mine)} {sub} launches in the trace, expected >= "
                             f"{(K + probe) * g}"}
        timed = mine[len(mine) - (K + probe) * g:len(mine) - probe * g][pos::g]
        dur = [(int(x["End_Timestamp"]) - int(x["Start_Timestamp"])) / 1e3 for x in timed]
        avg = sum(dur) / len(dur)
        legs[leg] = {"kernel": timed[0]["Kernel_Name"][:120], "launches": len(dur),
                     "avg_us": round(avg, 2), "median_us": round(statistics.median(dur), 2),
                     "min_us": round(min(dur), 2), "max_us": round(max(dur), 2),
                     "first_half_avg_us": round(sum(dur[:len(dur) // 2]) / max(1, len(dur) // 2), 2),
                     "second_half_avg_us": round(sum(dur[len(dur) // 2:]) /
                                                 max(1, len(dur) - len(dur) // 2), 2),
                     "durations_us": [round(x, 1) for x in dur[:64]],
                     "frac_kernel_time": round(w.alg_bytes(leg) / (avg * 1e-6) / 1e9 /
                                               HBM_PEAK_GBS, 4)}
        s0, e1 = int(timed[0]["Start_Timestamp"]), int(timed[-1]["End_Timestamp"])
        lo = s0 if lo is None else min(lo, s0)
        hi = e1 if hi is None else max(hi, e1)
    win = [x for x in rows if lo <= int(x["Start_Timestamp"]) and int(x["End_Timestamp"]) <= hi]
    gaps = [(int(win[i + 1]["Start_Timestamp"]) - int(win[i]["End_Timestamp"])) / 1e3
            for i in range(len(win) - 1)]
    busy = sum(int(x["End_Timestamp"]) - int(x["Start_Timestamp"]) for x in win) / 1e6
    span = (hi - lo) / 1e6
    return {"legs": legs, "dispatches_in_window": len(win),
            "window_ms_per_step": round(span / K, 4), "busy_ms_per_step": round(busy / K, 4),
            "idle_ms_per_step": round((span - busy) / K, 4),
            "median_gap_us": round(statistics.median(gaps), 2) if gaps else None,
            "max_gap_us": round(max(gaps), 2) if gaps else None,
            "settle_ms": settle_ms,
            "source": (f"rocprofv3 --kernel-trace --stats over a child run with this line's "
                       f"--steps {K} --warmup {a.warmup} --settle-ms {settle_ms} "
                       f"({time.perf_counter() - t0:.0f} s); the timed launches are the {K} "
                       f"per leg before the last {probe} (the per-leg event pass); the "
                       f"tracer itself adds ~2-3 us to each gap")}


def gpu_clocks(local):
    """The GPU's clock levels and power cap (sysfs of this device's PCI
    function; amd-smi reports the same values): current gfx / memory / fabric
    levels (the '*' entry of pp_dpm_*) and power1_cap / power1_average in W."""
    import glob
    import ctypes
    try:
        hip = ctypes.CDLL("libamdhip64.so")
        buf = ctypes.create_string_buffer(32)
        if hip.hipDeviceGetPCIBusId(buf, 32, local) != 0:
            return {"error": "hipDeviceGetPCIBusId failed"}
        base = "/sys/bus/pci/devices/" + buf.value.decode().lower()
    except OSError as e:
        return {"error": repr(e)}
    out = {"pci": base.rsplit("/", 1)[-1]}
    for name in ("pp_dpm_sclk", "pp_dpm_mclk", "pp_dpm_fclk", "pp_dpm_socclk",
                 "power_dpm_force_performance_level"):
        try:
            txt = open(os.path.join(base, name)).read().strip().splitlines()
        except OSError:
            continue
        cur = [x for x in txt if x.rstrip().endswith("*")]
        out[name] = (cur[0].split(":", 1)[1].strip(" *") if cur else txt[0].strip())
    for name in ("power1_cap", "power1_average", "power1_input"):
        for f in glob.glob(os.path.join(base, "hwmon", "hwmon*", name)):
            try:
                out[name + "_W"] = round(int(open(f).read()) / 1e6, 1)
            except (OSError, ValueError):
                pass
    return out


def pmc_passes(a, erase_pattern, seq=False):
    """Two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) over a short child
    run of this workload: ({(kernel name, counter): [values in launch
    order]}, error or None)."""
    import csv
    import glob
    import shutil
    import subprocess
    import tempfile

    prof = shutil.which("rocprofv3")
    if not prof:
        return None, "rocprofv3 not found"
    child = child_cmd(a, erase_pattern)
    env = dict(os.environ, TMPDIR="/tmp")
    vals = {}
    for cnt in ("FETCH_SIZE", "WRITE_SIZE"):
        d = tempfile.mkdtemp(prefix="storb_pmc_", dir="/tmp")
        try:
            cmd = ["timeout", "-s", "KILL", "150", prof, "--pmc", cnt, "--kernel-trace",
                   "--output-format", "csv", "-d", d, "-o", "run", "--", *child]
            r = subprocess.run(cmd, cwd="/tmp", env=env, stdout=subprocess.DEVNULL,
                               stderr=subprocess.PIPE, text=True)
            files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
            if r.returncode != 0 or not files:
                return None, (f"rocprofv3 --pmc {cnt} failed (rc {r.returncode}): "
                              f"{r.stderr.strip()[-300:]}")
            for row in csv.DictReader(open(files[0])):
                if row["Counter_Name"] == cnt:
                    vals.setdefault((row["Kernel_Name"], cnt), []).append(
                        float(row["Counter_Value"]))
        finally:
            shutil.rmtree(d, ignore_errors=True)
    return vals, None


def pmc_download_traffic(a, w):
    """HBM bytes of one download decode (--erase-pattern download's decode
    leg: the mixed-row descriptor launch plus any per-count launch), live,
    over a child run with download patterns: summed over the rs_apply_desc*
    launches of the run, divided by its number of decode calls (one
    rs_apply_desc_mix launch each). The descriptor copy kernel reads
    page-locked host memory and is not counted."""
    import statistics
    vals, err = pmc_passes(a, "download")
    if err:
        return {"traffic": None, "traffic_source": err}
    f = sum(v for (kn, c), xs in vals.items() if c == "FETCH_SIZE" and "rs_apply_desc" in kn
            for v in xs)
    wr = sum(v for (kn, c), xs in vals.items() if c == "WRITE_SIZE" and "rs_apply_desc" in kn
             for v in xs)
    calls = [len(xs) for (kn, c), xs in vals.items() if c == "FETCH_SIZE" and "rs_apply_desc_mix" in kn]
    if not calls or not calls[0]:
        return {"traffic": None, "traffic_source": "no rs_apply_desc_mix launches in the PMC passes"}
    b = (2 * f * 1024 + wr * 1024) / calls[0]
    per = [2 * x * 1024 for (kn, c), xs in vals.items() if c == "FETCH_SIZE"
           and "rs_apply_desc_mix" in kn for x in xs]
    return {"traffic": b, "decode_calls": calls[0],
            "mix_launch_read_bytes_median": statistics.median(per) if per else None,
            "traffic_source": "live: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over a 3-step "
                              "child run with --erase-pattern download; read = 2 x FETCH_SIZE"}


def pmc_traffic(a, w):
    """HBM bytes per launch measured in THIS run (roofline.traffic): two short
    child runs of the same workload under rocprofv3, one per counter
    (FETCH_SIZE and WRITE_SIZE do not fit one TCC pass), each under a hard
    time limit. gfx950 correction (MI355X_MICROARCH.md, HBM): read bytes =
    2 x FETCH_SIZE KiB for 16-B-per-lane streaming loads; WRITE_SIZE is exact
    for 16-B-per-lane stores. Per leg: median over that kernel's launches; a
    download-pattern decode leg (several launches): the sum over its
    rs_apply_desc* launches per call."""
    import statistics

    t0 = time.perf_counter()
    vals, err = pmc_passes(a, a.erase_pattern)
    if err:
        return {"traffic": None, "traffic_source": err}
    by_leg = {}
    for leg in w.legs:
        if leg == "decode" and w.sets is not None:
            calls = [len(xs) for (kn, c), xs in vals.items()
                     if c == "FETCH_SIZE" and "rs_apply_desc_mix" in kn]
            f = sum(v for (kn, c), xs in vals.items() if c == "FETCH_SIZE"
                    and "rs_apply_desc" in kn for v in xs)
            wr = sum(v for (kn, c), xs in vals.items() if c == "WRITE_SIZE"
                     and "rs_apply_desc" in kn for v in xs)
            if not calls or not calls[0]:
                by_leg[leg] = None
                continue
            b = (2 * f + wr) * 1024 / calls[0]
            by_leg[leg] = {"kernel": "rs_apply_desc*", "calls": calls[0], "bytes": b,
                           "vs_algorithmic": round(b / w.alg_bytes(leg), 5)}
            continue
        sub = leg_kernel_match(a, w, leg)
        f = [v for (kn, c), xs in vals.items() if c == "FETCH_SIZE" and sub in kn for v in xs]
        wr = [v for (kn, c), xs in vals.items() if c == "WRITE_SIZE" and sub in kn for v in xs]
        if not f or not wr:
            return {"traffic": None, "traffic_source": f"no {sub} launches in the PMC passes"}
        fk, wk = statistics.median(f), statistics.median(wr)
        b = 2 * fk * 1024 + wk * 1024
        by_leg[leg] = {"kernel": sub, "launches": len(f), "FETCH_SIZE_KiB": fk,
                       "WRITE_SIZE_KiB": wk, "bytes": b,
                       "vs_algorithmic": round(b / w.alg_bytes(leg), 5)}
    first = by_leg[w.legs[0]]
    if first is None:
        return {"traffic": None, "traffic_by_leg": by_leg,
                "traffic_source": "not measured: per-chunk patterns (several launches per leg)"}
    return {"traffic": first["bytes"], "traffic_by_leg": by_leg,
            "traffic_source": (f"live: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over a "
                               f"3-step child run of this workload ({time.perf_counter() - t0:.0f}"
                               f" s); read = 2 x FETCH_SIZE (gfx950), write = WRITE_SIZE")}


def jit_name(w, leg):
    nb, r0 = jit_blocks(w.k, leg_rows(w, leg))
    return (f"storb_bs_jit_k{w.k}_r{r0}_* (hipRTC)"
            + (f" x {nb} row blocks" if nb > 1 else ""))


def kernel_names(kernel, w):
    """The kernels the legs launch (rs_bitslice.hpp / rs_device.hpp)."""
    names = {}
    table = "lds" if kernel == "lds" else "perm"
    if "encode" in w.legs:
        bits = kernel == "auto" and (w.k, w.n) in ((16, 24), (32, 48), (64, 96))
        ks = "_ks" if (w.k, w.n) in ((16, 24), (32, 48)) else ""
        names["encode"] = (f"rs_encode_bitslice{ks}<{w.k},{w.n}>" if bits
                           else jit_name(w, "encode") if "encode" in w.jit_legs
                           else f"rs_apply_{table}<{min(w.k, 32)},{w.n - w.k}>")
    if "decode" in w.legs and w.sets is not None:
        mix = ({16: "rs_apply_desc_mix_ks<16, 2>", 32: "rs_apply_desc_mix_ks<32, 4>"}.get(w.k)
               or f"rs_apply_desc_mix<{min(w.k, 32)}>")
        names["decode"] = (f"{mix} (per-stripe descriptors: one "
                           f"launch for the stripes that lost 1-4 data shares, one per larger "
                           f"count; descriptors copied in by copy_u32x4_kernel)")
    elif "decode" in w.legs:
        e = sum(1 for x in w.erased if x < w.k)
        names["decode"] = (jit_name(w, "decode") if "decode" in w.jit_legs
                           else f"rs_apply_{table}<{min(w.k, 32)},{e}>")
    return names
