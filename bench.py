#!/usr/bin/env python3
"""Headline benchmark: device-resident RS encode+decode GiB/s on MI355X.

Metric (BASELINE.json): "GiB/s device-resident RS encode+decode, 1 MiB chunks
k=4 m=2, at 1/2/4/8 GPUs". m=2 is the PARITY count there, i.e. Storb's
k=4, m=6 (piece.rs:307-317 picks exactly that for a 1 MiB chunk).

Default (--config 2, the line the driver records). One step = one pass of
the hot path over one batch resident in HBM:
  encode: 1024 x 1 MiB chunks (k=4 data shards of 256 KiB -> 2 parity shards)
  decode: the same 1024 chunks with data shards {0, 1} erased (the RS(4,2)
          worst case), rebuilt in place from shares {2, 3, 4, 5}.
`value` = user bytes encoded + user bytes decoded, all ranks, / wall time.
Each rank owns its own 1024 chunks (independent objects partition across
GPUs, no collective on the data path): weak scaling. The 2 GiB per step
(+1 GiB parity) is well past the 256 MiB Infinity Cache, so the kernels
stream from HBM.

Other BASELINE configs (not the driver's line):
  --config 3  RS(8,4) [storb k=8,m=12] decode, 4096 x 256 KiB, erased {0,3,5}
  --config 4  10 000 x 1 MiB objects encoded, object i on rank i mod N
              (strong scaling: total work fixed)
  --config 5  RS(16,8) [storb k=16,m=24]: 128 x 8 MiB chunks (a 1 GiB object)
  --config 6  RS(32,16) [storb k=32,m=48]: 32 x 32 MiB chunks
  --config 7  RS(64,32) [storb k=64,m=96]: 8 x 128 MiB chunks (Storb's sizing of
              objects from ~160 GiB up, piece.rs:292-317)
              (5/6/7: --erase E loses data shares 0..E-1 for the decode leg)

Launch: python bench.py [--gpus N --steps K --warmup W]. One rank per GPU:
under torch.distributed.run (RANK/LOCAL_RANK/WORLD_SIZE env, which must agree
with --gpus), or, with --gpus N > 1 and no WORLD_SIZE, this script spawns the
N rank processes itself before touching the GPU (storb_amd/launch.py).
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

# RCCL across rank processes needs dmabuf IPC, the only kind the host driver
# supports. Set before torch (and HIP) load, so ranks started by
# torch.distributed.run get it as well as the ones storb_amd/launch.py spawns.
os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

from storb_amd import _lib, launch, partition  # noqa: E402

GIB = float(1 << 30)
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
METRIC = "GiB/s device-resident RS encode+decode, 1 MiB chunks k=4 m=2, at 1/2/4/8 GPUs"
SEED_BASE = 0x5709B


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--config", type=int, choices=[2, 3, 4, 5, 6, 7], default=2,
                   help="BASELINE config; 5 = the device-resident GPU half of config 5 "
                        "(1 GiB object -> 128 x 8 MiB chunks, storb k=16, m=24); 6 = "
                        "Storb's widest geometry (32 MiB chunks of 16-64 GiB objects, "
                        "storb k=32, m=48), 32 chunks per GPU")
    p.add_argument("--erase", type=int, default=None,
                   help="configs 5/6: data shares 0..E-1 lost per chunk for the decode leg "
                        "(default 2); E >= 3 takes the run-time-compiled bit-sliced decode")
    p.add_argument("--erase-pattern", choices=["fixed", "download"], default="fixed",
                   help="fixed: every chunk lost the same shares (--erase / the config's set); "
                        "download: each chunk keeps the first k+1 pieces to arrive from 10 "
                        "simulated fetch threads (download.rs:363-451, storb_amd/objects.py "
                        "download_arrivals), seeded, so the survivor set differs per chunk")
    p.add_argument("--fail", type=float, default=0.0,
                   help="--erase-pattern download: probability that a piece's miner is lost")
    p.add_argument("--chunks", type=int, default=None, help="chunks per GPU (config 2/3)")
    p.add_argument("--objects", type=int, default=10000, help="total objects (config 4)")
    p.add_argument("--kernel", choices=["auto", "perm", "lds"], default="auto",
                   help="auto = what the product runs (bit-sliced encoder for k=16/32, "
                        "v_perm tables otherwise); perm / lds force a table kernel")
    p.add_argument("--cpu-seconds", type=float, default=10.0,
                   help="bounded CPU-baseline sample (0 disables)")
    p.add_argument("--settle-ms", type=float, default=40.0,
                   help="untimed pre-roll of whole steps (at least this long) before the "
                        "warm-up steps: the first ~3-12 ms of load after an idle GPU run "
                        "slower while the power controller settles (DESIGN.md §5, "
                        "'Clock transient'); 0 disables")
    p.add_argument("--no-check", action="store_true")
    p.add_argument("--no-traffic", action="store_true",
                   help="skip the live rocprofv3 child passes: HBM traffic (--pmc FETCH_SIZE / "
                        "WRITE_SIZE) and the kernel trace of the timed region (needed when "
                        "this run is itself under rocprofv3)")
    p.add_argument("--minimal", action="store_true",
                   help="the timed line only (no traffic passes, copy ceiling, CPU baseline, "
                        "host path, hashing, repair); used for the traffic child runs")
    p.add_argument("--no-host-path", action="store_true")
    p.add_argument("--leg-events", choices=["each", "ends"], default="ends",
                   help="ends: HIP events only around the timed region, per-leg times "
                        "from a separate untimed pass; each: an event after every leg "
                        "inside the timed region (costs 2.5-3 %% of the step)")
    p.add_argument("--dist-backend", default="nccl",
                   help="nccl (= RCCL, one GPU per rank) or gloo (rehearsal of the "
                        "multi-rank logic with several ranks on one GPU, see "
                        "STORB_BENCH_DEVICE)")
    p.add_argument("--force-pg", action="store_true",
                   help="create the process group even at world size 1, so a one-GPU box "
                        "runs exactly the multi-rank sequence (init_process_group with "
                        "device_id, all_gather_object, device all_reduce, barrier)")
    return p.parse_args(argv)


def _cpu_where(cpu):
    """Clock and NUMA node of logical CPU `cpu` (from /proc and /sys)."""
    mhz, node = None, None
    try:
        cur = None
        for line in open("/proc/cpuinfo"):
            if line.startswith("processor"):
                cur = int(line.split(":")[1])
            elif line.startswith("cpu MHz") and cur == cpu:
                mhz = float(line.split(":")[1])
                break
    except (OSError, ValueError):
        pass
    try:
        for name in os.listdir(f"/sys/devices/system/cpu/cpu{cpu}"):
            if name.startswith("node") and name[4:].isdigit():
                node = int(name[4:])
    except OSError:
        pass
    return {"cpu": cpu, "cpu_mhz": mhz, "numa_node": node}


def _ssbd_run(run, secs):
    """run(fresh=True, secs) on a fresh thread that first turns SSBD on for
    itself (PR_SET_SPECULATION_CTRL; irreversible for that thread only)."""
    import ctypes
    import threading
    res = {}

    def body():
        libc = ctypes.CDLL(None, use_errno=True)
        rc = libc.prctl(53, 0, 4, 0, 0)  # PR_SET_SPECULATION_CTRL, PR_SPEC_STORE_BYPASS, DISABLE
        if rc != 0:
            res["refused_errno"] = ctypes.get_errno()
            return
        v, c, e, a = run(True, secs)
        res.update({"value": v, "unit": "GiB/s", "calls": c, "seconds": round(e, 2),
                    "ipc": a.get("ipc"), "effective_ghz": a.get("effective_ghz"),
                    "l1_addmul_GBps": a.get("l1_addmul_GBps"),
                    "Speculation_Store_Bypass": a["speculation"].get("Speculation_Store_Bypass")})

    t = threading.Thread(target=body)
    t.start()
    t.join()
    return res


def _speculation_state():
    """The measuring thread's speculative-store-bypass state and seccomp mode
    (/proc/thread-self/status) and the kernel's global view (sysfs). With
    SSBD on (e.g. forced for every seccomp-filtered process, the kernel's
    default `spec_store_bypass_disable=seccomp`), a load waits for every
    older store's address: the oracle's byte-wise read-modify-write loop is
    exactly that pattern, while register-only and streaming-read code is not
    affected."""
    out = {}
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("microcode"):
                out["microcode"] = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        for line in open("/proc/thread-self/status"):
            key = line.split(":")[0]
            if key in ("Speculation_Store_Bypass", "SpeculationIndirectBranch", "Seccomp",
                       "Seccomp_filters"):
                out[key] = line.split(":", 1)[1].strip()
    except OSError:
        pass
    try:
        out["vulnerabilities_spec_store_bypass"] = open(
            "/sys/devices/system/cpu/vulnerabilities/spec_store_bypass").read().strip()
    except OSError:
        pass
    return out


def _proc_stat():
    """Per-CPU jiffies from /proc/stat: {cpu: (total, steal)}."""
    out = {}
    try:
        for line in open("/proc/stat"):
            if line.startswith("cpu") and line[3:4].isdigit():
                f = line.split()
                v = [int(x) for x in f[1:]]
                out[int(f[0][3:])] = (sum(v), v[7] if len(v) > 7 else 0)
    except (OSError, ValueError):
        pass
    return out


def _steal_frac(st0, st1, cpu):
    if cpu not in st0 or cpu not in st1:
        return None
    tot = st1[cpu][0] - st0[cpu][0]
    return round((st1[cpu][1] - st0[cpu][1]) / tot, 4) if tot > 0 else None


def cpu_baseline(k, n, chunk_bytes, erased, seconds, do_encode=True, do_decode=True,
                 survivor_sets=None):
    """Reference CPU path (C restatement of zfec, oracle/) on this host.

    Single thread, like the reference: upload.rs:418-420 encodes one object's
    chunks sequentially in one task and download.rs:505-529 decodes them
    sequentially. Sample: 8 distinct splitmix chunks of the benchmark's
    shape, cycled for `seconds` in a C loop on this thread
    (oracle/cpu_bench.c). `value`: every call allocates its outputs as
    zfec-rs does (a Vec per share, a Vec out -- piece.rs:329,384-386);
    `arithmetic_only`: the same loop with every buffer allocated once. Both
    carry the thread's own getrusage account (user / system seconds, minor
    faults, context switches) and the CPU, clock and NUMA node it ran on, so
    a figure that moves between boxes shows where.
    """
    from oracle import coracle  # test infrastructure: the baseline, never the product

    survivors = [i for i in range(n) if i not in erased][:k]
    sets = [sorted(x)[:k] for x in survivor_sets] if survivor_sets else [survivors]
    sample = np.concatenate([coracle.splitmix_bytes(SEED_BASE + i, chunk_bytes)
                             for i in range(8)])
    legs = int(do_encode) + int(do_decode)
    what = "+".join(x for x, on in (("encode", do_encode), ("decode", do_decode)) if on)

    def run(fresh, secs):
        st0 = _proc_stat()
        r = coracle.bench_roundtrip(k, n, sample, chunk_bytes, 8, sets, do_encode, do_decode,
                                    fresh, secs)
        st1 = _proc_stat()
        el = r["wall_s"]
        acct = {"user_s": round(r["user_s"], 3), "sys_s": round(r["sys_s"], 3),
                "thread_cpu_over_wall": round((r["user_s"] + r["sys_s"]) / el, 3),
                "minor_faults": r["minflt"], "major_faults": r["majflt"],
                "minor_faults_per_call": round(r["minflt"] / max(1, r["calls"]), 2),
                # the thread's own cycles / instructions (perf_event_open; null
                # where refused): effective clock and IPC over the sample, and
                # a dependent multiply-add chain's rate before / after it
                "effective_ghz": round(r["cycles"] / el / 1e9, 3) if r["cycles"] > 0 else None,
                "ipc": round(r["instructions"] / r["cycles"], 3) if r["cycles"] > 0 else None,
                "clock_probe_giter_per_s": [round(r["probe_before"], 3), round(r["probe_after"], 3)],
                # after the sample, this thread: the oracle's addmul on an
                # L1-resident block, sequential reads from L2 and from DRAM
                "l1_addmul_GBps": round(r["l1_addmul_gbs"], 2),
                "l2_read_GBps": round(r["l2_read_gbs"], 2),
                "dram_read_GBps": round(r["dram_read_gbs"], 2),
                "voluntary_switches": r["nvcsw"], "involuntary_switches": r["nivcsw"],
                **_cpu_where(r["cpu_start"]),
                # time the hypervisor ran something else on this vCPU: the
                # thread's own CPU time does not show it (/proc/stat steal)
                "cpu_steal_frac": _steal_frac(st0, st1, r["cpu_start"]),
                "speculation": _speculation_state()}
        if r["cpu_end"] != r["cpu_start"]:
            acct["cpu_end"] = r["cpu_end"]
        return round(legs * r["calls"] * chunk_bytes / GIB / el, 4), r["calls"], el, acct

    value, calls, el, acct = run(True, seconds)
    arith, acalls, ael, aacct = run(False, max(1.0, seconds / 2))
    ssbd = _ssbd_run(run, max(1.0, seconds / 4))
    shape = (f"{chunk_bytes >> 10} KiB chunks (k={k},n={n}"
             f"{', erased ' + (str(sorted(erased)) if not survivor_sets else 'per chunk (download patterns)') if do_decode else ''})")
    return {
        "value": value,
        "unit": "GiB/s",
        "cores": 1,
        "kind": "port",
        "sample": (f"{calls} x {what} of {shape}, {el:.1f} s, 1 thread, scalar table-driven "
                   f"zfec restatement -O2 (oracle/), per-call allocation as zfec-rs; host "
                   f"{platform.machine()}, {os.cpu_count()} logical CPUs visible"),
        "thread": acct,
        "arithmetic_only": {"value": arith, "unit": "GiB/s",
                            "sample": f"{acalls} x {what}, {ael:.1f} s, buffers allocated once",
                            "thread": aacct},
        # the same loop on a thread with Speculative Store Bypass Disable on
        # (prctl, that thread only): on some boxes of this pool the oracle's
        # byte-wise read-modify-write loop runs ~19x slower with store-bypass
        # speculation enabled (IPC 0.16 vs 3.06, tools/ssbd_probe.py,
        # DESIGN.md §5 Host variance); `value` stays the process as started,
        # as the reference would run
        "ssbd_on": ssbd,
    }


def cpu_baseline_threads(k, n, chunk_bytes, erased, threads=16, nchunks=256, seconds=3.0,
                         ssbd=True):
    """The same CPU path on `threads` host threads over independent chunks
    ("nproc threads on independent chunks"; 16 = this box's
    CPU share per GPU). Encode + decode round trips over `nchunks` distinct
    chunks, repeated until `seconds` have passed, bit-exact checked."""
    from oracle import coracle  # test infrastructure: the baseline, never the product

    data = np.concatenate([coracle.splitmix_bytes(SEED_BASE + i, chunk_bytes)
                           for i in range(nchunks)])
    passes = 0
    t0 = time.perf_counter()
    while True:
        bad = coracle.roundtrip_many(k, n, data, chunk_bytes, nchunks, sorted(erased), threads)
        if bad:
            raise SystemExit("threaded CPU baseline round trip failed")
        passes += 1
        if time.perf_counter() - t0 >= seconds:
            break
    el = time.perf_counter() - t0
    res = {"value": round(2 * passes * nchunks * chunk_bytes / GIB / el, 4), "unit": "GiB/s",
           "cores": threads, "kind": "port",
           "sample": f"{passes} passes x {nchunks} x encode+decode of {chunk_bytes >> 10} KiB "
                     f"chunks, {threads} threads, {el:.2f} s"}
    if ssbd:
        # the same from a thread with SSBD on: the C workers it starts inherit
        # it (cpu_baseline's ssbd_on, DESIGN.md §5 Host variance)
        import ctypes
        import threading
        out = {}

        def body():
            if ctypes.CDLL(None).prctl(53, 0, 4, 0, 0) != 0:
                out["refused"] = True
                return
            out.update(cpu_baseline_threads(k, n, chunk_bytes, erased, threads, nchunks,
                                            max(1.0, seconds / 2), ssbd=False))

        t = threading.Thread(target=body)
        t.start()
        t.join()
        res["ssbd_on"] = {x: out.get(x) for x in ("value", "sample", "refused") if x in out}
    return res


def cpu_quota():
    """The CPUs this process may actually use: affinity mask and the cgroup v2
    CPU quota (cpu.max 'quota period'), which can be far below nproc."""
    q = {"nproc": os.cpu_count()}
    try:
        q["affinity"] = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        q["affinity"] = None
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        q["cgroup_cpus"] = None if quota == "max" else round(int(quota) / int(period), 2)
    except (OSError, ValueError):
        q["cgroup_cpus"] = None
    return q


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def copy_ceiling(ctx, dev, stream, nbytes=1 << 30, reps=5):
    """Measured device-to-device copy rates (read + write bytes / time), the
    practical HBM ceiling SURVEY 8(d) asks to report beside the 8 TB/s spec:
    our own kernel as a copy (RS apply with k=1 and coefficient 1: the same
    load/store path, no GF work) and torch's copy_ for comparison."""
    src = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    dst = torch.empty_like(src)
    blk = 1 << 20
    one = np.ones((1, 1), dtype=np.uint8)

    def ours():
        ctx.apply_dev(one, [src.data_ptr()], [blk], [dst.data_ptr()], [blk], blk,
                      nbytes // blk, stream=stream.cuda_stream)

    def theirs():
        dst.copy_(src)

    rates = {}
    with torch.cuda.stream(stream):
        src.random_(0, 256)
        for name, f in (("rs_apply_copy", ours), ("torch_copy", theirs)):
            f()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(reps):
                f()
            e1.record(stream)
            stream.synchronize()
            rates[name] = round(2 * nbytes * reps / (e0.elapsed_time(e1) * 1e-3) / 1e9, 1)
    if not torch.equal(src, dst):
        raise SystemExit("copy ceiling: copy mismatch")
    return rates


def host_path_rate(ctx, k, n, chunk_bytes, nchunks=256, reps=3, erased=(), sets=None):
    """PCIe-inclusive encode: host bytes in, parity out (pipelined). Two
    figures: from pageable caller memory (staged through the context's pinned
    buffers by host copy threads) and from page-locked caller memory
    (storb_rs_host_alloc: DMA'd in place). Output buffers are allocated and
    touched before timing."""
    B = -(-chunk_bytes // k)
    nout = nchunks * (n - k) * B
    res = {}
    for mode in ("pageable", "pinned"):
        if mode == "pinned":
            src, dst = _lib.PinnedBuffer(nchunks * chunk_bytes), _lib.PinnedBuffer(nout)
            host, out = src.array, dst.array
        else:
            host, out = np.empty(nchunks * chunk_bytes, np.uint8), np.empty(nout, np.uint8)
        host[:] = np.frombuffer(np.random.default_rng(7).bytes(host.size), dtype=np.uint8)
        out[:] = 0
        ctx.encode_chunks(k, n, host, chunk_bytes, nchunks, out=out)  # warm
        t0 = time.perf_counter()
        for _ in range(reps):
            ctx.encode_chunks(k, n, host, chunk_bytes, nchunks, out=out)
        el = time.perf_counter() - t0
        res[mode] = round(reps * nchunks * chunk_bytes / GIB / el, 3)
        # upload path with Storb's piece ids (upload.rs:623) hashed on the GPU
        ids = np.zeros((nchunks, n, 32), np.uint8)
        ctx.encode_chunks_hashed(k, n, host, chunk_bytes, nchunks, out=out, hashes=ids)
        t0 = time.perf_counter()
        for _ in range(reps):
            ctx.encode_chunks_hashed(k, n, host, chunk_bytes, nchunks, out=out, hashes=ids)
        res["hashed" if mode == "pageable" else "hashed_pinned"] = round(
            reps * nchunks * chunk_bytes / GIB / (time.perf_counter() - t0), 3)
        if erased:
            # download side: every chunk lost `erased`, rebuilt from the first
            # k survivors (storb_rs_decode_chunks), host shares in, chunks out;
            # page-locked shares and output: the kernel reads and writes them
            # in place (zero-copy), pageable: staged through pinned buffers
            surv = [i for i in range(n) if i not in erased][:k]
            par = out.reshape(nchunks, n - k, B)
            dat = host.reshape(nchunks, k, B)
            chunks = [([dat[c, i] if i < k else par[c, i - k] for i in surv], surv)
                      for c in range(nchunks)]
            if mode == "pinned":
                rbuf = _lib.PinnedBuffer(nchunks * chunk_bytes)
                rec = rbuf.array.reshape(nchunks, chunk_bytes)
            else:
                rec = np.empty((nchunks, chunk_bytes), np.uint8)
            rec[:] = 0
            ctx.decode_chunks(k, n, B, 0, chunks, out=rec)  # warm
            if not np.array_equal(rec.reshape(-1), host):
                raise SystemExit(f"host decode_chunks round trip mismatch ({mode})")
            t0 = time.perf_counter()
            for _ in range(reps):
                ctx.decode_chunks(k, n, B, 0, chunks, out=rec)
            res["decode" if mode == "pageable" else "decode_pinned"] = round(
                reps * nchunks * chunk_bytes / GIB / (time.perf_counter() - t0), 3)
            if sets:
                # download side with a different survivor set per chunk (the
                # first k + 1 pieces to arrive, download.rs:363-451)
                dl = []
                for c in range(nchunks):
                    ids = sets[c % len(sets)]
                    dl.append(([dat[c, i] if i < k else par[c, i - k] for i in ids], ids))
                rec[:] = 0
                ctx.decode_chunks(k, n, B, 0, dl, out=rec)  # warm
                if not np.array_equal(rec.reshape(-1), host):
                    raise SystemExit(f"host decode_chunks (download patterns) mismatch ({mode})")
                t0 = time.perf_counter()
                for _ in range(reps):
                    ctx.decode_chunks(k, n, B, 0, dl, out=rec)
                res["decode_download" if mode == "pageable" else "decode_pinned_download"] = round(
                    reps * nchunks * chunk_bytes / GIB / (time.perf_counter() - t0), 3)
            if mode == "pinned":
                rec = None
                rbuf.free()
        if mode == "pinned":
            src.free()
            dst.free()
    return {"value": res["pageable"], "unit": "GiB/s", "pinned_value": res["pinned"],
            "decode_value": res.get("decode"), "decode_pinned_value": res.get("decode_pinned"),
            "decode_download_value": res.get("decode_download"),
            "decode_pinned_download_value": res.get("decode_pinned_download"),
            "hashed_value": res.get("hashed"), "hashed_pinned_value": res.get("hashed_pinned"),
            "what": f"storb_rs_encode_chunks: {nchunks} x {chunk_bytes >> 20} MiB host chunks "
                    "-> H2D -> encode -> D2H parity, one stream per copy direction; value = pageable caller "
                    "buffers (staged), pinned_value = page-locked caller buffers (zero-copy kernels); "
                    "hashed_value = storb_rs_encode_chunks_hashed (parity + every share's blake3 "
                    "id computed on the GPU), pageable; hashed_pinned_value = the same from "
                    "page-locked chunks (read in place by the encode kernel); "
                    f"decode_value = storb_rs_decode_chunks of the same chunks with shares "
                    f"{sorted(erased)} lost (host shares in, chunks out), pageable; "
                    "decode_pinned_value = the same from page-locked shares into a page-locked "
                    "output (zero-copy decode kernels, no host copies); *_download_value = the "
                    "same two with each chunk's own survivor set (--erase-pattern download)"}


def _contention_probe(seconds=0.05):
    """CPU the measuring thread gets over wall time on a pure host loop (numpy
    XOR over 4 MiB): well below 1 means the host descheduled it, and any
    per-call latency measured beside it is inflated."""
    a = np.arange(1 << 22, dtype=np.uint8)
    b = np.empty_like(a)
    t0, c0, it = time.perf_counter(), time.thread_time(), 0
    while time.perf_counter() - t0 < seconds:
        np.bitwise_xor(a, 0x5A, out=b)
        it += 1
    wall = time.perf_counter() - t0
    return round((time.thread_time() - c0) / wall, 3), round(it * a.size / wall / 1e9, 2)


def shim_path_rate(ctx, seconds=0.4):
    """The drop-in path as Storb reaches it. The unchanged piece.rs calls
    Fec::encode / Fec::decode once per chunk (piece.rs:328-329,383-386), which
    the zfec-rs shim maps onto storb_rs_encode / storb_rs_decode with
    pageable Vec buffers (integration/zfec-rs-mi355x/src/lib.rs:142-186).
    One thread, one chunk per call, Storb's own sizing of three object sizes
    (upload.rs:209 chunking, piece.rs:307-317 k and m). Two figures per call:
    `call` = the C call alone on pageable caller buffers; `shim` = what
    lib.rs does around it too (m fresh zeroed Vecs, the k data shares copied
    out of the chunk -- since round 4 one storb_rs_encode_shares call into
    m unzeroed Vecs, the data shares copied by the library during the
    kernel; decode: a fresh output Vec). Median per-call latency;
    decode loses data shares 0.. (2 at most) and gets the first k survivors
    by index, as decode_chunk hands them over (piece.rs:368-381)."""
    L = _lib.lib()
    res = {"what": "per-chunk storb_rs_encode / storb_rs_decode from one thread, pageable "
                   "buffers, as the zfec-rs shim calls them (lib.rs:142-186)"}
    # The calling thread runs on the GPU's socket, as storb_rs_ctx_create(-1)
    # arranges on a multi-socket node (a thread gets a GPU of its own node);
    # the numa entry below repeats the (4, 6) calls from each node.
    gnode = L.storb_rs_device_numa_node(ctx.device)
    by_node = _node_cpus()
    saved = os.sched_getaffinity(0)
    res["allowed_cpus_per_node"] = {str(k): len(v) for k, v in by_node.items()}
    if gnode >= 0 and gnode in by_node:
        os.sched_setaffinity(0, by_node[gnode])
        res["caller"] = f"pinned to the {len(by_node[gnode])} allowed CPUs of NUMA node {gnode} (the GPU's)"
    else:
        res["caller"] = "unpinned (GPU node unknown or not in the allowed CPU set)"
    try:
        return _shim_rows(ctx, L, res, seconds, by_node)
    finally:
        os.sched_setaffinity(0, saved)


def _shim_rows(ctx, L, res, seconds, by_node):
    cpu_ratio, xor_gbs = _contention_probe()
    res["host_probe"] = {"thread_cpu_over_wall": cpu_ratio, "numpy_xor_GBps": xor_gbs}
    rows = []
    for obj, chunk in ((1 << 20, 256 << 10), (16 << 20, 1 << 20), (1 << 30, 8 << 20)):
        k, n = _lib.get_k_and_m(chunk)
        B = -(-chunk // k)
        data = np.frombuffer(np.random.default_rng(chunk).bytes(chunk), dtype=np.uint8).copy()
        par = [np.zeros(B, np.uint8) for _ in range(n - k)]
        pp = (_lib.vp * (n - k))(*[x.ctypes.data for x in par])
        bo, po = _lib.sz(), _lib.sz()
        lost = list(range(min(2, n - k)))
        surv = [i for i in range(n) if i not in lost][:k]
        row = {"object_bytes": obj, "chunk_bytes": chunk, "k": k, "m_total": n,
               "lost": lost, "survivors": surv}

        def enc_call():
            rc = L.storb_rs_encode(ctx.handle, k, n, data.ctypes.data, chunk, pp,
                                   _lib.C.byref(bo), _lib.C.byref(po))
            if rc:
                raise SystemExit(f"shim_path: storb_rs_encode rc {rc}")

        def enc_shim():
            # lib.rs Fec::encode: m Vecs with capacity b (not zero-filled), all
            # m shares written by one storb_rs_encode_shares call (the data
            # shares copied by the library's host pool during the kernel)
            shares = [np.empty(B, np.uint8) for _ in range(n)]
            ptr = (_lib.vp * n)(*[x.ctypes.data for x in shares])
            rc = L.storb_rs_encode_shares(ctx.handle, k, n, data.ctypes.data, chunk, ptr,
                                          _lib.C.byref(bo), _lib.C.byref(po))
            if rc:
                raise SystemExit(f"shim_path: storb_rs_encode_shares rc {rc}")

        enc_call()
        allsh = [data[j * B:(j + 1) * B].copy() for j in range(k)] + [x.copy() for x in par]
        sh = [allsh[i] for i in surv]
        sp_ = (_lib.vp * k)(*[x.ctypes.data for x in sh])
        ids = (_lib.C.c_uint32 * k)(*surv)
        out = np.zeros(chunk, np.uint8)

        def dec_call():
            rc = L.storb_rs_decode(ctx.handle, k, n, sp_, ids, k, B, 0, out.ctypes.data)
            if rc:
                raise SystemExit(f"shim_path: storb_rs_decode rc {rc}")

        def dec_shim():
            o = np.empty(k * B, np.uint8)  # Vec::with_capacity(k*b - padding), filled by the call
            rc = L.storb_rs_decode(ctx.handle, k, n, sp_, ids, k, B, 0, o.ctypes.data)
            if rc:
                raise SystemExit(f"shim_path: storb_rs_decode rc {rc}")

        dec_call()
        if not np.array_equal(out, data):
            raise SystemExit(f"shim_path: decode round trip mismatch ({k},{n})")
        for name, f in (("encode_call", enc_call), ("encode_shim", enc_shim),
                        ("decode_call", dec_call), ("decode_shim", dec_shim)):
            f()
            lat = []
            t0, c0 = time.perf_counter(), time.thread_time()
            while time.perf_counter() - t0 < seconds or len(lat) < 11:
                t = time.perf_counter_ns()
                f()
                lat.append(time.perf_counter_ns() - t)
            wall = time.perf_counter() - t0
            lat.sort()
            us = lat[len(lat) // 2] / 1e3
            row[name] = {"median_us": round(us, 2), "p10_us": round(lat[len(lat) // 10] / 1e3, 2),
                         "GiBps": round(chunk / GIB / (us * 1e-6), 3), "calls": len(lat),
                         "thread_cpu_over_wall": round((time.thread_time() - c0) / wall, 3)}
        if (k, n) == (4, 6):
            row["numa"] = _shim_numa(ctx, {"encode_call": enc_call, "decode_call": dec_call},
                                     chunk, seconds, by_node)
        rows.append(row)
    res["geometries"] = rows
    return res


def pcie_ceiling(dev, nbytes=256 << 20, reps=4):
    """The box's PCIe copy rates, measured in this run (SDMA, page-locked
    host memory): H2D, D2H and both directions at once on two streams; and
    what that allows an RS(4,2) encode that moves 1.5 bytes per user byte
    (data in, parity out)."""
    h_in = torch.empty(nbytes, dtype=torch.uint8).pin_memory()
    h_out = torch.empty(nbytes, dtype=torch.uint8).pin_memory()
    d_in = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    d_out = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    s1, s2 = torch.cuda.Stream(device=dev), torch.cuda.Stream(device=dev)
    res = {}
    for name, ops in (("h2d", ((s1, d_in, h_in),)), ("d2h", ((s1, h_out, d_out),)),
                      ("both", ((s1, d_in, h_in), (s2, h_out, d_out)))):
        for st, dst, src in ops:  # warm
            with torch.cuda.stream(st):
                dst.copy_(src, non_blocking=True)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(reps):
            for st, dst, src in ops:
                with torch.cuda.stream(st):
                    dst.copy_(src, non_blocking=True)
        torch.cuda.synchronize(dev)
        res[name + "_GBps"] = round(len(ops) * reps * nbytes / (time.perf_counter() - t0) / 1e9, 1)
    res["rs42_encode_ceiling_GiBps_user"] = round(res["both_GBps"] * 1e9 / 1.5 / GIB, 2)
    res["what"] = (f"torch pinned copies, {nbytes >> 20} MiB x {reps}, SDMA; both = H2D and D2H "
                   f"at once on two streams; the RS(4,2) ceiling = both / 1.5 bytes moved per user "
                   f"byte (zero-copy kernels can exceed it: they overlap the two directions)")
    return res


def _node_cpus():
    """{numa node: [allowed logical CPUs]} for this process's affinity set."""
    out = {}
    for c in sorted(os.sched_getaffinity(0)):
        node = _cpu_where(c)["numa_node"]
        out.setdefault(node, []).append(c)
    return out


def _shim_numa(ctx, calls, chunk, seconds, by_node):
    """The same single calls with the calling thread pinned to the CPUs of the
    GPU's NUMA node, then to those of another node of the allowed set: a
    pageable call's host copies cross the socket link when the caller sits on
    the other node (storb_rs_device_numa_node says which is which)."""
    import ctypes
    libc = ctypes.CDLL(None)
    gnode = _lib.lib().storb_rs_device_numa_node(ctx.device)
    res = {"gpu_numa_node": gnode,
           "allowed_cpus_per_node": {str(k): len(v) for k, v in by_node.items()},
           "caller_cpu_during_default_run": _cpu_where(libc.sched_getcpu())}
    if gnode < 0 or gnode not in by_node:
        res["skipped"] = "GPU node unknown or not in the allowed CPU set"
        return res
    others = [n for n in by_node if n != gnode and n is not None]
    saved = os.sched_getaffinity(0)
    try:
        for label, node in (("caller_on_gpu_node", gnode),
                            ("caller_on_other_node", others[0] if others else None)):
            if node is None:
                res[label] = None
                continue
            os.sched_setaffinity(0, by_node[node])
            r = {"node": node}
            for name, f in calls.items():
                f()
                lat = []
                t0 = time.perf_counter()
                while time.perf_counter() - t0 < seconds or len(lat) < 11:
                    t = time.perf_counter_ns()
                    f()
                    lat.append(time.perf_counter_ns() - t)
                lat.sort()
                us = lat[len(lat) // 2] / 1e3
                r[name] = {"median_us": round(us, 2),
                           "GiBps": round(chunk / GIB / (us * 1e-6), 3)}
            res[label] = r
    finally:
        os.sched_setaffinity(0, saved)
    return res


def shard_hash_rate(ctx, w, stream, reps=3):
    """blake3 of every shard of the batch where encode left it (Storb's piece
    ids, upload.rs:623): data shares + parity shares, device-resident."""
    dev = w.data.device
    hd = torch.empty(w.N * w.k * 32, dtype=torch.uint8, device=dev)
    hp = torch.empty(w.N * (w.n - w.k) * 32, dtype=torch.uint8, device=dev)
    sp = stream.cuda_stream

    def go():
        ctx.blake3_batch_dev(w.dptr, w.B, w.N * w.k, w.B, hd.data_ptr(), stream=sp)
        ctx.blake3_batch_dev(w.pptr, w.B, w.N * (w.n - w.k), w.B, hp.data_ptr(), stream=sp)

    go()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        go()
    e1.record(stream)
    e1.synchronize()
    ms = e0.elapsed_time(e1) / reps
    nbytes = w.N * w.n * w.B
    res = {"value": round(nbytes / (ms * 1e-3) / 1e9, 1), "unit": "GB/s of shard bytes",
           "ms": round(ms, 4), "shards": w.N * w.n, "shard_bytes": w.B,
           "what": "blake3 (Storb piece id) of all data+parity shards, batched kernel"}
    res["encode_with_piece_ids"] = encode_hashed_rate(ctx, w, stream, hd, hp)
    return res


def encode_hashed_rate(ctx, w, stream, hd, hp, reps=5):
    """Encode plus every share's piece id (upload.rs:418-420 then :623), device
    resident, two ways: the encode kernel then the hash kernel over the shards
    it left in HBM (k*B read twice, parity written then read back), and
    storb_rs_encode_hashed_dev, which for (2, 3) / (4, 6) runs one kernel that
    hashes each share while it encodes (rs_encode_hash<k, n-k>, every byte
    crosses HBM once). Self-checked: both give the same parity and digests.
    Both are VALU-bound (blake3's compression), so the fused figure is
    reported against the two-kernel one, with the HBM bytes it moves."""
    k, n, B, N = w.k, w.n, w.B, w.N
    sp = stream.cuda_stream
    dev = w.data.device
    h = torch.empty(N * n * 32, dtype=torch.uint8, device=dev)

    def two():
        ctx.encode_batch_dev(k, n, B, N, w.dptr, w.pptr, stream=sp)
        ctx.blake3_batch_dev(w.dptr, B, N * k, B, hd.data_ptr(), stream=sp)
        ctx.blake3_batch_dev(w.pptr, B, N * (n - k), B, hp.data_ptr(), stream=sp)

    def fused():
        ctx.encode_hashed_dev(k, n, B, N, w.dptr, w.pptr, h.data_ptr(), stream=sp)

    two()
    par_ref = w.parity.clone()
    with torch.cuda.stream(stream):
        w.parity.zero_()
    fused()
    stream.synchronize()
    want = torch.cat([hd.view(N, k, 32), hp.view(N, n - k, 32)], dim=1).reshape(-1)
    ok = torch.equal(w.parity, par_ref) and torch.equal(h, want)
    del par_ref
    if not ok:
        raise SystemExit("encode_hashed_dev mismatch against encode + blake3")
    res = {"what": "device-resident encode + blake3 of all n shares per stripe",
           "self_check": "parity and digests equal between the two paths"}
    for name, go in (("two_kernels", two), ("one_call", fused)):
        go()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(reps):
            go()
        e1.record(stream)
        e1.synchronize()
        ms = e0.elapsed_time(e1) / reps
        res[name] = {"ms": round(ms, 4),
                     "GiBps_user": round(N * w.chunk / GIB / (ms * 1e-3), 1)}
    fused_kernel = (k, n) in ((2, 3), (4, 6)) and B % 1024 == 0 and B <= (256 << 10)
    res["one_call"]["kernel"] = (f"rs_encode_hash<{k},{n - k}>" if fused_kernel
                                 else "encode kernel + blake3_batch_kernel")
    res["one_call"]["hbm_GBps_algorithmic"] = round(
        N * n * B / (res["one_call"]["ms"] * 1e-3) / 1e9, 1)
    res["speedup"] = round(res["two_kernels"]["ms"] / res["one_call"]["ms"], 3)
    return res


def download_sets(k, n, nchunks, seed, fail=0.0):
    """Per-chunk survivor sets as Storb's download collects them: the first
    k + 1 pieces to arrive from 10 fetch threads (download.rs:363-451,
    storb_amd/objects.py download_arrivals); decode_chunk then sorts and
    takes the first k (piece.rs:368-381)."""
    from storb_amd import objects
    rng = np.random.default_rng(seed)
    sets = []
    while len(sets) < nchunks:
        fail_set = {i for i in range(n) if rng.random() < fail} if fail > 0 else ()
        got = objects.download_arrivals(k, n, rng, fail=fail_set)
        if len(got) >= k:
            sets.append(got)
    return sets


def download_leg(ctx, w, stream, a, reps=100):
    """Storb's real download decode, device-resident, beside the headline
    (outside its timed region): the batch's chunks each keep their own
    survivor set (download_sets), and one storb_rs_decode_stripes_dev call
    rebuilds every chunk's lost data shares in place -- one mixed-row launch
    (rs_apply_desc_mix) for the chunks that lost 1-4 data shares, one more
    per larger count. Self-checked: lost rows wiped, rebuilt, compared with
    the pristine data. Calls back to back on one stream (each call's host
    work -- patterns, records, descriptor upload -- overlaps the previous
    call's kernels), HIP events around `reps` calls. Algorithmic bytes per
    call: sum over chunks with e > 0 lost data shares of (k + e) * B."""
    k, n, B, N = w.k, w.n, w.B, w.N
    sp = stream.cuda_stream
    sets = download_sets(k, n, N, SEED_BASE + 4242)
    lost = [[j for j in range(k) if j not in sorted(x)[:k]] for x in sets]
    ids, cnt = _lib.encode_stripe_shares(sets)
    w.encode()
    ref = w.data.clone()
    view = w.data.view(N, k, B)
    with torch.cuda.stream(stream):
        for si, ls in enumerate(lost):
            for e in ls:
                view[si, e].zero_()
    ctx.decode_stripes_dev_raw(k, n, B, N, ids, cnt, w.dptr, w.pptr, w.dptr, stream=sp)
    stream.synchronize()
    if not torch.equal(w.data, ref):
        raise SystemExit("download decode round trip mismatch")
    del ref
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def call():
        ctx.decode_stripes_dev_raw(k, n, B, N, ids, cnt, w.dptr, w.pptr, w.dptr, stream=sp)
    # the GPU idled through the self-check: the same settle pre-roll as the
    # headline's timed region (settle_device), or the first ms of calls run
    # through the power controller's transient
    settled = settle_device([call], stream, a.settle_ms)
    stream.synchronize()
    # the host's own cost of a call (patterns, records, descriptor upload,
    # launches): 3 calls into an idle descriptor ring, none waits on the GPU
    h0 = time.perf_counter()
    for _ in range(3):
        call()
    host_us = (time.perf_counter() - h0) * 1e6 / 3
    e0.record(stream)
    for _ in range(reps):
        call()
    e1.record(stream)
    stream.synchronize()
    ms = e0.elapsed_time(e1) / reps
    alg = sum((k + len(x)) * B for x in lost if x)
    hist = {}
    for x in lost:
        hist[len(x)] = hist.get(len(x), 0) + 1
    achieved = alg / (ms * 1e-3) / 1e9
    res = {"value": round(N * w.chunk / GIB / (ms * 1e-3), 2), "unit": "GiB/s",
           "what": "GiB/s of chunks reconstructed (device-resident), per-chunk survivor sets "
                   "from simulated download arrivals, one storb_rs_decode_stripes_dev per batch",
           "ms_per_call": round(ms, 4), "calls": reps, "settle": settled,
           "host_us_per_call": round(host_us, 1),
           "kernel": f"rs_apply_desc_mix<{min(k, 32)}>",
           "lost_data_shares_histogram": dict(sorted(hist.items())),
           "distinct_patterns": len({tuple(sorted(x)[:k]) for x in sets}),
           "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                        "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                        "algorithmic_bytes_per_call": alg}}
    if not a.no_traffic:
        # kernel time of the same mixed launch: a kernel-trace child run with
        # --erase-pattern download (its decode leg is this call), timed launches only
        kt = kernel_trace(a, w, a.settle_ms, "download",
                          [leg_kernel_match(a, w, "encode"), "rs_apply_desc_mix<"])
        if "legs" in kt:
            dk = kt["legs"]["decode"]
            # the child's own survivor sets (Workload, --erase-pattern download, rank 0)
            from storb_amd import objects
            rng = np.random.default_rng(SEED_BASE)
            alg_child = 0
            for _ in range(N):
                got = objects.download_arrivals(k, n, rng)
                e = sum(1 for j in range(k) if j not in sorted(got)[:k])
                alg_child += (k + e) * B if e else 0
            res["kernel_trace"] = {"kernel": dk["kernel"], "launches": dk["launches"],
                                   "avg_us": dk["avg_us"], "median_us": dk["median_us"],
                                   "algorithmic_bytes_per_launch": alg_child,
                                   "frac_kernel_time": round(alg_child / (dk["avg_us"] * 1e-6) /
                                                             1e9 / HBM_PEAK_GBS, 4),
                                   "call_overhead_us": round(ms * 1e3 - dk["avg_us"], 1),
                                   "source": kt["source"]}
        else:
            res["kernel_trace"] = kt
        t = pmc_download_traffic(a, w)
        res["roofline"]["traffic"] = t.get("traffic")
        res["roofline"]["traffic_source"] = t.get("traffic_source")
        if t.get("traffic"):
            res["roofline"]["traffic_vs_algorithmic"] = round(t["traffic"] / alg, 5)
    return res


def repair_rate(ctx, w, stream, reps=5):
    """Decode-based repair (repair.rs:44-277 today re-fetches a
    replica): regenerate one lost share of every stripe in place from the
    first k survivors. Two cases: a lost data share and a lost parity share.
    Algorithmic bytes per stripe: k*B read + 1*B written."""
    k, n, B, N = w.k, w.n, w.B, w.N
    sp = stream.cuda_stream
    res = {}
    for name, lost in (("data", 0), ("parity", n - 1)):
        surv = [i for i in range(n) if i != lost][:k]

        def go():
            ctx.repair_batch_dev(k, n, B, N, surv, [lost], w.dptr, w.pptr, stream=sp)

        go()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(reps):
            go()
        e1.record(stream)
        e1.synchronize()
        ms = e0.elapsed_time(e1) / reps
        gbs = N * (k + 1) * B / (ms * 1e-3) / 1e9
        res[name] = {"lost_share": lost, "ms": round(ms, 4), "GBps": round(gbs, 1),
                     "frac": round(gbs / HBM_PEAK_GBS, 4)}
    res["what"] = (f"storb_rs_repair_batch_dev: {N} stripes, one lost share each rebuilt in "
                   f"place from the first {k} survivors; bytes = k*B read + B written")
    return res


def _time_launches(stream, go, reps):
    go()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        go()
    e1.record(stream)
    e1.synchronize()
    return e0.elapsed_time(e1) / reps


def config3_assembly(ctx, w, stream, reps=5):
    """SURVEY 8(d) config 3, "full-chunk assembly reported separately", and
    its control erasure {9, 10, 11} (parity only: the first 8 survivors are
    the data shares, decode is pure assembly). decode_chunk returns a fresh
    chunk (piece.rs:363-387), so here the decode writes a separate chunk
    buffer: every data share, present or rebuilt, is written once, stored by
    the decode kernel from its own loads (fused assembly: k*B read + k*B
    written). (Copying the survivors first measured 0.503 vs 0.361 ms,
    profiles/r1_bench_config3_assembly.json.)"""
    k, n, B, N = w.k, w.n, w.B, w.N
    out = torch.empty_like(w.data)
    sp = stream.cuda_stream
    res = {}
    for erased in ([0, 3, 5], [9, 10, 11]):
        surv = [i for i in range(n) if i not in erased][:k]
        row = {"erased": erased, "survivors": surv}

        def go():
            ctx.decode_batch_dev(k, n, B, N, surv, w.dptr, w.pptr, out.data_ptr(), stream=sp)

        ms = _time_launches(stream, go, reps)
        if not torch.equal(out, w.data):
            raise SystemExit(f"config 3 assembly (erased {erased}) mismatch")
        with torch.cuda.stream(stream):
            out.zero_()
        gbs = N * 2 * k * B / (ms * 1e-3) / 1e9
        row["fused"] = {"ms": round(ms, 4), "GiBps_user": round(N * k * B / GIB / (ms * 1e-3), 1),
                        "GBps": round(gbs, 1), "frac": round(gbs / HBM_PEAK_GBS, 4)}
        res["control" if erased[0] >= k else "erased_data"] = row
    res["what"] = ("decode into a separate chunk buffer (decode_chunk semantics); bytes = "
                   "k*B read + k*B written per chunk; assembly inside the decode kernel")
    return res


def config4_storb_faithful(ctx, w, stream, reps=5):
    """SURVEY 8(d) config 4 secondary figure: Storb's own sizing of a 1 MiB
    object (upload.rs:209 piece_length(1 MiB) = 256 KiB chunks; piece.rs:307-317
    get_k_and_m(256 KiB) = (2, 3)): 4 chunks of 256 KiB per object, each k=2,
    m=3 (B = 128 KiB). The rank's objects are contiguous, so its chunks are
    too: one batched launch over 4*N stripes."""
    from storb_amd import piece as P
    plen = P.piece_length(w.chunk)
    k, n = P.get_k_and_m(plen)
    B = -(-plen // k)
    stripes = w.N * (w.chunk // plen)
    par = torch.empty(stripes * (n - k) * B, dtype=torch.uint8, device=w.data.device)
    sp = stream.cuda_stream

    def go():
        ctx.encode_batch_dev(k, n, B, stripes, w.dptr, par.data_ptr(), stream=sp)

    ms = _time_launches(stream, go, reps)
    gbs = stripes * n * B / (ms * 1e-3) / 1e9
    return {"chunk_bytes": plen, "k": k, "m_total": n, "shard_bytes": B, "stripes": stripes,
            "ms": round(ms, 4), "GiBps_user": round(w.N * w.chunk / GIB / (ms * 1e-3), 1),
            "GBps": round(gbs, 1), "frac": round(gbs / HBM_PEAK_GBS, 4),
            "kernel": f"rs_apply_perm<{k},{n - k}>",
            "what": "Storb-faithful sizing of the same objects: 1 MiB object -> 4 x 256 KiB "
                    "chunks, k=2, m=3, one batched launch; bytes = k*B read + (n-k)*B written"}


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
        return "rs_apply_desc_mix<"
    if leg in w.jit_legs:
        return f"storb_bs_jit_k{w.k}_r{jit_blocks(w.k, leg_rows(w, leg))[1]}_"
    if leg == "encode":
        if a.kernel == "auto" and (w.k, w.n) in ((16, 24), (32, 48), (64, 96)):
            return f"rs_encode_bitslice<{w.k}, {w.n}>"
        k, r = w.k, w.n - w.k
    else:
        k, r = w.k, sum(1 for x in w.erased if x < w.k)
    kb = 1
    while kb < min(k, 32):
        kb <<= 1
    return f"rs_apply_{'lds' if a.kernel == 'lds' else 'perm'}<{kb}, {r if r <= 8 else 16},"


def _child(a, erase_pattern, steps=3, warmup=1, settle_ms=0.0):
    """This workload as a short child run (the program rocprofv3 starts)."""
    child = [sys.executable, os.path.abspath(__file__), "--config", str(a.config),
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
               *_child(a, erase_pattern or a.erase_pattern, a.steps, a.warmup, settle_ms)]
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


def settle_device(legs, stream, ms):
    """Run whole steps, untimed, for at least `ms` of wall time. After an
    idle period the chip comes up at full clock and its power controller
    then pulls back: in the kernel traces (profiles/r5a_*) launches 3-12 ms
    into the load take 250-268 us against 238-242 us before and after, so a
    10 ms timed region that starts 4 ms after the load began (the driver's
    --steps 20 --warmup 5) measured that transient, not the kernel."""
    if ms <= 0:
        return {"ms": 0.0, "steps": 0}
    t0, n = time.perf_counter(), 0
    while (time.perf_counter() - t0) * 1e3 < ms:
        for _ in range(8):
            for f in legs:
                f()
        n += 8
        stream.synchronize()
    return {"ms": round((time.perf_counter() - t0) * 1e3, 1), "steps": n}


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


def _pmc_passes(a, erase_pattern, seq=False):
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
    child = _child(a, erase_pattern)
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
    vals, err = _pmc_passes(a, "download")
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
    vals, err = _pmc_passes(a, a.erase_pattern)
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
        names["encode"] = (f"rs_encode_bitslice<{w.k},{w.n}>" if bits
                           else jit_name(w, "encode") if "encode" in w.jit_legs
                           else f"rs_apply_{table}<{min(w.k, 32)},{w.n - w.k}>")
    if "decode" in w.legs and w.sets is not None:
        names["decode"] = (f"rs_apply_desc_mix<{min(w.k, 32)}> (per-stripe descriptors: one "
                           f"launch for the stripes that lost 1-4 data shares, one per larger "
                           f"count; descriptors copied in by copy_u32x4_kernel)")
    elif "decode" in w.legs:
        e = sum(1 for x in w.erased if x < w.k)
        names["decode"] = (jit_name(w, "decode") if "decode" in w.jit_legs
                           else f"rs_apply_{table}<{min(w.k, 32)},{e}>")
    return names


class Workload:
    """Device-resident buffers + the launches of one step."""

    def __init__(self, a, ctx, dev, sp, rank, world):
        self.ctx, self.sp = ctx, sp
        c = a.config
        if c == 2:
            self.k, self.n, chunk, self.erased = 4, 6, 1 << 20, [0, 1]
            N = a.chunks or 1024
            seed0 = SEED_BASE + rank * N
            self.legs = ("encode", "decode")
            self.metric = METRIC
            self.scaling = "weak"
            self.workload = (f"RS(k=4,m=2) [storb k=4,m=6] encode + decode(erased [0, 1]) "
                             f"of {N} x 1 MiB chunks per GPU, device-resident")
        elif c == 3:
            self.k, self.n, chunk, self.erased = 8, 12, 256 << 10, [0, 3, 5]
            N = a.chunks or 4096
            seed0 = SEED_BASE + rank * N
            self.legs = ("decode",)
            self.metric = ("GiB/s device-resident RS decode, 256 KiB chunks k=8 m=4, "
                           "3 data shards erased")
            self.scaling = "weak"
            self.workload = (f"RS(k=8,m=4) [storb k=8,m=12] decode, erased [0, 3, 5], "
                             f"survivors first 8 by index, {N} x 256 KiB chunks per GPU")
        elif c in (5, 6, 7):
            E = 2 if a.erase is None else a.erase
            if c == 5:
                self.k, self.n, chunk = 16, 24, 8 << 20
                N = a.chunks or 128
                what = "8 MiB chunks (a 1 GiB object)"
                self.metric = ("GiB/s device-resident RS encode+decode, 8 MiB chunks k=16 m=8 "
                               "(Storb's geometry for a 1 GiB object)")
            elif c == 6:
                self.k, self.n, chunk = 32, 48, 32 << 20
                N = a.chunks or 32
                what = "32 MiB chunks (objects of 16-64 GiB)"
                self.metric = ("GiB/s device-resident RS encode+decode, 32 MiB chunks k=32 m=16 "
                               "(Storb's geometry for objects of 16 GiB to ~160 GiB)")
            else:
                self.k, self.n, chunk = 64, 96, 128 << 20
                N = a.chunks or 8
                what = "128 MiB chunks (objects from ~160 GiB)"
                self.metric = ("GiB/s device-resident RS encode+decode, 128 MiB chunks k=64 m=32 "
                               "(Storb's widest geometry, objects from ~160 GiB)")
            if not 0 < E <= self.n - self.k:
                raise SystemExit(f"--erase must be in 1..{self.n - self.k}")
            self.erased = list(range(E))
            self.metric += f", {E} data shares lost"
            seed0 = SEED_BASE + rank * N
            self.legs = ("encode", "decode")
            self.scaling = "weak"
            self.workload = (f"RS(k={self.k},m={self.n - self.k}) [storb k={self.k},m={self.n}] "
                             f"encode + decode(erased {self.erased}) of {N} x {what} per GPU, "
                             f"device-resident")
        else:
            self.k, self.n, chunk, self.erased = 4, 6, 1 << 20, []
            mine = partition.objects_for_rank(a.objects, rank, world)
            N = len(mine)
            seed0 = None  # object i gets seed SEED_BASE + i (see _fill_strided)
            self.legs = ("encode",)
            self.metric = ("GiB/s batched RS(k=4,m=2) encode of 10 000 independent 1 MiB "
                           "objects, round-robin over GPUs")
            self.scaling = "strong"
            self.workload = (f"{a.objects} x 1 MiB objects, object i on rank i mod {world}; "
                             f"this rank {N} objects, one batched launch per step")
        self.chunk, self.N = chunk, N
        self.jit_legs = set()  # legs whose launches are run-time-compiled kernels
        k, n = self.k, self.n
        self.B = chunk // k
        self.survivors = [i for i in range(n) if i not in self.erased][:k]
        self.sets = None  # per-chunk collected pieces (--erase-pattern download)
        self.fixed_erased = list(self.erased)
        if a.erase_pattern == "download" and "decode" in self.legs:
            from storb_amd import objects
            rng = np.random.default_rng(SEED_BASE + rank)
            sets = []
            while len(sets) < N:
                fail = {i for i in range(n) if rng.random() < a.fail} if a.fail > 0 else ()
                got = objects.download_arrivals(k, n, rng, fail=fail)
                if len(got) >= k:  # fewer: reconstruct_chunk's Err, that chunk is not decoded
                    sets.append(got)
            self.sets = sets
            self.lost = [[j for j in range(k) if j not in sorted(s_)[:k]] for s_ in sets]
            self.set_ids, self.set_cnt = _lib.encode_stripe_shares(sets)
            hist = {}
            for x in self.lost:
                hist[len(x)] = hist.get(len(x), 0) + 1
            self.pattern_stats = {"distinct_patterns": len({tuple(sorted(s_)[:k]) for s_ in sets}),
                                  "lost_data_shares_histogram": dict(sorted(hist.items())),
                                  "fail_probability": a.fail, "fetch_threads": 10,
                                  "latency": "lognormal(0, 0.5) per fetch"}
            self.erased = "download"
            self.workload += (f"; decode: per-chunk survivors from simulated download arrivals "
                              f"({self.pattern_stats['distinct_patterns']} distinct patterns)")
        self.data = torch.empty(N * k * self.B, dtype=torch.uint8, device=dev)
        self.parity = torch.empty(N * (n - k) * self.B, dtype=torch.uint8, device=dev)
        self.dptr, self.pptr = self.data.data_ptr(), self.parity.data_ptr()
        if c == 4:
            self._fill_strided(rank, world)
        else:
            ctx.fill_splitmix_dev(self.dptr, chunk, N, chunk, seed0, stream=sp)
        if "decode" in self.legs and "encode" not in self.legs:
            self.encode()  # config 3 needs parity to decode from

    def _fill_strided(self, rank, world):
        # One launch per object keeps the seed = SEED_BASE + global object index
        # exact; only done once at setup.
        for j in range(self.N):
            i = rank + j * world
            self.ctx.fill_splitmix_dev(self.dptr + j * self.chunk, self.chunk, 1, self.chunk,
                                       SEED_BASE + i, stream=self.sp)

    def encode(self):
        self.ctx.encode_batch_dev(self.k, self.n, self.B, self.N, self.dptr, self.pptr,
                                  stream=self.sp)

    def decode(self):
        if self.sets is not None:
            self.ctx.decode_stripes_dev_raw(self.k, self.n, self.B, self.N, self.set_ids,
                                            self.set_cnt, self.dptr, self.pptr, self.dptr,
                                            stream=self.sp)
            return
        self.ctx.decode_batch_dev(self.k, self.n, self.B, self.N, self.survivors, self.dptr,
                                  self.pptr, self.dptr, stream=self.sp)

    def lost_rows(self):
        """Per stripe, the data shares the decode leg rebuilds."""
        if self.sets is not None:
            return self.lost
        return [[x for x in self.erased if x < self.k]] * self.N

    def alg_bytes(self, leg):
        # encode reads k*B, writes (n-k)*B per stripe; decode with
        # e erased data shards reads k*B and writes e*B (stripes with e = 0
        # are not touched by an in-place decode).
        k, n, B, N = self.k, self.n, self.B, self.N
        if leg == "encode":
            return N * n * B
        if self.sets is not None:
            return sum((k + len(x)) * B for x in self.lost if x)
        e = sum(1 for x in self.erased if x < k)
        return N * (k + e) * B


def rank_info(rank, world, local, dev, use_pg):
    """Who ran: every rank's GPU (ordinal + PCI bus) and the process group's
    own rank count, so a scaling line cannot silently be a 1-rank number."""
    props = torch.cuda.get_device_properties(dev)
    me = {"rank": rank, "device": local, "name": props.name,
          "pci_bus": getattr(props, "pci_bus_id", None), "host": platform.node()}
    if not use_pg:
        return {"world_size": 1, "backend": None, "pg_ranks": 1, "ranks": [me]}
    ranks = [None] * world
    dist.all_gather_object(ranks, me)
    return {"world_size": world, "backend": dist.get_backend(),
            "pg_ranks": dist.get_world_size(), "ranks": ranks,
            "distinct_gpus": len({(r["host"], r["device"]) for r in ranks})}


def line_extras(rank, world, minimal, config):
    """The bounded, untimed extras this rank adds to its line, all run after
    the last barrier of the timed region. Rank 0 always carries the
    single-thread CPU baseline (N > 1 lines too: the driver's scaling lines
    need it beside the GPU figure); the heavier ones (live PMC traffic passes,
    copy ceiling, threaded CPU baselines, PCIe-inclusive and per-call host
    rates, hashing, repair) only at world size 1, where no other rank waits."""
    if rank != 0 or minimal:
        return set()
    ex = {"cpu_baseline"}
    if world > 1:
        return ex
    ex |= {"traffic", "copy_ceiling", "kernel_trace"}
    if config in (2, 5, 6):
        ex |= {"cpu_threads", "host_path", "shim_path", "hashing", "repair", "download"}
    if config == 3:
        ex.add("assembly")
    if config == 4:
        ex.add("storb_faithful")
    return ex


def init_pg(a, world, dev):
    """One process group per job: RCCL ('nccl') with each rank bound to its
    GPU, or gloo for the rehearsal with several ranks on one GPU. --force-pg
    at world size 1 creates a one-rank group so the exact multi-rank sequence
    runs on a one-GPU box."""
    if world == 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(launch.free_port()))
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
    if a.dist_backend == "nccl":
        dist.init_process_group("nccl", device_id=dev)
    else:
        dist.init_process_group(a.dist_backend)
    if dist.get_world_size() != world:
        raise SystemExit(f"process group has {dist.get_world_size()} ranks, expected {world}")


def main():
    a = parse()
    # One process per GPU. Decided before any GPU call: with --gpus N > 1 and
    # no WORLD_SIZE in the environment this process only spawns the N ranks
    # (storb_amd/launch.py); under torch.distributed.run it is one of them.
    plan = launch.plan_launch(a.gpus, os.environ, torch.cuda.device_count(), a.dist_backend)
    if plan.action == "spawn":
        sys.exit(launch.spawn_ranks([os.path.abspath(__file__), *sys.argv[1:]], plan.world))
    world, rank, local = plan.world, plan.rank, plan.device
    # STORB_BENCH_DEVICE pins every rank to one GPU (multi-rank rehearsal on a
    # single-GPU box with --dist-backend gloo); by default rank i uses GPU i.
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    use_pg = world > 1 or a.force_pg
    if use_pg:
        init_pg(a, world, dev)
    ranks = rank_info(rank, world, local, dev, use_pg)

    ctx = _lib.Context(local)
    ctx.set_kernel({"auto": _lib.KERNEL_AUTO, "perm": _lib.KERNEL_PERM,
                    "lds": _lib.KERNEL_LDS}[a.kernel])
    stream = torch.cuda.Stream(device=dev)
    sp = stream.cuda_stream
    w = Workload(a, ctx, dev, sp, rank, world)
    stream.synchronize()

    if not a.no_check and w.erased:
        # Self-consistency at full size: wipe the erased shards, rebuild them
        # in place from parity, compare with the pristine copy. Bit-exactness
        # against the oracle is covered by tests/test_gpu_parity.py.
        ref = w.data.clone()
        w.encode()
        view = w.data.view(w.N, w.k, w.B)
        with torch.cuda.stream(stream):
            if w.sets is not None:
                for si, lost in enumerate(w.lost):
                    for e in lost:
                        view[si, e].zero_()
            else:
                for e in w.erased:
                    if e < w.k:
                        view[:, e].zero_()
        w.decode()
        stream.synchronize()
        if not torch.equal(w.data, ref):
            raise SystemExit("decode round trip mismatch")
        del ref

    # A decode matrix the table kernel is VALU-bound on gets its own compiled
    # bit-sliced kernel (rs_jit.cpp); the first decode queued its compile.
    # Let it finish so the timed steps run what a steady-state download runs.
    # (Config 7's k = 64 encode runs compiled kernels too.) One pass of every
    # leg queues them; wait for the compiles.
    for _ in range(2):  # a matrix is compiled once asked for twice (rs_jit.cpp)
        for leg in w.legs:
            getattr(w, leg)()
    stream.synchronize()
    _lib.jit_wait()
    # Which legs run compiled kernels (for the kernel names and the PMC match).
    for leg in w.legs:
        j0 = _lib.jit_stats()["launches"]
        getattr(w, leg)()
        stream.synchronize()
        if _lib.jit_stats()["launches"] > j0:
            w.jit_legs.add(leg)
    jit0 = _lib.jit_stats()
    legs = [getattr(w, leg) for leg in w.legs]
    clocks0 = gpu_clocks(local) if rank == 0 and not a.minimal else None
    settled = settle_device(legs, stream, a.settle_ms)
    for _ in range(a.warmup):
        for f in legs:
            f()
    stream.synchronize()

    # Timed region: K steps with one HIP event at each end on the launch
    # stream (a timing event after every leg costs 2.5-3 % of the step:
    # profiles/r1_leg_events.txt). GPU time per step = region / K.
    e_start = torch.cuda.Event(enable_timing=True)
    e_end = torch.cuda.Event(enable_timing=True)
    each = a.leg_events == "each"
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(len(legs) + 1)]
          for _ in range(a.steps if each else 0)]
    if use_pg:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e_start.record(stream)
    for i in range(a.steps):
        if each:
            ev[i][0].record(stream)
        for j, f in enumerate(legs):
            f()
            if each:
                ev[i][j + 1].record(stream)
    e_end.record(stream)
    stream.synchronize()
    torch.cuda.synchronize()
    if use_pg:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    gpu_ms = e_start.elapsed_time(e_end) / a.steps
    clocks1 = gpu_clocks(local) if rank == 0 and not a.minimal else None
    jit1 = _lib.jit_stats()
    if not each:
        # Per-leg split (which kernel took what) from an untimed pass of the
        # same steps with an event after every leg; reported, not used for
        # `value` or `achieved`.
        n_probe = min(a.steps, 50)
        ev = [[torch.cuda.Event(enable_timing=True) for _ in range(len(legs) + 1)]
              for _ in range(n_probe)]
        for i in range(n_probe):
            ev[i][0].record(stream)
            for j, f in enumerate(legs):
                f()
                ev[i][j + 1].record(stream)
        stream.synchronize()
    leg_ms = [sum(e[j].elapsed_time(e[j + 1]) for e in ev) / len(ev) for j in range(len(legs))]
    units = w.N * w.chunk * len(legs)  # user bytes per step on this rank
    mine = {"rank": rank, "elapsed_s": round(elapsed, 6), "gpu_ms_per_step": round(gpu_ms, 4),
            "units_per_step": units}
    if use_pg:
        tdev = dev if a.dist_backend == "nccl" else torch.device("cpu")
        t = torch.tensor([elapsed, float(units)], dtype=torch.float64, device=tdev)
        tmax = t[:1].clone()
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        tsum = t[1:].clone()
        dist.all_reduce(tsum, op=dist.ReduceOp.SUM)
        elapsed, units_all = float(tmax.item()), float(tsum.item())
        per_rank = [None] * world
        dist.all_gather_object(per_rank, mine)
    else:
        units_all = float(units)
        per_rank = [mine]
    value = a.steps * units_all / GIB / elapsed
    alg = {leg: w.alg_bytes(leg) for leg in w.legs}
    # algorithmic bytes of one step / GPU time of one step in the timed region
    # (config 2: every launch is rs_apply_perm<4,2> with 1.5 GiB, so this is
    # also bytes per launch / average launch duration)
    achieved = sum(alg.values()) / (gpu_ms * 1e-3) / 1e9

    out = {
        "metric": w.metric,
        "value": round(value, 3),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(elapsed / a.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": w.scaling,
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic: splitmix64 bytes, seed 0x5709B + object index, resident in HBM",
        "config": {
            "workload": w.workload,
            "baseline_config": a.config,
            "k": w.k, "m_total": w.n, "parity": w.n - w.k, "chunk_bytes": w.chunk,
            "shard_bytes": w.B, "chunks_per_gpu": w.N, "erased": w.erased,
            "erase_pattern": a.erase_pattern,
            "patterns": getattr(w, "pattern_stats", None),
            "survivors": w.survivors if w.erased and w.sets is None else None,
            "kernel": a.kernel,
            "parallelism": f"independent objects, {world} GPU(s), no collectives",
        },
        "launch": ranks,
        "per_rank": per_rank,
        "settle": dict(settled, why="untimed whole steps before the warm-up: the power "
                                    "controller's transient after an idle GPU (settle_device)"),
        "roofline": {
            "bound": "hbm",
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": None,
            "traffic_source": "not measured (N > 1, --minimal or --no-traffic)",
            "kernel": kernel_names(a.kernel, w),
            "gpu_ms_per_step": round(gpu_ms, 4),
            "launch_ms": round(gpu_ms / len(legs), 4),
            "leg_ms": {leg: round(ms, 4) for leg, ms in zip(w.legs, leg_ms)},
            "leg_ms_source": ("events after every leg inside the timed region" if each else
                              "separate untimed pass with an event after every leg"),
            "alg_bytes_per_launch": alg,
            "kernel_match": {leg: leg_kernel_match(a, w, leg) for leg in w.legs},
            # download patterns: one mixed-row launch for the stripes that lost
            # 1-4 data shares, one per larger count (decode_stripes.cpp)
            "launches_per_leg": {leg: ((1 if any(0 < len(x) <= 4 for x in w.lost) else 0) +
                                       len({len(x) for x in w.lost if len(x) > 4})
                                       if leg == "decode" and w.sets is not None
                                       else jit_blocks(w.k, leg_rows(w, leg))[0]
                                       if leg in w.jit_legs else 1) for leg in w.legs},
            "copy_ceiling_gbs": None,
            "jit": {"launches_in_run": jit1["launches"] - jit0["launches"],
                    "compiled": jit1["compiled"], "compile_ms": round(jit1["compile_ms"], 1),
                    "fallbacks": jit1["fallbacks"]},
        },
        "cpu_baseline": None,
    }
    ex = line_extras(rank, world, a.minimal, a.config)
    if clocks0 is not None:
        out["roofline"]["gpu_clocks"] = {"before_settle": clocks0, "after_timed_region": clocks1}
    if "kernel_trace" in ex and not a.no_traffic:
        kt = kernel_trace(a, w, a.settle_ms)
        if "legs" in kt:
            # without the pre-roll: what a short region right after idle measures
            kt0 = kernel_trace(a, w, 0.0)
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
            out["roofline"].update(pmc_traffic(a, w))
    if "copy_ceiling" in ex:
        out["roofline"]["copy_ceiling_gbs"] = copy_ceiling(ctx, dev, stream)
    if "cpu_baseline" in ex and a.cpu_seconds > 0:
        out["cpu_baseline"] = cpu_baseline(w.k, w.n, w.chunk, set(w.fixed_erased), a.cpu_seconds,
                                           do_encode="encode" in w.legs,
                                           do_decode="decode" in w.legs,
                                           survivor_sets=w.sets[:64] if w.sets else None)
        out["cpu_baseline"]["cpu_model"] = cpu_model()
        out["cpu_baseline"]["measured_by"] = f"rank 0 of {world}, after the timed region"
    if "cpu_threads" in ex and a.cpu_seconds > 0:
        # the same code on threads over independent chunks -- at
        # this box's CPU share per GPU (16) and at nproc (every logical CPU the
        # OS reports; the cgroup quota, if any, is stated beside it).
        er = set(w.fixed_erased) if w.sets is None else set(w.lost[0])
        nch = max(32, (256 << 20) // w.chunk)
        out["cpu_baseline_threads"] = cpu_baseline_threads(w.k, w.n, w.chunk, er,
                                                           threads=16, nchunks=nch)
        nproc = os.cpu_count() or 1
        out["cpu_baseline_nproc"] = cpu_baseline_threads(
            w.k, w.n, w.chunk, er, threads=nproc, nchunks=max(nch, nproc))
        out["cpu_baseline_nproc"]["cpu_quota"] = cpu_quota()
    if "host_path" in ex and not a.no_host_path:
        pc = pcie_ceiling(dev)
        out["pcie_inclusive"] = host_path_rate(ctx, w.k, w.n, w.chunk,
                                               nchunks=max(8, (256 << 20) // w.chunk),
                                               erased=[e for e in w.fixed_erased if e < w.k],
                                               sets=w.sets or download_sets(
                                                   w.k, w.n, 64, SEED_BASE + 4343))
        out["pcie_inclusive"]["pcie_ceiling"] = pc
    if "shim_path" in ex:
        out["shim_path"] = shim_path_rate(ctx)
    if "hashing" in ex:
        out["shard_hashing"] = shard_hash_rate(ctx, w, stream)
    if "repair" in ex:
        out["repair"] = repair_rate(ctx, w, stream)
    if "download" in ex and w.sets is None and "decode" in w.legs:
        out["download_decode"] = download_leg(ctx, w, stream, a)
    if "assembly" in ex:
        out["assembly"] = config3_assembly(ctx, w, stream)
    if "storb_faithful" in ex:
        out["storb_faithful"] = config4_storb_faithful(ctx, w, stream)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if use_pg:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
