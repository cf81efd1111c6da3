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

After the timed region: every rank at once runs the host-inclusive leg
(pcie_inclusive_all_ranks: host chunks in, parity / chunks out, pageable and
page-locked, configs 2 and 5 geometry); rank 0 alone adds the CPU baseline
and, at world size 1, the side legs (benchkit/legs.py). Each rank process is
pinned to its GPU's NUMA node first (--pin numa).

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
from benchkit import GIB, HBM_PEAK_GBS, SEED_BASE, cpu as bcpu, device as bdev  # noqa: E402
from benchkit import host as bhost, legs as blegs, prof  # noqa: E402
from benchkit.ranks import all_rank_leg, init_pg, line_extras, rank_info  # noqa: E402

METRIC = "GiB/s device-resident RS encode+decode, 1 MiB chunks k=4 m=2, at 1/2/4/8 GPUs"


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
    p.add_argument("--host-mib", type=int, default=256,
                   help="MiB of host chunks per rank and geometry in the all-rank "
                        "host-inclusive leg (pcie_inclusive_all_ranks)")
    p.add_argument("--pin", choices=["numa", "none"], default="numa",
                   help="numa: pin each rank process to its GPU's NUMA node before it "
                        "allocates (the CPU-baseline legs run on the original CPU set)")
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
        st0 = bcpu.proc_stat()
        r = coracle.bench_roundtrip(k, n, sample, chunk_bytes, 8, sets, do_encode, do_decode,
                                    fresh, secs)
        st1 = bcpu.proc_stat()
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
                **bcpu.cpu_where(r["cpu_start"]),
                # time the hypervisor ran something else on this vCPU: the
                # thread's own CPU time does not show it (/proc/stat steal)
                "cpu_steal_frac": bcpu.steal_frac(st0, st1, r["cpu_start"]),
                "speculation": bcpu.speculation_state()}
        if r["cpu_end"] != r["cpu_start"]:
            acct["cpu_end"] = r["cpu_end"]
        return round(legs * r["calls"] * chunk_bytes / GIB / el, 4), r["calls"], el, acct

    value, calls, el, acct = run(True, seconds)
    arith, acalls, ael, aacct = run(False, max(1.0, seconds / 2))
    ssbd = bcpu.ssbd_run(run, max(1.0, seconds / 4))
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
        # speculation enabled (IPC 0.16 vs 3.06, profiles/r4y_ssbd_probe.jsonl,
        # DESIGN.md §5 Host variance); `value` stays the process as started,
        # as the reference would run
        "ssbd_on": ssbd,
        # the figure defined identically on every box (SSBD on for the
        # measuring thread), quoted for GPU/CPU ratios:
        # `value` depends on whether the box leaves store-bypass speculation
        # enabled for the process, which moves this loop 19x
        "comparable": {"value": ssbd.get("value"), "unit": "GiB/s",
                       "definition": "the same 1-thread loop with Speculative Store Bypass "
                                     "Disable on for the measuring thread (prctl)"},
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
    # the rank process onto its GPU's socket before it allocates anything or
    # the library starts its host threads
    pin = bcpu.pin_rank(local, a.pin)
    allowed = pin.pop("allowed")
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
    # bit-sliced kernel (rs_jit.cpp), compiled once asked for twice: two
    # passes of every leg queue the compiles; wait for them, so the timed
    # steps run what a steady-state download runs (config 7's k = 64 encode
    # runs compiled kernels too). Then note which legs launch compiled kernels.
    for _ in range(2):
        for leg in w.legs:
            getattr(w, leg)()
    stream.synchronize()
    _lib.jit_wait()
    for leg in w.legs:
        j0 = _lib.jit_stats()["launches"]
        getattr(w, leg)()
        stream.synchronize()
        if _lib.jit_stats()["launches"] > j0:
            w.jit_legs.add(leg)
    jit0 = _lib.jit_stats()
    legs = [getattr(w, leg) for leg in w.legs]
    clocks0 = prof.gpu_clocks(local) if rank == 0 and not a.minimal else None
    settled = bdev.settle_device(legs, stream, a.settle_ms)
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
    clocks1 = prof.gpu_clocks(local) if rank == 0 and not a.minimal else None
    jit1 = _lib.jit_stats()
    if not each:
        # Per-leg split (which kernel took what) from an untimed pass of the
        # same steps with an event after every leg; reported, not used for
        # `value` or `achieved`.
        ev = [[torch.cuda.Event(enable_timing=True) for _ in range(len(legs) + 1)]
              for _ in range(min(a.steps, 50))]
        for e in ev:
            e[0].record(stream)
            for j, f in enumerate(legs):
                f()
                e[j + 1].record(stream)
        stream.synchronize()
    leg_ms = [sum(e[j].elapsed_time(e[j + 1]) for e in ev) / len(ev) for j in range(len(legs))]
    units = w.N * w.chunk * len(legs)  # user bytes per step on this rank
    mine = {"rank": rank, "elapsed_s": round(elapsed, 6), "gpu_ms_per_step": round(gpu_ms, 4),
            "units_per_step": units, "gpu_numa_node": pin["gpu_numa_node"],
            "cpus": pin["cpus"]}
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
        "roofline": {
            "bound": "hbm",
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": None,
            "traffic_source": "not measured (N > 1, --minimal or --no-traffic)",
            "kernel": prof.kernel_names(a.kernel, w),
            "gpu_ms_per_step": round(gpu_ms, 4),
            "launch_ms": round(gpu_ms / len(legs), 4),
            "leg_ms": {leg: round(ms, 4) for leg, ms in zip(w.legs, leg_ms)},
            "leg_ms_source": ("events after every leg inside the timed region" if each else
                              "separate untimed pass with an event after every leg"),
            "alg_bytes_per_launch": alg,
            "kernel_match": {leg: prof.leg_kernel_match(a, w, leg) for leg in w.legs},
            # download patterns: one mixed-row launch for the stripes that lost
            # 1-4 data shares, one per larger count (decode_stripes.cpp)
            "launches_per_leg": {leg: ((1 if any(0 < len(x) <= 4 for x in w.lost) else 0) +
                                       len({len(x) for x in w.lost if len(x) > 4})
                                       if leg == "decode" and w.sets is not None
                                       else prof.jit_blocks(w.k, prof.leg_rows(w, leg))[0]
                                       if leg in w.jit_legs else 1) for leg in w.legs},
            "copy_ceiling_gbs": None,
            "jit": {"launches_in_run": jit1["launches"] - jit0["launches"],
                    "compiled": jit1["compiled"], "compile_ms": round(jit1["compile_ms"], 1),
                    "fallbacks": jit1["fallbacks"]},
        },
        "cpu_baseline": None,
        "launch": ranks,
        "per_rank": per_rank,
        "settle": dict(settled, why="untimed whole steps before the warm-up: the power "
                                    "controller's transient after an idle GPU (settle_device)"),
    }
    if clocks0 is not None:
        out["roofline"]["gpu_clocks"] = {"before_settle": clocks0, "after_timed_region": clocks1}
    if all_rank_leg(a.minimal, a.config, a.no_host_path):
        # every rank, host memory in and out, all at once (after the timed
        # region: nothing here touches `value`)
        barrier = dist.barrier if use_pg else (lambda: None)
        rec = bhost.all_ranks_host_leg(ctx, dev, rank, world, barrier, mib=a.host_mib)
        recs, pins = [rec], [pin]
        if use_pg:
            recs, pins = [None] * world, [None] * world
            dist.all_gather_object(recs, rec)
            dist.all_gather_object(pins, pin)
        out["pcie_inclusive_all_ranks"] = bhost.aggregate_all_ranks(recs, pins)
    ex = line_extras(rank, world, a.minimal, a.config)
    blegs.side_legs(out, a, ctx, dev, stream, w, ex)
    if "cpu_baseline" in ex and a.cpu_seconds > 0:
        # the reference's CPU path runs unpinned: the rank's original CPU set
        with bcpu.affinity(allowed):
            out["cpu_baseline"] = cpu_baseline(
                w.k, w.n, w.chunk, set(w.fixed_erased), a.cpu_seconds,
                do_encode="encode" in w.legs, do_decode="decode" in w.legs,
                survivor_sets=w.sets[:64] if w.sets else None)
        out["cpu_baseline"]["cpu_model"] = bcpu.cpu_model()
        out["cpu_baseline"]["measured_by"] = f"rank 0 of {world}, after the timed region"
    if "cpu_threads" in ex and a.cpu_seconds > 0:
        # the same code on threads over independent chunks -- at
        # this box's CPU share per GPU (16) and at nproc (every logical CPU the
        # OS reports; the cgroup quota, if any, is stated beside it).
        er = set(w.fixed_erased) if w.sets is None else set(w.lost[0])
        nch = max(32, (256 << 20) // w.chunk)
        nproc = os.cpu_count() or 1
        with bcpu.affinity(allowed):
            out["cpu_baseline_threads"] = cpu_baseline_threads(w.k, w.n, w.chunk, er,
                                                               threads=16, nchunks=nch)
            out["cpu_baseline_nproc"] = cpu_baseline_threads(
                w.k, w.n, w.chunk, er, threads=nproc, nchunks=max(nch, nproc))
        out["cpu_baseline_nproc"]["cpu_quota"] = bcpu.cpu_quota()
    if rank == 0:
        print(json.dumps(out), flush=True)
    if use_pg:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
