"""Device-resident side legs of the bench line, run after the timed region:
the copy ceiling, piece-id hashing, Storb's download decode, decode-based
repair, config 3's assembly and config 4's Storb-faithful sizing, and the
settle pre-roll."""
from __future__ import annotations

import time

import numpy as np
import torch

from storb_amd import _lib

from . import GIB, HBM_PEAK_GBS, SEED_BASE
from .prof import kernel_trace, leg_kernel_match, pmc_download_traffic


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
           "kernel": ({16: "rs_apply_desc_mix_ks<16, 2>", 32: "rs_apply_desc_mix_ks<32, 4>"}.get(k)
                      or f"rs_apply_desc_mix<{min(k, 32)}>"),
           "lost_data_shares_histogram": dict(sorted(hist.items())),
           "distinct_patterns": len({tuple(sorted(x)[:k]) for x in sets}),
           "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                        "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                        "algorithmic_bytes_per_call": alg}}
    if not a.no_traffic:
        # kernel time of the same mixed launch: a kernel-trace child run with
        # --erase-pattern download (its decode leg is this call), timed launches only
        kt = kernel_trace(a, w, a.settle_ms, "download",
                          [leg_kernel_match(a, w, "encode"), "rs_apply_desc_mix"])
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


def time_launches(stream, go, reps):
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

        ms = time_launches(stream, go, reps)
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

    ms = time_launches(stream, go, reps)
    gbs = stripes * n * B / (ms * 1e-3) / 1e9
    return {"chunk_bytes": plen, "k": k, "m_total": n, "shard_bytes": B, "stripes": stripes,
            "ms": round(ms, 4), "GiBps_user": round(w.N * w.chunk / GIB / (ms * 1e-3), 1),
            "GBps": round(gbs, 1), "frac": round(gbs / HBM_PEAK_GBS, 4),
            "kernel": f"rs_apply_perm<{k},{n - k}>",
            "what": "Storb-faithful sizing of the same objects: 1 MiB object -> 4 x 256 KiB "
                    "chunks, k=2, m=3, one batched launch; bytes = k*B read + (n-k)*B written"}


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
