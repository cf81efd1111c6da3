"""Host-inclusive legs of the bench line: PCIe-inclusive batch encode /
decode (storb_rs_encode_chunks / storb_rs_decode_chunks), the per-chunk calls
as the zfec-rs shim makes them, the box's PCIe ceiling, and the concurrent
all-rank host leg (every rank at once)."""
from __future__ import annotations

import hashlib
import os
import time

import numpy as np
import torch

from storb_amd import _lib

from . import GIB, SEED_BASE
from .cpu import cpu_where, node_cpus


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
            # the library call as a compiled binding makes it: share pointers
            # marshalled once, outside the timed loop (_lib.decode_chunks_raw)
            mp, mi, mc, keep = _lib.marshal_chunks(chunks, B)
            t0 = time.perf_counter()
            for _ in range(reps):
                ctx.decode_chunks_raw(k, n, B, 0, mp, mi, mc, rec)
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
                mp, mi, mc, keep = _lib.marshal_chunks(dl, B)
                t0 = time.perf_counter()
                for _ in range(reps):
                    ctx.decode_chunks_raw(k, n, B, 0, mp, mi, mc, rec)
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
                    "same two with each chunk's own survivor set (--erase-pattern download); "
                    "decode calls timed as a compiled binding makes them: the share pointer "
                    "arrays built once before the timed loop (_lib.decode_chunks_raw)"}


def contention_probe(seconds=0.05):
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
    by_node = node_cpus()
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
    cpu_ratio, xor_gbs = contention_probe()
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
           "caller_cpu_during_default_run": cpu_where(libc.sched_getcpu())}
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


ALL_RANK_GEOMETRIES = (
    # (name, chunk bytes): Storb's sizing of each (piece.rs:307-317)
    ("config2", 1 << 20),   # 1 MiB chunks -> k=4, m=6 (BASELINE configs 2 / 4)
    ("config5", 8 << 20),   # 8 MiB chunks of a 1 GiB object -> k=16, m=24 (config 5)
)


def all_ranks_host_leg(ctx, dev, rank, world, barrier, mib=256, reps=3, lost=(0, 1)):
    """Every rank at once, host memory in and out (config 5's
    scaling limit is host-side -- PCIe, pinned memory, host threads -- not the
    device). Each rank encodes its own `mib` MiB of chunks from host memory
    (storb_rs_encode_chunks: H2D, encode, parity D2H) and rebuilds them with
    data shares `lost` erased (storb_rs_decode_chunks: the first k survivors
    by index in, chunks out), from pageable and from page-locked buffers, at
    config 2's and config 5's geometry -- the concurrent per-object loops of
    upload.rs:418-420 / download.rs:505-529, one rank per GPU. Every timed
    leg starts after a barrier, so all ranks run it together; each rank times
    its own `reps` calls. Aggregate = sum of user bytes over ranks / the
    slowest rank's time. Inputs are splitmix64 chunks, seed SEED_BASE + global
    chunk index (rank * chunks + c), filled on the device and copied out
    (untimed); every rank checks its decodes byte for byte against the input
    and reports a sha256 of its parity (pageable and page-locked must agree;
    tests/test_gpu_dist.py recomputes it with the oracle). Returns this rank's
    record; the caller gathers them (aggregate_all_ranks)."""
    me = {"rank": rank, "device": int(dev.index), "geometries": {}}
    for name, chunk in ALL_RANK_GEOMETRIES:
        k, n = _lib.get_k_and_m(chunk)
        B = -(-chunk // k)
        nch = max(1, (mib << 20) // chunk)
        surv = [i for i in range(n) if i not in lost][:k]
        d = torch.empty(nch * chunk, dtype=torch.uint8, device=dev)
        ctx.fill_splitmix_dev(d.data_ptr(), chunk, nch, chunk, SEED_BASE + rank * nch)
        ctx.sync()
        src = d.cpu().numpy()
        del d
        row = {"k": k, "m_total": n, "chunk_bytes": chunk, "chunks": nch, "lost": list(lost),
               "survivors": surv, "bytes_per_rep": nch * chunk, "reps": reps}
        digests = {}
        for mode in ("pageable", "pinned"):
            bufs = []
            if mode == "pinned":
                bufs = [_lib.PinnedBuffer(nch * chunk), _lib.PinnedBuffer(nch * (n - k) * B),
                        _lib.PinnedBuffer(nch * chunk)]
                host, par, rec = (b.array for b in bufs)
                rec = rec.reshape(nch, chunk)
            else:
                host = np.empty(nch * chunk, np.uint8)
                par = np.empty(nch * (n - k) * B, np.uint8)
                rec = np.empty((nch, chunk), np.uint8)
            host[:] = src
            par[:] = 0
            rec[:] = 0
            ctx.encode_chunks(k, n, host, chunk, nch, out=par)  # warm; the parity digested
            digests[mode] = hashlib.sha256(par).hexdigest()
            barrier()
            t0 = time.perf_counter()
            for _ in range(reps):
                ctx.encode_chunks(k, n, host, chunk, nch, out=par)
            row[f"encode_{mode}_s"] = time.perf_counter() - t0
            dat, pv = host.reshape(nch, k, B), par.reshape(nch, n - k, B)
            chunks = [([dat[c, i] if i < k else pv[c, i - k] for i in surv], surv)
                      for c in range(nch)]
            ctx.decode_chunks(k, n, B, 0, chunks, out=rec)  # warm
            row[f"roundtrip_{mode}"] = bool(np.array_equal(rec.reshape(-1), src))
            mp, mi, mc, keep = _lib.marshal_chunks(chunks, B)  # outside the timed loop
            barrier()
            t0 = time.perf_counter()
            for _ in range(reps):
                ctx.decode_chunks_raw(k, n, B, 0, mp, mi, mc, rec)
            row[f"decode_{mode}_s"] = time.perf_counter() - t0
            del chunks, dat, pv, host, par, rec, keep
            for b in bufs:
                b.free()
        row["parity_sha256"] = digests["pageable"]
        row["parity_modes_agree"] = digests["pageable"] == digests["pinned"]
        me["geometries"][name] = row
    return me


def aggregate_all_ranks(records, pins):
    """The gathered per-rank records of all_ranks_host_leg as one line entry:
    per geometry and leg, aggregate GiB/s = sum of bytes / max rank time, and
    every rank's own rate; per rank, its CPU set and its GPU's NUMA node."""
    out = {"ranks": len(records), "geometries": {}}
    for name, _ in ALL_RANK_GEOMETRIES:
        rows = [r["geometries"][name] for r in records]
        g = {x: rows[0][x] for x in ("k", "m_total", "chunk_bytes", "chunks", "lost", "reps")}
        for leg in ("encode_pageable", "encode_pinned", "decode_pageable", "decode_pinned"):
            secs = [r[f"{leg}_s"] for r in rows]
            tot = sum(r["bytes_per_rep"] * r["reps"] for r in rows)
            g[leg] = {"aggregate_GiBps": round(tot / GIB / max(secs), 3),
                      "per_rank_GiBps": [round(r["bytes_per_rep"] * r["reps"] / GIB / s, 3)
                                         for r, s in zip(rows, secs)],
                      "slowest_rank_s": round(max(secs), 4)}
        g["bit_exact"] = all(r["roundtrip_pageable"] and r["roundtrip_pinned"] and
                             r["parity_modes_agree"] for r in rows)
        g["parity_sha256_per_rank"] = [r["parity_sha256"] for r in rows]
        out["geometries"][name] = g
    out["per_rank"] = [{"rank": r["rank"], "device": r["device"],
                        "gpu_numa_node": p.get("gpu_numa_node"), "cpus": p.get("cpus"),
                        "pinned": p.get("pinned")} for r, p in zip(records, pins)]
    out["what"] = ("every rank at once after a barrier: storb_rs_encode_chunks (host chunks -> "
                   "H2D -> encode -> parity D2H) and storb_rs_decode_chunks (first k survivors "
                   "-> chunks, data shares lost) from pageable and page-locked buffers; "
                   "aggregate = sum of user bytes / slowest rank; each rank pinned to its GPU's "
                   "NUMA node (per_rank.cpus); decode share pointers marshalled before the "
                   "timed loop, as a compiled binding passes them")
    return out
