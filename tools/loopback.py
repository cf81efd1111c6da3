#!/usr/bin/env python3
"""BASELINE config 5: loopback upload -> store -> retrieve -> reconstruct.

One validator (this process) and N miner processes on 127.0.0.1 speak
Storb's formats (storb_amd/wire.py). The object is chunked as the reference
does (upload.rs:209,333-383: chunk = piece_length(object len)); each chunk is
RS-encoded on the GPU with every shard's blake3 id computed on the device
(storb_rs_encode_chunks_hashed: pinned H2D of data, D2H of parity and ids
only); pieces go to miners over the store framing and each miner's ack must
equal the id; one miner is killed (seeded); download gathers k+1 pieces per
chunk in piece_idx order (download.rs:336-451), verifies blake3, and
reconstructs with decode_chunk's rule (sort, first k) on the GPU
(storb_rs_decode). The reference itself cannot run this offline (live
chain, network-fetched crsqlite, >100-chunk channel hang,
download.rs:26,500) -- see SURVEY.md fact 9.

usage: python tools/loopback.py [--size BYTES] [--miners N] [--gpus G]   (one JSON line)
       python tools/loopback.py miner --store-port P --http-port Q --dir D
"""
from __future__ import annotations

import argparse
import http.server
import json
import os
import random
import shutil
import socket
import socketserver
import subprocess
import sys
import tempfile
import threading
import time
from concurrent.futures import ThreadPoolExecutor
from urllib.parse import parse_qs, urlparse

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

from storb_amd import _lib, objects, wire  # noqa: E402

GIB = float(1 << 30)
HANDSHAKE = bytes(96)  # opaque HandshakePayload bytes (auth out of scope)


# ------------------------------------------------------------------ miner
def miner_main(a):
    store = wire.ObjectStore(a.dir)

    class StoreHandler(socketserver.BaseRequestHandler):
        def handle(self):
            sock = self.request
            sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            while True:
                frame = wire.read_store_frame(sock)
                if frame is None:
                    return
                _, piece = frame
                h = _lib.blake3(piece)  # lib.rs:265
                store.write(h.hex(), piece)
                sock.sendall(h + b"\n")

    class PieceHandler(http.server.BaseHTTPRequestHandler):
        protocol_version = "HTTP/1.1"

        def do_GET(self):
            u = urlparse(self.path)
            q = parse_qs(u.query)
            try:
                if u.path != "/piece" or "handshake" not in q:
                    raise ValueError
                hexhash = q["piecehash"][0]
                if len(bytes.fromhex(hexhash)) != wire.HASH_LEN:
                    raise ValueError
                # routes.rs:188-206: bincode PieceResponse, piece bytes by sendfile
                store.send_piece_response(self.connection, hexhash,
                                          b"HTTP/1.1 200 OK\r\nContent-Length: %d\r\n\r\n")
            except (OSError, ValueError, KeyError):
                body = b"error"
                self.send_response(500)
                self.send_header("Content-Length", str(len(body)))
                self.end_headers()
                self.wfile.write(body)

        def log_message(self, *args):
            pass

    class TS(socketserver.ThreadingMixIn, socketserver.TCPServer):
        daemon_threads = True
        allow_reuse_address = True

    class HS(http.server.ThreadingHTTPServer):
        daemon_threads = True

    s1 = TS(("127.0.0.1", a.store_port), StoreHandler)
    s2 = HS(("127.0.0.1", a.http_port), PieceHandler)
    threading.Thread(target=s1.serve_forever, daemon=True).start()
    threading.Thread(target=s2.serve_forever, daemon=True).start()
    print("ready", flush=True)
    while True:
        time.sleep(3600)


# -------------------------------------------------------------- validator
def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def splitmix_bytes(seed: int, n: int) -> np.ndarray:
    i = np.arange(1, -(-n // 8) + 1, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + i * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z ^= z >> np.uint64(31)
    return z.view(np.uint8)[:n]


def run(a, inspect=None):
    """One loopback round trip; returns the JSON-able result. inspect (tests):
    called as inspect(obj, metas, miner_dirs) before the miners' stores are
    removed -- metas[c] holds chunk c's (k, m, B, padlen, off, len), its GPU
    piece ids and the miner of every piece."""
    tmp = tempfile.mkdtemp(prefix="storb_loop_")
    miners = []
    for m in range(a.miners):
        sp, hp = free_port(), free_port()
        proc = subprocess.Popen([sys.executable, os.path.abspath(__file__), "miner",
                                 "--store-port", str(sp), "--http-port", str(hp),
                                 "--dir", os.path.join(tmp, f"miner{m}")],
                                stdout=subprocess.PIPE, text=True)
        miners.append({"proc": proc, "store": sp, "http": hp,
                       "dir": os.path.join(tmp, f"miner{m}")})
    for m in miners:
        if m["proc"].stdout.readline().strip() != "ready":
            raise SystemExit("miner failed to start")
    try:
        return _run(a, miners, inspect)
    finally:
        for m in miners:
            if m["proc"].poll() is None:
                m["proc"].kill()
            m["proc"].wait()
        shutil.rmtree(tmp, ignore_errors=True)


def _run(a, miners, inspect=None):
    M = len(miners)
    # one context per GPU; chunks partition across them. With
    # more contexts than devices they share devices (multi-GPU rehearsal).
    ngpu = a.gpus or max(1, _lib.device_count())
    ctxs = objects.device_contexts(ngpu)
    ctx = ctxs[0]
    obj = splitmix_bytes(0x5709B + a.seed, a.size)
    chunks = objects.chunk_spans(a.size)
    chunk_size = chunks[0][1]
    metas = []  # per chunk: k, m, B, padlen, piece hashes, miner per piece

    # A running validator has warm contexts (pinned staging and device
    # buffers allocated, tables built): one untimed encode + reconstruct of
    # the same geometry first, so the clock sees the steady state.
    if not a.cold:
        w = objects.encode_object(obj, contexts=ctxs)
        objects.reconstruct_object(
            w.chunks, [{i: sh[i] for i in range(1, cv.k + 1)} for cv, sh in zip(w.chunks, w.data)],
            contexts=ctxs)
        del w

    # ---- upload: GPU encode + GPU piece ids (objects.encode_object: one
    # batched call per run of equal chunks), then the store framing
    t0 = time.perf_counter()
    enc = objects.encode_object(obj, contexts=ctxs)
    t_encode = time.perf_counter() - t0

    per_miner = [[] for _ in range(M)]
    for ci, ((off, ln), cv, pv, sh) in enumerate(zip(chunks, enc.chunks, enc.pieces, enc.data)):
        n = cv.m
        metas.append({"k": cv.k, "m": n, "B": cv.chunk_size, "padlen": cv.padlen, "off": off,
                      "len": ln, "hashes": [p.piece_hash for p in pv],
                      "miner": [(ci * n + i) % M for i in range(n)]})
        for i in range(n):
            per_miner[(ci * n + i) % M].append((ci, i, sh[i]))

    def upload(m):
        s = socket.create_connection(("127.0.0.1", miners[m]["store"]))
        s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        bad = 0
        for ci, i, piece in per_miner[m]:
            ack = wire.send_piece(s, HANDSHAKE, piece)
            bad += ack != metas[ci]["hashes"][i]
        s.close()
        return bad

    with ThreadPoolExecutor(M) as ex:
        ack_mismatch = sum(ex.map(upload, range(M)))
    t_upload = time.perf_counter() - t0
    if ack_mismatch:
        raise SystemExit(f"{ack_mismatch} miner acks differ from the GPU piece ids")

    # ---- a seeded miner failure
    dead = random.Random(a.kill_seed).randrange(M)
    miners[dead]["proc"].kill()
    miners[dead]["proc"].wait()

    # ---- download: > k unique pieces per chunk, blake3-verified, then decode
    t1 = time.perf_counter()
    tls = threading.local()

    def fetch(m, hexhash):
        conns = getattr(tls, "conns", None)
        if conns is None:
            conns = tls.conns = {}
        c = conns.get(m)
        if c is None:
            c = conns[m] = wire.PieceClient("127.0.0.1", miners[m]["http"])
        status, body = c.get(hexhash, HANDSHAKE.hex())
        if status != 200:
            raise IOError("miner error")
        return body

    def gather(ci):
        meta = metas[ci]
        got = {}
        for i in range(meta["m"]):  # get_pieces_by_chunk: ORDER BY piece_idx
            if len(got) > meta["k"]:
                break
            h = meta["hashes"][i]
            try:
                body = fetch(meta["miner"][i], h.hex())
                got[i] = wire.deserialise_piece_response(body, h)  # blake3 check
            except (OSError, ValueError):
                if hasattr(tls, "conns"):
                    c = tls.conns.pop(meta["miner"][i], None)
                    if c is not None:
                        c.close()
        return ci, got

    with ThreadPoolExecutor(16) as ex:
        gathered = dict(ex.map(gather, range(len(chunks))))
    t_fetch = time.perf_counter() - t1

    needed_parity = 0
    for ci, meta in enumerate(metas):
        if len(gathered[ci]) < meta["k"]:
            raise SystemExit(f"chunk {ci}: not enough pieces ({len(gathered[ci])} < {meta['k']})")
        needed_parity += any(i >= meta["k"] for i in sorted(gathered[ci])[:meta["k"]])
    t2 = time.perf_counter()
    # reconstruct_chunk per chunk (first k by index), batched per run of
    # equal chunks straight into the object buffer
    out = objects.reconstruct_object(enc.chunks, [gathered[ci] for ci in range(len(metas))],
                                     contexts=ctxs)
    t_decode = time.perf_counter() - t2
    t_download = time.perf_counter() - t1
    ok = bool(np.array_equal(out, obj))
    # the same reconstruct into a download buffer the validator reuses (the
    # fresh one above is first-touched page by page as the chunks land in it;
    # the bench's pcie_inclusive decode figures write pre-touched buffers)
    t3 = time.perf_counter()
    again = objects.reconstruct_object(enc.chunks, [gathered[ci] for ci in range(len(metas))],
                                       contexts=ctxs, out=out)
    t_decode_reused = time.perf_counter() - t3
    ok = ok and bool(np.array_equal(again, obj))
    nshards = sum(m["m"] for m in metas)
    res = {
        "config": "BASELINE 5 loopback (validator + miners on 127.0.0.1)",
        "object_bytes": a.size, "chunks": len(chunks), "chunk_bytes": chunk_size,
        "k_m": sorted({(m["k"], m["m"]) for m in metas}), "shards": nshards,
        "shard_bytes_total": sum(m["m"] * m["B"] for m in metas), "miners": M,
        "killed_miner": dead, "chunks_decoded_through_parity": needed_parity,
        "bit_exact": ok, "ack_mismatch": ack_mismatch,
        "t_encode_s": round(t_encode, 4), "t_upload_s": round(t_upload, 4),
        "t_fetch_s": round(t_fetch, 4), "t_decode_s": round(t_decode, 4),
        "t_download_s": round(t_download, 4),
        "encode_GiBps": round(a.size / GIB / t_encode, 3),
        "upload_GiBps": round(a.size / GIB / t_upload, 3),
        "download_GiBps": round(a.size / GIB / t_download, 3),
        "end_to_end_GiBps": round(a.size / GIB / (t_upload + t_download), 3),
        # the two GPU legs (host in / host out, PCIe included) apart from the
        # harness's Python socket legs, which bound the end-to-end figure
        "gpu_legs": {"encode_with_piece_ids_GiBps": round(a.size / GIB / t_encode, 3),
                     "batched_reconstruct_GiBps": round(a.size / GIB / t_decode, 3),
                     "batched_reconstruct_reused_out_GiBps": round(a.size / GIB / t_decode_reused, 3),
                     "what": "objects.encode_object (storb_rs_encode_chunks_hashed) and "
                             "objects.reconstruct_object (storb_rs_decode_chunks), host "
                             "buffers in and out, PCIe included; reused_out = the same into "
                             "an already-touched object buffer"},
        "harness_legs": {"store_framing_upload_s": round(t_upload - t_encode, 4),
                         "python_fetch_s": round(t_fetch, 4),
                         "what": "Python sockets / HTTP of this harness (wire.py), not the "
                                 "GPU path: the end-to-end figure is bound by these"},
        "devices": [c.device for c in ctxs], "contexts": len(ctxs), "warm": not a.cold,
        "visible_gpus": _lib.device_count(),
    }
    if inspect is not None:
        inspect(obj, metas, [m["dir"] for m in miners])
    return res


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "miner":
        p = argparse.ArgumentParser()
        p.add_argument("role")
        p.add_argument("--store-port", type=int, required=True)
        p.add_argument("--http-port", type=int, required=True)
        p.add_argument("--dir", required=True)
        miner_main(p.parse_args())
        return
    p = argparse.ArgumentParser()
    p.add_argument("--size", type=int, default=1 << 30)
    p.add_argument("--miners", type=int, default=8)
    p.add_argument("--seed", type=int, default=1)
    p.add_argument("--kill-seed", type=int, default=7)
    p.add_argument("--cold", action="store_true",
                   help="no untimed warm-up (first-call staging allocation inside the clock)")
    p.add_argument("--gpus", type=int, default=0,
                   help="contexts to spread the chunks over, one per GPU (0 = every "
                        "visible GPU; more than visible = several per device)")
    a = p.parse_args()
    res = run(a)
    print(json.dumps(res), flush=True)
    if not res["bit_exact"]:
        sys.exit(1)


if __name__ == "__main__":
    main()
