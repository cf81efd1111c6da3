#!/usr/bin/env python3
"""Randomised differential test of every host and device entry point against
the CPU oracle (test infrastructure: the oracle is the checker only).

Each round draws a geometry ((k, n) from Storb's sizings plus odd ones), a
chunk length (1 byte .. 6 MiB, ragged), an entry point (single encode /
decode / repair, batched encode_chunks[_hashed] / decode_chunks (page-locked:
scattered or arena shares, decoded in place), device
batched encode / decode / repair / encode with piece ids) and page-locked or
pageable buffers, and
compares the result byte for byte with the oracle. Runs for --seconds and
prints one JSON line; exits non-zero on the first mismatch.

    python tools/fuzz.py --seconds 60 [--seed S]
"""
import argparse
import json
import os
import random
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import coracle  # noqa: E402  (the checker)
from storb_amd import _lib  # noqa: E402

GEOS = [(1, 2), (2, 3), (4, 6), (8, 12), (16, 24), (32, 48), (3, 5), (5, 9), (6, 7), (10, 20),
        (1, 1), (7, 7), (20, 30), (40, 60), (64, 96)]


def rnd(rng, n):
    return np.frombuffer(rng.randbytes(n), dtype=np.uint8).copy()


def pinned_copy(a, keep):
    b = _lib.PinnedBuffer(max(1, a.size))
    keep.append(b)
    arr = b.array[:a.size]
    arr[:] = a
    return arr


def check(cond, what):
    if not cond:
        raise AssertionError(what)


TRACE = None  # --trace FILE: each round's tag, written before it runs


def one(ctx, rng, stats):
    k, n = rng.choice(GEOS)
    L = rng.choice([1, 15, 16, 17, 4095, 65536, 65537, (1 << 20) - 3, 3 << 20,
                    rng.randint(1, 6 << 20), 1 << 20, 256 << 10])
    L = max(L, 1)
    data = rnd(rng, L)
    shares, B, pad = coracle.encode(k, n, data)
    keep = []
    pin = rng.random() < 0.4
    api = rng.choice(["encode", "decode", "repair", "encode_chunks", "hashed", "decode_chunks",
                      "dev_encode", "dev_decode", "dev_repair", "dev_hashed"])
    stats[api] = stats.get(api, 0) + 1
    tag = f"{api} k={k} n={n} L={L} pinned={pin}"
    if TRACE:
        TRACE.write(tag + "\n")
        TRACE.flush()
    if api == "encode":
        src = pinned_copy(data, keep) if pin else data
        par = [pinned_copy(np.zeros(B, np.uint8), keep) if pin else np.zeros(B, np.uint8)
               for _ in range(n - k)]
        check(ctx.encode_into(k, n, src, par) == (B, pad), tag)
        check(all(np.array_equal(par[i], shares[k + i]) for i in range(n - k)), tag)
    elif api == "decode":
        ids = rng.sample(range(n), rng.randint(k, n))
        sh = [pinned_copy(shares[i], keep) if pin else shares[i] for i in ids]
        out = pinned_copy(np.zeros(L, np.uint8), keep) if pin else np.zeros(L, np.uint8)
        ctx.decode_into(k, n, sh, ids, B, pad, out)
        check(np.array_equal(out, data), tag + f" ids={sorted(ids)[:k]}")
    elif api == "repair":
        ids = rng.sample(range(n), k)
        rest = [i for i in range(n) if i not in ids]
        if not rest:
            return
        tg = rng.sample(rest, rng.randint(1, len(rest)))
        got = ctx.repair(k, n, [shares[i] for i in ids], ids, B, tg)
        check(all(np.array_equal(np.frombuffer(g, np.uint8), shares[t]) for g, t in zip(got, tg)),
              tag + f" targets={tg}")
    elif api in ("encode_chunks", "hashed"):
        cnt = rng.randint(1, max(1, min(40, (48 << 20) // max(L, 1))))
        objs = [data] + [rnd(rng, L) for _ in range(cnt - 1)]
        host = np.concatenate(objs)
        if pin:
            host = pinned_copy(host, keep)
        want = np.concatenate([coracle.encode(k, n, o)[0][k:].reshape(-1) for o in objs]) \
            if n > k else np.zeros(0, np.uint8)
        if api == "encode_chunks":
            if n == k:
                return
            out = (pinned_copy(np.zeros(want.size, np.uint8), keep) if pin
                   else np.zeros(want.size, np.uint8))
            ctx.encode_chunks(k, n, host, L, cnt, out=out)
            check(np.array_equal(out[:want.size], want), tag + f" cnt={cnt}")
        else:
            if n == k or B > (16 << 20):
                return
            par, ids = ctx.encode_chunks_hashed(k, n, host, L, cnt)
            check(np.array_equal(par[:want.size], want), tag + f" cnt={cnt}")
            for c in (0, cnt - 1):
                sh = coracle.encode(k, n, objs[c])[0]
                for i in (0, n - 1):
                    check(ids[c, i].tobytes() == _lib.blake3(sh[i]), tag + f" id c={c} i={i}")
    elif api == "decode_chunks":
        cnt = rng.randint(1, max(1, min(24, (32 << 20) // max(L, 1))))
        objs = [data] + [rnd(rng, L) for _ in range(cnt - 1)]
        batch = []
        arena = pin and rng.random() < 0.5  # every chunk's shares at one stride
        if arena:
            ar = pinned_copy(np.zeros(cnt * n * B, np.uint8), keep).reshape(cnt, n, B)
        for c, o in enumerate(objs):
            sh = coracle.encode(k, n, o)[0]
            ids = rng.sample(range(n), rng.randint(k, n))
            if rng.random() < 0.5:  # several chunks with one erasure pattern
                ids = list(range(n - k, n))
            if arena:
                ar[c] = sh
                batch.append(([ar[c, i] for i in ids], ids))
            else:
                batch.append(([pinned_copy(sh[i], keep) if pin else sh[i] for i in ids], ids))
        out = (pinned_copy(np.zeros(cnt * L, np.uint8), keep).reshape(cnt, L) if pin
               else None)
        got = ctx.decode_chunks(k, n, B, pad, batch, out=out)
        check(all(np.array_equal(got[c], objs[c]) for c in range(cnt)),
              tag + f" cnt={cnt} arena={arena}")
    elif api == "dev_hashed":
        # storb_rs_encode_hashed_dev: the fused kernel for (2, 3) / (4, 6)
        # with whole-KiB shares up to 256 KiB, two kernels otherwise
        if n == k:
            return
        ns = rng.randint(1, 40)
        Bd = rng.choice([1024, 2048, 3072, 5 << 10, 64 << 10, 255 << 10, 256 << 10, 1000, 16,
                         512 << 10])
        if ns * n * Bd > (64 << 20):
            ns = max(1, (64 << 20) // (n * Bd))
        pad_d = rng.choice([0, 0, 16, 4096])
        ds, ps = k * Bd + pad_d, (n - k) * Bd + pad_d
        host = rnd(rng, ns * ds)
        d = torch.from_numpy(host).cuda()
        p = torch.zeros(ns * ps, dtype=torch.uint8, device="cuda")
        h = torch.zeros(ns * n * 32, dtype=torch.uint8, device="cuda")
        ctx.encode_hashed_dev(k, n, Bd, ns, d.data_ptr(), p.data_ptr(), h.data_ptr(),
                              ds if pad_d else 0, ps if pad_d else 0)
        ctx.sync()
        par, ids = p.cpu().numpy(), h.cpu().numpy().reshape(ns, n, 32)
        for s_ in sorted({0, ns - 1, rng.randrange(ns)}):
            sh = coracle.encode(k, n, host[s_ * ds:s_ * ds + k * Bd])[0]
            for i in range(k, n):
                o = s_ * ps + (i - k) * Bd
                check(np.array_equal(par[o:o + Bd], sh[i]), tag + f" hashed_dev s={s_} i={i} B={Bd}")
            for t in range(n):
                check(ids[s_, t].tobytes() == _lib.blake3(sh[t].tobytes()),
                      tag + f" hashed_dev id s={s_} t={t} B={Bd}")
    else:
        ns = rng.randint(1, 6)
        Bd = rng.choice([16, 1024, 4096 + 16, 32 << 10, B - B % 16 or 16])
        host = rnd(rng, ns * k * Bd)
        d = torch.from_numpy(host).cuda()
        p = torch.zeros(ns * max(n - k, 1) * Bd, dtype=torch.uint8, device="cuda")
        ctx.encode_batch_dev(k, n, Bd, ns, d.data_ptr(), p.data_ptr())
        ctx.sync()
        par = p.cpu().numpy()
        want = np.concatenate([coracle.encode(k, n, host[s * k * Bd:(s + 1) * k * Bd])[0][k:]
                               .reshape(-1) for s in range(ns)]) if n > k else np.zeros(0)
        check(np.array_equal(par[:want.size], want), tag + f" dev ns={ns} B={Bd}")
        if api == "dev_decode" and n > k:
            ids = rng.sample(range(n), k)
            lost = [i for i in range(k) if i not in ids]
            v = d.view(ns, k, Bd)
            for i in lost:
                v[:, i].fill_(0xA5)
            ctx.decode_batch_dev(k, n, Bd, ns, ids, d.data_ptr(), p.data_ptr(), d.data_ptr())
            ctx.sync()
            check(np.array_equal(d.cpu().numpy(), host), tag + f" dev decode ids={sorted(ids)}")
        elif api == "dev_repair" and n > k:
            ids = rng.sample(range(n), k)
            rest = [i for i in range(n) if i not in ids]
            tg = rng.sample(rest, rng.randint(1, min(4, len(rest))))
            v, pv = d.view(ns, k, Bd), p.view(ns, n - k, Bd)
            for t in tg:
                (v[:, t] if t < k else pv[:, t - k]).fill_(0x5A)
            ctx.repair_batch_dev(k, n, Bd, ns, ids, tg, d.data_ptr(), p.data_ptr())
            ctx.sync()
            check(np.array_equal(d.cpu().numpy(), host), tag + f" dev repair data tg={tg}")
            check(np.array_equal(p.cpu().numpy()[:want.size], want), tag + f" dev repair par tg={tg}")
    for b in keep:
        b.free()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=60)
    ap.add_argument("--seed", type=int, default=int(time.time()) & 0xFFFF)
    ap.add_argument("--trace", default=None)
    a = ap.parse_args()
    # The oracle's byte-wise loop runs ~15x slower on hosts whose store-bypass
    # speculation mispredicts it: SSBD on for this thread
    # (threads started later inherit it), as tests/batch_oracle.py does.
    import ctypes
    ctypes.CDLL(None, use_errno=True).prctl(53, 0, 4, 0, 0)  # PR_SET_SPECULATION_CTRL, STORE_BYPASS, DISABLE
    global TRACE
    if a.trace:
        TRACE = open(a.trace, "a")
    rng = random.Random(a.seed)
    ctx = _lib.Context(0)
    ctx.default_stream = torch.cuda.current_stream(0).cuda_stream
    stats, rounds = {}, 0
    t0 = time.time()
    last = t0
    while time.time() - t0 < a.seconds:
        one(ctx, rng, stats)
        rounds += 1
        if time.time() - last > 20:
            print(json.dumps({"progress_rounds": rounds}), flush=True)
            last = time.time()
    print(json.dumps({"seed": a.seed, "rounds": rounds, "per_api": stats, "mismatches": 0}),
          flush=True)


if __name__ == "__main__":
    main()
