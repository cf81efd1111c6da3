#!/usr/bin/env python3
"""The storb_rs_host_register / _unregister GPU checks, run in a child
process of their own by tests/test_gpu_runtime.py and
tests/test_gpu_patterns.py.

Registering caller memory creates a device mapping of it; unregistering
tears that mapping down and frees its device addresses. This round saw two
illegal-address faults in torch host->device copies later in a pytest
process that had run these checks early (cause not found; no
stale mapping visible to HIP, the removed register_probe). Running the checks in
their own process keeps whatever registration does to the process's GPU
address space out of the rest of the suite. Each case is oracle-exact.

usage: python tests/registered_ranges.py direct_paths | each_chunk_own_range
"""
import os
import random
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import coracle  # noqa: E402  (the checker)
from storb_amd import _lib  # noqa: E402


def rnd(n, seed):
    return np.frombuffer(np.random.default_rng(seed).bytes(n), dtype=np.uint8).copy()


def page_aligned(nbytes, align=4096):
    raw = np.zeros(nbytes + align, dtype=np.uint8)
    off = (-raw.ctypes.data) % align
    return raw, raw[off:off + nbytes]


def oracle_stripes(k, n, B, ns, seed):
    data = rnd(ns * k * B, seed)
    par = coracle.encode_parity_many(k, n, data, k * B, ns, threads=8)
    return data.reshape(ns, k, B), par.reshape(ns, n - k, B)


def direct_paths(ctx):
    """storb_rs_host_register'd caller memory (mapped) used in place at
    interior offsets by encode, decode and encode_chunks."""
    k, n, B = 4, 6, 64 << 10
    L = k * B
    raw, buf = page_aligned(16 << 20)
    base = buf.ctypes.data
    lib = _lib.lib()
    assert lib.storb_rs_host_register(base, buf.nbytes) == _lib.OK
    try:
        assert _lib.host_is_pinned(buf[4096:4096 + L])
        data = buf[4096:4096 + L]                  # interior, 16-B aligned
        data[:] = rnd(L, 11)
        want, _, _ = coracle.encode(k, n, data)
        parity = [buf[(1 << 20) + i * B:(1 << 20) + (i + 1) * B] for i in range(n - k)]
        ctx.encode_into(k, n, data, parity)
        for i in range(n - k):
            assert np.array_equal(parity[i], want[k + i]), i
        # decode: survivors {1, 3, 4, 5} from registered memory into registered out
        surv = [1, 3, 4, 5]
        sh = [buf[(2 << 20) + j * B:(2 << 20) + (j + 1) * B] for j in range(len(surv))]
        for j, s in enumerate(surv):
            sh[j][:] = want[s]
        out = buf[(3 << 20):(3 << 20) + L]
        out[:] = 0
        ctx.decode_into(k, n, sh, surv, B, 0, out)
        assert np.array_equal(out, data)
        # batch encode: chunks and parity both registered
        nch, cl = 6, 512 << 10
        chunks = buf[(4 << 20):(4 << 20) + nch * cl]
        chunks[:] = rnd(nch * cl, 12)
        pout = buf[(8 << 20):(8 << 20) + nch * (n - k) * (cl // k)]
        ctx.encode_chunks(k, n, chunks, cl, nch, out=pout)
        want_p = coracle.encode_parity_many(k, n, chunks, cl, nch)
        assert np.array_equal(pout, want_p)
    finally:
        assert lib.storb_rs_host_unregister(base) == _lib.OK
    assert not _lib.host_is_pinned(buf[4096:4096 + L])
    del raw


def each_chunk_own_range(ctx):
    """shares of consecutive chunks in separate registered ranges
    at equal spacing -- a device address is taken per range, never derived
    from another chunk's mapping."""
    k, n, B, cnt = 4, 6, 64 << 10, 8
    data, par = oracle_stripes(k, n, B, cnt, 99)
    # one host allocation, one registered range per chunk (equal spacing)
    span = n * B + 4096
    host = np.zeros(cnt * span + 4096, np.uint8)
    base = (-host.ctypes.data) % 4096
    regs = []
    try:
        for ch in range(cnt):
            seg = host[base + ch * span: base + ch * span + n * B]
            seg[:k * B] = data[ch].reshape(-1)
            seg[k * B:] = par[ch].reshape(-1)
            rc = _lib.lib().storb_rs_host_register(seg.ctypes.data, seg.nbytes)
            assert rc == 0
            regs.append(seg)
        out_buf = _lib.PinnedBuffer(cnt * k * B)
        out = out_buf.array.reshape(cnt, k * B)
        rng = random.Random(3)
        chunks = []
        for ch in range(cnt):
            lost = rng.sample(range(k), 2)
            ids = [i for i in range(n) if i not in lost]
            chunks.append(([regs[ch][i * B:(i + 1) * B] for i in ids], ids))
        got = ctx.decode_chunks(k, n, B, 0, chunks, out=out)
        for ch in range(cnt):
            assert np.array_equal(got[ch], data[ch].reshape(-1)), ch
        out_buf.free()
    finally:
        for seg in regs:
            _lib.lib().storb_rs_host_unregister(seg.ctypes.data)


def main():
    torch.zeros(1, device="cuda:0")  # torch's HIP runtime first (storb_amd/_lib.py)
    case = sys.argv[1]
    ctx = _lib.Context(0)
    try:
        {"direct_paths": direct_paths, "each_chunk_own_range": each_chunk_own_range}[case](ctx)
    finally:
        ctx.close()
    print(f"{case} ok")


if __name__ == "__main__":
    main()
