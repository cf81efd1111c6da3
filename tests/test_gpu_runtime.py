"""GPU runtime contracts of the C ABI (round-2 ADVICE / VERDICT items):

* the coefficient-table cache never blocks and never frees a table a queued
  kernel still reads: thousands of distinct erasure patterns on two streams
  through a tiny LRU cache (STORB_RS_TABLE_CACHE), bit-exact;
* hip_stream = NULL runs on the HIP null stream and storb_rs_sync waits for
  it (read back on a separate non-blocking stream);
* caller ranges made page-locked with storb_rs_host_register are used in
  place by the zero-copy paths (interior offsets), matching the oracle.
"""
import itertools
import os
import random

import numpy as np
import pytest
import torch

from oracle import coracle
from storb_amd import _lib

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


def run_registered_case(case):
    """tests/registered_ranges.py CASE in a child process (see its docstring)."""
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    r = subprocess.run([sys.executable, os.path.join(here, "registered_ranges.py"), case],
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0 and f"{case} ok" in r.stdout, (r.returncode, r.stdout[-2000:],
                                                          r.stderr[-4000:])


def rnd(n, seed):
    return np.frombuffer(np.random.default_rng(seed).bytes(n), dtype=np.uint8).copy()


def oracle_stripes(k, n, B, nstripes, seed):
    """Data and parity regions (packed, stripe-major) built by the oracle."""
    data = rnd(nstripes * k * B, seed)
    par = np.empty((nstripes, n - k, B), np.uint8)
    for s in range(nstripes):
        shares, b, pad = coracle.encode(k, n, data[s * k * B:(s + 1) * k * B])
        assert (b, pad) == (B, 0)
        par[s] = shares[k:]
    return data, par.reshape(-1)


def test_table_cache_5000_patterns_two_streams(monkeypatch):
    """5,000 distinct survivor sets of RS(8,16) (storb k=8, m=16), decoded into
    separate buffers on two alternating streams, with an 8-entry table cache:
    tables are evicted while kernels that read them may still be queued."""
    monkeypatch.setenv("STORB_RS_TABLE_CACHE", "8")
    k, n, B, ns = 8, 16, 4096, 2
    ctx = _lib.Context(0)
    try:
        data_h, par_h = oracle_stripes(k, n, B, ns, 77)
        data = torch.from_numpy(data_h).to(DEV)
        par = torch.from_numpy(par_h).to(DEV)
        subsets = [c for c in itertools.combinations(range(n), k) if c != tuple(range(k))]
        random.Random(3).shuffle(subsets)
        subsets = subsets[:5000]
        streams = [torch.cuda.Stream(device=DEV), torch.cuda.Stream(device=DEV)]
        torch.cuda.synchronize()
        W = 64
        pool = torch.empty((W, data.numel()), dtype=torch.uint8, device=DEV)
        for w0 in range(0, len(subsets), W):
            batch = subsets[w0:w0 + W]
            for s in streams:
                s.wait_stream(torch.cuda.current_stream())  # pool reuse after the check
            for i, surv in enumerate(batch):
                st = streams[i & 1]
                ctx.decode_batch_dev(k, n, B, ns, list(surv), data.data_ptr(), par.data_ptr(),
                                     pool[i].data_ptr(), stream=st.cuda_stream)
            for s in streams:
                torch.cuda.current_stream().wait_stream(s)
            bad = (pool[:len(batch)] != data).any(dim=1).nonzero().flatten().tolist()
            assert not bad, [batch[i] for i in bad]
            pool[:len(batch)].zero_()
        torch.cuda.synchronize()
    finally:
        ctx.close()


def test_first_pattern_does_not_block_the_host():
    """A new pattern's tables are uploaded stream-ordered: the call returns
    while earlier work on the same stream is still running."""
    ctx = _lib.Context(0)
    try:
        k, n, B, ns = 4, 6, 1 << 20, 512
        st = torch.cuda.Stream(device=DEV)
        d = torch.empty(ns * k * B, dtype=torch.uint8, device=DEV)
        p = torch.empty(ns * (n - k) * B, dtype=torch.uint8, device=DEV)
        ctx.fill_splitmix_dev(d.data_ptr(), k * B, ns, k * B, 1, stream=st.cuda_stream)
        ctx.encode_batch_dev(k, n, B, ns, d.data_ptr(), p.data_ptr(), stream=st.cuda_stream)
        st.synchronize()
        ref = d.clone()
        # queue ~2 ms of encodes, then a decode with a never-seen pattern
        for _ in range(8):
            ctx.encode_batch_dev(k, n, B, ns, d.data_ptr(), p.data_ptr(), stream=st.cuda_stream)
        ctx.decode_batch_dev(k, n, B, ns, [1, 3, 4, 5], d.data_ptr(), p.data_ptr(),
                             d.data_ptr(), stream=st.cuda_stream)
        still_busy = not st.query()
        st.synchronize()
        assert torch.equal(d, ref)
        assert still_busy, "decode with a new pattern waited for the stream"
    finally:
        ctx.close()


def test_null_stream_sync_contract():
    """stream=None -> NULL -> HIP null stream; ctx.sync() waits for it, so a
    read on an unrelated non-blocking stream afterwards sees the results."""
    ctx = _lib.Context(0)
    try:
        assert ctx.default_stream is None
        k, n, B, ns = 4, 6, 256 << 10, 256
        data_h, par_h = oracle_stripes(k, n, B, 4, 9)
        d = torch.from_numpy(np.tile(data_h, ns // 4)).to(DEV)
        p = torch.zeros(ns * (n - k) * B, dtype=torch.uint8, device=DEV)
        torch.cuda.synchronize()
        ctx.encode_batch_dev(k, n, B, ns, d.data_ptr(), p.data_ptr())  # NULL stream
        ctx.sync()
        side = torch.cuda.Stream(device=DEV)
        with torch.cuda.stream(side):
            got = p.to("cpu", non_blocking=False)
        side.synchronize()
        assert np.array_equal(got.numpy(), np.tile(par_h, ns // 4))
    finally:
        ctx.close()


def page_aligned(nbytes, align=4096):
    raw = np.zeros(nbytes + align, dtype=np.uint8)
    off = (-raw.ctypes.data) % align
    return raw, raw[off:off + nbytes]


def test_host_register_direct_paths():
    """storb_rs_host_register'd caller memory (mapped) used in place at
    interior offsets by encode, decode and encode_chunks; oracle-exact. Runs
    in a child process (tests/registered_ranges.py)."""
    run_registered_case("direct_paths")


def test_streamed_call_gives_up_resets_and_streams_again(monkeypatch):
    """the streamed single call's give-up path, forced.

    The test knob (read once per context, storb_amd/csrc/ctx.hpp) makes a
    workgroup wait at most 20 ms (2,000,000 s_memrealtime ticks) for its
    slice's ready word and the host at most 200 ms for a done word, and makes
    the host sleep 100 ms before publishing slice 1 in the first streamed call
    -- a host descheduled past the device's wait. Slice 1's workgroups give up
    and exit without writing; the host drains the stream, resets the slice
    counters and redoes the call on the sliced path (host_calls.cpp streamed).
    The result must equal the oracle's, and the next calls must stream again
    (the counters were reset: a stale count would leave a done word unset)."""
    monkeypatch.setenv("STORB_RS_TEST_STREAM_STALL", "2000000,200,1,100000,1")
    ctx = _lib.Context(0)
    monkeypatch.delenv("STORB_RS_TEST_STREAM_STALL")
    try:
        k, n = 4, 6
        data = rnd(1 << 20, 31)  # B = 256 KiB: 4 slices of 64 KiB per share
        want, B, pad = coracle.encode(k, n, data)
        got, b, p = ctx.encode(k, n, data)
        assert (b, p) == (B, pad)
        assert got == [bytes(w) for w in want[k:]]
        st = ctx.stats()
        assert st["stream_fallbacks"] == 1 and st["sliced_calls"] == 1, st
        assert st["streamed_calls"] == 0, st
        for seed in (32, 33):  # streams again, exact
            d = rnd(1 << 20, seed)
            assert ctx.encode(k, n, d)[0] == [bytes(w) for w in coracle.encode(k, n, d)[0][k:]]
        shares = [bytes(w) for w in want]
        idx = [2, 3, 4, 5]
        assert ctx.decode(k, n, [shares[i] for i in idx], idx, B, pad) == data.tobytes()
        st = ctx.stats()
        assert st["stream_fallbacks"] == 1 and st["streamed_calls"] == 3, st
    finally:
        ctx.close()


@pytest.mark.parametrize("k,n,L", [(4, 6, 1 << 20), (4, 6, (1 << 20) - 5), (2, 3, 256 << 10),
                                   (16, 24, 8 << 20), (8, 12, 3 << 20 | 17), (1, 2, 4097),
                                   (3, 3, 1000), (32, 48, 32 << 20)])
def test_encode_shares_all_n_shares_match_oracle(ctx, k, n, L):
    """storb_rs_encode_shares: every share of zfec-rs Fec::encode's result
    (piece.rs:329) -- data shares zero-padded, then parity -- from one call,
    the data shares copied by the host pool while the kernel runs."""
    data = rnd(L, 40 + k)
    want, B, pad = coracle.encode(k, n, data)
    got, b, p = ctx.encode_shares(k, n, data)
    assert (b, p) == (B, pad)
    for i in range(n):
        assert got[i].tobytes() == bytes(want[i]), i


def _nodes():
    """{numa node: [allowed CPUs]} of this process."""
    out = {}
    for c in sorted(os.sched_getaffinity(0)):
        node = -1
        try:
            for name in os.listdir(f"/sys/devices/system/cpu/cpu{c}"):
                if name.startswith("node") and name[4:].isdigit():
                    node = int(name[4:])
        except OSError:
            pass
        out.setdefault(node, []).append(c)
    return out


def test_single_calls_stage_on_each_callers_node(ctx):
    """The single calls stage on the calling thread's NUMA node (ctx.hpp
    pin_in_node): the same context called from a thread pinned to each node
    of the allowed set -- one pair of staging buffers per node, the kernel
    reading each over the fabric -- encodes and decodes oracle-exact, for the
    streamed (4, 6), the wide (16, 24) and the repair path, and the device's
    node is reported."""
    assert _lib.lib().storb_rs_device_numa_node(ctx.device) >= -1
    saved = os.sched_getaffinity(0)
    try:
        for node, cpus in _nodes().items():
            os.sched_setaffinity(0, cpus)
            for k, n, L in ((4, 6, 1 << 20), (16, 24, 8 << 20), (2, 3, 100001)):
                data = rnd(L, 70 + k + node)
                want, B, pad = coracle.encode(k, n, data)
                got, b, p = ctx.encode(k, n, data)
                assert (b, p) == (B, pad)
                for i in range(n - k):
                    assert got[i] == bytes(want[k + i]), (node, k, i)
                surv = list(range(n - k, n))  # the last k shares: data lost 0 .. n-k-1
                out = ctx.decode(k, n, [bytes(want[i]) for i in surv], surv, B, pad)
                assert out == data.tobytes(), (node, k, surv)
            sh, B, _ = coracle.encode(4, 6, rnd(1 << 18, 9))
            rep = ctx.repair(4, 6, [bytes(sh[i]) for i in (1, 2, 3, 4)], [1, 2, 3, 4], B, [0, 5])
            assert rep == [bytes(sh[0]), bytes(sh[5])], node
    finally:
        os.sched_setaffinity(0, saved)


def test_staging_node_env_placements():
    """STORB_RS_STAGING_NODE=-1 (runtime placement, the pre-round-4 staging)
    and =0 (every call on node 0) in child processes: oracle-exact."""
    import subprocess
    import sys
    code = ("import numpy as np\n"
            "from oracle import coracle\n"
            "from storb_amd import _lib\n"
            "c = _lib.Context(0)\n"
            "for k, n, L in ((4, 6, 1 << 20), (16, 24, 8 << 20)):\n"
            "    d = np.frombuffer(np.random.default_rng(L).bytes(L), dtype=np.uint8).copy()\n"
            "    want, B, pad = coracle.encode(k, n, d)\n"
            "    got, b, p = c.encode(k, n, d)\n"
            "    assert all(got[i] == bytes(want[k + i]) for i in range(n - k))\n"
            "    surv = list(range(n - k, n))\n"
            "    assert c.decode(k, n, [bytes(want[i]) for i in surv[:k]], surv[:k], B, pad) == d.tobytes()\n"
            "c.close()\n"
            "print('staging ok')\n")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for v in ("-1", "0"):
        env = dict(os.environ, STORB_RS_STAGING_NODE=v)
        r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True,
                           timeout=240, env=env, cwd=root)
        assert r.returncode == 0 and "staging ok" in r.stdout, (v, r.stdout[-2000:],
                                                               r.stderr[-3000:])
