"""Context teardown and async-op lifetime (VERDICT r3 "next" item 1).

Round 3 saw two hipErrorIllegalAddress faults surface at a pageable
host->device copy after contexts had been destroyed (DESIGN.md §7 has the
analysis). This pins the teardown contract in one GPU test:

* a context whose coefficient-table cache was filled from two streams
  (stream-ordered pool memory, hipMallocAsync) and whose async slots are in
  use is destroyed while one op is still referenced and unfinished;
* a pageable H2D copy and a device synchronisation afterwards are clean;
* the default pool's used bytes are back where they were before the context;
* the unfinished op raises ECLOSED from test() / finish() instead of touching
  the destroyed context, and an op dropped after close is collected cleanly.

Ops are the storb_rs_encode_async / _decode_async calls that an async
integration would await per chunk (upload.rs:418-420, download.rs:464)."""
import gc

import numpy as np
import pytest

from oracle import coracle
from storb_amd import _lib

pytestmark = pytest.mark.gpu


def _patterns(k, n, count):
    """count distinct survivor sets: two data shares lost, the first k of the
    remaining shares by index (decode_chunk's selection, piece.rs:368-381)."""
    out = []
    for a in range(k):
        for b in range(a + 1, k):
            out.append([i for i in range(n) if i not in (a, b)][:k])
            if len(out) == count:
                return out
    return out


def test_close_with_tables_on_two_streams_and_an_unfinished_op():
    import torch
    torch.cuda.synchronize()
    base_used, _ = _lib.device_pool_stats(0)
    ctx = _lib.Context(0)
    ctx.set_kernel(_lib.KERNEL_PERM)  # every pattern gets device tables
    k, n, B, ns = 8, 12, 64 << 10, 4
    data = torch.randint(0, 256, (ns * k * B,), dtype=torch.uint8, device="cuda:0")
    par = torch.zeros(ns * (n - k) * B, dtype=torch.uint8, device="cuda:0")
    out = torch.zeros_like(data)
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    for i, surv in enumerate(_patterns(k, n, 24)):
        s = streams[i % 2]
        s.wait_stream(torch.cuda.current_stream())
        ctx.decode_batch_dev(k, n, B, ns, surv, data.data_ptr(), par.data_ptr(), out.data_ptr(),
                             stream=s.cuda_stream)
    st = ctx.stats()
    assert st["tables"] >= 24
    used_with_tables, _ = _lib.device_pool_stats(0)
    assert used_with_tables > base_used
    # async slots: finished ops, then ops left in flight; one stays referenced
    rng = np.random.default_rng(7)
    chunk = rng.integers(0, 256, 8 << 20, dtype=np.uint8)
    want = coracle.encode(16, 24, chunk)[0][16:]
    done = ctx.encode_async(16, 24, chunk)
    assert [bytes(w) for w in want] == done.finish()[0]
    held = ctx.encode_async(16, 24, chunk)
    dropped = ctx.encode_async(4, 6, chunk[: 1 << 20])
    assert ctx.stats()["live_ops"] == 2
    ctx.close()
    # a pageable host->device copy and a device-wide sync after the teardown
    host = rng.integers(0, 256, 3 << 20, dtype=np.uint8)
    dev = torch.from_numpy(host).to("cuda:0")
    torch.cuda.synchronize()
    assert torch.equal(dev.cpu(), torch.from_numpy(host))
    used_after, _ = _lib.device_pool_stats(0)
    assert used_after == base_used, (base_used, used_with_tables, used_after)
    # the unfinished op: detached, raises instead of touching freed memory
    with pytest.raises(_lib.StorbRsError) as e:
        held.test()
    assert e.value.code == _lib.ECLOSED
    with pytest.raises(_lib.StorbRsError) as e:
        held.finish()
    assert e.value.code == _lib.ECLOSED
    # an op dropped after close: its finalizer frees it without the context
    del dropped
    gc.collect()
    torch.cuda.synchronize()
    for s in streams:
        s.synchronize()


def test_page_locked_output_of_an_op_outliving_its_context():
    """The kernel writes a page-locked caller output in place; closing the
    context waits for it, and the buffer can be freed afterwards."""
    import torch
    ctx = _lib.Context(0)
    rng = np.random.default_rng(8)
    chunk = rng.integers(0, 256, 4 << 20, dtype=np.uint8)
    want, B, _ = coracle.encode(8, 12, chunk)
    bufs = [_lib.PinnedBuffer(B) for _ in range(4)]
    op = ctx.encode_async(8, 12, chunk, parity=[b.array for b in bufs])
    ctx.close()
    for b, w in zip(bufs, want[8:]):  # written in place by the kernel before close returned
        assert b.array[:B].tobytes() == bytes(w)
    for b in bufs:
        b.free()
    with pytest.raises(_lib.StorbRsError):
        op.finish()
    torch.cuda.synchronize()
