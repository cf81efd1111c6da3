"""GPU parity of the asynchronous single-chunk calls (storb_rs_encode_async /
storb_rs_decode_async, host_async.cpp): the async forms of the calls the
zfec-rs shim makes per chunk (piece.rs:329 Fec::encode, piece.rs:384-386
Fec::decode), for an integration that awaits them inside the tokio tasks of
upload.rs:418-420 / download.rs:464 instead of blocking a worker thread.

Every result is compared byte for byte with the oracle (oracle/, the restated
zfec): many ops in flight at once on two contexts, finished in random order,
inputs overwritten right after the start call returns (the call stages them),
notify callbacks counted, page-locked outputs written in place, and the
64-op limit per context."""
import random
import threading

import numpy as np
import pytest

from oracle import coracle
from storb_amd import _lib

pytestmark = pytest.mark.gpu

GEOS = [(2, 3), (3, 5), (4, 6), (8, 12), (16, 24), (32, 48), (17, 26), (10, 20)]


def rnd(rng, n):
    return np.frombuffer(rng.randbytes(n), dtype=np.uint8).copy()


@pytest.fixture(scope="module")
def ctxs():
    cs = [_lib.Context(0), _lib.Context(0)]
    yield cs
    for c in cs:
        c.close()


def test_async_encode_many_in_flight(ctxs):
    rng = random.Random(11)
    fired = []
    lock = threading.Lock()

    def note(i):
        def f():
            with lock:
                fired.append(i)
        return f

    ops = []
    for i in range(48):
        k, n = rng.choice(GEOS)
        L = rng.choice([1, 17, 4096, 65536 + 3, 1 << 20, rng.randint(1, 3 << 20)])
        data = rnd(rng, L)
        want, B, pad = coracle.encode(k, n, data)
        op = rng.choice(ctxs).encode_async(k, n, data, notify=note(i))
        data[:] = 0x5A  # staged by the call: overwriting must not matter
        ops.append((i, op, want[k:], B, pad))
    rng.shuffle(ops)
    for i, op, want, B, pad in ops:
        got, b, p = op.finish()
        assert (b, p) == (B, pad), i
        assert [bytes(w) for w in want] == got, i
    assert sorted(fired) == list(range(48))


def test_async_decode_many_in_flight(ctxs):
    rng = random.Random(12)
    ops = []
    for i in range(40):
        k, n = rng.choice(GEOS)
        L = rng.choice([33, 4096 * 3 + 5, 1 << 20, rng.randint(1, 2 << 20)])
        data = rnd(rng, L)
        shares, B, pad = coracle.encode(k, n, data)
        lost = set(rng.sample(range(n), rng.randint(0, n - k)))
        idx = [j for j in range(n) if j not in lost]
        rng.shuffle(idx)
        given = [np.frombuffer(bytes(shares[j]), dtype=np.uint8).copy() for j in idx]
        op = rng.choice(ctxs).decode_async(k, n, given, idx, B, pad)
        for g in given:
            g[:] = 0xA5  # staged by the call
        ops.append((i, op, data))
    rng.shuffle(ops)
    for i, op, data in ops:
        assert op.finish() == data.tobytes(), i


def test_async_without_device_work_completes_at_once(ctxs):
    """k = 1 (parity is the data) and decodes with every data share present
    are host copies: done, and notified, before the call returns."""
    c = ctxs[0]
    fired = []
    data = np.arange(50000, dtype=np.uint32).view(np.uint8)[:70001].copy()
    op = c.encode_async(1, 3, data, notify=lambda: fired.append(1))
    assert fired == [1] and op.test()
    got, B, pad = op.finish()
    assert got == [data.tobytes()] * 2 and (B, pad) == (data.size, 0)
    shares, B, pad = coracle.encode(4, 6, data)
    op = c.decode_async(4, 6, [bytes(s) for s in shares], list(range(6)), B, pad,
                        notify=lambda: fired.append(2))
    assert fired == [1, 2] and op.test()
    assert op.finish() == data.tobytes()


def test_async_page_locked_outputs_in_place(ctxs):
    c = ctxs[1]
    rng = random.Random(13)
    k, n = 8, 12
    data = rnd(rng, 8 << 20)
    want, B, pad = coracle.encode(k, n, data)
    bufs = [_lib.PinnedBuffer(B) for _ in range(n - k)]
    op = c.encode_async(k, n, data, parity=[b.array for b in bufs])
    op.finish()
    for b, w in zip(bufs, want[k:]):
        assert b.array[:B].tobytes() == bytes(w)
    for b in bufs:
        b.free()


def test_async_op_limit_and_errors(ctxs):
    c = ctxs[0]
    rng = random.Random(14)
    data = rnd(rng, 256 << 10)
    want = coracle.encode(4, 6, data)[0][4:]
    ops = [c.encode_async(4, 6, data) for _ in range(64)]
    with pytest.raises(_lib.StorbRsError) as e:
        c.encode_async(4, 6, data)
    assert e.value.code == 7  # STORB_RS_EBUSY
    for op in ops:
        assert op.finish()[0] == [bytes(w) for w in want]
    # slots are reused after finish
    assert c.encode_async(4, 6, data).finish()[0] == [bytes(w) for w in want]
    with pytest.raises(_lib.StorbRsError):
        c.encode_async(5, 4, data)  # k > n
    with pytest.raises(_lib.StorbRsError):
        c.decode_async(4, 6, [data[:1000]] * 3, [0, 1, 2], 1000, 0)  # fewer than k
