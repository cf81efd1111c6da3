"""GPU parity: the MI355X path vs the CPU oracle, through the C ABI.

Bit-exact for every byte (integer GF(2^8) work). The oracle is the C
restatement of zfec (oracle/), which tests/test_oracle.py pins against the
Appendix-B KATs and the reference's own round-trip tests (parity bytes are
otherwise unpinned -- no zfec-rs binary exists offline).
"""
import itertools
import random

import numpy as np
import pytest
import torch

from oracle import coracle
from storb_amd import _lib

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


def rnd(n, seed):
    return np.frombuffer(np.random.default_rng(seed).bytes(n), dtype=np.uint8).copy()


def to_dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


def oracle_parity(k, n, data):
    shares, B, pad = coracle.encode(k, n, data)
    return shares[k:], B, pad


# ------------------------------------------------------------- host API
HOST_CASES = [(1, 2), (2, 3), (3, 5), (4, 6), (6, 9), (8, 12), (16, 24), (32, 48),
              (5, 5), (17, 40), (64, 96)]
LENS = [1, 2, 13, 15, 16, 17, 255, 1000, 4097, 65536 + 5]


@pytest.mark.parametrize("k,n", HOST_CASES)
def test_host_encode_matches_oracle(ctx, k, n):
    for L in LENS:
        data = rnd(L, 1000 * k + L)
        parity, B, pad = ctx.encode(k, n, data)
        want, wB, wpad = oracle_parity(k, n, data)
        assert (B, pad) == (wB, wpad)
        assert len(parity) == n - k
        for i in range(n - k):
            assert parity[i] == want[i].tobytes(), (k, n, L, i)


def test_host_encode_edge_patterns(ctx):
    for k, n in [(4, 6), (8, 12)]:
        for fill in (0x00, 0xFF):
            data = np.full(k * 1024 + 3, fill, dtype=np.uint8)
            parity, _, _ = ctx.encode(k, n, data)
            want, _, _ = oracle_parity(k, n, data)
            assert all(parity[i] == want[i].tobytes() for i in range(n - k))


@pytest.mark.parametrize("k,n", [(1, 2), (2, 3), (3, 5), (4, 6), (6, 9), (8, 12)])
def test_host_decode_every_erasure_pattern(ctx, k, n):
    data = rnd(k * 333 + 1, k * 7 + n)
    shares, B, pad = coracle.encode(k, n, data)
    for subset in itertools.combinations(range(n), k):
        order = list(subset)
        random.Random(sum(subset)).shuffle(order)  # any order is accepted
        out = ctx.decode(k, n, [shares[i] for i in order], order, B, pad)
        assert out == data.tobytes(), subset


def test_host_decode_large_k_sampled(ctx):
    rng = random.Random(5)
    for k, n in [(16, 24), (32, 48), (64, 96)]:
        data = rnd(k * 512 + 7, k)
        shares, B, pad = coracle.encode(k, n, data)
        for _ in range(12):
            subset = rng.sample(range(n), k + rng.randrange(0, n - k + 1))
            out = ctx.decode(k, n, [shares[i] for i in subset], subset, B, pad)
            assert out == data.tobytes()
            # the chosen k (first k by index) must equal the oracle's choice
            assert out == coracle.decode(k, n, [shares[i] for i in subset], subset, B, pad)


def test_host_errors(ctx):
    with pytest.raises(_lib.StorbRsError) as e:
        ctx.encode(0, 2, b"x")
    assert e.value.code == _lib.EINVAL
    with pytest.raises(_lib.StorbRsError):
        ctx.encode(3, 2, b"x")
    with pytest.raises(_lib.StorbRsError):
        ctx.encode(2, 257, b"x")
    with pytest.raises(_lib.StorbRsError) as e:
        ctx.encode(4, 6, b"")
    assert e.value.code == _lib.EINVAL
    shares, B, pad = coracle.encode(4, 6, rnd(100, 1))
    with pytest.raises(_lib.StorbRsError) as e:
        ctx.decode(4, 6, [shares[i] for i in (0, 1, 2)], [0, 1, 2], B, pad)
    assert e.value.code == _lib.ENOTENOUGH
    with pytest.raises(_lib.StorbRsError) as e:
        ctx.decode(4, 6, [shares[i] for i in (0, 1, 1, 2)], [0, 1, 1, 2], B, pad)
    assert e.value.code == _lib.ENOTENOUGH
    with pytest.raises(_lib.StorbRsError) as e:
        ctx.decode(4, 6, [shares[i] for i in (0, 1, 2, 3)], [0, 1, 2, 6], B, pad)
    assert e.value.code == _lib.EINVAL


def test_host_encode_chunks_pipeline(ctx):
    for k, n, L, cnt in [(4, 6, 1 << 20, 70), (4, 6, (1 << 20) + 3, 9), (6, 9, 3 << 20, 5),
                         (16, 24, 8 << 20, 3), (1, 2, 9000, 11)]:
        data = rnd(L * cnt, L + cnt)
        par = ctx.encode_chunks(k, n, data, L, cnt)
        B = -(-L // k)
        par = par.reshape(cnt, n - k, B)
        for c in range(cnt):
            want, _, _ = oracle_parity(k, n, data[c * L:(c + 1) * L])
            assert np.array_equal(par[c], want), (k, n, L, c)


def test_host_encode_chunks_pinned_direct(ctx):
    """Caller buffers from storb_rs_host_alloc are DMA'd in place; every mix
    of pinned / pageable input and output gives the oracle's parity."""
    for k, n, L, cnt in [(4, 6, 1 << 20, 150), (16, 24, 8 << 20, 10), (4, 6, 4096, 7)]:
        B = -(-L // k)
        src = _lib.PinnedBuffer(L * cnt)
        dst = _lib.PinnedBuffer(cnt * (n - k) * B)
        src.array[:] = rnd(L * cnt, 5 * L + cnt)
        assert _lib.host_is_pinned(src.array) and _lib.host_is_pinned(dst.array)
        want = np.concatenate([oracle_parity(k, n, src.array[c * L:(c + 1) * L])[0].reshape(-1)
                               for c in range(cnt)])
        pageable_in = src.array.copy()
        assert not _lib.host_is_pinned(pageable_in)
        for inp in (src.array, pageable_in):
            for out in (dst.array, None):
                if out is not None:
                    out[:] = 0
                got = ctx.encode_chunks(k, n, inp, L, cnt, out=out)
                assert np.array_equal(got[:want.size], want), (k, n, L, out is None)
        par, hashes = ctx.encode_chunks_hashed(k, n, src.array, L, cnt)
        assert np.array_equal(par, want)
        assert bytes(hashes[0, k]) == _lib.blake3(want[:B])
        src.free()
        dst.free()


@pytest.mark.parametrize("zc", [True, False])
def test_single_call_pinned_and_staged(zc, monkeypatch):
    """storb_rs_encode / storb_rs_decode (the zfec-rs shim's per-chunk
    calls) on page-locked caller buffers (used in place) and on pageable
    ones (staged), through the zero-copy kernel path and the DMA path."""
    monkeypatch.setenv("STORB_RS_ZC_MAX", str(64 << 20) if zc else "0")
    c = _lib.Context(0)
    for k, n, B in [(4, 6, 256 << 10), (16, 24, 512 << 10), (1, 2, 65536), (8, 12, 4096)]:
        L = k * B
        pin = [_lib.PinnedBuffer(B) for _ in range(n)]     # n shares
        pout = _lib.PinnedBuffer(L)
        src = _lib.PinnedBuffer(L)
        src.array[:] = rnd(L, k + n + B)
        want = oracle_parity(k, n, src.array)[0]
        for data in (src.array, src.array.copy()):
            for par in ([pin[k + i].array for i in range(n - k)],
                        [np.zeros(B, np.uint8) for _ in range(n - k)]):
                for p in par:
                    p[:] = 0
                assert c.encode_into(k, n, data, par) == (B, 0)
                assert all(np.array_equal(par[i], want[i]) for i in range(n - k)), (k, n)
        for i in range(k):
            pin[i].array[:] = src.array[i * B:(i + 1) * B]
        for i in range(n - k):
            pin[k + i].array[:] = want[i]
        ids = list(range(min(2, n - k), n))[:k]          # lose the first data shares
        for shares in ([pin[i].array for i in ids], [pin[i].array.copy() for i in ids]):
            for out in (pout.array, np.empty(L, np.uint8)):
                out[:] = 0
                c.decode_into(k, n, shares, ids, B, 0, out)
                assert np.array_equal(out, src.array), (k, n, ids)
        for b in pin + [pout, src]:
            b.free()
    c.close()


@pytest.mark.parametrize("k,n,L", [(4, 6, (3 << 20) + 5), (16, 24, (8 << 20) - 77),
                                   (3, 5, (1 << 20) + 1), (8, 12, 4 << 20)])
def test_single_call_large_ragged(ctx, k, n, L):
    """Chunks big enough for the sliced single-call pipeline (column slices
    of a share, pack / kernel / unpack overlapped), with ragged lengths so
    the zero padding and the truncated last row fall inside a slice."""
    data = rnd(L, L % 1000)
    par, B, pad = ctx.encode(k, n, data)
    want, wB, wpad = oracle_parity(k, n, data)
    assert (B, pad) == (wB, wpad)
    for i in range(n - k):
        assert par[i] == want[i].tobytes(), (k, n, L, i)
    shares = coracle.encode(k, n, data)[0]
    for lost in ([0], list(range(min(n - k, k))), [k - 1]):
        ids = [i for i in range(n) if i not in lost][:k]
        got = ctx.decode(k, n, [shares[i] for i in ids], ids, B, pad)
        assert got == data.tobytes(), (k, n, L, lost)


@pytest.mark.parametrize("k,n", [(2, 3), (3, 5), (4, 6), (8, 12), (16, 24), (32, 48)])
def test_single_call_streamed_slices(ctx, k, n):
    """The streamed single calls (host_calls.cpp streamed: one launch gated
    per 64 KiB-per-share slice on host-written words; the table kernel for
    k <= 32 and <= 8 rows, the bit-sliced encoders for (16, 24) / (32, 48)) from pageable
    buffers, at lengths that put the slice edges, the zero padding and the
    truncated last row everywhere: one slice, exact slice multiples, one byte
    over, a ragged 16-B column count, and more than 16 slices (the slice
    grows). Every call is oracle-exact, and the calls are repeated so the
    per-slice counters run across geometries and slice counts."""
    rng = random.Random(k * 100 + n)
    S64 = 64 << 10
    lengths = [1000, k * S64, k * S64 + 1, k * (3 * S64 + 4096 + 48) - 7, k * 20 * S64 + 333]
    if k >= 16:
        lengths = [1000, k * S64, k * (3 * S64 + 48) - 7, k * 18 * S64 + 5]
    for rep in range(2):
        for L in lengths:
            data = rnd(L, L + rep)
            par, B, pad = ctx.encode(k, n, data)
            want, wB, wpad = oracle_parity(k, n, data)
            assert (B, pad) == (wB, wpad)
            for i in range(n - k):
                assert par[i] == want[i].tobytes(), (k, n, L, i)
            shares = coracle.encode(k, n, data)[0]
            lost = rng.sample(range(k), rng.randint(1, min(n - k, k, 8)))
            ids = [i for i in range(n) if i not in lost]
            rng.shuffle(ids)
            got = ctx.decode(k, n, [shares[i] for i in ids], ids, B, pad)
            assert got == data.tobytes(), (k, n, L, lost)


def test_host_decode_chunks_batch(ctx):
    """Batched download-side decode: every chunk its own survivor set
    (all-data, data+parity mixes, parity-only, extra shares beyond k, any
    order); each chunk must equal the original bytes (decode_chunk's first-k
    rule), including the truncated tail of the padding."""
    rng = random.Random(11)
    for k, n, L, cnt in [(4, 6, (1 << 20) - 5, 40), (8, 12, 256 << 10, 25), (16, 24, 777777, 9),
                         (2, 3, 4096, 12), (1, 2, 100, 5)]:
        data = rnd(L * cnt, 3 * L + k)
        chunks, want = [], []
        for c in range(cnt):
            chunk = data[c * L:(c + 1) * L]
            shares, B, pad = coracle.encode(k, n, chunk)
            m = rng.randint(k, n)
            ids = rng.sample(range(n), m)
            if c % 7 == 0:
                ids = list(range(k))                       # nothing erased
            elif c % 7 == 1 and n - k >= 1:
                ids = list(range(n - 1, n - 1 - min(n, k + 1), -1))  # parity first
            chunks.append(([shares[i] for i in ids], ids))
            want.append(chunk)
        got = ctx.decode_chunks(k, n, B, pad, chunks)
        for c in range(cnt):
            assert np.array_equal(got[c], want[c]), (k, n, L, c, chunks[c][1])
    # fewer than k shares in one chunk: the whole call reports ENOTENOUGH
    shares, B, pad = coracle.encode(4, 6, rnd(4096, 1))
    with pytest.raises(_lib.StorbRsError) as e:
        ctx.decode_chunks(4, 6, B, pad, [([shares[i] for i in range(4)], [0, 1, 2, 3]),
                                         ([shares[i] for i in (0, 4, 5)], [0, 4, 5])])
    assert e.value.code == _lib.ENOTENOUGH


@pytest.mark.parametrize("zc", [True, False])
def test_host_decode_chunks_page_locked(zc, monkeypatch):
    """storb_rs_decode_chunks with page-locked shares and output (the
    download path with receive buffers from storb_rs_host_alloc): the decode
    kernel reads the survivors over PCIe in place and writes rebuilt rows and
    surviving data shares straight into the output (STORB_RS_ZC_BATCH=1,
    default), or the staged pipeline (=0). Shares in an arena with regular
    strides (one launch per run of chunks), scattered shares (one launch per
    chunk), a pageable share in one chunk (that pattern's group is staged),
    and padded chunks (staged: the last row is truncated). Oracle-exact."""
    monkeypatch.setenv("STORB_RS_ZC_BATCH", "1" if zc else "0")
    c = _lib.Context(0)
    rng = random.Random(5)
    for k, n, B, cnt, pad in [(4, 6, 256 << 10, 12, 0), (16, 24, 512 << 10, 6, 0),
                              (8, 12, 64 << 10, 9, 0), (4, 6, 64 << 10, 5, 3)]:
        L = k * B - pad
        data = rnd(L * cnt, 7 * k + B + pad)
        arena = _lib.PinnedBuffer(cnt * n * B)
        A = arena.array.reshape(cnt, n, B)
        for ch in range(cnt):
            shares, b, p = coracle.encode(k, n, data[ch * L:(ch + 1) * L])
            assert (b, p) == (B, pad)
            A[ch] = shares
        out = _lib.PinnedBuffer(cnt * L)
        lost = [0, 1] if k > 2 else [0]
        pattern = [i for i in range(n) if i not in lost][:k]
        scratch = _lib.PinnedBuffer(cnt * n * B)
        slots = scratch.array.reshape(cnt * n, B)
        for layout in ("arena", "scattered", "mixed"):
            perm = rng.sample(range(cnt * n), cnt * n)       # share (ch, i) -> scratch slot
            chunks = []
            for ch in range(cnt):
                ids = list(pattern)
                if ch % 3 == 2:
                    ids = list(range(n - k, n))              # another pattern
                if layout == "arena":
                    shares = [A[ch, i] for i in ids]
                else:
                    shares = []
                    for i in ids:
                        slots[perm[ch * n + i]] = A[ch, i]
                        shares.append(slots[perm[ch * n + i]])
                if layout == "mixed" and ch == 1:
                    shares[0] = np.array(shares[0])          # pageable copy
                chunks.append((shares, ids))
            o = out.array[:cnt * L].reshape(cnt, L)
            o[:] = 0x5A
            got = c.decode_chunks(k, n, B, pad, chunks, out=o)
            for ch in range(cnt):
                assert np.array_equal(got[ch], data[ch * L:(ch + 1) * L]), (k, n, layout, ch)
            # a caller stride wider than the chunk (aligned: still zero-copy), gap untouched
            st = L + 4096
            wide = _lib.PinnedBuffer((cnt - 1) * st + L)
            wide.array[:] = 0x77
            got = c.decode_chunks(k, n, B, pad, chunks, out=wide.array, out_stride=st)
            for ch in range(cnt):
                assert np.array_equal(got[ch], data[ch * L:(ch + 1) * L]), (k, n, layout, "wide", ch)
                if ch + 1 < cnt:
                    assert (wide.array[ch * st + L:(ch + 1) * st] == 0x77).all()
            wide.free()
        for buf in (arena, scratch, out):
            buf.free()
    c.close()


# ----------------------------------------------------------- device API
def dev_encode_check(ctx, k, n, B, ns, kernel=_lib.KERNEL_PERM, offset=0):
    ctx.set_kernel(kernel)
    host = rnd(ns * k * B, k * 31 + n + B)
    buf = torch.zeros(ns * k * B + offset, dtype=torch.uint8, device=DEV)
    buf[offset:] = to_dev(host)
    par = torch.zeros(ns * (n - k) * B + offset, dtype=torch.uint8, device=DEV)
    ctx.encode_batch_dev(k, n, B, ns, buf.data_ptr() + offset, par.data_ptr() + offset)
    ctx.sync()
    got = par[offset:].cpu().numpy().reshape(ns, n - k, B)
    for s in range(ns):
        want, wB, _ = oracle_parity(k, n, host[s * k * B:(s + 1) * k * B])
        assert wB == B
        assert np.array_equal(got[s], want), (k, n, B, s)
    ctx.set_kernel(_lib.KERNEL_AUTO)


@pytest.mark.parametrize("k,n,B,ns", [(4, 6, 4096, 37), (4, 6, 16, 5), (2, 3, 8192, 9),
                                      (1, 2, 4096, 3), (8, 12, 4096 + 16, 7),
                                      (16, 24, 2048, 6), (32, 48, 1024, 3), (6, 9, 4096, 4),
                                      (3, 7, 512, 5), (12, 20, 1008, 3)])
def test_dev_encode_matches_oracle(ctx, k, n, B, ns):
    dev_encode_check(ctx, k, n, B, ns)


@pytest.mark.parametrize("k,n,B,ns", [(4, 6, 4096, 9), (8, 12, 2048, 5), (3, 5, 1024, 4),
                                      (16, 24, 512, 3)])
def test_dev_encode_lds_variant_identical(ctx, k, n, B, ns):
    dev_encode_check(ctx, k, n, B, ns, kernel=_lib.KERNEL_LDS)


@pytest.mark.parametrize("k,n,B,ns,off", [(4, 6, 13, 5, 0), (4, 6, 1000, 3, 0),
                                          (4, 6, 4096, 3, 3), (7, 10, 999, 4, 1)])
def test_dev_encode_unaligned_byte_path(ctx, k, n, B, ns, off):
    dev_encode_check(ctx, k, n, B, ns, offset=off)


@pytest.mark.parametrize("k,n,B,ns", [(40, 60, 256, 3), (64, 96, 512, 2), (200, 256, 64, 2),
                                      (33, 34, 128, 2), (10, 40, 256, 2)])
def test_dev_encode_tiled_large_matrices(ctx, k, n, B, ns):
    dev_encode_check(ctx, k, n, B, ns)


# Storb's wide full-chunk geometries take the bit-sliced encoder under AUTO
# (rs_bitslice.hpp; (64, 96) as one row-split launch): one 16-B column,
# ragged tiles, exact 8 KiB tiles.
@pytest.mark.parametrize("k,n", [(16, 24), (32, 48), (64, 96)])
@pytest.mark.parametrize("B,ns", [(16, 3), (1040, 4), (8192, 3), (3 * 8192 + 48, 2),
                                  (16 * 1024 + 1024, 2)])
def test_dev_encode_bitslice_matches_oracle(ctx, k, n, B, ns):
    dev_encode_check(ctx, k, n, B, ns, kernel=_lib.KERNEL_AUTO)


@pytest.mark.parametrize("k,n,B,ns", [(16, 24, 512 << 10, 9), (32, 48, 1 << 20, 3),
                                      (64, 96, 2 << 20, 2)])
def test_bitslice_identical_to_table_kernel(ctx, k, n, B, ns):
    """AUTO (bit-sliced) and forced PERM (v_perm tables) encodes agree byte
    for byte on the config-5 share size, splitmix input."""
    data = torch.empty(ns * k * B, dtype=torch.uint8, device=DEV)
    ctx.fill_splitmix_dev(data.data_ptr(), k * B, ns, k * B, 0x5709B)
    outs = []
    for kern in (_lib.KERNEL_AUTO, _lib.KERNEL_PERM):
        ctx.set_kernel(kern)
        par = torch.full((ns * (n - k) * B,), 0xA5, dtype=torch.uint8, device=DEV)
        ctx.encode_batch_dev(k, n, B, ns, data.data_ptr(), par.data_ptr())
        ctx.sync()
        outs.append(par)
    ctx.set_kernel(_lib.KERNEL_AUTO)
    assert torch.equal(outs[0], outs[1])
    # and one stripe against the oracle
    want, _, _ = oracle_parity(k, n, data[:k * B].cpu().numpy())
    assert np.array_equal(outs[0][:(n - k) * B].cpu().numpy().reshape(n - k, B), want)


@pytest.mark.parametrize("k,n,erased", [(8, 12, (0, 3, 5)), (8, 12, (9, 10, 11)),
                                        (4, 6, (0, 1)), (4, 6, (2, 5)), (16, 24, tuple(range(8))),
                                        (6, 9, (1, 4, 8)), (40, 60, tuple(range(0, 40, 2))),
                                        (2, 3, (0,)), (1, 2, (0,))])
@pytest.mark.parametrize("inplace", [True, False])
def test_dev_decode_roundtrip(ctx, k, n, erased, inplace):
    B, ns = 1024, 6
    host = rnd(ns * k * B, k + n + len(erased))
    data = to_dev(host)
    par = torch.zeros(ns * (n - k) * B, dtype=torch.uint8, device=DEV)
    ctx.encode_batch_dev(k, n, B, ns, data.data_ptr(), par.data_ptr())
    survivors = [i for i in range(n) if i not in erased]
    random.Random(k).shuffle(survivors)
    view = data.view(ns, k, B)
    for e in erased:
        if e < k:
            view[:, e].fill_(0xA5)  # garbage in the lost slots
    out = data if inplace else torch.full_like(data, 0x5A)
    ctx.decode_batch_dev(k, n, B, ns, survivors, data.data_ptr(), par.data_ptr(),
                         out.data_ptr())
    ctx.sync()
    assert np.array_equal(out.cpu().numpy(), host)


FUSED_CASES = [(4, 6, (0, 1)), (4, 6, ()), (4, 6, (4, 5)), (8, 12, (0, 3, 5)),
               (8, 12, (9, 10, 11)), (16, 24, (0, 1)), (16, 24, tuple(range(0, 16, 2))),
               (3, 5, (2,)), (12, 18, (11,)), (2, 3, (1,))]


@pytest.mark.parametrize("k,n,erased", FUSED_CASES)
@pytest.mark.parametrize("B,ns", [(4096 * 2, 5), (4096 * 3 + 16 * 5, 3)])
@pytest.mark.parametrize("mode", ["fused", "lds", "strided"])
def test_dev_decode_separate_output_assembly(ctx, monkeypatch, k, n, erased, B, ns, mode):
    """decode_chunk returns a fresh chunk (piece.rs:363-387): decode into a
    separate buffer stores every surviving data share from the decode
    kernel's own loads (fused assembly, k <= 16) -- full tiles and a ragged
    last tile, nothing missing (pure assembly) and a strided output --
    byte-identical to the LDS comparison variant (which copies the survivors
    first), and every stripe equals the input."""
    host = rnd(ns * k * B, 7 * k + n + B + len(erased))
    data = to_dev(host)
    par = torch.zeros(ns * (n - k) * B, dtype=torch.uint8, device=DEV)
    ctx.encode_batch_dev(k, n, B, ns, data.data_ptr(), par.data_ptr())
    survivors = [i for i in range(n) if i not in erased]
    random.Random(B + k).shuffle(survivors)
    view = data.view(ns, k, B)
    for e in erased:
        if e < k:
            view[:, e].fill_(0xA5)
    pad = 3 * 16 if mode == "strided" else 0
    ostride = k * B + pad
    out = torch.full((ns * ostride,), 0x5A, dtype=torch.uint8, device=DEV)
    if mode == "lds":
        ctx.set_kernel(_lib.KERNEL_LDS)
    try:
        ctx.decode_batch_dev(k, n, B, ns, survivors, data.data_ptr(), par.data_ptr(),
                             out.data_ptr(), out_stride=ostride if pad else 0)
        ctx.sync()
    finally:
        ctx.set_kernel(_lib.KERNEL_AUTO)
    got = out.cpu().numpy().reshape(ns, ostride)
    assert np.array_equal(got[:, :k * B].reshape(-1), host)
    assert (got[:, k * B:] == 0x5A).all()  # the stride gap is never written


def test_dev_decode_not_enough(ctx):
    d = torch.zeros(4 * 64, dtype=torch.uint8, device=DEV)
    p = torch.zeros(2 * 64, dtype=torch.uint8, device=DEV)
    with pytest.raises(_lib.StorbRsError) as e:
        ctx.decode_batch_dev(4, 6, 64, 1, [0, 1, 2], d.data_ptr(), p.data_ptr(), d.data_ptr())
    assert e.value.code == _lib.ENOTENOUGH


def test_apply_dev_regenerates_a_lost_share(ctx):
    """Decode-based repair: rebuild parity share 10 of an
    RS(8,12) stripe from 8 survivors in one apply launch."""
    k, n, B, ns = 8, 12, 2048, 4
    host = rnd(ns * k * B, 77)
    enc = coracle.enc_matrix(k, n)
    shares = [coracle.encode(k, n, host[s * k * B:(s + 1) * k * B])[0] for s in range(ns)]
    surv = [1, 2, 4, 6, 7, 8, 9, 11]
    # share 10 = enc[10] . data, data = inv(enc[surv]) . survivors
    from oracle import zfec_np
    dinv = zfec_np._mat_inv(enc[surv])
    coef = zfec_np._mat_mul(enc[10:11], dinv)
    srcs = [to_dev(np.stack([shares[s][i] for s in range(ns)]).reshape(-1)) for i in surv]
    out = torch.zeros(ns * B, dtype=torch.uint8, device=DEV)
    ctx.apply_dev(coef, [t.data_ptr() for t in srcs], [B] * k, [out.data_ptr()], [B], B, ns)
    ctx.sync()
    want = np.stack([shares[s][10] for s in range(ns)]).reshape(-1)
    assert np.array_equal(out.cpu().numpy(), want)


@pytest.mark.parametrize("k,n,lost", [(4, 6, (0, 5)), (4, 6, (4, 5)), (8, 12, (0, 3, 10)),
                                      (8, 12, (9, 10, 11)), (16, 24, (0, 7, 15, 16, 20, 23)),
                                      (2, 3, (2,)), (1, 2, (0,)), (40, 60, (1, 2, 45, 59)),
                                      (17, 40, tuple(range(17, 40)))])
def test_dev_repair_batch_regenerates_lost_shares(ctx, k, n, lost):
    """storb_rs_repair_batch_dev: lost data AND parity shares rebuilt in
    place from the first k survivors; each must equal the oracle's share."""
    B, ns = 1040, 5
    host = rnd(ns * k * B, 31 * k + n)
    data = to_dev(host)
    par = torch.zeros(ns * (n - k) * B, dtype=torch.uint8, device=DEV)
    ctx.encode_batch_dev(k, n, B, ns, data.data_ptr(), par.data_ptr())
    ctx.sync()
    want_par = par.cpu().numpy().copy()
    for s in range(ns):  # the encode itself against the oracle
        w, _, _ = oracle_parity(k, n, host[s * k * B:(s + 1) * k * B])
        assert np.array_equal(want_par.reshape(ns, n - k, B)[s], w)
    dv, pv = data.view(ns, k, B), par.view(ns, n - k, B)
    for t in lost:
        (dv[:, t] if t < k else pv[:, t - k]).fill_(0xA5)
    survivors = [i for i in range(n) if i not in lost]
    random.Random(n).shuffle(survivors)
    targets = list(lost)
    random.Random(k).shuffle(targets)
    ctx.repair_batch_dev(k, n, B, ns, survivors, targets, data.data_ptr(), par.data_ptr())
    ctx.sync()
    assert np.array_equal(data.cpu().numpy(), host)
    assert np.array_equal(par.cpu().numpy(), want_par)


def test_repair_rejects_bad_targets(ctx):
    d = torch.zeros(4 * 64, dtype=torch.uint8, device=DEV)
    p = torch.zeros(2 * 64, dtype=torch.uint8, device=DEV)
    for targets in ([1], [6], [5, 5]):  # a share read / out of range / repeated
        with pytest.raises(_lib.StorbRsError) as e:
            ctx.repair_batch_dev(4, 6, 64, 1, [0, 1, 2, 3], targets, d.data_ptr(), p.data_ptr())
        assert e.value.code == _lib.EINVAL
    with pytest.raises(_lib.StorbRsError) as e:
        ctx.repair_batch_dev(4, 6, 64, 1, [0, 1, 2], [4], d.data_ptr(), p.data_ptr())
    assert e.value.code == _lib.ENOTENOUGH


@pytest.mark.parametrize("k,n", [(4, 6), (8, 12), (16, 24), (3, 5)])
def test_host_repair_matches_oracle(ctx, k, n):
    rng = random.Random(k * n)
    data = rnd(k * 777 + 5, k + 3 * n)
    shares, B, _ = coracle.encode(k, n, data)
    for _ in range(8):
        have = rng.sample(range(n), k + rng.randrange(0, n - k + 1))
        used = sorted(have)[:k]
        targets = rng.sample([i for i in range(n) if i not in used],
                             rng.randrange(1, n - k + 1))
        got = ctx.repair(k, n, [shares[i] for i in have], have, B, targets)
        for t, g in zip(targets, got):
            assert g == shares[t].tobytes(), (k, n, have, t)


def test_fill_splitmix_matches_oracle(ctx):
    for L, cnt, stride in [(1 << 20, 3, 1 << 20), (13, 5, 16), (1001, 2, 1001)]:
        buf = torch.zeros(cnt * stride, dtype=torch.uint8, device=DEV)
        ctx.fill_splitmix_dev(buf.data_ptr(), L, cnt, stride, 0x5709B)
        ctx.sync()
        got = buf.cpu().numpy().reshape(cnt, stride)
        for o in range(cnt):
            assert np.array_equal(got[o, :L], coracle.splitmix_bytes(0x5709B + o, L))


# -------------------------------------------------- BASELINE full sizes
# Every stripe of every batch is compared with the C oracle run on host
# threads (tests/batch_oracle.py): the inputs as the
# oracle generates them, the parity of every chunk, and every reconstructed
# chunk -- plus the size-independent properties (round trips, linearity,
# partition invariance).
@pytest.mark.slow
def test_config2_full_size_encode_decode(ctx):
    """Config 2: 1024 x 1 MiB RS(4,2) [storb k=4,m=6], device-resident:
    inputs, all 1024 stripes' parity and all 1024 rebuilt chunks (data shards
    0,1 lost, rebuilt in place from {2,3,4,5}) against the oracle."""
    import batch_oracle as BO
    k, n, L, N = 4, 6, 1 << 20, 1024
    B = L // k
    data = torch.empty(N * L, dtype=torch.uint8, device=DEV)
    par = torch.empty(N * 2 * B, dtype=torch.uint8, device=DEV)
    ctx.fill_splitmix_dev(data.data_ptr(), L, N, L, 0x5709B)
    ctx.encode_batch_dev(k, n, B, N, data.data_ptr(), par.data_ptr())
    ctx.sync()
    host = BO.splitmix_chunks(0x5709B, L, N)
    assert BO.first_mismatch(data.cpu().numpy(), host, L) is None
    want = BO.parity_all(k, n, host, L, N)
    assert BO.first_mismatch(par.cpu().numpy(), want, 2 * B) is None
    v = data.view(N, k, B)
    v[:, 0].zero_()
    v[:, 1].zero_()
    ctx.decode_batch_dev(k, n, B, N, [2, 3, 4, 5], data.data_ptr(), par.data_ptr(),
                         data.data_ptr())
    ctx.sync()
    assert BO.first_mismatch(data.cpu().numpy(), host, L) is None


@pytest.mark.slow
def test_config3_full_size_decode_three_erased(ctx):
    """Config 3: RS(8,4) [storb k=8,m=12], 4096 x 256 KiB, erase {0,3,5}
    (survivors {1,2,4,6,7,8,9,10}) and the parity-only control {9,10,11}: all
    4096 stripes' parity and every reconstructed chunk against the oracle's
    own decode of the same shares."""
    import batch_oracle as BO
    k, n, L, N = 8, 12, 256 << 10, 4096
    B = L // k
    data = torch.empty(N * L, dtype=torch.uint8, device=DEV)
    par = torch.empty(N * 4 * B, dtype=torch.uint8, device=DEV)
    ctx.fill_splitmix_dev(data.data_ptr(), L, N, L, 0x5709B)
    ctx.encode_batch_dev(k, n, B, N, data.data_ptr(), par.data_ptr())
    ctx.sync()
    host = data.cpu().numpy()
    assert BO.first_mismatch(host, BO.splitmix_chunks(0x5709B, L, N), L) is None
    hpar = par.cpu().numpy()
    assert BO.first_mismatch(hpar, BO.parity_all(k, n, host, L, N), 4 * B) is None
    for erased in [(0, 3, 5), (9, 10, 11)]:
        surv = [i for i in range(n) if i not in erased][:k]
        out = torch.empty_like(data)
        ctx.decode_batch_dev(k, n, B, N, surv, data.data_ptr(), par.data_ptr(),
                             out.data_ptr())
        ctx.sync()
        wiped = host.reshape(N, k, B).copy()
        for e in erased:
            if e < k:
                wiped[:, e] = 0  # the oracle must not read the lost shares
        want = BO.decode_all(k, n, wiped.reshape(-1), hpar, B, N, surv)
        assert BO.first_mismatch(out.cpu().numpy(), want, L) is None, erased
        assert BO.first_mismatch(want, host, L) is None, erased


@pytest.mark.slow
def test_config4_round_robin_objects_match_single_batch(ctx):
    """Config 4: 10,000 x 1 MiB objects, RS(4,2) [storb k=4,m=6]. Each of 8
    (virtual) ranks encodes only its objects i = rank (mod 8) -- the
    multi-GPU partition, here on one device -- and every object's parity
    equals the single-batch encode of all 10,000 and the oracle's parity of
    that object (all 10,000 compared)."""
    import batch_oracle as BO
    from storb_amd import partition

    k, n, L, N, W = 4, 6, 1 << 20, 10000, 8
    B = L // k
    data = torch.empty(N * L, dtype=torch.uint8, device=DEV)
    ctx.fill_splitmix_dev(data.data_ptr(), L, N, L, 0x5709B)
    whole = torch.empty(N * 2 * B, dtype=torch.uint8, device=DEV)
    ctx.encode_batch_dev(k, n, B, N, data.data_ptr(), whole.data_ptr())
    parts = torch.full_like(whole, 0x5A)
    for rank in range(W):
        objs = partition.objects_for_rank(N, rank, W)
        # objects rank, rank+W, ...: a strided batch (stride W objects)
        ctx.encode_batch_dev(k, n, B, len(objs), data.data_ptr() + rank * L,
                             parts.data_ptr() + rank * 2 * B, data_stride=W * L,
                             parity_stride=W * 2 * B)
    ctx.sync()
    assert torch.equal(whole, parts)
    host = data.cpu().numpy()
    del data
    for s in (0, 7, 4999, N - 1):  # the device fill is the oracle's generator
        assert np.array_equal(host[s * L:(s + 1) * L], coracle.splitmix_bytes(0x5709B + s, L))
    want = BO.parity_all(k, n, host, L, N)
    assert BO.first_mismatch(whole.cpu().numpy(), want, 2 * B) is None


@pytest.mark.slow
def test_config5_full_size_linearity_and_max_erasure(ctx):
    """Config 5's GPU half: 128 x 8 MiB chunks, storb k=16, m=24 (bit-sliced
    encoder under AUTO). All 128 stripes' parity against the oracle; the code
    is linear (parity(a ^ b) == parity(a) ^ parity(b)); decoding with all 8
    parity shares standing in for data shares 0..7 (the most erasures) and
    with Storb's 2-lost download case returns every chunk as the oracle's
    own decode of the same shares does."""
    import batch_oracle as BO
    k, n, L, N = 16, 24, 8 << 20, 128
    B = L // k
    a = torch.empty(N * L, dtype=torch.uint8, device=DEV)
    b = torch.empty_like(a)
    ctx.fill_splitmix_dev(a.data_ptr(), L, N, L, 1)
    ctx.fill_splitmix_dev(b.data_ptr(), L, N, L, 0x5709B)
    c = a ^ b
    pars = []
    for x in (a, b, c):
        p = torch.empty(N * 8 * B, dtype=torch.uint8, device=DEV)
        ctx.encode_batch_dev(k, n, B, N, x.data_ptr(), p.data_ptr())
        pars.append(p)
    ctx.sync()
    assert torch.equal(pars[0] ^ pars[1], pars[2])
    host = a.cpu().numpy()
    assert BO.first_mismatch(host, BO.splitmix_chunks(1, L, N), L) is None
    hpar = pars[0].cpu().numpy()
    assert BO.first_mismatch(hpar, BO.parity_all(k, n, host, L, N), 8 * B) is None
    for lost in (list(range(8)), [0, 1]):
        surv = [i for i in range(n) if i not in lost][:k]
        out = torch.full_like(a, 0xA5)
        ctx.decode_batch_dev(k, n, B, N, surv, a.data_ptr(), pars[0].data_ptr(),
                             out.data_ptr())
        ctx.sync()
        wiped = host.reshape(N, k, B).copy()
        wiped[:, lost] = 0
        want = BO.decode_all(k, n, wiped.reshape(-1), hpar, B, N, surv)
        assert BO.first_mismatch(out.cpu().numpy(), want, L) is None, lost
        assert BO.first_mismatch(want, host, L) is None, lost
    ref = a.clone()
    a.view(N, k, B)[:, :8].fill_(0xA5)
    ctx.decode_batch_dev(k, n, B, N, list(range(8, 24)), a.data_ptr(), pars[0].data_ptr(),
                         a.data_ptr())
    ctx.sync()
    assert torch.equal(a, ref)


@pytest.mark.parametrize("k,n,erased", [(1, 256, (0,)), (255, 256, (0,)),
                                        (128, 256, tuple(range(0, 128, 1)))])
def test_max_share_count_roundtrip(ctx, k, n, erased):
    """zfec's limit n = 256 (the most shares a GF(2^8) code has): encode
    against the oracle, then decode with `erased` data shares lost (k = 128
    with all 128 data shares rebuilt from parity: a 128 x 128 inverse tiled
    over 16 x 32 kernel slots)."""
    B, ns = 256, 2
    dev_encode_check(ctx, k, n, B, ns)
    host = rnd(ns * k * B, n + k)
    data = to_dev(host)
    par = torch.zeros(ns * (n - k) * B, dtype=torch.uint8, device=DEV)
    ctx.set_kernel(_lib.KERNEL_AUTO)
    ctx.encode_batch_dev(k, n, B, ns, data.data_ptr(), par.data_ptr())
    surv = [i for i in range(n) if i not in erased]
    data.view(ns, k, B)[:, list(erased)] = 0
    ctx.decode_batch_dev(k, n, B, ns, surv, data.data_ptr(), par.data_ptr(), data.data_ptr())
    ctx.sync()
    assert np.array_equal(data.cpu().numpy(), host)



def test_concurrent_calls_per_thread_and_shared_context():
    """The shim's threading model (one context per tokio worker thread,
    INTEGRATION.md) and a context shared by several threads (calls serialise
    on its mutex): 8 threads mixing single-chunk encodes and decodes of
    several Storb geometries, bit-exact against the oracle."""
    import threading

    shared = _lib.Context(0)
    geos = [(4, 6, 1 << 20), (2, 3, 256 << 10), (1, 2, 65536), (16, 24, (3 << 20) + 7),
            (8, 12, 777)]
    errors = []

    def worker(t):
        ctx = _lib.Context(0) if t % 2 == 0 else shared
        rng = random.Random(t)
        try:
            for it in range(10):
                k, n, L = geos[(t + it) % len(geos)]
                data = rnd(L, 77 * t + it)
                par, B, pad = ctx.encode(k, n, data)
                want = oracle_parity(k, n, data)[0]
                assert all(par[i] == want[i].tobytes() for i in range(n - k)), (t, k, n, L)
                shares = coracle.encode(k, n, data)[0]
                ids = rng.sample(range(n), k)
                assert ctx.decode(k, n, [shares[i] for i in ids], ids, B, pad) == data.tobytes()
        except Exception as e:
            errors.append(f"thread {t}: {e!r}")
        finally:
            if ctx is not shared:
                ctx.close()

    th = [threading.Thread(target=worker, args=(t,)) for t in range(8)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    shared.close()
    assert not errors, errors[:3]


@pytest.mark.parametrize("zc", ["1", "0"])
def test_host_batches_reuse_staging_slots(zc, monkeypatch):
    """Several 64 MiB batches per call, so each double-buffer slot of the
    staged pipelines (host_batch.cpp Staging: H2D, kernels and D2H on a
    stream each, event-ordered per slot; non-temporal host copies) is reused:
    pageable encode (with and without piece ids) against the oracle's parity,
    pageable and page-locked download-pattern decode against the data."""
    monkeypatch.setenv("STORB_RS_ZC_BATCH", zc)
    ctx = _lib.Context(0)
    try:
        k, n, L, cnt = 4, 6, 1 << 20, 200  # 200 MiB: four batches
        B = L // k
        data = rnd(L * cnt, 4242 + int(zc))
        want = coracle.encode_parity_many(k, n, data, L, cnt, threads=8).reshape(cnt, n - k, B)
        par = ctx.encode_chunks(k, n, data, L, cnt).reshape(cnt, n - k, B)
        assert np.array_equal(par, want)
        ids = np.zeros((cnt, n, 32), np.uint8)
        par2 = np.zeros_like(par.reshape(-1))
        ctx.encode_chunks_hashed(k, n, data, L, cnt, out=par2, hashes=ids)
        assert np.array_equal(par2.reshape(cnt, n - k, B), want)
        for c in (0, 63, 64, 127, 128, cnt - 1):  # a chunk in every batch
            assert bytes(ids[c, 0]) == _lib.blake3(data[c * L:c * L + B].tobytes())
            assert bytes(ids[c, k]) == _lib.blake3(want[c, 0].tobytes())
        rng = random.Random(7)
        dat = data.reshape(cnt, k, B)
        chunks = []
        for c in range(cnt):
            sel = rng.sample(range(n), k + 1)
            chunks.append(([dat[c, i] if i < k else want[c, i - k] for i in sel], sel))
        got = ctx.decode_chunks(k, n, B, 0, chunks)
        assert np.array_equal(got.reshape(-1), data)
        pin = _lib.PinnedBuffer(L * cnt)
        try:
            rec = pin.array.reshape(cnt, L)
            rec[:] = 0
            ctx.decode_chunks(k, n, B, 0, chunks, out=rec)
            assert np.array_equal(rec.reshape(-1), data)
        finally:
            rec = None
            pin.free()
    finally:
        ctx.close()
