"""Object-level callers (storb_amd/objects.py) against the reference's
per-chunk semantics: upload.rs produce_bytes chunking and consume_bytes
piece / chunk hashes and metadata rows, piece.rs get_infohash_by_identity,
and the download side's first-k-by-index reconstruction.

Checks: chunking and sizing against the oracle's restatement of piece.rs
(CPU); the infohash against the restated blake3 (CPU); on the GPU, every
piece byte against the oracle's zfec parity, every piece hash against the
restated blake3, the chunk hash as blake3 over the piece hashes in piece
order, and round trips under random erasures.
"""
import random

import numpy as np
import pytest

from oracle import coracle
from oracle.blake3_ref import blake3 as ref_blake3
from storb_amd import _lib, objects
from storb_amd.piece import PieceError, PieceType


@pytest.mark.parametrize("total", [1, 16 << 10, (1 << 20) + 7, 10 * (1 << 20) + 12345,
                                   256 << 20, (1 << 30) + 1])
def test_chunk_spans_follow_produce_bytes(total):
    spans = objects.chunk_spans(total)
    size = coracle.piece_length(total)
    assert spans[0][0] == 0 and sum(ln for _, ln in spans) == total
    assert all(o2 == o1 + l1 for (o1, l1), (o2, _) in zip(spans, spans[1:]))
    full = {ln for _, ln in spans[:-1]}
    assert len(full) <= 1 and spans[-1][1] <= spans[0][1]
    assert spans[0][1] == min(size, total)
    for _, ln in spans:
        assert _lib.get_k_and_m(ln) == coracle.get_k_and_m(ln)


def test_infohash_by_identity():
    owner = bytes(range(32))
    hashes = [bytes([i]) * 32 for i in range(7)]
    want = ref_blake3(owner + b"".join(hashes))
    assert objects.get_infohash_by_identity(hashes, owner) == want
    assert objects.get_infohash_by_identity([], owner) == ref_blake3(owner)


def _obj(n, seed):
    return np.frombuffer(np.random.default_rng(seed).bytes(n), dtype=np.uint8).copy()


@pytest.mark.gpu
@pytest.mark.parametrize("total", [1, 100, (64 << 10) + 1, 10 * (1 << 20) + 12345, 20 << 20])
def test_encode_object_matches_per_chunk_reference(ctx, total):
    data = _obj(total, total % 977)
    enc = objects.encode_object(data, ctx)
    spans = objects.chunk_spans(total)
    assert len(enc.chunks) == len(spans)
    for (off, ln), cv, pv, sh in zip(spans, enc.chunks, enc.pieces, enc.data):
        k, m = _lib.get_k_and_m(ln)
        shares, B, pad = coracle.encode(k, m, data[off:off + ln])
        assert (cv.k, cv.m, cv.chunk_size, cv.padlen, cv.original_chunk_size) == (k, m, B, pad, ln)
        assert len(sh) == len(pv) == m
        for i in range(m):
            assert np.array_equal(np.asarray(sh[i]), shares[i]), (total, off, i)
            # the product's host hasher (pinned to the published vectors in
            # test_blake3.py) for every piece; the pure-Python restatement on
            # the first piece of each chunk (it is slow on MiB pieces)
            assert pv[i].piece_hash == _lib.blake3(shares[i]), (total, off, i)
            if i == 0:
                assert pv[i].piece_hash == ref_blake3(shares[i].tobytes()), (total, off)
            assert pv[i].piece_size == B
            assert pv[i].piece_type == (PieceType.Data if i < k else PieceType.Parity)
        assert cv.chunk_hash == ref_blake3(b"".join(p.piece_hash for p in pv))
    assert enc.piece_hashes() == [p.piece_hash for ps in enc.pieces for p in ps]


@pytest.mark.gpu
def test_reconstruct_object_under_erasures(ctx):
    total = 24 * (1 << 20) + 999
    data = _obj(total, 5)
    enc = objects.encode_object(data, ctx)
    rng = random.Random(3)
    fetched = []
    for cv, sh in zip(enc.chunks, enc.data):
        keep = rng.sample(range(cv.m), rng.randint(cv.k, cv.m))
        fetched.append({i: np.asarray(sh[i]).tobytes() for i in keep})
    assert np.array_equal(objects.reconstruct_object(enc.chunks, fetched, ctx), data)
    # a chunk short of k pieces: reconstruct_chunk's ReconstructionError
    bad = [dict(f) for f in fetched]
    cv0 = enc.chunks[1]
    bad[1] = {i: bad[1][i] for i in sorted(bad[1])[:cv0.k - 1]}
    with pytest.raises(PieceError) as e:
        objects.reconstruct_object(enc.chunks, bad, ctx)
    assert (e.value.chunk_idx, e.value.k, e.value.got) == (1, cv0.k, cv0.k - 1)


@pytest.mark.gpu
@pytest.mark.parametrize("nctx", [2, 3, 5])
def test_object_calls_partitioned_over_contexts(ctx, nctx):
    """Chunks of one object spread over several contexts (one per GPU on a
    node; here several share the one device) give the same shares, piece
    ids, rows and reconstruction as one context -- including runs shorter
    than the context count and the short tail chunk."""
    ctxs = objects.device_contexts(nctx)
    try:
        for total in (40 << 20, 9 * (1 << 20) + 7):
            data = _obj(total, nctx + total % 13)
            one = objects.encode_object(data, ctx)
            many = objects.encode_object(data, contexts=ctxs)
            assert one.chunks == many.chunks and one.pieces == many.pieces
            for a, b in zip(one.data, many.data):
                assert all(np.array_equal(np.asarray(x), np.asarray(y)) for x, y in zip(a, b))
            rng = random.Random(nctx)
            fetched = []
            for cv, sh in zip(many.chunks, many.data):
                keep = rng.sample(range(cv.m), cv.k)
                fetched.append({i: np.asarray(sh[i]).tobytes() for i in keep})
            assert np.array_equal(objects.reconstruct_object(many.chunks, fetched,
                                                             contexts=ctxs), data)
    finally:
        for c in ctxs:
            c.close()


def test_slices_cover_every_chunk_once():
    for cnt in range(1, 40):
        for parts in range(1, 12):
            sl = objects._slices(cnt, parts)
            assert len(sl) == min(cnt, parts)
            assert sl[0][0] == 0 and sl[-1][1] == cnt
            assert all(a < b for a, b in sl) and all(sl[i][1] == sl[i + 1][0]
                                                      for i in range(len(sl) - 1))
            sizes = [b - a for a, b in sl]
            assert max(sizes) - min(sizes) <= 1
