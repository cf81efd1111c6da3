"""Object-level callers of the erasure stage, batched on the MI355X path.

Storb's validator drives the chunk -> shard stage one chunk at a time:

* upload (crates/storb_validator/src/upload.rs): ``produce_bytes`` cuts the
  body into chunks of ``piece_length(total)`` bytes, the last one short
  (:333-383); ``consume_bytes`` runs ``encode_chunk`` on each (:420), hashes
  every piece with blake3 (``upload_piece_to_miner``, :623), folds the piece
  hashes of a chunk into its ``chunk_hash`` in piece order (:424, :538, :564)
  and records ``ChunkValue`` / ``PieceValue`` rows (:567-594, metadata
  models.rs:46-53, :96-102); the object's infohash is
  ``get_infohash_by_identity`` (storb_base piece.rs:257-276).
* download (download.rs:336-465): per chunk, pieces in ``piece_idx`` order
  until more than k are in hand, then ``reconstruct_chunk`` (first k by
  index, piece.rs:441-481).

Here the same results come from whole-object calls: every run of chunks of
one geometry is ONE ``storb_rs_encode_chunks_hashed`` (parity and every
piece id on the GPU) or ONE ``storb_rs_decode_chunks``. Bytes, hashes and
metadata rows are identical to the per-chunk path (tests/test_objects.py).

Several GPUs (BASELINE config 5 on 8 x MI355X, SURVEY 8(e): chunks of a single
huge object partition across the devices of a node): pass ``contexts`` (one
``Context`` per device, e.g. ``device_contexts()``) and every run is cut into
one contiguous slice of chunks per context, all slices in flight at once
(one host thread per context; the calls release the GIL). No data moves
between devices: each slice is host in / host out on its own GPU.
"""
from __future__ import annotations

import heapq
from concurrent.futures import ThreadPoolExecutor
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import _lib
from .piece import PieceError, PieceType, get_infohash_by_identity  # noqa: F401 (re-export)


@dataclass
class ChunkValue:
    """metadata::models::ChunkValue (models.rs:46-53)."""
    chunk_hash: bytes
    k: int
    m: int
    chunk_size: int           # EncodedChunk.chunk_size = share bytes B
    padlen: int
    original_chunk_size: int


@dataclass
class PieceValue:
    """metadata::models::PieceValue (models.rs:96-102) without the miner list."""
    piece_hash: bytes
    piece_size: int
    piece_type: PieceType


@dataclass
class EncodedObject:
    chunks: List[ChunkValue]
    pieces: List[List[PieceValue]]
    # piece bytes, per chunk in piece order: data shares are views of the
    # (zero-padded) chunk, parity shares views of the parity batch
    data: List[List[np.ndarray]]

    def piece_hashes(self) -> List[bytes]:
        """All piece hashes in chunk, then piece order (upload.rs:603-607)."""
        return [p.piece_hash for ps in self.pieces for p in ps]


def chunk_spans(total: int) -> List[Tuple[int, int]]:
    """(offset, length) of the chunks produce_bytes emits (upload.rs:333-383):
    chunk size piece_length(total), the last chunk short."""
    if total <= 0:
        return []
    size = _lib.piece_length(total)
    return [(o, min(size, total - o)) for o in range(0, total, size)]


def _runs(spans: Sequence[Tuple[int, int]]):
    """Maximal runs of consecutive chunks of one length."""
    i = 0
    while i < len(spans):
        j = i
        while j < len(spans) and spans[j][1] == spans[i][1]:
            j += 1
        yield i, j
        i = j


def device_contexts(ndev: Optional[int] = None) -> List[_lib.Context]:
    """One context per visible device (the first `ndev` of them)."""
    n = _lib.device_count() if ndev is None else ndev
    return [_lib.Context(d % max(_lib.device_count(), 1)) for d in range(n)]


def _slices(cnt: int, parts: int) -> List[Tuple[int, int]]:
    """Split chunks [0, cnt) into <= parts contiguous non-empty ranges."""
    parts = max(1, min(parts, cnt))
    q, r = divmod(cnt, parts)
    out, a = [], 0
    for i in range(parts):
        b = a + q + (i < r)
        out.append((a, b))
        a = b
    return out


def _fan_out(ctxs, cnt: int, call) -> None:
    """call(ctx, a, b) for one contiguous slice of [0, cnt) per context, the
    slices concurrently; the first error is raised."""
    sl = _slices(cnt, len(ctxs))
    if len(sl) == 1:
        call(ctxs[0], *sl[0])
        return
    with ThreadPoolExecutor(len(sl)) as ex:
        for f in [ex.submit(call, c, a, b) for c, (a, b) in zip(ctxs, sl)]:
            f.result()


def encode_object(data, ctx: Optional[_lib.Context] = None,
                  contexts: Optional[Sequence[_lib.Context]] = None) -> EncodedObject:
    """encode_chunk + piece hashing + ChunkValue / PieceValue for a whole
    object; one batched GPU call per run of equal-length chunks (per
    context, when `contexts` spreads the run over several GPUs)."""
    ctxs = list(contexts) if contexts else [ctx or _lib.thread_context()]
    buf = data if isinstance(data, np.ndarray) else np.frombuffer(bytes(data), np.uint8)
    buf = np.ascontiguousarray(buf, dtype=np.uint8).reshape(-1)
    spans = chunk_spans(buf.size)
    chunks: List[ChunkValue] = []
    pieces: List[List[PieceValue]] = []
    shares: List[List[np.ndarray]] = []
    for c0, c1 in _runs(spans):
        off, ln = spans[c0]
        cnt = c1 - c0
        k, m = _lib.get_k_and_m(ln)
        B = _lib.block_size(k, ln)
        par = np.empty((cnt, m - k, B), np.uint8)
        ids = np.empty((cnt, m, 32), np.uint8)

        def enc(cx, a, b, off=off, ln=ln, k=k, m=m, par=par, ids=ids):
            cx.encode_chunks_hashed(k, m, buf[off + a * ln:off + b * ln], ln, b - a,
                                    out=par[a:b].reshape(-1), hashes=ids[a:b])

        _fan_out(ctxs, cnt, enc)
        for c in range(cnt):
            chunk = buf[off + c * ln:off + (c + 1) * ln]
            if B * k != ln:
                chunk = np.concatenate([chunk, np.zeros(B * k - ln, np.uint8)])
            sh = [chunk[i * B:(i + 1) * B] for i in range(k)] + [par[c, i] for i in range(m - k)]
            hashes = [ids[c, i].tobytes() for i in range(m)]
            chunks.append(ChunkValue(chunk_hash=_lib.blake3(b"".join(hashes)), k=k, m=m,
                                     chunk_size=B, padlen=B * k - ln, original_chunk_size=ln))
            pieces.append([PieceValue(hashes[i], B, PieceType.Data if i < k else PieceType.Parity)
                           for i in range(m)])
            shares.append(sh)
    return EncodedObject(chunks, pieces, shares)


FETCH_THREADS = 10  # download.rs:28 THREAD_COUNT


def download_arrivals(k: int, m: int, rng: np.random.Generator, fail=(), sigma: float = 0.5,
                      threads: int = FETCH_THREADS) -> List[int]:
    """The pieces of one chunk that produce_chunk collects, in arrival order
    (download.rs:363-451), simulated: the m pieces are queued in piece_idx
    order (:424-428, get_pieces_by_chunk is ORDER BY piece_idx); `threads`
    workers each take the next queued piece when free (:378-383) and fetch it
    in a lognormal(0, sigma) time; a piece whose miner is in `fail` yields
    nothing (:403-405); the collector keeps pieces until more than k unique
    ones are in hand (:434-451), i.e. the first k + 1 to arrive (all that
    arrive, if fewer). decode_chunk then sorts them and uses the first k by
    index (piece.rs:368-381) -- see download_survivors."""
    fail = set(fail)
    heap = []
    nxt = 0
    for _ in range(min(threads, m)):
        heapq.heappush(heap, (float(rng.lognormal(0.0, sigma)), nxt))
        nxt += 1
    got: List[int] = []
    while heap:
        t, idx = heapq.heappop(heap)
        if idx not in fail:
            got.append(idx)
        if nxt < m:  # the worker that finished takes the next queued piece
            heapq.heappush(heap, (t + float(rng.lognormal(0.0, sigma)), nxt))
            nxt += 1
    collected: List[int] = []
    for idx in got:
        if len(collected) > k:  # `unique_pieces.len() > k` -> break (:443-447)
            break
        collected.append(idx)
    return collected


def download_survivors(k: int, m: int, rng: np.random.Generator, fail=(),
                       sigma: float = 0.5) -> List[int]:
    """The k shares decode_chunk hands to Fec::decode for one downloaded chunk
    (first k by index of the pieces collected, piece.rs:368-381); fewer than k
    means reconstruct_chunk's Err (piece.rs:462-473)."""
    return sorted(download_arrivals(k, m, rng, fail, sigma))[:k]


def reconstruct_object(chunks: Sequence[ChunkValue], fetched: Sequence[Dict[int, bytes]],
                       ctx: Optional[_lib.Context] = None,
                       contexts: Optional[Sequence[_lib.Context]] = None,
                       out: Optional[np.ndarray] = None) -> np.ndarray:
    """The download side: fetched[c] maps piece_idx -> piece bytes of chunk c
    (any subset); each chunk rebuilds from its first k pieces by index
    (reconstruct_chunk); PieceError if a chunk has fewer than k. One batched
    GPU call per run of chunks of one geometry. Returns the object's bytes
    as a uint8 array (no extra copy into a bytes object), written into `out`
    when given (a download buffer the caller reuses: a fresh one is first
    touched page by page while the decoded chunks land in it)."""
    ctxs = list(contexts) if contexts else [ctx or _lib.thread_context()]
    for ci, (cv, got) in enumerate(zip(chunks, fetched)):
        if len(got) < cv.k:
            raise PieceError(ci, cv.k, len(got))
    total = sum(cv.original_chunk_size for cv in chunks)
    if out is None:
        out = np.empty(total, np.uint8)
    elif out.dtype != np.uint8 or not out.flags.c_contiguous or out.size < total:
        raise ValueError("out: a contiguous uint8 buffer of the object's size")
    out = out[:total]
    geo = [(cv.k, cv.m, cv.chunk_size, cv.padlen, cv.original_chunk_size) for cv in chunks]
    off = 0
    i = 0
    while i < len(chunks):
        j = i
        while j < len(chunks) and geo[j] == geo[i]:
            j += 1
        k, m, B, pad, ln = geo[i]
        batch = []
        for c in range(i, j):
            ids = sorted(fetched[c])
            batch.append(([fetched[c][x] for x in ids], ids))
        dst = out[off:off + (j - i) * ln].reshape(j - i, ln)

        def dec(cx, a, b, k=k, m=m, B=B, pad=pad, batch=batch, dst=dst):
            cx.decode_chunks(k, m, B, pad, batch[a:b], out=dst[a:b])

        _fan_out(ctxs, j - i, dec)
        off += (j - i) * ln
        i = j
    return out
