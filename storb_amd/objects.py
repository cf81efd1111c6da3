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
"""
from __future__ import annotations

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


def encode_object(data, ctx: Optional[_lib.Context] = None) -> EncodedObject:
    """encode_chunk + piece hashing + ChunkValue / PieceValue for a whole
    object; one batched GPU call per run of equal-length chunks."""
    ctx = ctx or _lib.thread_context()
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
        par, ids = ctx.encode_chunks_hashed(k, m, buf[off:off + cnt * ln], ln, cnt)
        par = par.reshape(cnt, m - k, B)
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


def reconstruct_object(chunks: Sequence[ChunkValue], fetched: Sequence[Dict[int, bytes]],
                       ctx: Optional[_lib.Context] = None) -> np.ndarray:
    """The download side: fetched[c] maps piece_idx -> piece bytes of chunk c
    (any subset); each chunk rebuilds from its first k pieces by index
    (reconstruct_chunk); PieceError if a chunk has fewer than k. One batched
    GPU call per run of chunks of one geometry. Returns the object's bytes
    as a uint8 array (no extra copy into a bytes object)."""
    ctx = ctx or _lib.thread_context()
    for ci, (cv, got) in enumerate(zip(chunks, fetched)):
        if len(got) < cv.k:
            raise PieceError(ci, cv.k, len(got))
    total = sum(cv.original_chunk_size for cv in chunks)
    out = np.empty(total, np.uint8)
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
        ctx.decode_chunks(k, m, B, pad, batch, out=out[off:off + (j - i) * ln].reshape(j - i, ln))
        off += (j - i) * ln
        i = j
    return out
