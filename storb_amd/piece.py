"""Python mirror of crates/storb_base/src/piece.rs over the MI355X path.

Same names, argument meaning and error behaviour as the reference:
``piece_length`` (piece.rs:292-303), ``get_k_and_m`` (:307-317),
``encode_chunk`` (:320-361), ``decode_chunk`` (:363-387),
``reconstruct_data`` (:389-438), ``reconstruct_chunk`` (:441-481),
``get_infohash_by_identity`` (:257-276) and the carrier types (:157-213). Rust ``.expect()`` panics raise :class:`Panic`;
``Result::Err(PieceError)`` raises :class:`PieceError`.
The C++ mirror of the same file is include/storb_piece.hpp.
"""
from __future__ import annotations

import enum
from dataclasses import dataclass, field, replace
from typing import List, Optional, Sequence

from . import _lib
from .fec import Chunk, Fec, FecError

PIECE_LENGTH_FUNC_MIN_SIZE = 16 * 1024          # constants.rs:5
PIECE_LENGTH_FUNC_MAX_SIZE = 256 * 1024 * 1024  # constants.rs:6


class Panic(RuntimeError):
    """A Rust panic (``.expect`` on Err) in the reference."""


class PieceType(enum.IntEnum):
    Data = 0
    Parity = 1


@dataclass
class Piece:
    chunk_idx: int
    piece_size: int
    piece_idx: int
    piece_type: PieceType
    data: bytes


@dataclass
class EncodedChunk:
    pieces: List[Piece]
    chunk_idx: int
    k: int  # number of data blocks
    m: int  # total blocks (data + parity)
    chunk_size: int
    padlen: int
    original_chunk_size: int


class PieceError(Exception):
    """ReconstructionError(chunk_idx, k, got)."""

    def __init__(self, chunk_idx: int, k: int, got: int):
        self.chunk_idx, self.k, self.got = chunk_idx, k, got
        super().__init__(f"Not enough pieces to reconstruct chunk {chunk_idx}, "
                         f"expected k={k} but got {got} pieces")


def piece_length(content_length: int, min_size: Optional[int] = None,
                 max_size: Optional[int] = None) -> int:
    lo = PIECE_LENGTH_FUNC_MIN_SIZE if min_size is None else min_size
    hi = PIECE_LENGTH_FUNC_MAX_SIZE if max_size is None else max_size
    v = _lib.piece_length(content_length, 1, 2**64 - 1)
    return min(max(v, lo), hi)


def get_k_and_m(chunk_size: int):
    return _lib.get_k_and_m(chunk_size)


def encode_chunk(chunk: bytes, chunk_idx: int) -> EncodedChunk:
    chunk = bytes(chunk)
    chunk_size = len(chunk)
    piece_size = piece_length(chunk_size)
    k, m = get_k_and_m(chunk_size)
    try:
        encoder = Fec.new(k, m)
    except FecError as e:
        raise Panic(f"Failed to create encoder: {e}") from e
    try:
        encoded, padlen = encoder.encode(chunk)
    except FecError as e:
        raise Panic(f"Failed to encode chunk: {e}") from e
    zfec_chunk_size = -(-chunk_size // k)
    pieces = [Piece(chunk_idx=chunk_idx, piece_size=piece_size, piece_idx=i,
                    piece_type=PieceType.Data if i < k else PieceType.Parity,
                    data=c.data) for i, c in enumerate(encoded)]
    return EncodedChunk(pieces=pieces, chunk_idx=chunk_idx, k=k, m=m,
                        chunk_size=zfec_chunk_size, padlen=padlen,
                        original_chunk_size=chunk_size)


def decode_chunk(encoded_chunk: EncodedChunk) -> bytes:
    k, m = int(encoded_chunk.k), int(encoded_chunk.m)
    pieces = sorted(encoded_chunk.pieces, key=lambda p: p.piece_idx)
    if len(pieces) > k:  # zfec decode requires exactly k blocks
        pieces = pieces[:k]
    to_decode = [Chunk.new(p.data, p.piece_idx) for p in pieces]
    try:
        decoder = Fec.new(k, m)
    except FecError as e:
        raise Panic(f"Failed to create decoder: {e}") from e
    try:
        return decoder.decode(to_decode, int(encoded_chunk.padlen))
    except FecError as e:
        raise Panic(f"Failed to decode chunk: {e}") from e


def reconstruct_data(pieces: Sequence[Piece], chunks: Sequence[EncodedChunk]) -> bytes:
    out = []
    for chunk in chunks:
        relevant = sorted((p for p in pieces if p.chunk_idx == chunk.chunk_idx),
                          key=lambda p: p.piece_idx)
        if len(relevant) < chunk.k:
            return b""  # piece.rs:411-421: empty Vec signals the error
        out.append(decode_chunk(replace(chunk, pieces=relevant)))
    return b"".join(out)


def reconstruct_chunk(chunk: EncodedChunk) -> bytes:
    relevant = sorted((p for p in chunk.pieces if p.chunk_idx == chunk.chunk_idx),
                      key=lambda p: p.piece_idx)
    if len(relevant) < chunk.k:
        raise PieceError(chunk.chunk_idx, chunk.k, len(relevant))
    return decode_chunk(replace(chunk, pieces=relevant))


def get_infohash_by_identity(piece_hashes: Sequence[bytes], owner_account_id: bytes) -> bytes:
    """piece.rs:257-276: blake3(owner account id || piece hashes...)."""
    return _lib.blake3(bytes(owner_account_id) + b"".join(bytes(h) for h in piece_hashes))
