"""zfec-rs API mirror (``Fec``, ``Chunk``) over the MI355X C ABI.

Mirrors the surface Storb uses (crates/storb_base/src/piece.rs:9,328-329,
375,383-386): ``Fec.new(k, m)`` with m the TOTAL share count,
``Fec.encode(data) -> (chunks, padlen)`` returning all m shares in index
order, ``Fec.decode(chunks, padlen) -> bytes``, ``Chunk(data, index)``.
Errors raise :class:`FecError` (zfec-rs returns ``Err`` which Storb
``.expect()``s).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Sequence, Tuple

from . import _lib


class FecError(ValueError):
    pass


@dataclass
class Chunk:
    data: bytes
    index: int

    @classmethod
    def new(cls, data: bytes, index: int) -> "Chunk":
        return cls(bytes(data), int(index))


class Fec:
    def __init__(self, k: int, m: int):
        if not _lib.check_params(k, m):
            raise FecError(f"invalid parameters k={k}, m={m}")
        self.k, self.m = int(k), int(m)

    @classmethod
    def new(cls, k: int, m: int) -> "Fec":
        return cls(k, m)

    def encode(self, data) -> Tuple[List[Chunk], int]:
        buf = bytes(data)
        if not buf:
            raise FecError("empty input")
        # storb_rs_encode_shares, as the Rust shim's Fec::encode: every share
        # (data shares zero-padded, then parity) written by one call
        shares, B, pad = _lib.thread_context().encode_shares(self.k, self.m, buf)
        return [Chunk(s.tobytes(), i) for i, s in enumerate(shares)], pad

    def decode(self, chunks: Sequence[Chunk], padlen: int) -> bytes:
        if len(chunks) < self.k:
            raise FecError(f"need {self.k} chunks, got {len(chunks)}")
        B = len(chunks[0].data)
        if any(len(c.data) != B for c in chunks):
            raise FecError("chunks of different lengths")
        try:
            return _lib.thread_context().decode(self.k, self.m, [c.data for c in chunks],
                                                [c.index for c in chunks], B, padlen)
        except _lib.StorbRsError as e:
            if e.code in (_lib.EINVAL, _lib.ENOTENOUGH):
                raise FecError(str(e)) from e
            raise
