"""storb_amd -- MI355X-native chunk->shard Reed-Solomon path for Storb.

Scope: exactly the erasure-coding stage of crates/storb_base (the zfec-rs
calls in piece.rs). The product is the HIP library storb_amd/lib/
libstorb_rs.so behind the C ABI include/storb_rs.h; this package is its
Python binding (``_lib``), a zfec-rs mirror (``fec``) and a piece.rs mirror
(``piece``). There is no CPU fallback.
"""
from . import _lib
from ._lib import Context, StorbRsError, build, device_count, thread_context
from .fec import Chunk, Fec, FecError
from .piece import (EncodedChunk, Panic, Piece, PieceError, PieceType, decode_chunk,
                    encode_chunk, get_k_and_m, piece_length, reconstruct_chunk,
                    reconstruct_data)

__all__ = [
    "Context", "StorbRsError", "build", "device_count", "thread_context", "Chunk", "Fec",
    "FecError", "EncodedChunk", "Panic", "Piece", "PieceError", "PieceType",
    "decode_chunk", "encode_chunk", "get_k_and_m", "piece_length", "reconstruct_chunk",
    "reconstruct_data",
]
