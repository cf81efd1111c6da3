"""Python transliteration of the zfec-rs shim (integration/zfec-rs-mi355x/src/lib.rs).

TEST INFRASTRUCTURE. The Rust crate cannot be compiled in this image (no
cargo / rustc), so its logic is restated here statement for statement and run
against a *backend* with the C ABI's contract (include/storb_rs.h
storb_rs_block_size / storb_rs_encode_shares / storb_rs_decode, return codes 0 / 1 / 2):

* `LibBackend` -- the real libstorb_rs.so through ctypes (needs a gfx950 GPU);
* `OracleBackend` -- the CPU oracle (oracle/coracle.py) wrapped in that same
  contract, so the shim's own logic (share slicing and zero padding, the b and
  padding checks, error mapping) is tested on CPU.

Line references are to lib.rs; `piece.rs` means crates/storb_base/src/piece.rs
of the reference, whose calls (piece.rs:328-329,375,383-386) this API serves.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

EINVAL, ENOTENOUGH = 1, 2


class ShimError(Exception):
    """lib.rs `Error { code, message }` (lib.rs:53-84)."""

    def __init__(self, code: int, message: str = ""):
        super().__init__(f"zfec-rs(mi355x) error {code}: {message}")
        self.code = code


@dataclass
class Chunk:
    """lib.rs:113-124: `pub struct Chunk { pub data: Vec<u8>, pub index: usize }`."""
    data: bytearray
    index: int


class OracleBackend:
    """The C ABI's contract over the CPU oracle (checker only)."""

    def block_size(self, k: int, length: int) -> int:  # storb_rs_block_size
        return (length + k - 1) // k if k else 0

    def check_params(self, k: int, n: int) -> int:  # storb_rs_check_params
        return 0 if 1 <= k <= n <= 256 else EINVAL

    def encode_shares(self, k, n, data: bytes, shares_out: list) -> tuple[int, int, int]:
        from oracle import coracle
        if self.check_params(k, n) or len(data) == 0:
            return EINVAL, 0, 0
        shares, B, pad = coracle.encode(k, n, data)
        for i, out in enumerate(shares_out):
            out[:B] = shares[i].tobytes()
        return 0, B, pad

    def decode(self, k, n, shares: list, idx: list, block: int, padlen: int, out) -> int:
        from oracle import coracle
        if self.check_params(k, n) or block == 0 or padlen >= k * block:
            return EINVAL
        if any(i >= n for i in idx):
            return EINVAL
        first = sorted(range(len(idx)), key=lambda i: idx[i])[:k]
        if len(first) < k or len({idx[i] for i in first}) < k:
            return ENOTENOUGH
        rec = coracle.decode(k, n, [np.frombuffer(bytes(shares[i]), np.uint8) for i in first],
                             [idx[i] for i in first], block, padlen)
        out[:len(rec)] = rec
        return 0


class LibBackend:
    """libstorb_rs.so through ctypes, the externs lib.rs's Fec uses."""

    def __init__(self, ctx_handle):
        from storb_amd import _lib
        self.L = _lib.lib()
        self.ctx = ctx_handle

    def block_size(self, k, length):
        return int(self.L.storb_rs_block_size(k, length))

    def check_params(self, k, n):
        return int(self.L.storb_rs_check_params(k, n))

    def encode_shares(self, k, n, data: bytes, shares_out: list):
        buf = (C.c_uint8 * max(1, len(data))).from_buffer_copy(data or b"\0")
        outs = [(C.c_uint8 * max(1, len(p))).from_buffer(p) for p in shares_out]
        ptrs = (C.c_void_p * max(1, len(outs)))(*[C.addressof(o) for o in outs])
        b, pad = C.c_size_t(), C.c_size_t()
        rc = self.L.storb_rs_encode_shares(self.ctx, k, n, C.addressof(buf), len(data), ptrs,
                                           C.byref(b), C.byref(pad))
        return int(rc), int(b.value), int(pad.value)

    def decode(self, k, n, shares, idx, block, padlen, out):
        bufs = [(C.c_uint8 * max(1, len(s))).from_buffer(s) for s in shares]
        ptrs = (C.c_void_p * max(1, len(bufs)))(*[C.addressof(b) for b in bufs])
        ids = (C.c_uint32 * max(1, len(idx)))(*idx)
        o = (C.c_uint8 * max(1, len(out))).from_buffer(out)
        return int(self.L.storb_rs_decode(self.ctx, k, n, ptrs, ids, len(idx), block, padlen,
                                          C.addressof(o)))


class Fec:
    """lib.rs:126-187 `pub struct Fec { k, m }`; m is the TOTAL share count."""

    def __init__(self, k: int, m: int, backend):
        # lib.rs:134-139: k > 256 || m > 256 || storb_rs_check_params != 0 -> Err(code 1)
        if k > 256 or m > 256 or backend.check_params(k, m) != 0:
            raise ShimError(EINVAL, "invalid argument")
        self.k, self.m, self.be = k, m, backend

    def encode(self, data: bytes) -> tuple[list[Chunk], int]:
        """lib.rs Fec::encode: m Vecs of capacity b (uninitialised in Rust;
        here filled with 0xCD so an unwritten byte shows), every share --
        data shares zero-padded, then parity -- written by one
        storb_rs_encode_shares call; returns all m shares in index order and
        padlen."""
        k, m = self.k, self.m
        b = self.be.block_size(k, len(data))
        bufs = [bytearray(b"\xcd" * b) for _ in range(m)]
        rc, _block, pad = self.be.encode_shares(k, m, bytes(data), bufs)
        if rc != 0:
            raise ShimError(rc)
        return [Chunk(bufs[i], i) for i in range(m)], pad

    def decode(self, encoded_data: list[Chunk], padding: int) -> bytes:
        """lib.rs:166-186: Err(2) below k shares; b from the first share; Err(1)
        for b == 0, padding >= k*b or shares of unequal length; output
        k*b - padding bytes."""
        k = self.k
        if len(encoded_data) < k:
            raise ShimError(ENOTENOUGH)
        b = len(encoded_data[0].data)
        if b == 0 or padding >= k * b or any(len(c.data) != b for c in encoded_data):
            raise ShimError(EINVAL)
        out = bytearray(b"\xcd" * (k * b - padding))  # Vec::with_capacity: not zero-filled
        rc = self.be.decode(k, self.m, [c.data for c in encoded_data],
                            [c.index for c in encoded_data], b, padding, out)
        if rc != 0:
            raise ShimError(rc)
        return bytes(out)


def decode_chunk(pieces: list[tuple[int, bytes]], k: int, m: int, padlen: int, backend) -> bytes:
    """piece.rs:363-387 decode_chunk over this shim: sort by piece_idx, keep
    the first k (or all if fewer), wrap as Chunk::new(data.clone(), idx)."""
    srt = sorted(pieces, key=lambda p: p[0])
    if len(srt) > k:
        srt = srt[:k]
    chunks = [Chunk(bytearray(d), i) for i, d in srt]
    return Fec(k, m, backend).decode(chunks, padlen)
