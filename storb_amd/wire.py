"""Storb's wire and storage formats on either side of the RS stage
(SURVEY.md 8(f).3), for the loopback harness (tools/loopback.py).

* Store stream (validator -> miner), upload.rs:47-122 and
  crates/storb_miner/src/lib.rs:158-285:
  [u64 BE len(handshake)] [bincode HandshakePayload] [u64 BE piece_len]
  [piece bytes]; the miner answers blake3(piece) as 32 raw bytes + b"\\n".
  The reference runs it over a QUIC bi-stream; the harness uses one TCP
  stream per miner with the same framing, frame after frame (QUIC transport
  and the sr25519 handshake verification are out of scope: the payload is
  carried and skipped, not verified).
* Retrieve (miner -> validator), crates/storb_miner/src/routes.rs:101-207,
  download.rs:47-164: GET /piece?piecehash=<hex>&handshake=<hex> returns
  bincode{fixint, LE}(PieceResponse{piece_hash: [u8; 32], piece_data:
  Vec<u8>}) = [32 B hash][u64 LE len][data] (piece.rs:202-255); the
  validator checks blake3(data) == piece_hash (download.rs:158-161).
* Miner object store, crates/storb_miner/src/store.rs:18-66:
  store_dir/<hex[0:2]>/<hex[2:]> holds the raw piece bytes.
"""
from __future__ import annotations

import os
import socket
import struct

from . import _lib

HASH_LEN = 32


def recv_exact(sock: socket.socket, n: int) -> bytes:
    buf = bytearray(n)
    view = memoryview(buf)
    got = 0
    while got < n:
        r = sock.recv_into(view[got:], n - got)
        if r == 0:
            raise EOFError("connection closed")
        got += r
    return bytes(buf)


def send_piece(sock: socket.socket, handshake: bytes, piece) -> bytes:
    """One store frame (upload.rs:88-100); returns the miner's 32-byte ack."""
    piece = memoryview(piece)
    sock.sendall(struct.pack(">Q", len(handshake)) + handshake +
                 struct.pack(">Q", len(piece)))
    sock.sendall(piece)
    ack = recv_exact(sock, HASH_LEN + 1)
    if ack[-1:] != b"\n":
        raise ValueError("bad ack delimiter")
    return ack[:HASH_LEN]


def read_store_frame(sock: socket.socket):
    """Miner side of one store frame: (handshake, piece) or None at EOF."""
    try:
        hdr = recv_exact(sock, 8)
    except EOFError:
        return None
    (hlen,) = struct.unpack(">Q", hdr)
    handshake = recv_exact(sock, hlen)
    (plen,) = struct.unpack(">Q", recv_exact(sock, 8))
    return handshake, recv_exact(sock, plen)


def serialise_piece_response(piece_hash: bytes, data: bytes) -> bytes:
    """piece.rs:220-234: bincode fixint little-endian PieceResponse."""
    assert len(piece_hash) == HASH_LEN
    return piece_hash + struct.pack("<Q", len(data)) + data


def deserialise_piece_response(buf, piece_hash: bytes) -> memoryview:
    """piece.rs:238-255 + download.rs:121-164: locate the hash, decode the
    Vec<u8>, reject trailing bytes, and check blake3(data) == piece_hash.
    Returns a zero-copy view of the piece inside `buf` (no slice copies:
    fetch threads hold the GIL for every copy of a shard)."""
    mv = memoryview(buf).cast("B")
    pos = 0 if bytes(mv[:HASH_LEN]) == piece_hash else bytes(buf).find(piece_hash)
    if pos < 0:
        raise ValueError("piece hash not found in response")
    rest = mv[pos + HASH_LEN:]
    if len(rest) < 8:
        raise ValueError("truncated response")
    (n,) = struct.unpack("<Q", rest[:8])
    if len(rest) != 8 + n:
        raise ValueError("trailing or missing bytes in response")
    data = rest[8:]
    if _lib.blake3(data) != piece_hash:
        raise ValueError("piece hash mismatch")
    return data


class PieceClient:
    """Keep-alive HTTP/1.1 GET /piece client for one miner (the retrieve
    request of download.rs:47-164). Reads the body with recv_into into one
    preallocated buffer: http.client's reads cost the fetch threads about
    half their throughput in GIL-held copies."""

    def __init__(self, host: str, port: int, timeout: float = 10.0):
        self.sock = socket.create_connection((host, port), timeout=timeout)
        self.sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        self.host = f"{host}:{port}"

    def get(self, hexhash: str, handshake_hex: str):
        """Returns (status, body bytearray)."""
        self.sock.sendall((f"GET /piece?piecehash={hexhash}&handshake={handshake_hex} "
                           f"HTTP/1.1\r\nHost: {self.host}\r\n\r\n").encode())
        head = bytearray()
        while True:
            end = head.find(b"\r\n\r\n")
            if end >= 0:
                break
            more = self.sock.recv(65536)
            if not more:
                raise ConnectionError("connection closed in response headers")
            head += more
        lines = bytes(head[:end]).split(b"\r\n")
        status = int(lines[0].split()[1])
        length = None
        for ln in lines[1:]:
            k, _, v = ln.partition(b":")
            if k.strip().lower() == b"content-length":
                length = int(v)
        if length is None:
            raise ValueError("response without Content-Length")
        body = bytearray(length)
        view = memoryview(body)
        got = len(head) - (end + 4)
        if got > length:
            raise ValueError("unexpected bytes after the response body")
        view[:got] = head[end + 4:]
        while got < length:
            r = self.sock.recv_into(view[got:], length - got)
            if r == 0:
                raise ConnectionError("connection closed in response body")
            got += r
        return status, body

    def close(self):
        self.sock.close()


class ObjectStore:
    """store.rs:18-66: <dir>/<hash[0:2]>/<hash[2:]>."""

    def __init__(self, path: str):
        self.path = path
        if not os.path.exists(path):
            os.makedirs(path)
            for i in range(256):
                os.makedirs(os.path.join(path, f"{i:02x}"), exist_ok=True)

    def _file(self, hexhash: str) -> str:
        return os.path.join(self.path, hexhash[:2], hexhash[2:])

    def write(self, hexhash: str, data) -> str:
        f = self._file(hexhash)
        os.makedirs(os.path.dirname(f), exist_ok=True)  # store.rs:50-53
        with open(f, "wb") as fh:
            fh.write(data)
        return f

    def read(self, hexhash: str) -> bytes:
        with open(self._file(hexhash), "rb") as fh:
            return fh.read()

    def send_piece_response(self, sock: socket.socket, hexhash: str, http_head: bytes) -> None:
        """Writes `http_head` and the bincode PieceResponse of the stored
        piece to sock, the piece bytes with sendfile (no copy through
        Python). Raises OSError/ValueError before writing anything if the
        piece is missing."""
        with open(self._file(hexhash), "rb") as fh:
            size = os.fstat(fh.fileno()).st_size
            prefix = bytes.fromhex(hexhash) + struct.pack("<Q", size)
            sock.sendall(http_head % (len(prefix) + size) + prefix)
            off = 0
            while off < size:
                off += os.sendfile(sock.fileno(), fh.fileno(), off, size - off)
