"""BLAKE3 (hash mode, 32-byte output) restated from the published spec --
CPU ORACLE, test infrastructure only.

Storb identifies every shard by blake3(shard bytes) (upload.rs:623,
crates/storb_miner/src/lib.rs:265-283, download.rs:158-161) using the crate
blake3 1.8.2 (reference Cargo.lock:1099-1107), which is not available in this
image (no Python or C blake3 either). This is a direct restatement of the
BLAKE3 paper / reference implementation: 7-round BLAKE2s-derived compression,
1024-byte chunks of 64-byte blocks, left-balanced binary tree, flags
CHUNK_START/CHUNK_END/PARENT/ROOT. Pinned by the published vectors in
tests/test_blake3.py (empty input, "abc", and entries of the official
test_vectors.json whose input is bytes i % 251).
"""
from __future__ import annotations

IV = (0x6A09E667, 0xBB67AE85, 0x3C6EF372, 0xA54FF53A,
      0x510E527F, 0x9B05688C, 0x1F83D9AB, 0x5BE0CD19)
MSG_PERM = (2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8)
CHUNK_START, CHUNK_END, PARENT, ROOT = 1, 2, 4, 8
BLOCK_LEN, CHUNK_LEN = 64, 1024
M32 = 0xFFFFFFFF


def _rotr(x, n):
    return ((x >> n) | (x << (32 - n))) & M32


def _g(s, a, b, c, d, mx, my):
    s[a] = (s[a] + s[b] + mx) & M32
    s[d] = _rotr(s[d] ^ s[a], 16)
    s[c] = (s[c] + s[d]) & M32
    s[b] = _rotr(s[b] ^ s[c], 12)
    s[a] = (s[a] + s[b] + my) & M32
    s[d] = _rotr(s[d] ^ s[a], 8)
    s[c] = (s[c] + s[d]) & M32
    s[b] = _rotr(s[b] ^ s[c], 7)


def compress(cv, block_words, counter, block_len, flags):
    s = list(cv) + list(IV[:4]) + [counter & M32, (counter >> 32) & M32, block_len, flags]
    m = list(block_words)
    for r in range(7):
        _g(s, 0, 4, 8, 12, m[0], m[1])
        _g(s, 1, 5, 9, 13, m[2], m[3])
        _g(s, 2, 6, 10, 14, m[4], m[5])
        _g(s, 3, 7, 11, 15, m[6], m[7])
        _g(s, 0, 5, 10, 15, m[8], m[9])
        _g(s, 1, 6, 11, 12, m[10], m[11])
        _g(s, 2, 7, 8, 13, m[12], m[13])
        _g(s, 3, 4, 9, 14, m[14], m[15])
        if r < 6:
            m = [m[i] for i in MSG_PERM]
    for i in range(8):
        s[i] ^= s[i + 8]
        s[i + 8] ^= cv[i]
    return s


def _words(block: bytes):
    block = block + bytes(BLOCK_LEN - len(block))
    return [int.from_bytes(block[4 * i:4 * i + 4], "little") for i in range(16)]


def _chunk_output(chunk: bytes, counter: int):
    """(cv, block_words, block_len, flags) of the chunk's last block."""
    cv = list(IV)
    blocks = [chunk[i:i + BLOCK_LEN] for i in range(0, len(chunk), BLOCK_LEN)] or [b""]
    for bi, blk in enumerate(blocks):
        flags = (CHUNK_START if bi == 0 else 0) | (CHUNK_END if bi == len(blocks) - 1 else 0)
        if bi == len(blocks) - 1:
            return cv, _words(blk), len(blk), flags
        cv = compress(cv, _words(blk), counter, len(blk), flags)[:8]


def _parent_words(left, right):
    return list(left) + list(right)


def blake3(data: bytes) -> bytes:
    data = bytes(data)
    chunks = [data[i:i + CHUNK_LEN] for i in range(0, len(data), CHUNK_LEN)] or [b""]
    if len(chunks) == 1:
        cv, w, bl, fl = _chunk_output(chunks[0], 0)
        out = compress(cv, w, 0, bl, fl | ROOT)
        return b"".join(x.to_bytes(4, "little") for x in out[:8])
    nodes = []
    for c, ch in enumerate(chunks):
        cv, w, bl, fl = _chunk_output(ch, c)
        nodes.append(compress(cv, w, c, bl, fl)[:8])
    # left-balanced tree = pairwise merging with the odd node carried up
    while len(nodes) > 2:
        nxt = [compress(IV, _parent_words(nodes[i], nodes[i + 1]), 0, BLOCK_LEN, PARENT)[:8]
               for i in range(0, len(nodes) - 1, 2)]
        if len(nodes) % 2:
            nxt.append(nodes[-1])
        nodes = nxt
    out = compress(IV, _parent_words(nodes[0], nodes[1]), 0, BLOCK_LEN, PARENT | ROOT)
    return b"".join(x.to_bytes(4, "little") for x in out[:8])


def hexdigest(data: bytes) -> str:
    return blake3(data).hex()
