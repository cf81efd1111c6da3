"""CPU ORACLE, numpy twin (test infrastructure only).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import anything under oracle/, and only as the checker. The product path
(storb_amd) never imports it.

An independent second restatement of zfec's fec.c (the algorithm behind
zfec-rs @3f3a3720, reference Cargo.toml:81) used to cross-check the C oracle
and to emit the committed fixtures in tests/golden/. Unlike the C oracle it
derives the generator two different ways:

* ``enc_matrix_gauss``    V[k..n) * inverse(V[0..k)) by Gauss-Jordan;
* ``enc_matrix_lagrange`` the closed form enc[r][j] = prod_{l!=j}
  (x_r + x_l) / (x_j + x_l) with x_0 = 0, x_i = alpha^(i-1)
  (SURVEY.md Appendix A.2).

PARITY UNPINNED: no zfec-rs output exists offline; see oracle/zfec_oracle.h.
"""
from __future__ import annotations

import math
from typing import Sequence

import numpy as np

PRIM_POLY = 0x11D  # x^8+x^4+x^3+x^2+1, fec.c Pp = "101110001"


def _tables():
    exp = np.zeros(510, dtype=np.uint8)
    log = np.zeros(256, dtype=np.int32)
    x = 1
    for i in range(255):
        exp[i] = x
        log[x] = i
        x <<= 1
        if x & 0x100:
            x ^= PRIM_POLY
    exp[255:510] = exp[0:255]
    log[0] = 255
    inv = np.zeros(256, dtype=np.uint8)
    for a in range(1, 256):
        inv[a] = exp[(255 - log[a]) % 255]
    la = log[:, None].astype(np.int64)
    lb = log[None, :].astype(np.int64)
    mul = exp[(la + lb) % 255].astype(np.uint8)
    mul[0, :] = 0
    mul[:, 0] = 0
    return exp, log, inv, mul


GF_EXP, GF_LOG, GF_INV, GF_MUL = _tables()


def gf_mul(a: int, b: int) -> int:
    return int(GF_MUL[a, b])


def gf_inv(a: int) -> int:
    return int(GF_INV[a])


def _mat_inv(m: np.ndarray) -> np.ndarray:
    k = m.shape[0]
    a = np.concatenate([m.astype(np.uint8), np.eye(k, dtype=np.uint8)], axis=1)
    for col in range(k):
        piv = next((r for r in range(col, k) if a[r, col]), None)
        if piv is None:
            raise ValueError("singular matrix")
        if piv != col:
            a[[col, piv]] = a[[piv, col]]
        a[col] = GF_MUL[gf_inv(int(a[col, col])), a[col]]
        for r in range(k):
            if r != col and a[r, col]:
                a[r] ^= GF_MUL[int(a[r, col]), a[col]]
    return a[:, k:].copy()


def _mat_mul(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    out = np.zeros((a.shape[0], b.shape[1]), dtype=np.uint8)
    for i in range(a.shape[0]):
        for j in range(b.shape[1]):
            acc = 0
            for t in range(a.shape[1]):
                acc ^= int(GF_MUL[a[i, t], b[t, j]])
            out[i, j] = acc
    return out


def vandermonde(k: int, n: int) -> np.ndarray:
    v = np.zeros((n, k), dtype=np.uint8)
    v[0, 0] = 1
    for row in range(n - 1):
        for col in range(k):
            v[row + 1, col] = GF_EXP[(row * col) % 255]
    return v


def check_params(k: int, n: int) -> None:
    if k < 1 or n < 1 or n > 256 or k > n:
        raise ValueError(f"invalid (k={k}, n={n})")


def enc_matrix_gauss(k: int, n: int) -> np.ndarray:
    check_params(k, n)
    v = vandermonde(k, n)
    top_inv = _mat_inv(v[:k])
    enc = np.zeros((n, k), dtype=np.uint8)
    enc[:k] = np.eye(k, dtype=np.uint8)
    if n > k:
        enc[k:] = _mat_mul(v[k:], top_inv)
    return enc


def _point(i: int) -> int:
    return 0 if i == 0 else int(GF_EXP[(i - 1) % 255])


def enc_matrix_lagrange(k: int, n: int) -> np.ndarray:
    check_params(k, n)
    enc = np.zeros((n, k), dtype=np.uint8)
    enc[:k] = np.eye(k, dtype=np.uint8)
    for r in range(k, n):
        xr = _point(r)
        for j in range(k):
            xj = _point(j)
            num, den = 1, 1
            for l in range(k):
                if l == j:
                    continue
                xl = _point(l)
                num = gf_mul(num, xr ^ xl)
                den = gf_mul(den, xj ^ xl)
            enc[r, j] = gf_mul(num, gf_inv(den))
    return enc


enc_matrix = enc_matrix_gauss


def encode(k: int, n: int, data: bytes | np.ndarray):
    """Fec::encode: returns (shares[n, B] uint8, B, padlen)."""
    check_params(k, n)
    buf = np.frombuffer(bytes(data), dtype=np.uint8) if not isinstance(data, np.ndarray) else data.astype(np.uint8)
    if buf.size == 0:
        raise ValueError("empty chunk")
    B = -(-buf.size // k)
    padlen = B * k - buf.size
    shards = np.zeros(k * B, dtype=np.uint8)
    shards[: buf.size] = buf
    shards = shards.reshape(k, B)
    enc = enc_matrix(k, n)
    out = np.zeros((n, B), dtype=np.uint8)
    out[:k] = shards
    for r in range(k, n):
        acc = np.zeros(B, dtype=np.uint8)
        for j in range(k):
            acc ^= GF_MUL[int(enc[r, j])][shards[j]]
        out[r] = acc
    return out, B, padlen


def decode(k: int, n: int, shares: Sequence[np.ndarray], idx: Sequence[int], padlen: int) -> bytes:
    """decode_chunk semantics: sort by index, first k, Fec::decode."""
    check_params(k, n)
    order = sorted(range(len(idx)), key=lambda i: idx[i])[:k]
    if len(order) < k:
        raise ValueError("not enough shares")
    sel = [int(idx[i]) for i in order]
    if len(set(sel)) != k or any(s >= n for s in sel):
        raise ValueError("duplicate or out-of-range share index")
    enc = enc_matrix(k, n)
    rows = np.stack([enc[s] for s in sel])
    mats = np.stack([np.asarray(shares[i], dtype=np.uint8) for i in order])
    dinv = _mat_inv(rows)
    B = mats.shape[1]
    data = np.zeros((k, B), dtype=np.uint8)
    for r in range(k):
        acc = np.zeros(B, dtype=np.uint8)
        for c in range(k):
            acc ^= GF_MUL[int(dinv[r, c])][mats[c]]
        data[r] = acc
    flat = data.reshape(-1)
    return flat[: k * B - padlen].tobytes()


def piece_length(content_length: int, min_size: int | None = None, max_size: int | None = None) -> int:
    """piece.rs:292-303 (f64 log2, saturating `as i32`, masked shift)."""
    min_size = 16 * 1024 if min_size is None else min_size
    max_size = 256 * 1024 * 1024 if max_size is None else max_size
    e = (math.log2(content_length) if content_length > 0 else -math.inf) * 0.5 + 8.39
    if math.isnan(e):
        ei = 0
    elif e <= -(2**31):
        ei = -(2**31)
    elif e >= 2**31 - 1:
        ei = 2**31 - 1
    else:
        ei = int(e)
    length = 1 << (ei & 63)
    return max(min_size, min(length, max_size))


def get_k_and_m(chunk_size: int):
    """piece.rs:307-317 (m is the TOTAL share count)."""
    ps = piece_length(chunk_size)
    k = math.ceil(chunk_size / ps)
    return k, k + math.ceil(k / 2.0)


def splitmix_bytes(seed: int, length: int) -> np.ndarray:
    """Same stream as zo_splitmix_fill / the device fill kernel."""
    words = -(-length // 8)
    i = np.arange(1, words + 1, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + i * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z ^= z >> np.uint64(31)
    return z.astype("<u8").view(np.uint8)[:length].copy()
