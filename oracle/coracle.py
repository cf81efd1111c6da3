"""ctypes binding for the C oracle (oracle/_build/libzfec_oracle.so).

TEST INFRASTRUCTURE ONLY -- the checker and the timed CPU baseline; see
oracle/zfec_oracle.h for what it restates and its parity status.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from typing import Sequence

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "_build", "libzfec_oracle.so")
_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _SO


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            build()
        L = C.CDLL(_SO)
        u8p = C.POINTER(C.c_uint8)
        L.zo_gf_mul.restype = C.c_uint8
        L.zo_gf_mul.argtypes = [C.c_uint8, C.c_uint8]
        L.zo_gf_inv.restype = C.c_uint8
        L.zo_gf_inv.argtypes = [C.c_uint8]
        L.zo_gf_exp.restype = C.c_uint8
        L.zo_gf_exp.argtypes = [C.c_uint]
        L.zo_fec_new.argtypes = [C.c_uint, C.c_uint, u8p]
        L.zo_invert_mat.argtypes = [u8p, C.c_uint]
        L.zo_encode.argtypes = [C.c_uint, C.c_uint, C.c_void_p, C.c_size_t, C.c_void_p,
                                C.POINTER(C.c_size_t), C.POINTER(C.c_size_t)]
        L.zo_encode_parity.argtypes = [C.c_uint, C.c_uint, C.c_void_p, C.c_size_t,
                                       C.POINTER(C.c_void_p), C.POINTER(C.c_size_t),
                                       C.POINTER(C.c_size_t)]
        L.zo_decode.argtypes = [C.c_uint, C.c_uint, C.POINTER(C.c_void_p), C.POINTER(C.c_uint),
                                C.c_uint, C.c_size_t, C.c_size_t, C.c_void_p]
        L.zo_piece_length.restype = C.c_uint64
        L.zo_piece_length.argtypes = [C.c_uint64, C.c_uint64, C.c_uint64]
        L.zo_get_k_and_m.argtypes = [C.c_uint64, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
        L.zo_splitmix_fill.argtypes = [C.c_uint64, C.c_void_p, C.c_size_t]
        L.zo_decode_many.argtypes = [C.c_uint, C.c_uint, C.c_void_p, C.c_void_p, C.c_size_t,
                                     C.c_uint, C.c_void_p, C.c_void_p, C.c_int]
        L.zo_encode_many.argtypes = [C.c_uint, C.c_uint, C.c_void_p, C.c_size_t, C.c_uint,
                                     C.c_void_p, C.c_int]
        L.zo_bench_roundtrip.argtypes = [C.c_uint, C.c_uint, C.c_void_p, C.c_size_t, C.c_uint,
                                         C.POINTER(C.c_uint), C.c_uint, C.c_int, C.c_int,
                                         C.c_int, C.c_double, C.c_void_p]
        L.zo_roundtrip_many.argtypes = [C.c_uint, C.c_uint, C.c_void_p, C.c_size_t, C.c_uint,
                                        C.POINTER(C.c_uint), C.c_uint, C.c_int]
        _lib = L
    return _lib


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data


def enc_matrix(k: int, n: int) -> np.ndarray:
    out = np.zeros(n * k, dtype=np.uint8)
    rc = lib().zo_fec_new(k, n, out.ctypes.data_as(C.POINTER(C.c_uint8)))
    if rc != 0:
        raise ValueError(f"invalid (k={k}, n={n})")
    return out.reshape(n, k)


def encode(k: int, n: int, data) -> tuple[np.ndarray, int, int]:
    buf = np.frombuffer(bytes(data), dtype=np.uint8) if not isinstance(data, np.ndarray) else np.ascontiguousarray(data, dtype=np.uint8)
    if buf.size == 0 or k < 1:
        raise ValueError("empty chunk or k < 1")
    B = -(-buf.size // k)
    shares = np.zeros(n * B, dtype=np.uint8)
    b, p = C.c_size_t(), C.c_size_t()
    rc = lib().zo_encode(k, n, _ptr(buf), buf.size, _ptr(shares), C.byref(b), C.byref(p))
    if rc != 0:
        raise ValueError(f"zo_encode failed rc={rc}")
    return shares.reshape(n, B), b.value, p.value


def encode_parity_many(k: int, n: int, data: np.ndarray, chunk_len: int, nchunks: int,
                       threads: int = 1) -> np.ndarray:
    B = -(-chunk_len // k)
    out = np.zeros(nchunks * (n - k) * B, dtype=np.uint8)
    rc = lib().zo_encode_many(k, n, _ptr(data), chunk_len, nchunks, _ptr(out), threads)
    if rc != 0:
        raise ValueError("zo_encode_many failed")
    return out


def decode_many(k: int, n: int, data: np.ndarray, parity: np.ndarray, block: int,
                nchunks: int, survivors, threads: int = 1) -> np.ndarray:
    """Whole-batch decode (zo_decode_many): chunk c rebuilt from the survivors
    (sorted, k of them) among its data shares (data, k*block per chunk) and
    parity shares (parity, (n-k)*block per chunk); returns nchunks*k*block."""
    surv = sorted(survivors)[:k]
    sv = (C.c_uint * k)(*surv)
    out = np.zeros(nchunks * k * block, dtype=np.uint8)
    rc = lib().zo_decode_many(k, n, _ptr(np.ascontiguousarray(data)),
                              _ptr(np.ascontiguousarray(parity)), block, nchunks, sv,
                              _ptr(out), threads)
    if rc != 0:
        raise ValueError(f"zo_decode_many failed ({rc})")
    return out


def decode(k: int, n: int, shares: Sequence[np.ndarray], idx: Sequence[int], block: int,
           padlen: int) -> bytes:
    arrs = [np.ascontiguousarray(s, dtype=np.uint8) for s in shares]
    ptrs = (C.c_void_p * max(1, len(arrs)))(*[a.ctypes.data for a in arrs])
    ids = (C.c_uint * max(1, len(idx)))(*idx)
    out = np.zeros(max(1, k * block - padlen), dtype=np.uint8)
    rc = lib().zo_decode(k, n, ptrs, ids, len(arrs), block, padlen, _ptr(out))
    if rc == -2:
        raise ValueError("not enough / duplicate shares")
    if rc != 0:
        raise ValueError(f"invalid decode parameters rc={rc}")
    return out[: k * block - padlen].tobytes()


def piece_length(n: int, min_size: int = 0, max_size: int = 0) -> int:
    return int(lib().zo_piece_length(n, min_size, max_size))


def get_k_and_m(n: int) -> tuple[int, int]:
    k, m = C.c_uint64(), C.c_uint64()
    lib().zo_get_k_and_m(n, C.byref(k), C.byref(m))
    return k.value, m.value


def splitmix_bytes(seed: int, length: int) -> np.ndarray:
    out = np.zeros(length, dtype=np.uint8)
    lib().zo_splitmix_fill(seed, _ptr(out), length)
    return out


def roundtrip_many(k: int, n: int, data: np.ndarray, chunk_len: int, nchunks: int,
                   erased, threads: int) -> int:
    """Threaded encode+decode round trips; returns the number of failures."""
    er = (C.c_uint * max(1, len(erased)))(*erased)
    return int(lib().zo_roundtrip_many(k, n, _ptr(data), chunk_len, nchunks, er, len(erased),
                                       threads))


class BenchStats(C.Structure):
    """zo_bench_t (oracle/zfec_oracle.h)."""
    _fields_ = [("wall_s", C.c_double), ("user_s", C.c_double), ("sys_s", C.c_double),
                ("minflt", C.c_long), ("majflt", C.c_long), ("nvcsw", C.c_long),
                ("nivcsw", C.c_long), ("calls", C.c_ulonglong), ("cpu_start", C.c_int),
                ("cpu_end", C.c_int), ("bad", C.c_int), ("cycles", C.c_longlong),
                ("instructions", C.c_longlong), ("probe_before", C.c_double),
                ("probe_after", C.c_double), ("l1_addmul_gbs", C.c_double),
                ("l2_read_gbs", C.c_double), ("dram_read_gbs", C.c_double)]


def bench_roundtrip(k: int, n: int, chunks: np.ndarray, chunk_len: int, nsample: int,
                    survivor_sets, do_encode: bool, do_decode: bool, fresh: bool,
                    seconds: float) -> dict:
    """The CPU baseline loop in C on the calling thread (oracle/cpu_bench.c)
    with that thread's getrusage accounting. fresh: per-call buffers as
    zfec-rs allocates them; else every buffer allocated once."""
    sets = [list(s)[:k] for s in survivor_sets]
    flat = (C.c_uint * (k * len(sets)))(*[i for s in sets for i in s])
    st = BenchStats()
    buf = np.ascontiguousarray(chunks, dtype=np.uint8)
    rc = lib().zo_bench_roundtrip(k, n, buf.ctypes.data, chunk_len, nsample, flat, len(sets),
                                  int(do_encode), int(do_decode), int(fresh), float(seconds),
                                  C.addressof(st))
    if rc != 0 or st.bad:
        raise ValueError(f"zo_bench_roundtrip rc={rc} bad={st.bad}")
    return {f: getattr(st, f) for f, _ in BenchStats._fields_}
