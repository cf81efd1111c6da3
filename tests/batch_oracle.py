"""Whole-batch oracle checks for the BASELINE-size GPU tests (VERDICT r5
item 4): the C oracle (oracle/zfec_oracle.c, test infrastructure) run on
host threads over EVERY stripe of a device batch, instead of a sampled few.

The oracle's byte-wise table loop runs ~19x slower on hosts that leave
store-bypass speculation enabled for the process (DESIGN.md §5 Host
variance); the calls below run from a thread that turns Speculative Store
Bypass Disable on for itself first (prctl; the oracle's worker threads
inherit it), which only changes its speed."""
import ctypes
import os
import threading

import numpy as np

from oracle import coracle

THREADS = max(1, min(16, os.cpu_count() or 1))  # the GPU box's CPU share


def _ssbd_thread(fn, *args):
    res = {}

    def body():
        ctypes.CDLL(None).prctl(53, 0, 4, 0, 0)  # PR_SET_SPECULATION_CTRL: best effort
        try:
            res["v"] = fn(*args)
        except BaseException as e:  # re-raised in the caller
            res["e"] = e

    t = threading.Thread(target=body)
    t.start()
    t.join()
    if "e" in res:
        raise res["e"]
    return res["v"]


def splitmix_chunks(seed0: int, chunk: int, nchunks: int) -> np.ndarray:
    """The synthetic inputs as the oracle generates them: chunk c =
    splitmix64(seed0 + c) (the device fill kernel's contract)."""
    out = np.empty(nchunks * chunk, np.uint8)
    for c in range(nchunks):
        out[c * chunk:(c + 1) * chunk] = coracle.splitmix_bytes(seed0 + c, chunk)
    return out


def parity_all(k: int, n: int, data: np.ndarray, chunk: int, nchunks: int) -> np.ndarray:
    """Parity of every chunk (nchunks x (n-k) x B, packed), oracle, threaded."""
    return _ssbd_thread(coracle.encode_parity_many, k, n, np.ascontiguousarray(data), chunk,
                        nchunks, THREADS)


def decode_all(k: int, n: int, data: np.ndarray, parity: np.ndarray, block: int,
               nchunks: int, survivors) -> np.ndarray:
    """Every chunk rebuilt by the oracle from `survivors` among its data
    shares (data) and parity shares (parity)."""
    return _ssbd_thread(coracle.decode_many, k, n, data, parity, block, nchunks, survivors,
                        THREADS)


def first_mismatch(got: np.ndarray, want: np.ndarray, per: int):
    """Index of the first unit of `per` bytes that differs, or None."""
    if np.array_equal(got, want):
        return None
    g, w = got.reshape(-1, per), want.reshape(-1, per)
    return int(np.nonzero((g != w).any(axis=1))[0][0])
