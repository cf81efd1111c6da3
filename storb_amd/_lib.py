"""ctypes binding of the C ABI in include/storb_rs.h (libstorb_rs.so).

There is no fallback: if the HIP library is missing, importing this module
raises. Host-only entry points (sizing, generator matrix, parameter checks)
work without a GPU; every compute entry point needs a gfx950 device.

With PyTorch in the same process, import torch before this library is
loaded: PyTorch-ROCm ships its own HIP runtime (torch/lib/libamdhip64.so,
ROCm 7.0) beside the image's /opt/rocm 7.2 one linked here. The two coexist
when torch's is loaded first; the other way round torch finds no GPU
("No HIP GPUs are available"). bench.py, smoke() and tests/conftest.py do so.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
import threading
import weakref
from typing import Optional, Sequence

import numpy as np

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(PKG_DIR, "lib", "libstorb_rs.so")

OK, EINVAL, ENOTENOUGH, EDEVICE, ENOMEM, ENODEV = range(6)
EAGAIN, EBUSY, ECLOSED = 6, 7, 8
KERNEL_AUTO, KERNEL_PERM, KERNEL_LDS = 0, 1, 2


class StorbRsError(RuntimeError):
    def __init__(self, code: int, detail: str = ""):
        self.code = code
        msg = lib().storb_rs_strerror(code).decode()
        super().__init__(f"{msg}{': ' + detail if detail else ''} (code {code})")


def build(jobs: int = 8) -> str:
    """Compile the HIP library in-tree for gfx950 (make -C storb_amd)."""
    subprocess.run(["make", "-s", f"-j{jobs}", "-C", PKG_DIR], check=True)
    return LIB_PATH


_lib = None
_lock = threading.Lock()

u8p = C.POINTER(C.c_uint8)
vp = C.c_void_p
sz = C.c_size_t


class JitStats(C.Structure):
    """storb_rs_jit_stats_t (include/storb_rs.h)."""
    _fields_ = [("compiled", C.c_uint64), ("failed", C.c_uint64), ("pending", C.c_uint64),
                ("launches", C.c_uint64), ("fallbacks", C.c_uint64), ("compile_ms", C.c_double),
                ("evicted", C.c_uint64), ("loaded", C.c_uint64), ("refused", C.c_uint64)]


class CtxStats(C.Structure):
    """storb_rs_ctx_stats_t (include/storb_rs.h)."""
    _fields_ = [("streamed_calls", C.c_uint64), ("stream_fallbacks", C.c_uint64),
                ("sliced_calls", C.c_uint64), ("live_ops", C.c_uint64), ("tables", C.c_uint64),
                ("device_syncs", C.c_uint64), ("caller_node", C.c_int32),
                ("device_node", C.c_int32)]


NOTIFY_FN = C.CFUNCTYPE(None, vp)  # storb_rs_notify_fn


def _declare(L):
    L.storb_rs_version.restype = C.c_char_p
    L.storb_rs_strerror.restype = C.c_char_p
    L.storb_rs_strerror.argtypes = [C.c_int]
    L.storb_rs_device_count.restype = C.c_int
    L.storb_rs_ctx_create.argtypes = [C.c_int, C.POINTER(vp)]
    L.storb_rs_ctx_destroy.argtypes = [vp]
    L.storb_rs_ctx_destroy.restype = None
    L.storb_rs_ctx_device.argtypes = [vp]
    L.storb_rs_last_error.argtypes = [vp]
    L.storb_rs_last_error.restype = C.c_char_p
    L.storb_rs_check_params.argtypes = [C.c_uint32, C.c_uint32]
    L.storb_rs_enc_matrix.argtypes = [C.c_uint32, C.c_uint32, vp]
    L.storb_rs_block_size.argtypes = [C.c_uint32, sz]
    L.storb_rs_block_size.restype = sz
    L.storb_piece_length.argtypes = [C.c_uint64, C.c_uint64, C.c_uint64]
    L.storb_piece_length.restype = C.c_uint64
    L.storb_get_k_and_m.argtypes = [C.c_uint64, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
    L.storb_get_k_and_m.restype = None
    L.storb_rs_encode.argtypes = [vp, C.c_uint32, C.c_uint32, vp, sz, C.POINTER(vp),
                                  C.POINTER(sz), C.POINTER(sz)]
    L.storb_rs_encode_shares.argtypes = [vp, C.c_uint32, C.c_uint32, vp, sz, C.POINTER(vp),
                                         C.POINTER(sz), C.POINTER(sz)]
    L.storb_rs_ctx_stats.argtypes = [vp, C.POINTER(CtxStats)]
    L.storb_rs_device_pool_stats.argtypes = [C.c_int, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
    L.storb_rs_decode.argtypes = [vp, C.c_uint32, C.c_uint32, C.POINTER(vp),
                                  C.POINTER(C.c_uint32), C.c_uint32, sz, sz, vp]
    L.storb_rs_encode_chunks.argtypes = [vp, C.c_uint32, C.c_uint32, vp, sz, C.c_uint32, vp]
    L.storb_rs_encode_chunks_hashed.argtypes = [vp, C.c_uint32, C.c_uint32, vp, sz, C.c_uint32,
                                                vp, vp]
    L.storb_rs_encode_batch_dev.argtypes = [vp, C.c_uint32, C.c_uint32, sz, C.c_uint32,
                                            vp, sz, vp, sz, vp]
    L.storb_rs_decode_batch_dev.argtypes = [vp, C.c_uint32, C.c_uint32, sz, C.c_uint32,
                                            C.POINTER(C.c_uint32), C.c_uint32, vp, sz, vp,
                                            sz, vp, sz, vp]
    L.storb_rs_decode_stripes_dev.argtypes = [vp, C.c_uint32, C.c_uint32, sz, C.c_uint32,
                                              C.POINTER(C.c_uint32), C.POINTER(C.c_uint32), vp,
                                              sz, vp, sz, vp, sz, vp]
    L.storb_rs_repair_batch_dev.argtypes = [vp, C.c_uint32, C.c_uint32, sz, C.c_uint32,
                                            C.POINTER(C.c_uint32), C.c_uint32,
                                            C.POINTER(C.c_uint32), C.c_uint32, vp, sz, vp,
                                            sz, vp]
    L.storb_rs_repair.argtypes = [vp, C.c_uint32, C.c_uint32, C.POINTER(vp),
                                  C.POINTER(C.c_uint32), C.c_uint32, sz,
                                  C.POINTER(C.c_uint32), C.c_uint32, C.POINTER(vp)]
    L.storb_rs_apply_dev.argtypes = [vp, C.c_uint32, C.c_uint32, vp, C.POINTER(vp),
                                     C.POINTER(sz), C.POINTER(vp), C.POINTER(sz), sz,
                                     C.c_uint32, vp]
    L.storb_rs_fill_splitmix_dev.argtypes = [vp, vp, sz, C.c_uint32, sz, C.c_uint64, vp]
    L.storb_blake3.argtypes = [vp, sz, vp]
    L.storb_blake3.restype = None
    L.storb_rs_blake3_batch_dev.argtypes = [vp, vp, sz, C.c_uint32, sz, vp, vp]
    L.storb_rs_device_numa_node.argtypes = [C.c_int]
    L.storb_rs_select_device.argtypes = [C.c_int, C.POINTER(C.c_int), C.c_int, C.c_uint64]
    L.storb_rs_encode_hashed_dev.argtypes = [vp, C.c_uint32, C.c_uint32, sz, C.c_uint32,
                                             vp, sz, vp, sz, vp, vp]
    L.storb_rs_decode_chunks.argtypes = [vp, C.c_uint32, C.c_uint32, sz, sz, C.c_uint32,
                                         C.POINTER(vp), C.POINTER(C.c_uint32),
                                         C.POINTER(C.c_uint32), vp, sz]
    L.storb_rs_host_alloc.argtypes = [sz, C.POINTER(vp)]
    L.storb_rs_host_free.argtypes = [vp]
    L.storb_rs_host_register.argtypes = [vp, sz]
    L.storb_rs_host_unregister.argtypes = [vp]
    L.storb_rs_host_is_pinned.argtypes = [vp, sz]
    L.storb_rs_encode_async.argtypes = [vp, C.c_uint32, C.c_uint32, vp, sz, C.POINTER(vp),
                                        C.POINTER(sz), C.POINTER(sz), NOTIFY_FN, vp,
                                        C.POINTER(vp)]
    L.storb_rs_decode_async.argtypes = [vp, C.c_uint32, C.c_uint32, C.POINTER(vp),
                                        C.POINTER(C.c_uint32), C.c_uint32, sz, sz, vp,
                                        NOTIFY_FN, vp, C.POINTER(vp)]
    L.storb_rs_op_test.argtypes = [vp]
    L.storb_rs_op_finish.argtypes = [vp]
    L.storb_rs_notify_fd.argtypes = [vp]
    L.storb_rs_notify_fd.restype = None
    L.storb_rs_set_kernel.argtypes = [vp, C.c_int]
    L.storb_rs_sync.argtypes = [vp]
    L.storb_rs_jit_stats.argtypes = [C.POINTER(JitStats)]
    L.storb_rs_code_object_calls.argtypes = [vp, sz, C.c_char_p, sz]
    L.storb_rs_jit_wait.argtypes = []
    L.storb_rs_jit_prepare_decode.argtypes = [C.c_uint32, C.c_uint32, C.POINTER(C.c_uint32),
                                              C.c_uint32, C.c_int, C.c_int]


def lib():
    global _lib
    if _lib is None:
        with _lock:
            if _lib is None:
                if not os.path.exists(LIB_PATH):
                    raise ImportError(
                        f"{LIB_PATH} is missing: the MI355X library must be built "
                        "(python -c 'import __graft_entry__ as g; g.build()'); there is "
                        "no CPU fallback")
                L = C.CDLL(LIB_PATH)
                _declare(L)
                _lib = L
    return _lib


# ------------------------------------------------------------ host-only
def version() -> str:
    return lib().storb_rs_version().decode()


def device_count() -> int:
    return int(lib().storb_rs_device_count())


def device_numa_node(device: int) -> int:
    """NUMA node of the socket GPU `device` hangs off (-1 unknown)."""
    return lib().storb_rs_device_numa_node(device)


def select_device(caller_node: int, device_nodes: Sequence[int], ticket: int) -> int:
    """The device storb_rs_ctx_create(-1) gives the ticket-th context of a
    thread on NUMA node caller_node, for any topology (no device access)."""
    arr = (C.c_int * max(1, len(device_nodes)))(*device_nodes)
    return lib().storb_rs_select_device(caller_node, arr, len(device_nodes), ticket)


def device_pool_stats(device: int = 0) -> tuple[int, int]:
    """(used, reserved) bytes of the device's default stream-ordered pool."""
    u, r = C.c_uint64(), C.c_uint64()
    rc = lib().storb_rs_device_pool_stats(device, C.byref(u), C.byref(r))
    if rc != OK:
        raise StorbRsError(rc, "storb_rs_device_pool_stats")
    return int(u.value), int(r.value)


def check_params(k: int, n: int) -> bool:
    if not (0 <= k < 2**32 and 0 <= n < 2**32):
        return False
    return lib().storb_rs_check_params(k, n) == OK


def enc_matrix(k: int, n: int) -> np.ndarray:
    out = np.zeros(n * k, dtype=np.uint8)
    rc = lib().storb_rs_enc_matrix(k, n, out.ctypes.data)
    if rc != OK:
        raise StorbRsError(rc, f"(k={k}, n={n})")
    return out.reshape(n, k)


def block_size(k: int, length: int) -> int:
    return int(lib().storb_rs_block_size(k, length))


def piece_length(content_length: int, min_size: int = 0, max_size: int = 0) -> int:
    return int(lib().storb_piece_length(content_length, min_size, max_size))


def get_k_and_m(chunk_size: int) -> tuple[int, int]:
    k, m = C.c_uint64(), C.c_uint64()
    lib().storb_get_k_and_m(chunk_size, C.byref(k), C.byref(m))
    return int(k.value), int(m.value)


def blake3(data) -> bytes:
    """Host BLAKE3 digest (32 bytes) -- Storb's shard identity."""
    buf = _as_u8(data)
    out = np.zeros(32, dtype=np.uint8)
    lib().storb_blake3(buf.ctypes.data if buf.size else None, buf.size, out.ctypes.data)
    return out.tobytes()


def _as_u8(data) -> np.ndarray:
    if isinstance(data, np.ndarray):
        return np.ascontiguousarray(data, dtype=np.uint8).reshape(-1)
    if isinstance(data, memoryview) and data.contiguous:
        return np.frombuffer(data.cast("B"), dtype=np.uint8)  # zero-copy view
    return np.frombuffer(bytes(data), dtype=np.uint8)


def marshal_chunks(chunks, block: int):
    """chunks[c] = (shares, idx) -> (ptrs uint64, idx uint32, cnt uint32, keep):
    the arrays storb_rs_decode_chunks takes (Context.decode_chunks_raw).
    `keep` holds the share arrays the pointers point into; keep it alive."""
    keep, ptrs, idx, cnt = [], [], [], []
    for shares, ids in chunks:
        assert len(shares) == len(ids)
        cnt.append(len(ids))
        idx.extend(int(i) for i in ids)
        for sh in shares:
            a = sh if (type(sh) is np.ndarray and sh.dtype == np.uint8 and sh.flags.c_contiguous
                       ) else _as_u8(sh)
            assert a.nbytes >= block
            keep.append(a)
            ptrs.append(a.__array_interface__["data"][0])
    return (np.array(ptrs, dtype=np.uint64), np.array(idx, dtype=np.uint32),
            np.array(cnt, dtype=np.uint32), keep)


def jit_stats() -> dict:
    """Counters of the run-time-compiled bit-sliced kernels (rs_jit.cpp)."""
    st = JitStats()
    rc = lib().storb_rs_jit_stats(C.byref(st))
    if rc != OK:
        raise StorbRsError(rc, "storb_rs_jit_stats")
    return {f: getattr(st, f) for f, _ in JitStats._fields_}


def code_object_calls(code: bytes) -> tuple[int, str]:
    """storb_rs_code_object_calls: (1 call / 0 none / -1 unreadable, why)."""
    why = C.create_string_buffer(512)
    buf = C.create_string_buffer(bytes(code), len(code))
    r = lib().storb_rs_code_object_calls(buf, len(code), why, 512)
    return r, why.value.decode()


def jit_wait():
    """Block until no kernel compile is pending."""
    lib().storb_rs_jit_wait()


def jit_prepare_decode(k: int, n: int, share_idx: Sequence[int], assemble: bool = False,
                       wait: bool = True):
    """Compile (or queue) the decode kernel of one erasure pattern ahead of
    the calls that need it; no GPU needed."""
    ids = (C.c_uint32 * max(len(share_idx), 1))(*share_idx)
    rc = lib().storb_rs_jit_prepare_decode(k, n, ids, len(share_idx), int(assemble), int(wait))
    if rc != OK:
        raise StorbRsError(rc, "storb_rs_jit_prepare_decode")


class PinnedBuffer:
    """Page-locked host bytes from storb_rs_host_alloc, viewed as a numpy
    array. storb_rs_encode_chunks DMAs such buffers in place."""

    def __init__(self, nbytes: int):
        p = vp()
        rc = lib().storb_rs_host_alloc(nbytes, C.byref(p))
        if rc != OK:
            raise StorbRsError(rc, "storb_rs_host_alloc")
        self._p = p
        self.nbytes = nbytes
        self.array = np.ctypeslib.as_array(C.cast(p, C.POINTER(C.c_uint8)), shape=(nbytes,))

    def free(self):
        if getattr(self, "_p", None):
            self.array = None
            lib().storb_rs_host_free(self._p)
            self._p = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def host_is_pinned(arr: np.ndarray) -> bool:
    return bool(lib().storb_rs_host_is_pinned(arr.ctypes.data, arr.nbytes))


class Context:
    """One storb_rs_ctx: a GPU, its streams, staging and table caches."""

    def __init__(self, device: int = -1):
        h = vp()
        rc = lib().storb_rs_ctx_create(device, C.byref(h))
        if rc != OK:
            raise StorbRsError(rc, "storb_rs_ctx_create")
        self._h = h
        # Async ops started here and not finished: close() detaches them
        # (storb_rs_ctx_destroy waits for their device work; finish() then
        # raises ECLOSED instead of touching the destroyed context).
        self._ops = weakref.WeakSet()
        # hipStream_t used when a call passes stream=None. None here means
        # NULL at the ABI: the HIP null stream, which orders with torch's
        # default stream and which sync() waits for. Tests point it at
        # torch's current stream.
        self.default_stream: Optional[int] = None

    def _s(self, stream):
        return self.default_stream if stream is None else stream

    @property
    def handle(self):
        return self._h

    @property
    def device(self) -> int:
        return int(lib().storb_rs_ctx_device(self._h))

    def close(self):
        """Destroy the context. Unfinished AsyncOps of it are waited for and
        detached: their finish() / test() raise StorbRsError(ECLOSED)."""
        if getattr(self, "_h", None):
            lib().storb_rs_ctx_destroy(self._h)
            self._h = None
            for op in list(getattr(self, "_ops", ())):
                op._ctx_closed = True

    @property
    def closed(self) -> bool:
        return not getattr(self, "_h", None)

    def stats(self) -> dict:
        """storb_rs_ctx_stats: single-call path counters, live async ops, tables."""
        st = CtxStats()
        self._check(lib().storb_rs_ctx_stats(self._h, C.byref(st)), "storb_rs_ctx_stats")
        return {f: getattr(st, f) for f, _ in CtxStats._fields_}

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc: int, what: str):
        if rc != OK:
            detail = lib().storb_rs_last_error(self._h).decode()
            raise StorbRsError(rc, f"{what}: {detail}" if detail else what)

    # ---------------------------------------------------- host buffers
    def encode(self, k: int, n: int, data) -> tuple[list[bytes], int, int]:
        buf = _as_u8(data)
        B = block_size(k, buf.size) if k else 0
        p = max(n - k, 0)
        outs = [np.zeros(max(B, 1), dtype=np.uint8) for _ in range(p)]
        ptrs = (vp * max(p, 1))(*[o.ctypes.data for o in outs])
        b, pad = sz(), sz()
        rc = lib().storb_rs_encode(self._h, k, n, buf.ctypes.data if buf.size else None,
                                   buf.size, ptrs, C.byref(b), C.byref(pad))
        self._check(rc, "storb_rs_encode")
        return [o[: b.value].tobytes() for o in outs], int(b.value), int(pad.value)

    def encode_shares(self, k: int, n: int, data, shares: Optional[Sequence[np.ndarray]] = None):
        """storb_rs_encode_shares: all n shares (data shares zero-padded, then
        parity), zfec-rs Fec::encode's result. shares: optional caller-owned
        arrays (n of >= B bytes). Returns (shares, B, padlen)."""
        buf = _as_u8(data)
        B = block_size(k, buf.size) if k else 0
        outs = list(shares) if shares is not None else \
            [np.empty(max(B, 1), dtype=np.uint8) for _ in range(max(n, 0))]
        assert len(outs) == n
        ptrs = (vp * max(n, 1))(*[o.ctypes.data for o in outs])
        b, pad = sz(), sz()
        rc = lib().storb_rs_encode_shares(self._h, k, n, buf.ctypes.data if buf.size else None,
                                          buf.size, ptrs, C.byref(b), C.byref(pad))
        self._check(rc, "storb_rs_encode_shares")
        return [o[: b.value] for o in outs], int(b.value), int(pad.value)

    def decode(self, k: int, n: int, shares: Sequence, idx: Sequence[int], block: int,
               padlen: int) -> bytes:
        arrs = [_as_u8(s) for s in shares]
        ptrs = (vp * max(len(arrs), 1))(*[a.ctypes.data for a in arrs])
        ids = (C.c_uint32 * max(len(idx), 1))(*idx)
        outlen = max(k * block - padlen, 0)
        out = np.zeros(max(outlen, 1), dtype=np.uint8)
        rc = lib().storb_rs_decode(self._h, k, n, ptrs, ids, len(arrs), block, padlen,
                                   out.ctypes.data)
        self._check(rc, "storb_rs_decode")
        return out[:outlen].tobytes()

    def encode_into(self, k: int, n: int, data: np.ndarray, parity: Sequence[np.ndarray]):
        """storb_rs_encode into caller-owned parity buffers (n-k arrays of >=
        B bytes; page-locked ones are written in place by the kernel)."""
        buf = _as_u8(data)
        assert len(parity) == n - k
        ptrs = (vp * max(n - k, 1))(*[p.ctypes.data for p in parity])
        b, pad = sz(), sz()
        rc = lib().storb_rs_encode(self._h, k, n, buf.ctypes.data, buf.size, ptrs,
                                   C.byref(b), C.byref(pad))
        self._check(rc, "storb_rs_encode")
        return int(b.value), int(pad.value)

    def decode_into(self, k: int, n: int, shares: Sequence[np.ndarray], idx: Sequence[int],
                    block: int, padlen: int, out: np.ndarray):
        """storb_rs_decode into a caller-owned buffer of k*block - padlen bytes."""
        assert out.dtype == np.uint8 and out.flags.c_contiguous
        assert out.size >= k * block - padlen
        ptrs = (vp * max(len(shares), 1))(*[a.ctypes.data for a in shares])
        ids = (C.c_uint32 * max(len(idx), 1))(*idx)
        rc = lib().storb_rs_decode(self._h, k, n, ptrs, ids, len(shares), block, padlen,
                                   out.ctypes.data)
        self._check(rc, "storb_rs_decode")

    # ------------------------------------------------ asynchronous calls
    def encode_async(self, k: int, n: int, data, notify=None, parity=None) -> "AsyncOp":
        """storb_rs_encode_async: returns at once with an AsyncOp; `data` may be
        reused immediately. op.finish() -> (parity shares, B, padlen).
        parity: optional caller-owned output arrays (n-k of >= B bytes;
        page-locked ones are written in place by the kernel)."""
        buf = _as_u8(data)
        B = block_size(k, buf.size) if k else 0
        p = max(n - k, 0)
        outs = list(parity) if parity is not None else \
            [np.zeros(max(B, 1), dtype=np.uint8) for _ in range(p)]
        ptrs = (vp * max(p, 1))(*[o.ctypes.data for o in outs])
        b, pad = sz(), sz()
        op = AsyncOp(self, notify)
        rc = lib().storb_rs_encode_async(self._h, k, n, buf.ctypes.data if buf.size else None,
                                         buf.size, ptrs, C.byref(b), C.byref(pad), op._cb,
                                         op._user, C.byref(op._h))
        if rc != OK:
            op._abandon()  # no op was created
        self._check(rc, "storb_rs_encode_async")
        op._keep = outs
        op._result = lambda: ([o[: b.value].tobytes() for o in outs], int(b.value),
                              int(pad.value))
        op._started()
        return op

    def decode_async(self, k: int, n: int, shares: Sequence, idx: Sequence[int], block: int,
                     padlen: int, notify=None) -> "AsyncOp":
        """storb_rs_decode_async; op.finish() -> the chunk bytes."""
        arrs = [_as_u8(s) for s in shares]
        ptrs = (vp * max(len(arrs), 1))(*[a.ctypes.data for a in arrs])
        ids = (C.c_uint32 * max(len(idx), 1))(*idx)
        outlen = max(k * block - padlen, 0)
        out = np.zeros(max(outlen, 1), dtype=np.uint8)
        op = AsyncOp(self, notify)
        rc = lib().storb_rs_decode_async(self._h, k, n, ptrs, ids, len(arrs), block, padlen,
                                         out.ctypes.data, op._cb, op._user, C.byref(op._h))
        if rc != OK:
            op._abandon()  # no op was created
        self._check(rc, "storb_rs_decode_async")
        op._keep = out
        op._result = lambda: out[:outlen].tobytes()
        op._started()
        return op

    def repair(self, k: int, n: int, shares: Sequence, idx: Sequence[int], block: int,
               targets: Sequence[int]) -> list[bytes]:
        """Regenerate shares `targets` (data or parity) of one stripe from the
        first k of the given shares by index (decode-based repair)."""
        arrs = [_as_u8(s) for s in shares]
        ptrs = (vp * max(len(arrs), 1))(*[a.ctypes.data for a in arrs])
        ids = (C.c_uint32 * max(len(idx), 1))(*idx)
        outs = [np.zeros(max(block, 1), dtype=np.uint8) for _ in targets]
        optr = (vp * max(len(outs), 1))(*[o.ctypes.data for o in outs])
        tg = (C.c_uint32 * max(len(targets), 1))(*targets)
        rc = lib().storb_rs_repair(self._h, k, n, ptrs, ids, len(arrs), block, tg,
                                   len(targets), optr)
        self._check(rc, "storb_rs_repair")
        return [o[:block].tobytes() for o in outs]

    def encode_chunks(self, k: int, n: int, data: np.ndarray, chunk_len: int,
                      nchunks: int, out: Optional[np.ndarray] = None) -> np.ndarray:
        buf = _as_u8(data)
        assert buf.size >= chunk_len * nchunks
        B = block_size(k, chunk_len)
        if out is None:
            out = np.empty(nchunks * (n - k) * B, dtype=np.uint8)
        assert out.dtype == np.uint8 and out.flags.c_contiguous
        assert out.size >= nchunks * (n - k) * B
        rc = lib().storb_rs_encode_chunks(self._h, k, n, buf.ctypes.data, chunk_len,
                                          nchunks, out.ctypes.data)
        self._check(rc, "storb_rs_encode_chunks")
        return out

    def encode_chunks_hashed(self, k: int, n: int, data: np.ndarray, chunk_len: int,
                             nchunks: int, out: Optional[np.ndarray] = None,
                             hashes: Optional[np.ndarray] = None):
        """(parity [nchunks*(n-k)*B], digests [nchunks, n, 32]) -- piece ids
        computed on the GPU. `out` / `hashes` reuse caller buffers."""
        buf = _as_u8(data)
        assert buf.size >= chunk_len * nchunks
        B = block_size(k, chunk_len)
        par = out if out is not None else np.empty(max(1, nchunks * (n - k) * B), np.uint8)
        assert par.dtype == np.uint8 and par.flags.c_contiguous
        assert par.size >= nchunks * (n - k) * B
        if hashes is None:
            hashes = np.empty((nchunks, n, 32), dtype=np.uint8)
        assert hashes.dtype == np.uint8 and hashes.flags.c_contiguous
        assert hashes.size >= nchunks * n * 32
        rc = lib().storb_rs_encode_chunks_hashed(self._h, k, n, buf.ctypes.data, chunk_len,
                                                 nchunks, par.ctypes.data, hashes.ctypes.data)
        self._check(rc, "storb_rs_encode_chunks_hashed")
        return par[:nchunks * (n - k) * B], hashes

    def decode_chunks(self, k: int, n: int, block: int, padlen: int, chunks,
                      out: Optional[np.ndarray] = None,
                      out_stride: Optional[int] = None) -> np.ndarray:
        """Batch of download-side reconstructions: chunks[c] = (shares, idx),
        shares[i] (block bytes) being share idx[i] of chunk c. Returns
        [nchunks, k*block - padlen] (decode_chunk per chunk, piece.rs:363-387).
        out_stride: bytes between chunks in `out` (default: packed)."""
        nch = len(chunks)
        outlen = k * block - padlen
        stride = outlen if out_stride is None else int(out_stride)
        assert stride >= outlen
        if out is None:
            out = np.empty(max(1, (nch - 1) * stride + outlen), dtype=np.uint8)
        assert out.dtype == np.uint8 and out.flags.c_contiguous
        assert out.size >= (nch - 1) * stride + outlen if nch else True
        ptrs, idx, cnt, keep = marshal_chunks(chunks, block)
        self.decode_chunks_raw(k, n, block, padlen, ptrs, idx, cnt, out, stride)
        del keep
        flat = out.reshape(-1)
        if stride == outlen:
            return flat[:nch * outlen].reshape(nch, outlen)
        return np.lib.stride_tricks.as_strided(flat, shape=(nch, outlen), strides=(stride, 1))

    def decode_chunks_raw(self, k: int, n: int, block: int, padlen: int, ptrs: np.ndarray,
                          idx: np.ndarray, cnt: np.ndarray, out: np.ndarray,
                          out_stride: Optional[int] = None) -> None:
        """decode_chunks with the shares already marshalled (marshal_chunks):
        ptrs (uint64 host addresses, chunk after chunk), idx (uint32 share
        indices in the same order), cnt (uint32 shares per chunk) -- the
        arrays a compiled binding hands storb_rs_decode_chunks directly
        (INTEGRATION.md). The caller keeps the shares alive. Timing this call
        times the library: decode_chunks' per-share Python loop costs ~2-5 ms
        per 1,024 shares, a third of a 256 MiB batch."""
        nch = int(cnt.size)
        outlen = k * block - padlen
        stride = outlen if out_stride is None else int(out_stride)
        assert stride >= outlen
        assert ptrs.dtype == np.uint64 and idx.dtype == np.uint32 and cnt.dtype == np.uint32
        assert ptrs.flags.c_contiguous and idx.flags.c_contiguous and cnt.flags.c_contiguous
        assert ptrs.size == idx.size == int(cnt.sum())
        assert out.dtype == np.uint8 and out.flags.c_contiguous
        assert out.size >= (nch - 1) * stride + outlen if nch else True
        rc = lib().storb_rs_decode_chunks(
            self._h, k, n, block, padlen, nch, C.cast(ptrs.ctypes.data, C.POINTER(vp)),
            C.cast(idx.ctypes.data, C.POINTER(C.c_uint32)),
            C.cast(cnt.ctypes.data, C.POINTER(C.c_uint32)), out.ctypes.data, stride)
        self._check(rc, "storb_rs_decode_chunks")

    # --------------------------------------------------- device buffers
    def encode_batch_dev(self, k: int, n: int, block: int, nstripes: int, d_data: int,
                         d_parity: int, data_stride: int = 0, parity_stride: int = 0,
                         stream: Optional[int] = None):
        rc = lib().storb_rs_encode_batch_dev(self._h, k, n, block, nstripes, d_data,
                                             data_stride, d_parity, parity_stride, self._s(stream))
        self._check(rc, "storb_rs_encode_batch_dev")

    def decode_batch_dev(self, k: int, n: int, block: int, nstripes: int,
                         share_idx: Sequence[int], d_data: int, d_parity: int, d_out: int,
                         data_stride: int = 0, parity_stride: int = 0, out_stride: int = 0,
                         stream: Optional[int] = None):
        ids = (C.c_uint32 * max(len(share_idx), 1))(*share_idx)
        rc = lib().storb_rs_decode_batch_dev(self._h, k, n, block, nstripes, ids,
                                             len(share_idx), d_data, data_stride, d_parity,
                                             parity_stride, d_out, out_stride, self._s(stream))
        self._check(rc, "storb_rs_decode_batch_dev")

    def decode_stripes_dev(self, k: int, n: int, block: int, share_idx: Sequence[Sequence[int]],
                           d_data: int, d_parity: int, d_out: int, data_stride: int = 0,
                           parity_stride: int = 0, out_stride: int = 0,
                           stream: Optional[int] = None):
        """storb_rs_decode_stripes_dev: share_idx[s] lists the shares stripe s
        offers (any order, >= k; its first k by index are used)."""
        ids, cnt = encode_stripe_shares(share_idx)
        self.decode_stripes_dev_raw(k, n, block, len(share_idx), ids, cnt, d_data, d_parity, d_out,
                                    data_stride, parity_stride, out_stride, stream)

    def decode_stripes_dev_raw(self, k: int, n: int, block: int, nstripes: int, ids, cnt,
                               d_data: int, d_parity: int, d_out: int, data_stride: int = 0,
                               parity_stride: int = 0, out_stride: int = 0,
                               stream: Optional[int] = None):
        """The same with prebuilt ctypes arrays (encode_stripe_shares), for
        callers that replay one set of patterns (benchmarks)."""
        rc = lib().storb_rs_decode_stripes_dev(self._h, k, n, block, nstripes, ids, cnt, d_data,
                                               data_stride, d_parity, parity_stride, d_out,
                                               out_stride, self._s(stream))
        self._check(rc, "storb_rs_decode_stripes_dev")

    def repair_batch_dev(self, k: int, n: int, block: int, nstripes: int,
                         share_idx: Sequence[int], targets: Sequence[int], d_data: int,
                         d_parity: int, data_stride: int = 0, parity_stride: int = 0,
                         stream: Optional[int] = None):
        ids = (C.c_uint32 * max(len(share_idx), 1))(*share_idx)
        tg = (C.c_uint32 * max(len(targets), 1))(*targets)
        rc = lib().storb_rs_repair_batch_dev(self._h, k, n, block, nstripes, ids,
                                             len(share_idx), tg, len(targets), d_data,
                                             data_stride, d_parity, parity_stride,
                                             self._s(stream))
        self._check(rc, "storb_rs_repair_batch_dev")

    def apply_dev(self, coef: np.ndarray, d_in: Sequence[int], in_stride: Sequence[int],
                  d_out: Sequence[int], out_stride: Sequence[int], block: int,
                  nstripes: int, stream: Optional[int] = None):
        coef = np.ascontiguousarray(coef, dtype=np.uint8)
        rows, k = coef.shape
        ins = (vp * k)(*d_in)
        inst = (sz * k)(*in_stride)
        outs = (vp * rows)(*d_out)
        outst = (sz * rows)(*out_stride)
        rc = lib().storb_rs_apply_dev(self._h, k, rows, coef.ctypes.data, ins, inst, outs,
                                      outst, block, nstripes, self._s(stream))
        self._check(rc, "storb_rs_apply_dev")

    def fill_splitmix_dev(self, d: int, obj_len: int, nobj: int, obj_stride: int = 0,
                          seed_base: int = 0, stream: Optional[int] = None):
        rc = lib().storb_rs_fill_splitmix_dev(self._h, d, obj_len, nobj, obj_stride,
                                              seed_base, self._s(stream))
        self._check(rc, "storb_rs_fill_splitmix_dev")

    def blake3_batch_dev(self, d_in: int, length: int, count: int, stride: int, d_out: int,
                         stream: Optional[int] = None):
        rc = lib().storb_rs_blake3_batch_dev(self._h, d_in, length, count, stride, d_out,
                                             self._s(stream))
        self._check(rc, "storb_rs_blake3_batch_dev")

    def encode_hashed_dev(self, k: int, n: int, block: int, nstripes: int, d_data: int,
                          d_parity: int, d_hashes: int, data_stride: int = 0,
                          parity_stride: int = 0, stream: Optional[int] = None):
        """Encode plus the blake3 piece id of every share: digest of share t of
        stripe s at d_hashes + (s*n + t)*32 (storb_rs_encode_hashed_dev)."""
        rc = lib().storb_rs_encode_hashed_dev(self._h, k, n, block, nstripes, d_data,
                                              data_stride, d_parity, parity_stride, d_hashes,
                                              self._s(stream))
        self._check(rc, "storb_rs_encode_hashed_dev")

    def set_kernel(self, variant: int):
        self._check(lib().storb_rs_set_kernel(self._h, variant), "storb_rs_set_kernel")

    def sync(self):
        self._check(lib().storb_rs_sync(self._h), "storb_rs_sync")


def encode_stripe_shares(share_idx: Sequence[Sequence[int]]):
    """(share_idx, nshares) ctypes arrays of storb_rs_decode_stripes_dev /
    storb_rs_decode_chunks: all stripes' share lists back to back + counts."""
    flat = [int(i) for ids in share_idx for i in ids]
    ids = (C.c_uint32 * max(1, len(flat)))(*flat)
    cnt = (C.c_uint32 * max(1, len(share_idx)))(*[len(x) for x in share_idx])
    return ids, cnt


_tls = threading.local()


class _Notifier:
    """One daemon thread that runs the Python `notify` callables of async ops.

    The C library wakes it without Python: an op's notify function is
    storb_rs_notify_fd (a C function, never garbage-collected), which writes
    to the op's eventfd from the HIP runtime thread. Nothing runs Python or
    takes the GIL on that thread; this thread polls the eventfds and calls
    the callables."""

    def __init__(self):
        import selectors
        self._sel = selectors.DefaultSelector()
        self._lock = threading.Lock()
        self._wake = os.eventfd(0, os.EFD_NONBLOCK | os.EFD_CLOEXEC)
        self._sel.register(self._wake, selectors.EVENT_READ, None)
        self._pending = []
        threading.Thread(target=self._run, name="storb_rs_notify", daemon=True).start()

    def watch(self, fd: int, op: "AsyncOp"):
        with self._lock:
            self._pending.append((fd, op))
        os.eventfd_write(self._wake, 1)

    def _run(self):
        import selectors
        while True:
            for key, _ in self._sel.select():
                if key.data is None:
                    try:
                        os.eventfd_read(self._wake)
                    except BlockingIOError:
                        pass
                    with self._lock:
                        todo, self._pending = self._pending, []
                    for fd, op in todo:
                        self._sel.register(fd, selectors.EVENT_READ, op)
                    continue
                self._sel.unregister(key.fd)
                os.close(key.fd)  # written once, by the op's notification
                key.data._fd = None
                key.data._fire()


_notifier: Optional[_Notifier] = None
_notifier_lock = threading.Lock()


def _get_notifier() -> _Notifier:
    global _notifier
    with _notifier_lock:
        if _notifier is None:
            _notifier = _Notifier()
        return _notifier


class _OpState:
    """What an AsyncOp's finalizer needs without the op: the C handle and
    whether finish() ran (an op dropped unfinished is finished here, so its
    staging slot is given back)."""

    def __init__(self):
        self.h = vp()
        self.done = False

    def finish_if_pending(self):
        if not self.done and self.h:
            self.done = True
            lib().storb_rs_op_finish(self.h)


class AsyncOp:
    """An in-flight storb_rs_*_async call: test() polls, finish() waits, writes
    the outputs and returns the call's result (exactly once). `notify` (a
    Python callable, optional) runs once when the device work is done: on the
    notifier thread (woken through an eventfd by storb_rs_notify_fd), or in
    the calling thread when the op needed no device work; always before
    finish() returns."""

    EAGAIN = 6

    def __init__(self, ctx: Context, notify=None):
        self._ctx = ctx  # keeps the context alive until finish
        self._ctx_closed = False  # set by ctx.close() while this op is unfinished
        ctx._ops.add(self)
        self._st = _OpState()
        self._h = self._st.h
        self._keep = None
        self._result = None
        self._notify = notify
        self._fired = not notify
        self._fire_lock = threading.Lock()
        self._fd = None
        if notify:
            self._fd = os.eventfd(0, os.EFD_NONBLOCK | os.EFD_CLOEXEC)
            fn = C.cast(lib().storb_rs_notify_fd, C.c_void_p).value
            self._cb, self._user = NOTIFY_FN(fn), C.c_void_p(self._fd)
        else:
            self._cb, self._user = C.cast(None, NOTIFY_FN), None
        self._fin = weakref.finalize(self, _OpState.finish_if_pending, self._st)

    def _started(self):
        """After the start call succeeded: hand the eventfd to the notifier
        thread, or notify now if the op is already complete."""
        if self._notify is None:
            return
        # The eventfd is closed only by the notifier thread, once the
        # notification's write has arrived: closing it here when the op
        # already tests done would let a notification that runs after the
        # completion event (nothing in HIP's contract orders a host function
        # before a later event on the stream) write into a closed descriptor
        # whose number the process may have reused.
        if self.test():
            self._fire()
        _get_notifier().watch(self._fd, self)

    def _abandon(self):
        self._st.done = True
        self._fin.detach()
        if self._fd is not None:
            os.close(self._fd)
            self._fd = None

    def _fire(self):
        with self._fire_lock:
            if self._fired:
                return
            self._fired = True
        self._notify()

    def fileno(self) -> int:
        """The eventfd that becomes readable when the device work is done
        (ops created with notify=...)."""
        return -1 if self._fd is None else self._fd

    def test(self) -> bool:
        if self._st.done:
            return True
        rc = lib().storb_rs_op_test(self._h)
        if rc == self.EAGAIN:
            return False
        if rc != OK:
            raise StorbRsError(rc, "storb_rs_op_test")
        return True

    def finish(self):
        if self._st.done:
            raise RuntimeError("op already finished")
        self._st.done = True
        rc = lib().storb_rs_op_finish(self._h)
        self._fin.detach()
        if self._notify is not None:
            self._fire()  # the stream is drained: the device work is done
        if rc != OK:
            raise StorbRsError(rc, "storb_rs_op_finish")
        return self._result()


def thread_context() -> Context:
    """Per-thread context (the Rust shim's OnceLock analogue)."""
    ctx = getattr(_tls, "ctx", None)
    if ctx is None:
        ctx = Context(-1)
        _tls.ctx = ctx
    return ctx
