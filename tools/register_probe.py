#!/usr/bin/env python3
"""Does a storb_rs_host_register'd range stay known to HIP after
storb_rs_host_unregister? (Diagnosis of the intermittent illegal-address
faults in torch host->device copies after tests/test_gpu_patterns.py's
registered-buffer test, profiles/r3_fault_notes.md.)

Registers sub-ranges of one numpy allocation exactly as that test does,
decodes from them (zero-copy), unregisters (return codes checked), then asks
the HIP runtime -- without launching anything -- whether the unregistered
addresses, and fresh numpy arrays that reuse the freed address range, are
still host-registered (hipHostGetDevicePointer / hipPointerGetAttributes).
No device work touches the freed memory, so a stale registration shows up as
a report, not as a fault.

usage (GPU box): python tools/register_probe.py
"""
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

from oracle import coracle  # noqa: E402  (checker)
from storb_amd import _lib  # noqa: E402


def hip_runtime():
    for line in open("/proc/self/maps"):
        if "libamdhip64" in line:
            return C.CDLL(line.split()[-1])
    raise SystemExit("libamdhip64 not loaded")


def main():
    torch.zeros(1, device="cuda:0")
    hip = hip_runtime()
    hip.hipHostGetDevicePointer.argtypes = [C.POINTER(C.c_void_p), C.c_void_p, C.c_uint]
    hip.hipPointerGetAttributes.argtypes = [C.c_void_p, C.c_void_p]

    def status(addr):
        d = C.c_void_p()
        e1 = hip.hipHostGetDevicePointer(C.byref(d), C.c_void_p(addr), 0)
        attr = (C.c_ubyte * 128)()
        e2 = hip.hipPointerGetAttributes(attr, C.c_void_p(addr))
        mtype = int.from_bytes(bytes(attr[:4]), "little")
        hip.hipGetLastError()  # the failed queries set HIP's last error; torch checks it
        return {"hipHostGetDevicePointer": e1, "dev": d.value, "hipPointerGetAttributes": e2,
                "memoryType": mtype}

    lib = _lib.lib()
    # device memory torch holds across the register / unregister sequence
    tens = [torch.full((sz,), 7, dtype=torch.uint8, device="cuda:0")
            for sz in (1 << 20, 3 << 20, 8 << 20, 64 << 20, 5 << 20, 2 << 20, 16 << 20)]
    torch.cuda.synchronize()
    c = _lib.Context(0)
    k, n, B, cnt = 4, 6, 64 << 10, 8
    rng = np.random.default_rng(99)
    data = np.frombuffer(rng.bytes(cnt * k * B), np.uint8).copy()
    par = coracle.encode_parity_many(k, n, data, k * B, cnt, threads=4).reshape(cnt, n - k, B)
    span = n * B + 4096
    host = np.zeros(cnt * span + 4096, np.uint8)
    base = (-host.ctypes.data) % 4096
    segs, rcs = [], []
    for ch in range(cnt):
        seg = host[base + ch * span: base + ch * span + n * B]
        seg[:k * B] = data[ch * k * B:(ch + 1) * k * B]
        seg[k * B:] = par[ch].reshape(-1)
        rcs.append(lib.storb_rs_host_register(seg.ctypes.data, seg.nbytes))
        segs.append(seg)
    out_buf = _lib.PinnedBuffer(cnt * k * B)
    out = out_buf.array.reshape(cnt, k * B)
    chunks = [([segs[ch][i * B:(i + 1) * B] for i in range(2, n)], list(range(2, n)))
              for ch in range(cnt)]
    got = c.decode_chunks(k, n, B, 0, chunks, out=out)
    ok = bool(np.array_equal(got.reshape(-1), data))
    addrs = [s.ctypes.data for s in segs]
    registered = [status(a) for a in addrs]
    unreg = [lib.storb_rs_host_unregister(a) for a in addrs]
    after = [status(a) for a in addrs]
    dev_ranges = [(r["dev"], r["dev"] + n * B) for r in registered if r["dev"]]
    tens_after = []
    for t in tens:
        a0, a1 = t.data_ptr(), t.data_ptr() + t.numel()
        st = status(a0)
        tens_after.append({"size": t.numel(), "memoryType": st["memoryType"],
                           "attr_rc": st["hipPointerGetAttributes"],
                           "overlaps_registered_dev_va": any(a0 < h and a1 > l for l, h in dev_ranges)})
    # new torch allocations after the unregistration: mapped? (no kernel reads them yet)
    new_t = [torch.empty(sz, dtype=torch.uint8, device="cuda:0") for sz in (4 << 20, 32 << 20, 3 << 20)]
    new_after = [{"size": t.numel(), **{k2: v for k2, v in status(t.data_ptr()).items()
                                        if k2 in ("memoryType", "hipPointerGetAttributes")},
                  "overlaps_registered_dev_va": any(t.data_ptr() < h and t.data_ptr() + t.numel() > l
                                                    for l, h in dev_ranges)} for t in new_t]
    lo, hi = host.ctypes.data, host.ctypes.data + host.nbytes
    del segs, chunks, seg, host
    out_buf.free()
    c.close()
    # fresh arrays: do any land on the freed range, and do they look registered?
    fresh = []
    keep = []
    host_n = cnt * span + 4096
    for size in (host_n, 2 << 20, 4 << 20, 1 << 20, host_n):
        a = np.ones(size, np.uint8)
        keep.append(a)
        p = a.ctypes.data
        overlap = p < hi and p + size > lo
        fresh.append({"size": size, "overlaps_freed_registered_range": overlap,
                      **status(p), **({"mid": status(p + size // 2)} if overlap else {})})
    print(json.dumps({"register_rc": rcs, "decode_ok": ok, "while_registered": registered[:2],
                      "unregister_rc": unreg, "after_unregister": after,
                      "registered_dev_va": [hex(l) for l, _ in dev_ranges],
                      "torch_tensors_after_unregister": tens_after,
                      "torch_new_tensors": new_after,
                      "torch_tensor_va": [hex(t.data_ptr()) for t in tens + new_t],
                      "fresh_arrays": fresh}, indent=1))


if __name__ == "__main__":
    main()
