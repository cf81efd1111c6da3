"""Time storb_rs_encode_chunks vs storb_rs_encode_chunks_hashed on the same
pageable chunks (one JSON line); run under rocprofv3 --kernel-trace
--memory-copy-trace to see where the hashed path spends its time."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from storb_amd import _lib  # noqa: E402

k, n, L = (int(x) for x in (sys.argv[1:4] if len(sys.argv) > 3 else (4, 6, 1 << 20)))
N = max(8, (256 << 20) // L)
ctx = _lib.Context(0)
host = np.frombuffer(np.random.default_rng(3).bytes(N * L), dtype=np.uint8).copy()
B = -(-L // k)
out = np.zeros(N * (n - k) * B, np.uint8)
ids = np.zeros((N, n, 32), np.uint8)
res = {}
for name, fn in (("plain", lambda: ctx.encode_chunks(k, n, host, L, N, out=out)),
                 ("hashed", lambda: ctx.encode_chunks_hashed(k, n, host, L, N, out=out,
                                                             hashes=ids))):
    fn()
    t0 = time.perf_counter()
    for _ in range(3):
        fn()
    res[name] = round(3 * N * L / (1 << 30) / (time.perf_counter() - t0), 2)
print(json.dumps({"k": k, "n": n, "chunk": L, "chunks": N, "GiBps": res}), flush=True)
