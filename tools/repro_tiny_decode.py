import sys, time, faulthandler
sys.path.insert(0, '.')
import numpy as np
from oracle import coracle
from storb_amd import _lib
faulthandler.dump_traceback_later(40, exit=True)
k, n, L = 32, 48, 17
ids_all = [list(range(16, 48)),
           [13, 46, 39, 29, 12, 47, 41, 3, 18, 22, 44, 17, 8, 43, 25, 20, 9, 45, 5, 36, 0, 14, 7, 2, 26, 37, 21, 27, 23, 35, 40, 16, 19, 33],
           [13, 25, 45, 46, 5, 15, 11, 30, 37, 44, 14, 16, 2, 21, 29, 33, 3, 47, 28, 34, 41, 17, 32, 1, 23, 8, 0, 36, 38, 19, 39, 26, 12, 10, 42, 27, 40, 9, 7]]
rng = np.random.default_rng(1)
objs = [rng.integers(0, 256, L, dtype=np.uint8) for _ in ids_all]
ctx = _lib.Context(0)
def run(sel, tag):
    batch, want = [], []
    for c in sel:
        sh, B, pad = coracle.encode(k, n, objs[c])
        batch.append(([sh[i] for i in ids_all[c]], ids_all[c]))
        want.append(objs[c])
    print('start', tag, flush=True)
    t = time.time()
    got = ctx.decode_chunks(k, n, B, pad, batch)
    print('done', tag, round(time.time() - t, 3), all(np.array_equal(g, w) for g, w in zip(got, want)), flush=True)
for c in range(3):
    run([c], f'chunk {c} alone')
run([0, 1, 2], 'all three')
ctx.close()
print('repro ok', flush=True)
