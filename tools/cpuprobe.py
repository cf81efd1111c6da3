import time, sys, os
sys.path.insert(0, os.getcwd())
t=time.time(); sum(range(30_000_000)); print("py_sum_s", round(time.time()-t,3))
import numpy as np
a=np.ones(1<<28,np.uint8); b=np.empty_like(a)
t=time.time(); b[:]=a; print("memcpy_GBps", round(a.nbytes/(time.time()-t)/1e9,2))
from oracle import coracle
d=coracle.splitmix_bytes(1,1<<20)
t=time.perf_counter(); n=0
while time.perf_counter()-t<2:
    coracle.encode(4,6,d); n+=1
print("oracle_encode_MiBps", round(n/(time.perf_counter()-t),1))
print(open("/proc/cpuinfo").read().count("processor"), [l for l in open("/proc/cpuinfo") if "MHz" in l][:3])
import ctypes as C
L = coracle.lib()
sh = np.zeros(6 * (1 << 18), np.uint8); bb = C.c_size_t(); pp = C.c_size_t()
t = time.perf_counter(); n = 0
while time.perf_counter() - t < 2:
    L.zo_encode(4, 6, d.ctypes.data, d.size, sh.ctypes.data, C.byref(bb), C.byref(pp)); n += 1
print("raw_zo_encode_MiBps", round(n / (time.perf_counter() - t), 1))
big = np.concatenate([coracle.splitmix_bytes(i, 1 << 20) for i in range(64)])
t = time.perf_counter()
out = coracle.encode_parity_many(4, 6, big, 1 << 20, 64, threads=1)
print("encode_many_1thr_MiBps", round(64 / (time.perf_counter() - t), 1))
t = time.perf_counter()
for _ in range(200):
    x = np.zeros(1 << 20, np.uint8); x[::4096] = 1
print("fault_1MiB_us", round((time.perf_counter() - t) / 200 * 1e6, 1))
