"""Timing of two or more builds of libmppi_hostrng.so on the drop-in's c3 draw (K = 65536, T = 64: 8.4 M
standard normals, 16 threads), alternating builds.  python tools/hostrng_ab.py LIB_A LIB_B [...]"""
import ctypes as C, numpy as np, time, sys
def load(p):
    L = C.CDLL(os.path.abspath(p))
    f = L.mppi_np_legacy_gauss; f.restype = C.c_int
    f.argtypes = [C.c_void_p, C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_double), C.c_void_p, C.c_int64, C.c_int]
    L.mppi_np_jump_config.restype = C.c_int
    return L
n = 65536 * 64 * 2
import os
out = np.empty(n)
for p in sys.argv[1:] * 2:
    L = load(p)
    print(p, "jump ready", L.mppi_np_jump_config(0))
    np.random.seed(0)
    ts = []
    for r in range(8):
        st = np.random.get_state()
        key = np.array(st[1], dtype=np.uint32); pos = C.c_int(int(st[2])); hg = C.c_int(0); g = C.c_double(0)
        t0 = time.perf_counter()
        rc = L.mppi_np_legacy_gauss(key.ctypes.data, C.byref(pos), C.byref(hg), C.byref(g), out.ctypes.data, n, 16)
        ts.append(time.perf_counter() - t0)
    print(p, "median ms", round(np.median(ts[2:]) * 1e3, 2), [round(t*1e3,1) for t in ts])
