"""The reference's noise draw, ``np.random.multivariate_normal(mu, Sigma, (K, T))`` on the legacy global
RandomState (control.py:154-164), with its standard-normal stream produced by ``csrc/np_legacy_gauss.c``
(threads over NumPy's polar attempts, same values and the same RNG state left behind) and the rest of
multivariate_normal done with NumPy's own calls in NumPy's order.  Small draws, a non-MT19937 global state
or a missing library use NumPy itself, which is the same stream.
"""
from __future__ import annotations

import ctypes as C
import os
import warnings

import numpy as np

_LIB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_lib", "libmppi_hostrng.so")
_MIN_NORMALS = 1 << 15   # below this NumPy's own loop is as fast as the threads' start-up
_lib = None   # loaded on the first large draw (checked again while the file is missing)


def _load():
    global _lib
    if _lib is None and os.path.exists(_LIB):
        lib = C.CDLL(_LIB)
        f = lib.mppi_np_legacy_gauss
        f.restype = C.c_int
        f.argtypes = [C.c_void_p, C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_double), C.c_void_p,
                      C.c_int64, C.c_int]
        _lib = lib
    return _lib


def _threads() -> int:
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    return max(1, min(16, n))


def legacy_standard_normal(n: int) -> np.ndarray | None:
    """n values of np.random.standard_normal(n) from the global state, advancing it as NumPy would; None when
    this path does not apply (the caller then uses NumPy)."""
    if n < _MIN_NORMALS:
        return None
    lib = _load()
    if lib is None:
        return None
    st = np.random.get_state()
    if st[0] != "MT19937":
        return None
    key = np.array(st[1], dtype=np.uint32, copy=True)
    pos, has_gauss, gauss = C.c_int(int(st[2])), C.c_int(int(st[3])), C.c_double(float(st[4]))
    out = np.empty(n, dtype=np.float64)
    rc = lib.mppi_np_legacy_gauss(key.ctypes.data, C.byref(pos), C.byref(has_gauss), C.byref(gauss),
                                  out.ctypes.data, n, _threads())
    if rc != 0:
        return None
    np.random.set_state(("MT19937", key, pos.value, has_gauss.value, gauss.value))
    return out


def multivariate_normal(mean, cov, size) -> np.ndarray:
    """np.random.multivariate_normal(mean, cov, size) (legacy RandomState, check_valid='warn', tol=1e-8):
    the same checks, the same draw, the same transform and the same values."""
    mean = np.array(mean)
    cov = np.array(cov)
    shape = [size] if isinstance(size, (int, np.integer)) else ([] if size is None else list(size))
    if len(mean.shape) != 1 or len(cov.shape) != 2 or cov.shape[0] != cov.shape[1] or mean.shape[0] != cov.shape[0]:
        return np.random.multivariate_normal(mean, cov, size)   # NumPy raises its own error
    final_shape = list(shape[:]) + [mean.shape[0]]
    n = int(np.prod(final_shape))
    z = legacy_standard_normal(n)
    if z is None:
        return np.random.multivariate_normal(mean, cov, size)
    x = z.reshape(-1, mean.shape[0])
    cov = cov.astype(np.double)
    (u, s, v) = np.linalg.svd(cov)
    psd = np.allclose(np.dot(v.T * s, v), cov, rtol=1e-8, atol=1e-8)
    if not psd:
        warnings.warn("covariance is not symmetric positive-semidefinite.", RuntimeWarning)
    x = np.dot(x, np.sqrt(s)[:, None] * v)
    x += mean
    x.shape = tuple(final_shape)
    return x
