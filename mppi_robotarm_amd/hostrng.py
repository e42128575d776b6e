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
        lib.mppi_np_log_params.restype = C.c_int
        lib.mppi_np_log_params.argtypes = [C.c_void_p, C.c_int]
        lib.mppi_np_jump_poly.restype = C.c_int
        lib.mppi_np_jump_poly.argtypes = [C.c_uint64, C.c_void_p]
        lib.mppi_np_poly_words.restype = C.c_int
        lib.mppi_np_log_mismatches.restype = C.c_int64
        lib.mppi_np_log_mismatches.argtypes = [C.c_void_p, C.c_void_p, C.c_int64]
        lib.mppi_np_dot2_fma.restype = None
        lib.mppi_np_dot2_fma.argtypes = [C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p]
        _lib = lib
    return _lib


def log_params():
    """glibc's log constants for the device draw (include/mppi_rocm.h mppi_np_*): NPLOG_NDATA float64 values read
    from this process's libm, accepted only after the C replica of the log (csrc/np_glibc_log.h) matched libm's
    log() on 600k inputs (np_legacy_gauss.c mppi_np_log_params); None when unavailable or mismatched (the
    device draw is then not used).  Cached."""
    global _log_params
    if _log_params is None:
        lib = _load()
        out = np.zeros(274)
        _log_params = out if lib is not None and lib.mppi_np_log_params(out.ctypes.data, 200000) == 0 else False
    return _log_params if _log_params is not False else None


_log_params = None
_jump_cache = {}


def jump_polys(block_stride: int, streams: int) -> np.ndarray | None:
    """x^(624 (block_stride s - 1)) mod P for s = 1 .. streams - 1 as a (streams - 1, 312) uint64 array (the
    MT19937 jump polynomials of the device draw's generator streams; np_legacy_gauss.c mppi_np_jump_poly), or
    None when the jump machinery is unavailable.  Cached per block stride (grown as needed)."""
    lib = _load()
    if lib is None:
        return None
    words = lib.mppi_np_poly_words()
    have = _jump_cache.get(block_stride)
    if have is None or have.shape[0] < streams - 1:
        out = np.zeros((max(streams - 1, 0), words), dtype=np.uint64)
        n0 = 0 if have is None else have.shape[0]
        if n0:
            out[:n0] = have
        for s in range(n0 + 1, streams):
            if lib.mppi_np_jump_poly(624 * (block_stride * s - 1), out[s - 1].ctypes.data) != 0:
                return None
        _jump_cache[block_stride] = have = out
    return have[:streams - 1]


def _threads() -> int:
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    return max(1, min(16, n))


def legacy_standard_normal(n: int, out: np.ndarray | None = None) -> np.ndarray | None:
    """n values of np.random.standard_normal(n) from the global state, advancing it as NumPy would, into `out`
    (a C-contiguous float64 array of at least n values, e.g. page-locked) or a fresh array; None when this path
    does not apply (the caller then uses NumPy; the state is untouched)."""
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
    if out is None:
        out = np.empty(n, dtype=np.float64)
    else:
        if out.dtype != np.float64 or not out.flags.c_contiguous or out.size < n or not out.flags.writeable:
            raise ValueError("out must be a writable C-contiguous float64 array of at least n values")
        out = out.reshape(-1)[:n]
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


_dot2_cache = {}


def dot2_model(m: np.ndarray) -> bool:
    """Whether this process's np.dot rounds an (n, 2) @ (2, 2) float64 product `z @ m` as
    fma(z1, m[1, j], z0 * m[0, j]) (np_legacy_gauss.c mppi_np_dot2_fma) — the operations the device draw applies
    for a general 2 x 2 transform (mppi_npgauss.hip, mppi_np_target.dot2).  The host BLAS picks its kernel at run
    time (CPU type, problem size), so it is pinned here, the way the log constants are: np.dot against the C
    model bit for bit on 4096 and 2^19 rows of standard normals (both sides of OpenBLAS's small-matrix limit,
    M N K = 10^6), and through the same product NumPy's draw makes (a C-contiguous (n, 2) float64 array times
    this m).  Cached per matrix."""
    m = np.ascontiguousarray(m, dtype=np.float64)
    key = m.tobytes()
    hit = _dot2_cache.get(key)
    if hit is None:
        lib = _load()
        hit = False
        if lib is not None and m.shape == (2, 2) and np.all(np.isfinite(m)):
            z = np.random.default_rng(0x5EED).standard_normal(1 << 20).reshape(-1, 2)
            ok = True
            for rows in (4096, 1 << 19):
                zz = np.ascontiguousarray(z[:rows])
                want = np.dot(zz, m)
                got = np.empty_like(want)
                lib.mppi_np_dot2_fma(zz.ctypes.data, rows, m.ctypes.data, got.ctypes.data)
                ok = ok and np.array_equal(want.view(np.uint64), got.view(np.uint64))
            hit = bool(ok)
        _dot2_cache[key] = hit
    return hit


def device_plan(mean, cov):
    """The device draw's transform of multivariate_normal (NumPy's svd of cov and its positive-semidefinite test,
    without the warning): (src, scale, mean, psd, mat) with mat None for a scaled column permutation
    (monomial_plan), or for du = 2 the whole matrix sqrt(s)[:, None] * v when dot2_model pins np.dot's rounding
    of it (src and scale then unused); None otherwise (the host draws)."""
    plan = monomial_plan(mean, cov)
    if plan is not None:
        return plan + (None,)
    mean = np.array(mean)
    cov = np.array(cov)
    if len(mean.shape) != 1 or cov.shape != (2, 2) or mean.shape[0] != 2:
        return None
    cov = cov.astype(np.double)
    (u, s, v) = np.linalg.svd(cov)
    m = np.sqrt(s)[:, None] * v
    if not dot2_model(m):
        return None
    psd = np.allclose(np.dot(v.T * s, v), cov, rtol=1e-8, atol=1e-8)
    return (np.arange(2, dtype=np.int64), np.ones(2), mean.astype(np.float64), bool(psd),
            np.ascontiguousarray(m, dtype=np.float64))


def monomial_plan(mean, cov):
    """monomial_transform without NumPy's positive-semidefinite warning: (src, scale, mean, psd) or None."""
    mean = np.array(mean)
    cov = np.array(cov)
    if len(mean.shape) != 1 or len(cov.shape) != 2 or cov.shape[0] != cov.shape[1] or mean.shape[0] != cov.shape[0]:
        return None
    cov = cov.astype(np.double)
    (u, s, v) = np.linalg.svd(cov)
    m = np.sqrt(s)[:, None] * v
    nz = m != 0
    if not np.all(nz.sum(axis=0) <= 1):   # a zero column (singular cov) is x = mean: z * 0 + mean
        return None
    psd = np.allclose(np.dot(v.T * s, v), cov, rtol=1e-8, atol=1e-8)
    src = np.argmax(nz, axis=0).astype(np.int64)
    return src, m[src, np.arange(m.shape[1])].astype(np.float64), mean.astype(np.float64), bool(psd)


def monomial_transform(mean, cov):
    """multivariate_normal's transform x = z @ (sqrt(s)[:, None] * v) + mean (NumPy's svd of cov, its
    positive-semidefinite check and warning) when that matrix has at most one nonzero per column: then
    x[..., j] = z[..., src[j]] * scale[j] + mean[j] exactly (the other products are exact zeros), so the
    device can apply it to the standard normals.  Returns (src, scale, mean) as float64 / int64 arrays, or None
    for another shape of transform (the caller keeps NumPy's np.dot).  Run.py's Sigma = 20 I and the chain's
    diagonal Sigma are of this kind."""
    plan = monomial_plan(mean, cov)
    if plan is None:
        return None
    if not plan[3]:
        warnings.warn("covariance is not symmetric positive-semidefinite.", RuntimeWarning)
    return plan[:3]


class StdNoise:
    """multivariate_normal(mean, cov, size) left untransformed: the standard normals z (final shape, NumPy's
    values, in the caller's buffer) and the scaled column permutation that makes them the draw.  eps(idx)
    evaluates one element of the draw as the device does."""

    def __init__(self, z: np.ndarray, src: np.ndarray, scale: np.ndarray, mean: np.ndarray):
        self.z, self.src, self.scale, self.mean = z, src, scale, mean

    def eps(self, k: int, t: int, d: int) -> float:
        return float(self.z[k, t, self.src[d]] * self.scale[d] + self.mean[d])


def multivariate_normal_std(mean, cov, size, out: np.ndarray) -> StdNoise | None:
    """np.random.multivariate_normal(mean, cov, size) for a caller that applies the transform itself (on the
    device): when the transform is a scaled column permutation (monomial_transform; NumPy's checks and
    warning included), the standard normals are drawn into `out` (float64, C-contiguous, at least the draw's
    size: e.g. page-locked) exactly as NumPy draws them, and StdNoise is returned; otherwise None and nothing
    is drawn (the caller then takes multivariate_normal).  The global RNG state moves as NumPy's would."""
    mean_a = np.array(mean)
    if len(mean_a.shape) != 1:
        return None
    shape = [size] if isinstance(size, (int, np.integer)) else ([] if size is None else list(size))
    final_shape = tuple(shape) + (mean_a.shape[0],)
    n = int(np.prod(final_shape))
    if n < _MIN_NORMALS or out.size < n:
        return None
    plan = monomial_transform(mean, cov)
    if plan is None:
        return None
    z = legacy_standard_normal(n, out=out)
    if z is None:   # NumPy's own draw of the same standard normals (multivariate_normal's first call)
        z = out.reshape(-1)[:n]
        z[:] = np.random.standard_normal(n)
    return StdNoise(z.reshape(final_shape), *plan)
