"""CPU ORACLE (ctypes wrapper of oracle/mppi_oracle.c) — test infrastructure only.

Loaded only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.
Builds ``oracle/_build/liboracle.so`` on first use if it is missing (gcc is on
both the build container and the GPU box).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "liboracle.so")
_lib = None

_dp = np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")
_fp = np.ctypeslib.ndpointer(dtype=np.float32, flags="C_CONTIGUOUS")


def build(force: bool = False) -> str:
    if force or not os.path.exists(LIB_PATH):
        subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        build()
        L = C.CDLL(LIB_PATH)
        L.oracle_rollout_costs_f64.argtypes = [
            _dp, _dp, _fp, C.c_long, C.c_long, C.c_int, C.c_int, C.c_int, _dp, C.c_int, C.c_double,
            C.c_double, C.c_double, _dp, _dp, _dp, C.c_long, C.c_long, _dp, _dp, C.c_int]
        L.oracle_rollout_costs_f64.restype = C.c_int
        L.oracle_weighted_noise_f64.argtypes = [_dp, _fp, C.c_long, C.c_long, C.c_int, C.c_int,
                                                C.c_double, _dp, _dp]
        L.oracle_weighted_noise_f64.restype = C.c_int
        L.oracle_rollout_traj_f64.argtypes = [_dp, _dp, C.c_int, C.c_int, C.c_double, _dp, _dp]
        L.oracle_rollout_traj_f64.restype = C.c_int
        L.oracle_max_threads.restype = C.c_int
        L.oracle_chain_rollout_costs_f64.argtypes = [
            _dp, _dp, _fp, C.c_long, C.c_long, C.c_long, C.c_int, C.c_int, C.c_int, C.c_int, _dp, C.c_int,
            C.c_double, C.c_double, C.c_double, _dp, _dp, _dp, C.c_long, C.c_long, _dp, _dp, C.c_int]
        L.oracle_chain_rollout_costs_f64.restype = C.c_int
        L.oracle_chain_weighted_noise_f64.argtypes = [_dp, _fp, C.c_long, C.c_long, C.c_long, C.c_int, C.c_int,
                                                      C.c_int, C.c_double, _dp, _dp]
        L.oracle_chain_weighted_noise_f64.restype = C.c_int
        L.oracle_chain_traj_f64.argtypes = [_dp, _dp, C.c_int, C.c_int, C.c_int, C.c_double, _dp, _dp]
        L.oracle_chain_traj_f64.restype = C.c_int
        _lib = L
    return _lib


def arm_array(arm) -> np.ndarray:
    return np.array([arm.m1, arm.m2, arm.l1, arm.l2, arm.lc1, arm.lc2, arm.g, arm.fk_l1, arm.fk_l2],
                    dtype=np.float64)


def rollout_costs(x0, u, eps, window, dt, lam, alpha, sigma, stage_w, term_w, arm,
                  k_exploit=None, k_offset=0, layout="KT", k_range=None, nthreads=0):
    """S for samples ``k_range`` (default all).  ``eps`` fp32, (K,T,2) for layout
    "KT" (reference order) or (T,K,2) for "TK" (device order)."""
    eps = np.ascontiguousarray(eps, dtype=np.float32)
    if layout == "KT":
        K, T, _ = eps.shape
        sk, st = T * 2, 2
    else:
        T, K, _ = eps.shape
        sk, st = 2, K * 2
    k0, k1 = (0, K) if k_range is None else k_range
    k_exploit = K if k_exploit is None else k_exploit
    S = np.zeros(k1 - k0)
    win = np.ascontiguousarray(np.asarray(window, dtype=np.float64)[:, :4])  # rows [x, y, dq1, dq2]
    rc = lib().oracle_rollout_costs_f64(
        np.ascontiguousarray(x0, np.float64), np.ascontiguousarray(u, np.float64), eps, sk, st,
        k0, k1, T, win, win.shape[0], dt, lam, alpha,
        np.ascontiguousarray(np.linalg.inv(sigma), np.float64),
        np.ascontiguousarray(stage_w, np.float64), np.ascontiguousarray(term_w, np.float64),
        int(k_exploit), int(k_offset), arm_array(arm), S, int(nthreads))
    if rc != 0:
        raise ValueError("oracle_rollout_costs_f64 failed")
    return S


def weighted_noise(S, eps, lam, layout="KT"):
    eps = np.ascontiguousarray(eps, dtype=np.float32)
    if layout == "KT":
        K, T, _ = eps.shape
        sk, st = T * 2, 2
    else:
        T, K, _ = eps.shape
        sk, st = 2, K * 2
    w = np.zeros(K)
    w_eps = np.zeros(T * 2)
    lib().oracle_weighted_noise_f64(np.ascontiguousarray(S, np.float64), eps, sk, st, K, T, lam, w, w_eps)
    return w, w_eps.reshape(T, 2)


def max_threads() -> int:
    return int(lib().oracle_max_threads())


# ---------------------------------------------------------------- n-link chain

def chain_array(P) -> np.ndarray:
    """ChainParams -> m[n], l[n], lc[n], I[n], fk[n], J[n], b[n], g (chain_oracle.c chain_setup)."""
    return np.concatenate([P.m, P.l, P.lc, P.I, P.fk, P.J, P.b, [P.g]]).astype(np.float64)


def _chain_strides(eps, layout):
    if layout == "KTN":
        K, T, n = eps.shape
        return K, T, n, T * n, n, 1
    if layout == "TKN":                      # the device order [T][K][n]
        T, K, n = eps.shape
        return K, T, n, n, K * n, 1
    T, n, K = eps.shape                      # "TNK": [T][n][K]
    return K, T, n, 1, n * K, K


def chain_rollout_costs(x0, u, eps, window, dt, lam, alpha, sigma, stage_w, term_w, P, k_exploit=None,
                        k_offset=0, layout="KTN", k_range=None, nthreads=0):
    """S of the chain for samples ``k_range`` (default all); eps fp32 (K,T,n) "KTN", (T,K,n) "TKN" (the device's)
    or (T,n,K) "TNK"."""
    eps = np.ascontiguousarray(eps, dtype=np.float32)
    K, T, n, sk, st, sd = _chain_strides(eps, layout)
    k0, k1 = (0, K) if k_range is None else k_range
    k_exploit = K if k_exploit is None else k_exploit
    S = np.zeros(k1 - k0)
    win = np.ascontiguousarray(np.asarray(window, dtype=np.float64)[:, :4])  # rows [x, y, dq1, dq2]
    rc = lib().oracle_chain_rollout_costs_f64(
        np.ascontiguousarray(x0, np.float64), np.ascontiguousarray(u, np.float64), eps, sk, st, sd, k0, k1, T, n,
        win, win.shape[0], dt, lam, alpha, np.ascontiguousarray(np.linalg.inv(sigma), np.float64),
        np.ascontiguousarray(stage_w, np.float64), np.ascontiguousarray(term_w, np.float64), int(k_exploit),
        int(k_offset), chain_array(P), S, int(nthreads))
    if rc != 0:
        raise ValueError("oracle_chain_rollout_costs_f64 failed")
    return S


def chain_weighted_noise(S, eps, lam, layout="KTN"):
    eps = np.ascontiguousarray(eps, dtype=np.float32)
    K, T, n, sk, st, sd = _chain_strides(eps, layout)
    w = np.zeros(K)
    w_eps = np.zeros(T * n)
    lib().oracle_chain_weighted_noise_f64(np.ascontiguousarray(S, np.float64), eps, sk, st, sd, K, T, n, lam, w,
                                          w_eps)
    return w, w_eps.reshape(T, n)


def chain_traj(x0, ctrl, dt, P):
    """States (N, T, 2n) for control rows ctrl (N, T, n)."""
    ctrl = np.ascontiguousarray(ctrl, dtype=np.float64)
    N, T, n = ctrl.shape
    out = np.zeros((N, T, 2 * n))
    lib().oracle_chain_traj_f64(np.ascontiguousarray(x0, np.float64), ctrl, N, T, n, dt, chain_array(P), out)
    return out
