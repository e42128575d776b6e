"""CPU ORACLE — test infrastructure only, never shipped, never on the product path.

Host restatement of the device noise generator (``noise="device"``, SURVEY §8
row f1: the on-device alternative to ``_calc_epsilon``, control.py:154-164,
which is not bit-equal to NumPy's stream by design).  It pins the COUNTER and
INDEX MAPPING of ``philox_noise_kernel`` (mppi_rocm.hip) and
``chain_philox_kernel`` (mppi_chain.hip): which Philox call and which output
word feeds which (t, k, d) element, for any shard offset, odd T and ragged K.

* ``philox4x32_10``: the published Philox4x32-10 (Salmon et al., SC'11,
  "Parallel random numbers: as easy as 1, 2, 3"; Random123's
  ``philox4x32`` with 10 rounds), vectorised over NumPy uint64.  Checked
  against Random123's known-answer vectors in tests/test_philox_ref.py.
* ``box_muller``: z = sqrt(-2 ln u0) (cos 2 pi u1, sin 2 pi u1) with the
  device's fp32 uniforms u0 = (a + 1) 2^-32, u1 = b 2^-32, evaluated in fp64
  (the device uses the fp32 hardware log2 / sqrt / sin / cos: agreement to
  ~1e-6 relative, far below what a wrong mapping would give).
"""
from __future__ import annotations

import numpy as np

M0, M1 = 0xD2511F53, 0xCD9E8D57
W0, W1 = 0x9E3779B9, 0xBB67AE85
MASK = 0xFFFFFFFF


def philox4x32_10(ctr, key):
    """ctr: 4 uint arrays (broadcastable), key: 2 uint arrays -> 4 uint64 arrays of 32-bit words."""
    c0, c1, c2, c3 = (np.asarray(x, dtype=np.uint64) & MASK for x in ctr)
    k0, k1 = (np.asarray(x, dtype=np.uint64) & MASK for x in key)
    for _ in range(10):
        p0 = c0 * np.uint64(M0)
        p1 = c2 * np.uint64(M1)
        hi0, lo0 = p0 >> np.uint64(32), p0 & np.uint64(MASK)
        hi1, lo1 = p1 >> np.uint64(32), p1 & np.uint64(MASK)
        c0, c1, c2, c3 = hi1 ^ c1 ^ k0, lo1, hi0 ^ c3 ^ k1, lo0
        k0 = (k0 + np.uint64(W0)) & np.uint64(MASK)
        k1 = (k1 + np.uint64(W1)) & np.uint64(MASK)
    return c0, c1, c2, c3


def box_muller(a, b):
    inv = np.float32(2.3283064365386963e-10)   # 2^-32, as the device
    u0 = np.minimum((a.astype(np.float32) + np.float32(1.0)) * inv, np.float32(1.0)).astype(np.float64)
    u1 = (b.astype(np.float32) * inv).astype(np.float64)
    r = np.sqrt(-2.0 * np.log(u0))
    return r * np.cos(2.0 * np.pi * u1), r * np.sin(2.0 * np.pi * u1)


def _key(seed, step):
    return (seed & MASK, ((seed >> 32) ^ (step >> 32)) & MASK)


def arm_noise(K_local, T, k_offset, seed, step, sigma):
    """philox_noise_kernel: eps[t][k][2] (device layout, fp64) of the 2-link arm.
    One Philox call per (global k, step pair t0 = 2i): words (x, y) -> step t0,
    (z, w) -> step t0 + 1; eps = L z with L = chol of Sigma's symmetric part."""
    S = np.asarray(sigma, dtype=np.float64)
    s01 = 0.5 * (S[0, 1] + S[1, 0])
    L00 = np.sqrt(S[0, 0])
    L10 = s01 / L00
    L11 = np.sqrt(S[1, 1] - L10 * L10)
    kg = np.arange(K_local, dtype=np.uint64) + np.uint64(k_offset)
    out = np.zeros((T, K_local, 2))
    for t0 in range(0, T, 2):
        r = philox4x32_10((kg & np.uint64(MASK), kg >> np.uint64(32), np.full_like(kg, t0), np.full_like(kg, step & MASK)),
                          _key(seed, step))
        for tt, (a, b) in ((t0, (r[0], r[1])), (t0 + 1, (r[2], r[3]))):
            if tt >= T:
                break
            z0, z1 = box_muller(a, b)
            out[tt, :, 0] = L00 * z0
            out[tt, :, 1] = L10 * z0 + L11 * z1
    return out


def chain_noise(K_local, T, n, k_offset, seed, step, sigma):
    """chain_philox_kernel: eps[t][d][k] (device layout, fp64) of the n-link chain.
    Calls (global k, counter word 2 = 4 t + call), call = 0, 1: words (x, y, z, w)
    -> z[4 call .. 4 call + 3] by Box-Muller pairs; eps = L z."""
    S = np.asarray(sigma, dtype=np.float64)
    L = np.linalg.cholesky(0.5 * (S + S.T))
    kg = np.arange(K_local, dtype=np.uint64) + np.uint64(k_offset)
    out = np.zeros((T, n, K_local))
    for t in range(T):
        z = np.zeros((8, K_local))
        for call in range(2):
            r = philox4x32_10((kg & np.uint64(MASK), kg >> np.uint64(32), np.full_like(kg, 4 * t + call),
                               np.full_like(kg, step & MASK)), _key(seed, step))
            z[4 * call], z[4 * call + 1] = box_muller(r[0], r[1])
            z[4 * call + 2], z[4 * call + 3] = box_muller(r[2], r[3])
        out[t] = L @ z[:n]
    return out
