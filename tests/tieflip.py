"""Test helper (checker side only): explain an fp32 cost outlier by nearest-waypoint ties.

The device evaluates the end effector in fp32; where the fp64 end effector lies
within fp32 resolution of the bisector between the two nearest window slots
(control.py:205-215's argmin), the device may pick the neighbour slot at that
step.  S then differs from the fp64 oracle by exactly that stage's cost
difference between the two slots (the state itself does not depend on the
pick).  ``tie_flip_residual`` recomputes, in fp64 with the chain oracle, the
per-step cost difference and the distance gap between the nearest and the
second-nearest slot for the given samples, and returns, per sample, the smallest
relative residual |S_dev - S_alt| / |S_alt| over every combination of flips at
its closest-tie steps (gap below ``gap_max``), with the largest gap that combination used.
An outlier is explained when the residual falls to the normal fp32 level and
the gaps used are below the fp32 position resolution of the trajectory.

``device_pick_residual`` is the exact form for the 7-link chain, whose kernel
can record the slot it picked at every step (ChainEngine.debug_slots): the fp64
cost recomputed with the device's own picks, and the gap at every step where a
pick differs from the fp64 argmin — no search over flip combinations.
"""
from __future__ import annotations

import numpy as np

import chain_oracle as CO


def tie_table(idx, x0, u, eps_tnk, win, dt, stage_w, term_w, P, exploit=None):
    """Per sample and step: (gap [m], cost of the second-nearest slot - cost of the nearest)."""
    idx = np.asarray(idx)
    e = np.asarray(eps_tnk)[:, :, idx].astype(np.float64).transpose(2, 0, 1)   # (m, T, n)
    m, T, n = e.shape
    q = np.tile(np.asarray(x0[:n], dtype=np.float64), (m, 1))
    dq = np.tile(np.asarray(x0[n:2 * n], dtype=np.float64), (m, 1))
    ex = np.ones(m, bool) if exploit is None else np.asarray(exploit)[idx]
    win = np.asarray(win, dtype=np.float64)
    gap = np.empty((m, T))
    delta = np.empty((m, T))
    rows = np.arange(m)
    for t in range(T):
        v = np.where(ex[:, None], u[t] + e[:, t], e[:, t])
        q, dq = CO.chain_forward_dynamics(q, dq, v, dt, P)
        x, y = CO.chain_fk(q, P)
        d = ((x[:, None] - win[:, 0]) ** 2 + (y[:, None] - win[:, 1]) ** 2) * 100
        order = np.argsort(d, axis=1, kind="stable")      # first minimum first, as list.index(min(d))
        j1, j2 = order[:, 0], order[:, 1]
        w = np.asarray(stage_w, dtype=np.float64)
        if t == T - 1:
            w = w + np.asarray(term_w, dtype=np.float64)   # the terminal cost uses the same slot

        def cost(j):
            r = win[j]
            return 10000 * (w[0] * (x - r[:, 0]) ** 2 + w[1] * (y - r[:, 1]) ** 2 +
                            w[2] * (dq[:, 0] - r[:, 2]) ** 2 + w[3] * (dq[:, 1] - r[:, 3]) ** 2)

        delta[:, t] = cost(j2) - cost(j1)
        gap[:, t] = np.sqrt(d[rows, j2] / 100) - np.sqrt(d[rows, j1] / 100)
    return gap, delta


def _walk(idx, x0, u, eps_tnk, dt, P, exploit):
    """fp64 oracle states of the samples idx, step by step: yields (t, x, y, dq)."""
    idx = np.asarray(idx)
    e = np.asarray(eps_tnk)[:, :, idx].astype(np.float64).transpose(2, 0, 1)   # (m, T, n)
    m, T, n = e.shape
    q = np.tile(np.asarray(x0[:n], dtype=np.float64), (m, 1))
    dq = np.tile(np.asarray(x0[n:2 * n], dtype=np.float64), (m, 1))
    ex = np.ones(m, bool) if exploit is None else np.asarray(exploit)[idx]
    for t in range(T):
        v = np.where(ex[:, None], u[t] + e[:, t], e[:, t])
        q, dq = CO.chain_forward_dynamics(q, dq, v, dt, P)
        x, y = CO.chain_fk(q, P)
        yield t, x, y, dq


def device_pick_residual(S_dev, S_ref, idx, x0, u, eps_tnk, win, dt, stage_w, term_w, P, slots, exploit=None):
    """(residual, largest gap [m] among the differing picks, number of differing steps) per sample
    of ``idx``: S_ref plus, at every step where the device's slot (``slots`` (K, T)) differs from
    the fp64 first minimum, that step's cost difference between the two slots."""
    idx = np.asarray(idx)
    win = np.asarray(win, dtype=np.float64)
    m = len(idx)
    rows = np.arange(m)
    alt = np.asarray(S_ref, dtype=np.float64)[idx].copy()
    gap = np.zeros(m)
    ndiff = np.zeros(m, dtype=np.int64)
    T = np.asarray(eps_tnk).shape[0]
    for t, x, y, dq in _walk(idx, x0, u, eps_tnk, dt, P, exploit):
        d = ((x[:, None] - win[:, 0]) ** 2 + (y[:, None] - win[:, 1]) ** 2) * 100
        j1 = np.argmin(d, axis=1)                       # first minimum, as list.index(min(d))
        jd = np.asarray(slots)[idx, t].astype(np.int64)
        w = np.asarray(stage_w, dtype=np.float64)
        if t == T - 1:
            w = w + np.asarray(term_w, dtype=np.float64)   # the terminal cost uses the same slot

        def cost(j):
            r = win[j]
            return 10000 * (w[0] * (x - r[:, 0]) ** 2 + w[1] * (y - r[:, 1]) ** 2 +
                            w[2] * (dq[:, 0] - r[:, 2]) ** 2 + w[3] * (dq[:, 1] - r[:, 3]) ** 2)

        diff = jd != j1
        alt += np.where(diff, cost(jd) - cost(j1), 0.0)
        g = np.sqrt(d[rows, jd] / 100) - np.sqrt(d[rows, j1] / 100)
        gap = np.maximum(gap, np.where(diff, g, 0.0))
        ndiff += diff
    res = np.abs(np.asarray(S_dev, dtype=np.float64)[idx] - alt) / np.abs(alt)
    return res, gap, ndiff


def tie_flip_residual(S_dev, S_ref, idx, x0, u, eps_tnk, win, dt, stage_w, term_w, P, exploit=None,
                      gap_max=1e-5, max_flips=10):
    """(residual, gap_used) per sample of ``idx``: every combination of neighbour picks
    at the (at most ``max_flips``) closest-tie steps whose gap is below ``gap_max``."""
    idx = np.asarray(idx)
    gap, delta = tie_table(idx, x0, u, eps_tnk, win, dt, stage_w, term_w, P, exploit)
    res = np.empty(len(idx))
    used = np.zeros(len(idx))
    for i in range(len(idx)):
        cand = np.argsort(gap[i], kind="stable")[:max_flips]
        cand = cand[gap[i, cand] < gap_max]
        m = len(cand)
        combos = ((np.arange(2 ** m)[:, None] >> np.arange(m)[None, :]) & 1).astype(bool)   # (2^m, m)
        s_alt = S_ref[idx[i]] + combos.astype(np.float64) @ delta[i, cand]
        rr = np.abs(S_dev[idx[i]] - s_alt) / np.abs(s_alt)
        b = int(np.argmin(rr))
        res[i] = rr[b]
        used[i] = float(gap[i, cand][combos[b]].max()) if combos[b].any() else 0.0
    return res, used
