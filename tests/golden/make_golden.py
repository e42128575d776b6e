"""Generate the golden fixtures for the MPPI hot path from the imported reference.

Run ONCE in the build container (where /root/reference exists); the outputs are
committed as small ``.npz`` files next to this script and are what every parity
test compares against.  Nothing here runs on the GPU box, and no reference source
is copied: the reference module is imported read-only from /root/reference and
only its *outputs* (plus the trajectory data files it ships) are stored.

How one fixture is captured (reference ``control.py``):
  * ``np.random.seed(seed)`` then ``calc_control_input`` is called once
    (control.py:67-152) with the instance methods below wrapped on the instance:
      - ``_calc_epsilon`` (control.py:154-164) returns the reference draw rounded
        to fp32 and back, so the fp64 oracle, the fp32 HIP kernel and the
        reference all consume bit-identical noise;
      - ``_compute_weights`` (control.py:297-314) records S and w;
      - ``_moving_median_filter`` (control.py:319-327) records raw and filtered
        w_eps.
  * ``u_new`` (the pre-shift update ``u += w_eps``, control.py:126) is rebuilt as
    ``u_prev_before + w_eps_filtered``: the same single fp64 add, same bits.
  * The reference's ``IPython`` import (control.py:7) is unused; an empty stub
    module stands in for it so ``import control`` succeeds.  matplotlib runs
    headless (Agg).

Usage:  python tests/golden/make_golden.py   (≈30 s)
"""
from __future__ import annotations

import contextlib
import io
import json
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"

RUNPY = dict(  # run.py:25-37
    param_exploration=0.0,
    param_lambda=100.0,
    param_alpha=0.98,
    sigma=np.array([[20.0, 0.0], [0.0, 20.0]]),
    stage_cost_weight=np.array([0.50, 0.50, 5.0, 5.0]),
    terminal_cost_weight=np.array([5.0, 5.0, 50.0, 50.0]),
)
DT_PLANT = 0.003                     # run.py:10
X0 = np.array([1.152198236517471885e00, -1.266101672070702344e00, 0.0, 0.0])  # run.py:14-15


def _import_reference():
    sys.dont_write_bytecode = True
    os.environ.setdefault("MPLBACKEND", "Agg")
    ip = types.ModuleType("IPython")
    ipd = types.ModuleType("IPython.display")
    ip.display = ipd
    sys.modules.setdefault("IPython", ip)
    sys.modules.setdefault("IPython.display", ipd)
    if REF not in sys.path:
        sys.path.insert(0, REF)
    import control  # noqa: E402
    import utils  # noqa: E402
    return control, utils


def _instrument(mppi, rec):
    orig_eps = mppi._calc_epsilon
    orig_w = mppi._compute_weights
    orig_f = mppi._moving_median_filter

    def eps_fp32(*a, **k):
        e = orig_eps(*a, **k)
        e = e.astype(np.float32).astype(np.float64)
        rec["eps"] = e.astype(np.float32)
        return e

    def weights(S):
        w = orig_w(S)
        rec["S"] = S.copy()
        rec["w"] = w.copy()
        return w

    def medfilt(xx, window_size):
        out = orig_f(xx=xx, window_size=window_size)
        rec["w_eps_raw"] = xx.copy()
        rec["w_eps_filt"] = out.copy()
        return out

    mppi._calc_epsilon = eps_fp32
    mppi._compute_weights = weights
    mppi._moving_median_filter = medfilt


def one_step(control, name, ref_path, path_name, K, T, seed, x0, prev_idx=0,
             u_prev=None, delta_t=0.006, sampled=False, **over):
    kw = dict(RUNPY)
    kw.update(over)
    mppi = control.MPPIControllerForPathTracking(
        delta_t=delta_t, ref_path=ref_path, horizon_step_T=T, number_of_samples_K=K,
        visualze_sampled_trajs=sampled, **kw)
    mppi.prev_waypoints_idx = prev_idx
    if u_prev is not None:
        mppi.u_prev = np.array(u_prev, dtype=np.float64).copy()
    u_before = mppi.u_prev.copy()
    rec = {}
    _instrument(mppi, rec)
    np.random.seed(seed)
    with contextlib.redirect_stdout(io.StringIO()):
        u0, u_seq, opt, samp = mppi.calc_control_input(observed_x=np.array(x0, dtype=np.float64))
    out = dict(
        path=np.array(path_name), K=np.int64(K), T=np.int64(T), seed=np.int64(seed),
        delta_t=np.float64(delta_t), x0=np.asarray(x0, np.float64), prev_idx=np.int64(prev_idx),
        u_prev=u_before, param_exploration=np.float64(kw["param_exploration"]),
        param_lambda=np.float64(kw["param_lambda"]), param_alpha=np.float64(kw["param_alpha"]),
        sigma=np.asarray(kw["sigma"], np.float64),
        stage_cost_weight=np.asarray(kw["stage_cost_weight"], np.float64),
        terminal_cost_weight=np.asarray(kw["terminal_cost_weight"], np.float64),
        sampled=np.bool_(sampled),
        eps=rec["eps"], S=rec["S"], w=rec["w"], w_eps_raw=rec["w_eps_raw"],
        w_eps_filt=rec["w_eps_filt"], u_new=u_before + rec["w_eps_filt"],
        u0=np.array(u0), u_seq=np.array(u_seq), optimal_traj=np.array(opt),
        prev_idx_after=np.int64(mppi.prev_waypoints_idx),
    )
    if sampled:
        out["sampled_traj"] = np.array(samp)
    np.savez_compressed(os.path.join(HERE, f"step_{name}.npz"), **out)
    print(f"step_{name}: K={K} T={T} argmin={int(np.argmin(rec['S']))} "
          f"prev {prev_idx}->{mppi.prev_waypoints_idx}")


def closed_loop(control, utils, name, ref_path, K, T, seed, ticks, sampled):
    """run.py:48-71 for `ticks` ticks (plant utils.py:14-38, dt=0.003)."""
    mppi = control.MPPIControllerForPathTracking(
        delta_t=DT_PLANT * 2, ref_path=ref_path, horizon_step_T=T, number_of_samples_K=K,
        visualze_sampled_trajs=sampled, **RUNPY)
    rec = {}
    _instrument(mppi, rec)
    q = X0[:2].copy()
    dq = X0[2:].copy()
    state = [q[0], q[1], dq[0], dq[1]]
    np.random.seed(seed)
    states, us, useqs, prevs, eps = [], [], [], [], []
    with contextlib.redirect_stdout(io.StringIO()):
        for _ in range(ticks):
            states.append(np.array(state, dtype=np.float64))
            u, u_seq, _, _ = mppi.calc_control_input(observed_x=state)
            eps.append(rec["eps"])
            us.append(np.array(u))
            useqs.append(np.array(u_seq))
            prevs.append(mppi.prev_waypoints_idx)
            dq += DT_PLANT * utils.Arm_Dynamic(q, dq, u)
            q += DT_PLANT * dq
            state = np.concatenate((q, dq))
    np.savez_compressed(
        os.path.join(HERE, f"loop_{name}.npz"), K=np.int64(K), T=np.int64(T),
        seed=np.int64(seed), ticks=np.int64(ticks), states=np.array(states),
        u=np.array(us), u_seq=np.array(useqs), prev_idx=np.array(prevs, dtype=np.int64),
        eps=np.array(eps), final_state=np.array(state))
    print(f"loop_{name}: ticks={ticks} final={state}")


def errors(control):
    """Exception classes the reference raises on the boundary's error paths."""
    res = {}
    ref_path = np.loadtxt(os.path.join(REF, "xydq_circle.txt"))[:, 0:4]
    with contextlib.redirect_stdout(io.StringIO()):
        # control.py:76-78 — end of path
        m = control.MPPIControllerForPathTracking(delta_t=0.006, ref_path=ref_path,
                                                  horizon_step_T=8, number_of_samples_K=4, **RUNPY)
        m.prev_waypoints_idx = ref_path.shape[0] - 1
        try:
            m.calc_control_input(observed_x=np.array([0.0, 0.0, 0.0, 0.0]))
            res["end_of_path"] = None
        except Exception as e:  # noqa: BLE001
            res["end_of_path"] = type(e).__name__
        # control.py:30 default sigma is singular → np.linalg.inv at :106
        m = control.MPPIControllerForPathTracking(delta_t=0.006, ref_path=ref_path,
                                                  horizon_step_T=8, number_of_samples_K=4)
        np.random.seed(0)
        try:
            import warnings
            with warnings.catch_warnings():
                warnings.simplefilter("ignore")
                m.calc_control_input(observed_x=X0.copy())
            res["default_sigma"] = None
        except Exception as e:  # noqa: BLE001
            res["default_sigma"] = type(e).__module__ + "." + type(e).__name__
        # control.py:157-159 — sigma shape
        m = control.MPPIControllerForPathTracking(delta_t=0.006, ref_path=ref_path,
                                                  horizon_step_T=8, number_of_samples_K=4,
                                                  **{**RUNPY, "sigma": np.eye(3)})
        try:
            m.calc_control_input(observed_x=X0.copy())
            res["sigma_shape"] = None
        except Exception as e:  # noqa: BLE001
            res["sigma_shape"] = type(e).__name__
    with open(os.path.join(HERE, "errors.json"), "w") as f:
        json.dump(res, f, indent=1, sort_keys=True)
    print("errors:", res)


def medfilt_vectors():
    """scipy.ndimage.median_filter(size=10, mode='reflect') known answers (control.py:325)."""
    from scipy.ndimage import median_filter
    rng = np.random.default_rng(123)
    cases = {}
    for n in (1, 2, 3, 5, 9, 10, 11, 20, 30, 64):
        x = rng.standard_normal(n)
        x[rng.integers(0, n)] = x[0]  # a tie
        cases[f"x{n}"] = x
        cases[f"y{n}"] = median_filter(x, size=10, mode="reflect")
    np.savez_compressed(os.path.join(HERE, "medfilt.npz"), **cases)


def main():
    control, utils = _import_reference()
    circle_full = np.loadtxt(os.path.join(REF, "xydq_circle.txt"))
    circle = circle_full[:, 0:4]
    traj = np.loadtxt(os.path.join(REF, "trajectory.txt"))[:, 0:4]
    traj1 = np.loadtxt(os.path.join(REF, "trajectory1.txt"))
    np.savez_compressed(os.path.join(HERE, "paths.npz"), xydq_circle=circle_full,
                        trajectory=traj, trajectory1=traj1)

    rng = np.random.default_rng(2024)
    # config 1: K=128 T=20, both paths named by BASELINE.json
    one_step(control, "c1_circle_k128_t20", circle, "xydq_circle", 128, 20, 0, X0)
    one_step(control, "c1_traj_k128_t20", traj, "trajectory", 128, 20, 1, X0)
    # run.py's shipped configuration, sampled trajectories on (run.py:36)
    one_step(control, "runpy_k100_t30", circle, "xydq_circle", 100, 30, 2, X0, sampled=True)
    # mid-path start (joint angles of trajectory1.txt row 700 + path joint velocities)
    i = 700
    x_mid = np.array([traj1[i, 0], traj1[i, 1], circle[i, 2], circle[i, 3]])
    u_mid = np.array([[10.0, -2.0]] * 32) + rng.normal(0.0, 1.0, (32, 2))
    one_step(control, "mid_k256_t32", circle, "xydq_circle", 256, 32, 3, x_mid,
             prev_idx=690, u_prev=u_mid)
    # window truncated by the path end (control.py:208-209 slice semantics)
    j = circle.shape[0] - 12
    x_end = np.array([traj1[1995, 0], traj1[1995, 1], circle[1995, 2], circle[1995, 3]])
    one_step(control, "end_k64_t16", circle, "xydq_circle", 64, 16, 4, x_end, prev_idx=j)
    # exploration split (control.py:98-101)
    one_step(control, "expl_k128_t20", circle, "xydq_circle", 128, 20, 5, X0,
             param_exploration=0.25)
    # non-degenerate soft-min weights (large lambda), gamma = 0
    one_step(control, "dense_k256_t24", circle, "xydq_circle", 256, 24, 6, x_mid,
             prev_idx=690, param_lambda=5.0e6, param_alpha=1.0)
    # non-degenerate weights with a gamma term and a general (non-diagonal) Sigma
    one_step(control, "sigma_k128_t20", circle, "xydq_circle", 128, 20, 7, X0,
             sigma=np.array([[20.0, 6.0], [6.0, 12.0]]), param_lambda=2.0e6, param_alpha=0.9)
    # short seeded closed loops of run.py's loop (run.py:48-71)
    closed_loop(control, utils, "runpy_k100_t30", circle, 100, 30, 11, 8, sampled=True)
    closed_loop(control, utils, "k64_t20", circle, 64, 20, 12, 25, sampled=False)
    errors(control)
    medfilt_vectors()


if __name__ == "__main__":
    main()
