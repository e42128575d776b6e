"""Closed-loop harness equal to the reference's driver loop (run.py:48-71).

Each tick: ``calc_control_input`` (the drop-in, HIP hot path), then the plant
``dq += dt * Arm_Dynamic(q, dq, u); q += dt * dq`` (utils.py:14-29, semi-implicit
Euler at dt = 0.003, run.py:53-55) and forward kinematics (utils.py:32-38), with
run.py's recording (tick 1 is not recorded, run.py:62-63).  The plant runs on
the host in fp64, as in the reference; only the controller's K x T work is on
the GPU.  Plots (run.py:120-173) are out of scope.

    python -m mppi_robotarm_amd.harness --ticks 200 [--noise device] [--K 4096]
"""
from __future__ import annotations

import argparse
import os
import time

import numpy as np

from .params import DT_PLANT, X0_RUNPY, ArmParams, runpy_config


def arm_dynamic(q, dq, u, arm: ArmParams = ArmParams()):
    """Plant joint accelerations, utils.py:14-29 (mass matrix as written there)."""
    c2 = np.cos(q[1])
    M11 = arm.m1 * arm.lc1 ** 2 + arm.l1 + arm.m2 * (arm.l1 ** 2 + arm.lc2 ** 2 + 2 * arm.l1 * arm.lc2 * c2) + arm.l2
    M22 = arm.m2 * arm.lc2 ** 2 + arm.l2
    M12 = arm.m2 * arm.l1 * arm.lc2 * c2 + arm.m2 * arm.lc2 ** 2 + arm.l2
    M = np.array([[M11, M12], [M12, M22]])
    h = arm.m2 * arm.l1 * arm.lc2 * np.sin(q[1])
    g1 = arm.m1 * arm.lc1 * arm.g * np.cos(q[0]) + arm.m2 * arm.g * (arm.lc2 * np.cos(q[0] + q[1])
                                                                   + arm.l1 * np.cos(q[0]))
    g2 = arm.m2 * arm.lc2 * arm.g * np.cos(q[0] + q[1])
    C = np.array([[-h * dq[1], -h * dq[0] - h * dq[1]], [h * dq[0], 0]])
    return np.linalg.inv(M).dot(u - C.dot(dq) - np.array([g1, g2]))


def forward_kinematics(q, arm: ArmParams = ArmParams()):
    """Elbow and end-effector positions, utils.py:32-38."""
    x1 = arm.l1 * np.cos(q[0])
    y1 = arm.l1 * np.sin(q[0])
    x2 = arm.l1 * np.cos(q[0]) + arm.l2 * np.cos(q[0] + q[1])
    y2 = arm.l1 * np.sin(q[0]) + arm.l2 * np.sin(q[0] + q[1])
    return x1, y1, x2, y2


def run_closed_loop(ref_path, ticks: int = 1500, controller=None, x0=X0_RUNPY, dt: float = DT_PLANT,
                    arm: ArmParams = ArmParams(), on_tick=None, **controller_kwargs):
    """run.py:39-71.  Returns the record arrays of run.py plus per-tick latency."""
    if controller is None:
        from .controller import MPPIControllerForPathTracking
        kw = runpy_config()
        kw.update(controller_kwargs)
        controller = MPPIControllerForPathTracking(ref_path=ref_path, **kw)
    q = np.array(x0[:2], dtype=np.float64)
    dq = np.array(x0[2:], dtype=np.float64)
    n = int(ticks) + 1
    rec = {k: np.zeros((n, 2)) for k in ("rq", "rx", "ry", "x", "y", "q", "u")}
    rec["t"] = np.zeros(n)
    rec["latency_s"] = np.zeros(n)
    state = [q[0], q[1], dq[0], dq[1]]                                  # run.py:23 (a list on tick 1)
    for k in range(1, int(ticks) + 1):
        t0 = time.perf_counter()
        u, _, _, _ = controller.calc_control_input(observed_x=state)  # run.py:49-51
        rec["latency_s"][k] = time.perf_counter() - t0
        dq += dt * arm_dynamic(q, dq, u, arm)                           # run.py:53
        q += dt * dq                                                    # run.py:55
        x1, y1, x2, y2 = forward_kinematics(q, arm)                     # run.py:57
        state = np.concatenate((q, dq))                                 # run.py:59
        if on_tick is not None:
            on_tick(k, state, u)
        if k == 1:                                                      # run.py:62-63
            continue
        rec["rq"][k] = q
        rec["rx"][k] = ref_path[k, 0:1]
        rec["ry"][k] = ref_path[k, 1:2]
        rec["x"][k] = [x1, x2]
        rec["y"][k] = [y1, y2]
        rec["q"][k] = q
        rec["u"][k] = u
        rec["t"][k] = k
    rec["final_state"] = state
    rec["controller"] = controller
    return rec


def main():
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--ticks", type=int, default=200)
    ap.add_argument("--K", type=int, default=100, help="number_of_samples_K (run.py: 100)")
    ap.add_argument("--T", type=int, default=30, help="horizon_step_T (run.py: 30)")
    ap.add_argument("--noise", choices=("numpy", "device"), default="numpy")
    ap.add_argument("--no-sampled", action="store_true", help="visualze_sampled_trajs=False")
    ap.add_argument("--seed", type=int, default=0)
    args = ap.parse_args()
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    path = np.load(os.path.join(root, "tests", "golden", "paths.npz"))["xydq_circle"][:, 0:4]
    np.random.seed(args.seed)
    rec = run_closed_loop(path, ticks=args.ticks, number_of_samples_K=args.K, horizon_step_T=args.T,
                          noise=args.noise, seed=args.seed, verbose=False,
                          visualze_sampled_trajs=not args.no_sampled)
    ks = np.arange(2, args.ticks + 1)
    err = np.hypot(rec["x"][ks, 1] - rec["rx"][ks, 0], rec["y"][ks, 1] - rec["ry"][ks, 0])
    lat = rec["latency_s"][2:] * 1e3
    print(f"ticks={args.ticks} K={args.K} T={args.T} noise={args.noise}: end-effector tracking error "
          f"mean {err.mean():.4e} max {err.max():.4e} m; control-step latency median {np.median(lat):.3f} ms "
          f"p90 {np.percentile(lat, 90):.3f} ms")


if __name__ == "__main__":
    main()
