"""Per-call wall time of ChainMPPIController at config 5 for precision "f32", "f64" and "auto" (the default),
with one-hot weights (lambda = 100, run.py's) and spread ones (lambda = 3e5): what precision="auto" costs.
Back to back from the config-5 start state, device noise, steady state (calls counted after warm-up).
    python tools/chain_auto_cost.py [--K 131072] [--calls 30] [--warm 8]
"""
import argparse
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from mppi_robotarm_amd.chain import CHAIN7_SIGMA, CHAIN7_X0, ChainMPPIController, gravity_torque  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--K", type=int, default=131072)
    ap.add_argument("--T", type=int, default=128)
    ap.add_argument("--calls", type=int, default=30)
    ap.add_argument("--warm", type=int, default=8)
    a = ap.parse_args()
    d = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden", "paths.npz"))
    path = d["xydq_circle"][:, :4]
    ug = gravity_torque(CHAIN7_X0[:7])
    print(f"K={a.K} T={a.T}: {a.calls} calls after {a.warm}, back to back, device noise")
    for lam in (100.0, 3.0e5):
        for prec in ("f32", "f64", "auto"):
            c = ChainMPPIController(0.006, path, a.T, a.K, 0.0, lam, 0.98, CHAIN7_SIGMA, precision=prec,
                                    device=0, verbose=False, noise="device", seed=11, u_init=np.tile(ug, (a.T, 1)))
            walls, precs, etas = [], [], []
            for i in range(a.warm + a.calls):
                c.u_prev[:] = ug                              # the same start nominal every call: a fixed regime
                c.prev_waypoints_idx = 0
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                c.calc_control_input(CHAIN7_X0.copy())
                t1 = time.perf_counter()
                if i >= a.warm:
                    walls.append((t1 - t0) * 1e3)
                    precs.append(c.last_precision)
                    etas.append(c.last_eta)
            c.close()
            w = np.array(walls)
            print(f"lambda={lam:g} precision={prec:4s}: median {np.median(w):7.3f} ms  p90 {np.percentile(w, 90):7.3f}"
                  f"  max {w.max():7.3f}  fp64 steps {precs.count('f64')}/{len(precs)}  eta median "
                  f"{np.median(etas):.3f}", flush=True)


if __name__ == "__main__":
    main()
