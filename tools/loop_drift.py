"""Diagnostic: the device closed loops of bench.py (fused steps on the updated nominal, fixed start state):
nominal range, non-finite rollouts and S every few steps.  WL=c3 (2-DoF arm) or c5 (7-link chain, fp32 and
fp64); RESET=M re-stages the start nominal every M steps (what bench.py does for c5)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT]
import numpy as np  # noqa: E402
import torch  # noqa: E402

torch.cuda.set_device(0)
path = dict(np.load(os.path.join(ROOT, "tests", "golden", "paths.npz")))["xydq_circle"][:, :4]
WL = os.environ.get("WL", "c5")
NSTEP = int(os.environ.get("NSTEP", 1500))
RESET = int(os.environ.get("RESET", 0))


def engines():
    if WL == "c3":
        from mppi_robotarm_amd.engine import RolloutEngine
        from mppi_robotarm_amd.params import ArmParams, X0_RUNPY
        K, T = 65536, 64
        yield "f32", K, RolloutEngine(K, T, 0.006, 100.0, 0.98, np.eye(2) * 20.0, [.5, .5, 5, 5], [5, 5, 50, 50], 0.0,
                                      ArmParams(), device=0), X0_RUNPY.copy(), np.array([[10.0, -2.0]] * T)
    else:
        from mppi_robotarm_amd.chain import CHAIN7_SIGMA, CHAIN7_X0, ChainEngine, ChainParams, gravity_torque
        K, T = 131072, 128
        for prec in ("f32", "f64"):
            yield prec, K, ChainEngine(K, T, 0.006, 100.0, 0.98, CHAIN7_SIGMA, [.5, .5, 5, 5], [5, 5, 50, 50], 0.0,
                                       ChainParams(), device=0, precision=prec), CHAIN7_X0.copy(), \
                np.tile(gravity_torque(CHAIN7_X0[:7]), (T, 1))


for prec, K, eng, x0, u in engines():
    eng.set_step_inputs(x0, path[0:30], u)
    noise = [eng.philox_noise(1234, i) for i in range(4)]
    S = torch.empty(K, dtype=torch.float64, device="cuda")
    for i in range(NSTEP):
        if RESET and i % RESET == 0:
            eng.set_step_inputs(x0, path[0:30], u)
        eng.rollout(noise[i % 4], S_out=S, fused_update=True)
        if i < 4 or i % max(1, NSTEP // 20) == 0 or i == NSTEP - 1:
            un = eng.nominal()
            s = S.cpu().numpy()
            print(f"{WL} {prec} step {i}: |u| max {np.abs(un).max():.4g} finite {np.isfinite(un).all()}  "
                  f"S min {np.nanmin(s) if np.isfinite(s).any() else np.nan:.6g} nan {np.isnan(s).sum()} "
                  f"inf {np.isinf(s).sum()}", flush=True)
            if not np.isfinite(un).all():
                break
    eng.close()
