"""Diagnostic: per-step state of the chain kernel (traj kernel, same ChainState::step)
vs the C oracle, to locate a dynamics discrepancy."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import chain_oracle as CO  # noqa: E402
import coracle  # noqa: E402
from mppi_robotarm_amd.chain import CHAIN7_SIGMA, CHAIN7_X0, ChainEngine, ChainParams, gravity_torque  # noqa: E402

torch.cuda.set_device(0)
paths = dict(np.load(os.path.join(ROOT, "tests", "golden", "paths.npz")))
for label, P, Po in [("J=b=0", ChainParams(J=(0.0,) * 7, b=(0.0,) * 7), CO.ChainParams(J=(0.0,) * 7, b=(0.0,) * 7)),
                     ("default", ChainParams(), CO.ChainParams())]:
    K, T = 8, 16
    eng = ChainEngine(K, T, 0.006, 100.0, 0.98, CHAIN7_SIGMA, [.5, .5, 5, 5], [5, 5, 50, 50], 0.0, P, device=0)
    u = np.tile(gravity_torque(CHAIN7_X0[:7], P), (T, 1))
    eng.set_step_inputs(CHAIN7_X0, paths["xydq_circle"][:30], u)
    still = eng.trajectories(base_u=u, K=1)[0].cpu().numpy()
    print(label, "gravity hold: max |x_t - x0|", np.abs(still - CHAIN7_X0[None]).max())
    noise = eng.philox_noise(7, 1)
    tr = eng.trajectories(base_u=u, noise=noise).cpu().numpy()          # (K, T, 14), control(t) = u[t-1] + eps[t-1]
    nz = noise.cpu().numpy()                                            # (T, 7, K)
    ctrl = np.roll(u[None] + nz.transpose(2, 0, 1), 1, axis=1)
    ref = coracle.chain_traj(CHAIN7_X0, ctrl, 0.006, Po)
    d = np.abs(tr - ref).max(axis=(0, 2))
    print(label, "per-step max |dx|:", " ".join(f"{v:.1e}" for v in d))
    eng.close()
