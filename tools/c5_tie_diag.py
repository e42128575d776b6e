"""Diagnostics for the config-5 parity test (tests/test_gpu_chain.py::test_chain_n7_against_c_oracle,
K = 131072, T = 128, lambda = 100): for every sample beyond 1e-3 of the fp64 oracle, its closest
nearest-waypoint ties (gap, cost step) and the residual left after the best flip combination at
two search settings.  python tools/c5_tie_diag.py [lps]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import chain_oracle as CO  # noqa: E402
import coracle  # noqa: E402
from tieflip import tie_flip_residual, tie_table  # noqa: E402
from mppi_robotarm_amd.chain import CHAIN7_SIGMA, CHAIN7_X0, ChainEngine, ChainParams, gravity_torque  # noqa: E402

W, TW = [0.5, 0.5, 5.0, 5.0], [5.0, 5.0, 50.0, 50.0]
lps = int(sys.argv[1]) if len(sys.argv) > 1 else 1
K, T, lam = 131072, 128, 100.0
torch.cuda.set_device(0)
P, x0, sig, ug = ChainParams(), CHAIN7_X0, CHAIN7_SIGMA, gravity_torque(CHAIN7_X0[:7])
eng = ChainEngine(K, T, 0.006, lam, 0.98, sig, W, TW, 0.0, P, device=0, lanes_per_sample=lps)
win = np.load(os.path.join(ROOT, "tests", "golden", "paths.npz"))["xydq_circle"][:30]
u = np.tile(ug, (T, 1)) + np.random.default_rng(4).normal(0, 0.3, (T, 7))
eng.set_step_inputs(x0, win, u)
noise = eng.philox_noise(11, 2)
S_dev = torch.empty(K, dtype=torch.float64, device="cuda")
eng.rollout(noise, S_out=S_dev)
S = S_dev.cpu().numpy()
nz = noise.cpu().numpy()
eng.close()
Sr = coracle.chain_rollout_costs(x0, u, nz, win, 0.006, lam, 0.98, sig, W, TW, CO.ChainParams(), layout="TNK")
rel = np.abs(S - Sr) / np.abs(Sr)
out = np.flatnonzero(rel > 1e-3)
print(f"lps {lps}: {len(out)} samples beyond 1e-3")
for gm, mf in ((1e-5, 10), (3e-5, 14)):
    res, gap = tie_flip_residual(S, Sr, out, x0, u, nz, win, 0.006, W, TW, CO.ChainParams(), gap_max=gm, max_flips=mf)
    print(f"  gap_max {gm:g} max_flips {mf}: residual max {res.max():.2e}, gap used max {gap.max():.2e}")
    bad = out[res > 2e-4]
    for i in bad:
        g, d = tie_table([i], x0, u, nz, win, 0.006, W, TW, CO.ChainParams())
        o = np.argsort(g[0], kind="stable")[:16]
        print(f"    sample {i}: S_dev {S[i]:.9g} S_ref {Sr[i]:.9g} rel {rel[i]:.2e} diff {S[i] - Sr[i]:.6g}")
        print("      closest ties (step, gap m, cost delta):", [(int(t), float(f"{g[0, t]:.2e}"), float(f"{d[0, t]:.4g}")) for t in o])
