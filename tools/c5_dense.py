"""Diagnostic: config 5 (7-link chain, K=131072 T=128) where the weights are spread.

For each lambda: the effective sample size of the fp64 weights, the device's
w_eps error against the C oracle, the S error of the samples that carry the
weight, and how much of it nearest-waypoint ties explain; then the fp32 state
drift of the trajectory kernel against the fp64 chain on a subset.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import chain_oracle as CO  # noqa: E402
import coracle  # noqa: E402
from mppi_robotarm_amd.chain import CHAIN7_SIGMA, CHAIN7_X0, ChainEngine, ChainParams, gravity_torque  # noqa: E402
from tieflip import tie_flip_residual  # noqa: E402

torch.cuda.set_device(0)
path = dict(np.load(os.path.join(ROOT, "tests", "golden", "paths.npz")))["xydq_circle"]
win = path[:30]
W, TW = [.5, .5, 5, 5], [5, 5, 50, 50]
K, T = int(os.environ.get("K", 131072)), int(os.environ.get("T", 128))
u = np.tile(gravity_torque(CHAIN7_X0[:7]), (T, 1))
lams = [float(x) for x in os.environ.get("LAMS", "3e4,6e4,1e5,3e5").split(",")]
for lam in lams:
    eng = ChainEngine(K, T, 0.006, lam, 0.98, CHAIN7_SIGMA, W, TW, 0.0, ChainParams(), device=0)
    eng.set_step_inputs(CHAIN7_X0, win, u)
    noise = eng.philox_noise(11, 2)
    S_dev = torch.empty(K, dtype=torch.float64, device="cuda")
    eng.rollout(noise, S_out=S_dev)
    w = eng.weighted_noise()
    S = S_dev.cpu().numpy()
    nz = noise.cpu().numpy().transpose(0, 2, 1)   # device [T][K][n] -> (T, n, K)
    Sr = coracle.chain_rollout_costs(CHAIN7_X0, u, nz, win, 0.006, lam, 0.98, CHAIN7_SIGMA, W, TW, CO.ChainParams(),
                                     layout="TNK")
    _, wr = coracle.chain_weighted_noise(Sr, nz, lam, layout="TNK")
    wt = np.exp(-(Sr - Sr.min()) / lam)
    ess = wt.sum() ** 2 / (wt ** 2).sum()
    urel = float(np.max(np.abs(w - wr)) / max(1.0, float(np.max(np.abs(wr)))))
    rel = np.abs(S - Sr) / np.abs(Sr)
    top = np.argsort(Sr)[:64]
    dS = (S - Sr)[top]
    print(f"lam={lam:g}: ESS {ess:.1f}  w_eps rel-err {urel:.2e}  |w_eps| max {np.abs(wr).max():.3f}  "
          f"S rel p50 {np.median(rel):.2e} p99 {np.percentile(rel, 99):.2e}; top-64 |dS| max {np.abs(dS).max():.3g} "
          f"(dS/lam {np.abs(dS).max() / lam:.2e}), rel max {rel[top].max():.2e}")
    bad = top[rel[top] > 1e-6]
    if len(bad):
        res, gap = tie_flip_residual(S, Sr, bad, CHAIN7_X0, u, nz, win, 0.006, W, TW, CO.ChainParams())
        for i, k in enumerate(bad[:12]):
            print(f"    k={k} rank {int(np.where(top == k)[0][0])} rel {rel[k]:.2e} dS {S[k] - Sr[k]:.3g} "
                  f"-> after ties {res[i]:.2e} (gap {gap[i]:.2e} m)")
    eng.close()

# fp32 state drift of the trajectory kernel (same dynamics as the rollout)
Kd = 2048
eng = ChainEngine(K, T, 0.006, 100.0, 0.98, CHAIN7_SIGMA, W, TW, 0.0, ChainParams(), device=0)
eng.set_step_inputs(CHAIN7_X0, win, u)
noise = eng.philox_noise(11, 2)
tr = eng.trajectories(u, noise, K=Kd).cpu().numpy().astype(np.float64)   # (Kd, T, 14)
nz = noise.cpu().numpy().transpose(0, 2, 1)[:, :, :Kd].astype(np.float64)   # device (T, K, 7) -> (T, 7, Kd)
ti = (np.arange(T) - 1) % T
ctrl = (u[ti][None] + nz[ti].transpose(2, 0, 1))                          # control(t) = u[t-1] + eps[t-1]
ref = CO.chain_rollout_trajectory(CHAIN7_X0, ctrl, 0.006, CO.ChainParams())
dq = np.abs(tr[..., :7] - ref[..., :7]).max(-1)
ddq = np.abs(tr[..., 7:] - ref[..., 7:]).max(-1)
for t in (0, 7, 31, 63, 127):
    if t < T:
        print(f"t={t}: |q err| p50 {np.median(dq[:, t]):.2e} p99 {np.percentile(dq[:, t], 99):.2e} max {dq[:, t].max():.2e};"
              f" |dq err| p50 {np.median(ddq[:, t]):.2e} p99 {np.percentile(ddq[:, t], 99):.2e} max {ddq[:, t].max():.2e}")
eng.close()
