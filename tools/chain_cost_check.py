"""Diagnostic: chain S at small T vs the oracle, with the worst sample dissected."""
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
path = dict(np.load(os.path.join(ROOT, "tests", "golden", "paths.npz")))["xydq_circle"]
win = path[:30]
P, Po = ChainParams(), CO.ChainParams()
W, TW = [.5, .5, 5, 5], [5, 5, 50, 50]
for T in (1, 2, 4):
    K = 4096
    eng = ChainEngine(K, T, 0.006, 100.0, 0.98, CHAIN7_SIGMA, W, TW, 0.0, P, device=0)
    u = np.tile(gravity_torque(CHAIN7_X0[:7], P), (T, 1))
    eng.set_step_inputs(CHAIN7_X0, win, u)
    noise = eng.philox_noise(7, 1)
    S_dev = torch.empty(K, dtype=torch.float64, device="cuda")
    eng.rollout(noise, S_out=S_dev)
    S = S_dev.cpu().numpy()
    nz = noise.cpu().numpy().transpose(0, 2, 1)   # device [T][K][n] -> (T, n, K)
    Sr = coracle.chain_rollout_costs(CHAIN7_X0, u, nz, win, 0.006, 100.0, 0.98, CHAIN7_SIGMA, W, TW, Po, layout="TNK")
    rel = np.abs(S - Sr) / np.abs(Sr)
    k = int(np.argmax(rel))
    print(f"T={T}: S rel max {rel.max():.2e} (#>1e-3: {(rel > 1e-3).sum()}) worst k={k} S_gpu {S[k]:.6g} S_ref {Sr[k]:.6g}")
    # dissect the worst sample with the NumPy oracle
    eps_k = nz[:, :, k].astype(np.float64)             # (T, 7)
    q, dq = CHAIN7_X0[None, :7].copy(), CHAIN7_X0[None, 7:].copy()
    for t in range(T):
        q, dq = CO.chain_forward_dynamics(q, dq, (u[t] + eps_k[t])[None], 0.006, Po)
        x, y = CO.chain_fk(q, Po)
        d = ((x[0] - win[:, 0]) ** 2 + (y[0] - win[:, 1]) ** 2) * 100
        j = int(np.argmin(d))
        srt = np.sort(d)
        print(f"   t={t}: ee ({x[0]:.5f},{y[0]:.5f}) nearest {j} d {srt[0]:.6g} next {srt[1]:.6g} rel gap {(srt[1]-srt[0])/srt[0]:.2e} dq01 ({dq[0,0]:.4f},{dq[0,1]:.4f})")
    eng.close()
