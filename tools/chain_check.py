"""Diagnostic: chain engine vs the oracles (prints errors and timings; the
asserting versions live in tests/test_gpu_chain.py).

    python tools/chain_check.py [K T]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import chain_oracle as CO  # noqa: E402
import coracle  # noqa: E402
from conftest import STEP_FIXTURES, load_step  # noqa: E402
from mppi_robotarm_amd.chain import (CHAIN7_SIGMA, CHAIN7_X0, ChainEngine, ChainMPPIController,  # noqa: E402
                                     ChainParams, gravity_torque)

torch.cuda.set_device(0)
paths = dict(np.load(os.path.join(ROOT, "tests", "golden", "paths.npz")))
W = [0.5, 0.5, 5.0, 5.0]
TW = [5.0, 5.0, 50.0, 50.0]

# 1. n = 2 through the chain engine against the reference's golden steps
P2 = ChainParams.from_arm2()
for name in STEP_FIXTURES:
    g = load_step(name)
    c = ChainMPPIController(float(g["delta_t"]), paths[str(g["path"])], int(g["T"]), int(g["K"]),
                            float(g["param_exploration"]), float(g["param_lambda"]), float(g["param_alpha"]),
                            g["sigma"], g["stage_cost_weight"], g["terminal_cost_weight"], chain=P2,
                            u_init=g["u_prev"])
    c.prev_waypoints_idx = int(g["prev_idx"])
    eps = g["eps"].astype(np.float64)
    c._calc_epsilon = lambda *a, e=eps, **k: e
    c.keep_costs = True
    try:
        u0, u_seq, opt, _ = c.calc_control_input(g["x0"])
        S = c.last_S
        print(f"n=2 {name:22s} S rel {np.max(np.abs(S - g['S']) / np.abs(g['S'])):.2e} argmin "
              f"{np.argmin(S) == np.argmin(g['S'])} u rel {np.max(np.abs(u_seq - g['u_seq'])) / max(1, np.abs(g['u_seq']).max()):.2e}")
    except Exception as ex:  # noqa: BLE001
        print(f"n=2 {name}: {type(ex).__name__}: {ex}")
    c.close()

# 2. n = 7 vs the C oracle
K = int(sys.argv[1]) if len(sys.argv) > 1 else 131072
T = int(sys.argv[2]) if len(sys.argv) > 2 else 128
P7 = ChainParams()
for (Kc, Tc, lam) in [(4096, 8, 100.0), (4096, 32, 100.0), (4096, 32, 1e9), (K, T, 100.0)]:
    eng = ChainEngine(Kc, Tc, 0.006, lam, 0.98, CHAIN7_SIGMA, W, TW, 0.0, P7, device=0)
    u = np.tile(gravity_torque(CHAIN7_X0[:7], P7), (Tc, 1))
    win = paths["xydq_circle"][:30]
    eng.set_step_inputs(CHAIN7_X0, win, u)
    noise = eng.philox_noise(7, 1)
    S_dev = torch.empty(Kc, dtype=torch.float64, device="cuda")
    eng.rollout(noise, S_out=S_dev)
    w = eng.weighted_noise()
    S = S_dev.cpu().numpy()
    nz = noise.cpu().numpy()
    t0 = time.time()
    Sr = coracle.chain_rollout_costs(CHAIN7_X0, u, nz, win, 0.006, lam, 0.98, CHAIN7_SIGMA, W, TW, CO.ChainParams(),
                                     layout="TNK")
    tc = time.time() - t0
    _, wr = coracle.chain_weighted_noise(Sr, nz, lam, layout="TNK")
    rel = np.abs(S - Sr) / np.abs(Sr)
    print(f"n=7 K={Kc} T={Tc} lam={lam:g} {eng.handoff}: S rel max {rel.max():.2e} p99 {np.percentile(rel, 99):.2e} "
          f"argmin {np.argmin(S) == np.argmin(Sr)} w_eps rel {np.abs(w - wr).max() / max(1, np.abs(wr).max()):.2e} "
          f"(C oracle {tc:.1f} s)")
    # timing: fused launches back to back
    nbuf = [eng.philox_noise(3, i) for i in range(4)]
    for i in range(3):
        eng.rollout(nbuf[i % 4], fused_update=True)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    n = 20
    for i in range(n):
        eng.rollout(nbuf[i % 4], fused_update=True)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / n
    print(f"    step {ms * 1e3:.1f} us  -> {Kc * Tc / (ms * 1e-3) / 1e9:.2f} G state-steps/s")
    eng.close()
