"""Diagnostic: one shard's partial row {rho, eta, N} from the device direct merge
against the same sums on the host from the shard's S and noise."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np, torch
from mppi_robotarm_amd.engine import RolloutEngine
from mppi_robotarm_amd.params import ArmParams, X0_RUNPY
torch.cuda.set_device(0)
path = np.load(os.path.join(ROOT, "tests", "golden", "paths.npz"))["xydq_circle"][:, :4]
K, T, lam = int(sys.argv[1]), int(sys.argv[2]), float(sys.argv[3])
e = RolloutEngine(K, T, 0.006, lam, 0.95, np.eye(2) * 20, [.5, .5, 5, 5], [5, 5, 50, 50], 0.0, ArmParams(), device=0)
print("lps", e.lanes_per_sample, "blocks", e.blocks, "threads", e.threads, e.handoff)
e.set_step_inputs(X0_RUNPY, path[:30], np.array([[10.0, -2.0]] * T))
nz = e.philox_noise(99, 1)
part = e.new_partial()
S = torch.empty(K, dtype=torch.float64, device="cuda")
e.rollout(nz, S_out=S, partial_out=part)
torch.cuda.synchronize()
p = part.cpu().numpy(); S = S.cpu().numpy(); eps = nz.cpu().numpy().astype(np.float64)   # [T][K][2]
rho = S.min(); w = np.exp(-(S - rho) / lam)
eta = w.sum(); N = np.einsum("k,tkd->td", w, eps).ravel()
print("rho", p[0], rho, "eta rel", abs(p[1] - eta) / eta)
rel = np.abs(p[2:] - N) / np.maximum(np.abs(N), 1e-30)
bad = np.argwhere(rel > 1e-6).ravel()
print("bad N columns", bad.tolist(), "max rel", rel.max())
