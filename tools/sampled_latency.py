"""The drop-in with run.py's own visualze_sampled_trajs=True at K = 65536, T = 64 (device noise): wall time
of calc_control_input back to back, and the cost of materialising the (K, T, 4) fp64 sampled_traj_list
(134 MB) on the host by three routes.  python tools/sampled_latency.py"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from mppi_robotarm_amd.controller import MPPIControllerForPathTracking  # noqa: E402
from mppi_robotarm_amd.params import X0_RUNPY, runpy_config  # noqa: E402

K, T = 65536, 64
torch.cuda.set_device(0)
path = np.load(os.path.join(ROOT, "tests", "golden", "paths.npz"))["xydq_circle"][:, :4]
kw = runpy_config()
kw.update(number_of_samples_K=K, horizon_step_T=T)     # visualze_sampled_trajs=True, as run.py
c = MPPIControllerForPathTracking(ref_path=path, noise="device", seed=0, verbose=False, device=0, **kw)
ts = []
for i in range(25):
    c.prev_waypoints_idx = 0
    t0 = time.perf_counter()
    out = c.calc_control_input(X0_RUNPY)
    ts.append(time.perf_counter() - t0)
    del out
print(f"calc_control_input with sampled trajectories: median {np.median(ts[5:]) * 1e3:7.2f} ms", flush=True)
tr = c._engine.trajectories(base_u=None, noise=c._noise_dev)
torch.cuda.synchronize()


def t(name, fn, n=10):
    v = []
    for _ in range(n):
        t0 = time.perf_counter()
        r = fn()
        v.append(time.perf_counter() - t0)
        del r
    print(f"  {name:48s} {np.median(v) * 1e3:7.2f} ms", flush=True)


t("trajectory launch + sync", lambda: (c._engine.trajectories(base_u=None, noise=c._noise_dev), torch.cuda.synchronize()))
t("np.zeros + [:] = tr.double().cpu().numpy()", lambda: np.zeros((K, T, 4)).__setitem__(slice(None), tr.double().cpu().numpy()))
t("tr.double().cpu().numpy()", lambda: tr.double().cpu().numpy())
t("tr.cpu().numpy().astype(float64)", lambda: tr.cpu().numpy().astype(np.float64))
pin = torch.empty((K, T, 4), dtype=torch.float64, pin_memory=True)
t("double() into a reused pinned buffer + numpy copy", lambda: pin.copy_(tr.double()).numpy().copy())
c.close()
