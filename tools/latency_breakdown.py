"""Where the drop-in's control-step latency goes (diagnostic tool, not product):
the phases of MPPIControllerForPathTracking.calc_control_input at the bench's
K, T with device noise, timed on the host with a device sync after each phase
(so each phase's GPU time lands in its own line), plus the untouched call.

    python tools/latency_breakdown.py [K T calls]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from mppi_robotarm_amd.controller import MPPIControllerForPathTracking  # noqa: E402
from mppi_robotarm_amd.params import X0_RUNPY, runpy_config  # noqa: E402


def main():
    a = [int(x) for x in sys.argv[1:]]
    K, T, n = (a + [65536, 64, 60][len(a):])[:3]
    torch.cuda.set_device(0)
    path = np.load(os.path.join(ROOT, "tests", "golden", "paths.npz"))["xydq_circle"][:, :4]
    kw = runpy_config()
    kw.update(number_of_samples_K=K, horizon_step_T=T, visualze_sampled_trajs=False)
    c = MPPIControllerForPathTracking(ref_path=path, noise="device", seed=0, verbose=False, device=0, **kw)
    x = X0_RUNPY.copy()
    whole = []
    for i in range(n):
        t0 = time.perf_counter()
        c.calc_control_input(x)
        whole.append(time.perf_counter() - t0)
        c.prev_waypoints_idx = 0
    eng = c._get_engine()
    sync = torch.cuda.synchronize
    ph = {k: [] for k in ("waypoint", "philox", "set_inputs", "rollout", "w_eps D2H", "median+update", "opt traj")}
    u = c.u_prev.copy()
    for i in range(n):
        t = time.perf_counter()
        c._get_nearest_waypoint(x[0], x[1], update_prev_idx=True)
        t1 = time.perf_counter(); ph["waypoint"].append(t1 - t)
        eng.philox_noise(0, i, out=c._noise_dev); sync()
        t2 = time.perf_counter(); ph["philox"].append(t2 - t1)
        eng.set_step_inputs(x, path[0:30], u); sync()
        t3 = time.perf_counter(); ph["set_inputs"].append(t3 - t2)
        eng.rollout(c._noise_dev); sync()
        t4 = time.perf_counter(); ph["rollout"].append(t4 - t3)
        w = eng.weighted_noise()
        t5 = time.perf_counter(); ph["w_eps D2H"].append(t5 - t4)
        w = c._moving_median_filter(xx=w, window_size=10)
        uu = u + w
        t6 = time.perf_counter(); ph["median+update"].append(t6 - t5)
        eng.trajectories(base_u=uu, K=1)[0].double().cpu().numpy()
        t7 = time.perf_counter(); ph["opt traj"].append(t7 - t6)
    print(f"K={K} T={T}: calc_control_input median {np.median(whole) * 1e3:.3f} ms")
    for k, v in ph.items():
        print(f"  {k:14s} {np.median(v) * 1e6:8.1f} us")
    c.close()


if __name__ == "__main__":
    main()
