"""Endurance of the drop-in's NumPy-noise path with the queued draw: N back-to-back calls at config 3 on the device
draw against the host-draw twin (numpy_noise_on_device=False), the caller touching np.random every 97th call;
the nominals and the final RNG state must be equal bit for bit."""
import sys
import time

import numpy as np

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from mppi_robotarm_amd.controller import MPPIControllerForPathTracking  # noqa: E402
from mppi_robotarm_amd.params import X0_RUNPY, runpy_config  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 500
path = np.load(__file__.rsplit("/tools/", 1)[0] + "/tests/golden/paths.npz")["xydq_circle"][:, :4]


def run(on_dev):
    kw = runpy_config()
    kw.update(number_of_samples_K=65536, horizon_step_T=64, visualze_sampled_trajs=False)
    c = MPPIControllerForPathTracking(ref_path=path, noise="numpy", verbose=False, device=0,
                                      numpy_noise_on_device=on_dev, **kw)
    np.random.seed(3)
    us, ts = [], []
    for i in range(N):
        if i % 97 == 96:
            np.random.rand(1)
        c.prev_waypoints_idx = 0
        t0 = time.perf_counter()
        us.append(c.calc_control_input(X0_RUNPY)[1].copy())
        ts.append(time.perf_counter() - t0)
    dt = float(np.median(ts[10:]))
    hits = getattr(c, "_npre_used", 0)
    c.close()
    return np.array(us), np.random.get_state(), dt, hits


a, sa, ta, hits = run(True)
b, sb, tb, _ = run(False)
same = np.array_equal(a, b) and np.array_equal(sa[1], sb[1]) and sa[2:] == sb[2:]
print(f"{N} calls: device draw median {ta * 1e3:.3f} ms/call ({hits} queued draws used), host draw "
      f"{tb * 1e3:.3f} ms/call; nominals and RNG state equal: {same}; finite: {bool(np.isfinite(a).all())}")
sys.exit(0 if same and np.isfinite(a).all() else 1)
