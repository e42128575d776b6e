"""Where the drop-in's time goes with the default NumPy noise (device draw): host time of each part of
calc_control_input, wrapped method by method, back to back at config 3."""
import sys
import time
from collections import defaultdict

import numpy as np

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from mppi_robotarm_amd.controller import MPPIControllerForPathTracking  # noqa: E402
from mppi_robotarm_amd.params import X0_RUNPY, runpy_config  # noqa: E402

acc = defaultdict(list)


def wrap(cls, name):
    f = getattr(cls, name)

    def g(*a, **k):
        t0 = time.perf_counter()
        try:
            return f(*a, **k)
        finally:
            acc[name].append(time.perf_counter() - t0)
    setattr(cls, name, g)


C = MPPIControllerForPathTracking
for n in ("_settle_predraw", "_device_reference_noise", "_dropin_step", "_queue_predraw", "_get_nearest_waypoint",
          "_get_engine"):
    wrap(C, n)
path = np.load(__file__.rsplit("/tools/", 1)[0] + "/tests/golden/paths.npz")["xydq_circle"][:, :4]
kw = runpy_config()
kw.update(number_of_samples_K=65536, horizon_step_T=64, visualze_sampled_trajs=False)
c = C(ref_path=path, noise="numpy", verbose=False, device=0, **kw)
np.random.seed(0)
tot = []
for i in range(30):
    c.prev_waypoints_idx = 0
    t0 = time.perf_counter()
    c.calc_control_input(X0_RUNPY)
    tot.append(time.perf_counter() - t0)
    if i == 9:
        acc.clear()
        tot.clear()
print(f"calc_control_input median {np.median(tot) * 1e3:.3f} ms; queued draws used {c._npre_used}")
for k, v in acc.items():
    print(f"  {k:26s} median {np.median(v) * 1e3:.3f} ms x {len(v)}")
c.close()
