"""Device NumPy-stream draw (include/mppi_rocm.h mppi_np_*): event time of one draw at config 3's size, and the
drop-in's calc_control_input with noise="numpy" (its default) back to back, device draw against host draw.
    python tools/npdraw_bench.py [K T [draw]]   (draw: the draw's timing only)"""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from mppi_robotarm_amd import hostrng  # noqa: E402
from mppi_robotarm_amd.engine import NpDeviceStream  # noqa: E402

K, T = (int(a) for a in sys.argv[1:3]) if len(sys.argv) > 2 else (65536, 64)
DRAW_ONLY = len(sys.argv) > 3 and sys.argv[3] == "draw"   # skip the drop-in legs (the host draw is slow at large K)
torch.cuda.set_device(0)
nd = NpDeviceStream(torch.device("cuda", 0))
sigma = np.eye(2) * 20.0
plan = hostrng.device_plan(np.zeros(2), sigma)
out = torch.empty((T, K, 2), dtype=torch.float32, device="cuda")
s = torch.cuda.current_stream()
np.random.seed(0)
t_first = time.perf_counter()
nd.draw(np.random.get_state(), (K, T, 2), plan, out, s.cuda_stream, 0, K, (2 * K, 2, 1))
np.random.set_state(nd.result())
print(f"first draw (jump polynomials, buffers): {(time.perf_counter() - t_first) * 1e3:.1f} ms")
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
dev, wall = [], []
for i in range(30):
    t0 = time.perf_counter()
    ev[0].record(s)
    nd.draw(np.random.get_state(), (K, T, 2), plan, out, s.cuda_stream, 0, K, (2 * K, 2, 1))
    ev[1].record(s)
    np.random.set_state(nd.result())
    wall.append(time.perf_counter() - t0)
    dev.append(ev[0].elapsed_time(ev[1]))
print(f"device draw K={K} T={T}: events median {np.median(dev[5:]):.3f} ms, wall median "
      f"{np.median(wall[5:]) * 1e3:.3f} ms (get_state / set_state included)")
nd.close()
if DRAW_ONLY:
    sys.exit(0)

from mppi_robotarm_amd.controller import MPPIControllerForPathTracking  # noqa: E402
from mppi_robotarm_amd.params import X0_RUNPY, runpy_config  # noqa: E402
path = np.load(__file__.rsplit("/tools/", 1)[0] + "/tests/golden/paths.npz")["xydq_circle"][:, :4]
for on_dev in (True, False):
    kw = runpy_config()
    kw.update(number_of_samples_K=K, horizon_step_T=T, visualze_sampled_trajs=False)
    c = MPPIControllerForPathTracking(ref_path=path, noise="numpy", verbose=False, device=0,
                                      numpy_noise_on_device=on_dev, **kw)
    np.random.seed(0)
    ts = []
    for i in range(25):
        c.prev_waypoints_idx = 0
        t0 = time.perf_counter()
        c.calc_control_input(X0_RUNPY)
        ts.append(time.perf_counter() - t0)
    print(f"calc_control_input noise='numpy' ({'device' if on_dev else 'host'} draw): "
          f"median {np.median(ts[5:]) * 1e3:.3f} ms")
    c.close()
