"""The drop-in with its default noise="numpy" (the reference's own RNG stream) at K = 65536, T = 64: the draw by
NumPy and by hostrng (threaded, same values; checked equal here on this host's libm), and calc_control_input's
wall time.  python tools/numpy_noise_latency.py"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from mppi_robotarm_amd import hostrng  # noqa: E402
from mppi_robotarm_amd.controller import MPPIControllerForPathTracking  # noqa: E402
from mppi_robotarm_amd.params import X0_RUNPY, runpy_config  # noqa: E402

K, T = 65536, 64
S = np.eye(2) * 20.0
print(f"host threads used by hostrng: {hostrng._threads()}", flush=True)


def med(fn, n=7):
    v = []
    for _ in range(n):
        t0 = time.perf_counter()
        fn()
        v.append(time.perf_counter() - t0)
    return np.median(v[1:]) * 1e3


for seed in (0, 1, 2):
    np.random.seed(seed)
    a = np.random.multivariate_normal(np.zeros(2), S, (K, T))
    sa = np.random.get_state()
    np.random.seed(seed)
    b = hostrng.multivariate_normal(np.zeros(2), S, (K, T))
    sb = np.random.get_state()
    same = np.array_equal(a, b) and np.array_equal(sa[1], sb[1]) and sa[2:] == sb[2:]
    print(f"seed {seed}: hostrng equals NumPy (values and state): {same}", flush=True)
    assert same
print(f"np.random.multivariate_normal      {med(lambda: np.random.multivariate_normal(np.zeros(2), S, (K, T))):8.2f} ms")
print(f"hostrng.multivariate_normal        {med(lambda: hostrng.multivariate_normal(np.zeros(2), S, (K, T))):8.2f} ms")
zbuf = torch.empty(K * T * 2, dtype=torch.float64).pin_memory().numpy()
print(f"hostrng.legacy_standard_normal     {med(lambda: hostrng.legacy_standard_normal(K * T * 2, out=zbuf)):8.2f} ms"
      "  (the drop-in's draw: standard normals into a page-locked buffer)")
print(f"hostrng.multivariate_normal_std    {med(lambda: hostrng.multivariate_normal_std(np.zeros(2), S, (K, T), zbuf)):8.2f} ms"
      "  (+ NumPy's svd / checks of Sigma)")
torch.cuda.set_device(0)
path = np.load(os.path.join(ROOT, "tests", "golden", "paths.npz"))["xydq_circle"][:, :4]
kw = runpy_config()
kw.update(number_of_samples_K=K, horizon_step_T=T, visualze_sampled_trajs=False)
c = MPPIControllerForPathTracking(ref_path=path, verbose=False, device=0, **kw)   # noise="numpy", the default


def call():
    c.prev_waypoints_idx = 0
    c.calc_control_input(X0_RUNPY)


print(f"calc_control_input, noise='numpy'  {med(call, 9):8.2f} ms", flush=True)
c.close()
