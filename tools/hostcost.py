"""Diagnostic: host cost of one launch through RolloutEngine.rollout vs a raw
ctypes call, and the device time per step each launch loop sustains (does the
host loop keep the GPU queue full?).  python tools/hostcost.py [K T]"""
import ctypes as C
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from mppi_robotarm_amd import _native as N  # noqa: E402
from mppi_robotarm_amd.engine import RolloutEngine  # noqa: E402
from mppi_robotarm_amd.params import X0_RUNPY, ArmParams  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
T = int(sys.argv[2]) if len(sys.argv) > 2 else 64
torch.cuda.set_device(0)
eng = RolloutEngine(K, T, 0.006, 100.0, 0.98, np.eye(2) * 20.0, [0.5, 0.5, 5, 5], [5, 5, 50, 50], 0.0, ArmParams(),
                    device=0)
path = np.load(os.path.join(ROOT, "tests", "golden", "paths.npz"))["xydq_circle"][:, :4]
eng.set_step_inputs(X0_RUNPY, path[:30], np.array([[10.0, -2.0]] * T))
stream = torch.cuda.current_stream()


def run(nbuf, mode, n=400):
    noise = [eng.philox_noise(1234, i) for i in range(nbuf)]
    ptrs = [C.c_void_p(z.data_ptr()) for z in noise]
    fn, ctx, fl = eng._lib.mppi_rollout, eng._ctx, N.MPPI_FLAG_FUSED_UPDATE
    for i in range(20):
        eng.rollout(noise[i % nbuf], fused_update=True)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    h0 = time.perf_counter()
    e0.record(stream)
    if mode == "engine":
        for i in range(n):
            eng.rollout(noise[i % nbuf], fused_update=True)
    else:
        for i in range(n):
            fn(ctx, ptrs[i % nbuf], None, None, fl)
    e1.record(stream)
    h1 = time.perf_counter()
    torch.cuda.synchronize()
    print(f"nbuf {nbuf:2d} {mode:6s}: host {1e6 * (h1 - h0) / n:6.1f} us/launch, device {1e3 * e0.elapsed_time(e1) / n:6.2f} us/step")


for nbuf in (8, 10):
    for mode in ("engine", "raw"):
        run(nbuf, mode)
