"""ChainMPPIController.calc_control_input wall time (config 5: K = 131072, T = 128, device noise), back to
back from a fixed state, with the per-phase split of one call.  python tools/chain_latency.py [K] [calls]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from mppi_robotarm_amd.chain import CHAIN7_X0, ChainMPPIController, gravity_torque  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 131072
n = int(sys.argv[2]) if len(sys.argv) > 2 else 40
torch.cuda.set_device(0)
path = np.load(os.path.join(ROOT, "tests", "golden", "paths.npz"))["xydq_circle"][:, :4]
for vis in (True, False):
    c = ChainMPPIController(0.006, path, 128, K, u_init=gravity_torque(CHAIN7_X0[:7]), device=0, noise="device",
                            visualize_optimal_traj=vis)
    u0 = c.u_prev.copy()
    ts = []
    for i in range(n + 5):
        c.u_prev[:] = u0            # the same start nominal each call (no plant: keeps the loop bounded)
        c.prev_waypoints_idx = 0
        t0 = time.perf_counter()
        c.calc_control_input(CHAIN7_X0)
        ts.append(time.perf_counter() - t0)
    c.close()
    ts = np.array(ts[5:]) * 1e6
    print(f"K={K} T=128 n=7 device noise, optimal_traj={vis}: back to back median {np.median(ts):8.1f} us "
          f"(p90 {np.percentile(ts, 90):8.1f})", flush=True)

# phases of one back-to-back call (host wall time of each engine call, the rest is Python), then the
# device time of the draw and of the fused launch alone (HIP events on the engine's stream)
c = ChainMPPIController(0.006, path, 128, K, u_init=gravity_torque(CHAIN7_X0[:7]), device=0, noise="device")
u0 = c.u_prev.copy()
c.calc_control_input(CHAIN7_X0)
eng = c._engine
acc = {}


def timed(name, fn):
    def w(*a, **k):
        t0 = time.perf_counter()
        out = fn(*a, **k)
        acc.setdefault(name, []).append(time.perf_counter() - t0)
        return out
    return w


for name in ("philox_noise", "set_step_inputs", "rollout", "wait_outputs"):
    setattr(eng, name, timed(name, getattr(eng, name)))
whole = []
for i in range(n):
    c.u_prev[:] = u0
    c.prev_waypoints_idx = 0
    t0 = time.perf_counter()
    c.calc_control_input(CHAIN7_X0)
    whole.append(time.perf_counter() - t0)
print(f"  whole call {np.median(whole) * 1e6:8.1f} us; engine calls (host wall time, medians):", flush=True)
tot = 0.0
for name, v in acc.items():
    m = float(np.median(v[-n:])) * 1e6
    tot += m
    print(f"    {name:16s} {m:8.1f} us", flush=True)
print(f"    Python / NumPy rest {np.median(whole) * 1e6 - tot:8.1f} us", flush=True)
s = torch.cuda.current_stream()
ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
kp, kr = [], []
for i in range(20):
    ev[0].record(s)
    eng.philox_noise(1, i, out=c._noise_dev)
    ev[1].record(s)
    eng.rollout(c._noise_dev)
    ev[2].record(s)
    torch.cuda.synchronize()
    kp.append(ev[0].elapsed_time(ev[1]) * 1e3)
    kr.append(ev[1].elapsed_time(ev[2]) * 1e3)
print(f"  device: Philox draw {np.median(kp):8.1f} us, rollout {np.median(kr):8.1f} us", flush=True)
c.close()
