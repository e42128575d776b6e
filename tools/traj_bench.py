"""Time the sampled-trajectory re-roll (traj_kernel / chain_traj_kernel) at a
full bench size (diagnostic tool, not product): HIP events around repeated
mppi_rollout_traj launches on the engine's stream.

    python tools/traj_bench.py [LIB.so]            (arm, K=65536 T=64)
    WORKLOAD=c5 python tools/traj_bench.py [LIB.so] (7-link chain, K=131072 T=128)
"""
import os
import sys

if len(sys.argv) > 1:
    os.environ["MPPI_LIB_PATH"] = os.path.abspath(sys.argv[1])
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

torch.cuda.set_device(0)
path = np.load(os.path.join(ROOT, "tests", "golden", "paths.npz"))["xydq_circle"][:, :4]
if os.environ.get("WORKLOAD") == "c5":
    from mppi_robotarm_amd.chain import CHAIN7_SIGMA, CHAIN7_X0, ChainEngine, gravity_torque
    K, T, W = 131072, 128, 14
    eng = ChainEngine(K, T, 0.006, 100.0, 0.98, CHAIN7_SIGMA, [0.5, 0.5, 5, 5], [5, 5, 50, 50], 0.0, device=0)
    eng.set_step_inputs(CHAIN7_X0, path[:30], np.tile(gravity_torque(CHAIN7_X0[:7]), (T, 1)))
else:
    from mppi_robotarm_amd.engine import RolloutEngine
    from mppi_robotarm_amd.params import X0_RUNPY, ArmParams
    K, T, W = 65536, 64, 4
    eng = RolloutEngine(K, T, 0.006, 100.0, 0.98, np.eye(2) * 20.0, [0.5, 0.5, 5, 5], [5, 5, 50, 50], 0.0,
                        ArmParams(), device=0)
    eng.set_step_inputs(X0_RUNPY, path[:30], np.array([[10.0, -2.0]] * T))
noise = eng.philox_noise(3, 0)
for _ in range(3):
    eng.trajectories(noise=noise)
torch.cuda.synchronize()
n = 20
s = torch.cuda.current_stream()
t = []
for _ in range(n):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(s)
    eng.trajectories(noise=noise)
    b.record(s)
    torch.cuda.synchronize()
    t.append(a.elapsed_time(b) * 1e3)
us = float(np.median(t))
wbytes = K * T * W * 4
rbytes = K * T * (W // 2 if W == 14 else 2) * 4 // (1 if W == 14 else 1)
print(f"K={K} T={T} traj median {us:.1f} us (min {min(t):.1f}); writes {wbytes / 1e6:.1f} MB -> "
      f"{wbytes / us / 1e3:.0f} GB/s; + noise reads {rbytes / 1e6:.1f} MB; total {(wbytes + rbytes) / us / 1e3:.0f} GB/s")
