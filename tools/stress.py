"""Endurance run (diagnostic, not a test): N fused device steps at c3 and c5,
checking after every chunk that no in-launch hand-off timed out and that the
nominal stays finite; then the bench line's throughput over the whole run.

    python tools/stress.py [steps]     (default 20000 arm steps, 2000 chain steps)
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from mppi_robotarm_amd.engine import RolloutEngine  # noqa: E402
from mppi_robotarm_amd.params import X0_RUNPY, ArmParams  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
torch.cuda.set_device(0)
path = np.load(os.path.join(ROOT, "tests", "golden", "paths.npz"))["xydq_circle"][:, :4]


def run(eng, steps, x0, u, label, chunk=1000, reset=0):
    """reset: re-stage the start nominal every `reset` steps (bench.py's c5 loop: the plant-less chain loop
    drifts into overflowing rollouts otherwise, tools/loop_drift.py)."""
    eng.set_step_inputs(x0, path[:30], u)
    noise = [eng.philox_noise(7, i) for i in range(8)]
    t0 = time.perf_counter()
    done = 0
    while done < steps:
        for i in range(min(chunk, steps - done)):
            if reset and (done + i) % reset == 0:
                eng.set_step_inputs(x0, path[:30], u)
            eng.rollout(noise[(done + i) % 8], fused_update=True)
        done += min(chunk, steps - done)
        eng.synchronize()                      # raises on a hand-off timeout
        assert np.all(np.isfinite(eng.nominal())), f"{label}: non-finite nominal after {done} steps"
    dt = time.perf_counter() - t0
    print(f"{label}: {steps} fused steps, {dt / steps * 1e6:.1f} us/step incl. chunk syncs, no timeout, finite",
          flush=True)


arm = RolloutEngine(65536, 64, 0.006, 100.0, 0.98, np.eye(2) * 20.0, [0.5, 0.5, 5, 5], [5, 5, 50, 50], 0.0,
                    ArmParams(), device=0)
run(arm, n, X0_RUNPY, np.array([[10.0, -2.0]] * 64), "c3 K=65536 T=64")
arm.close()
from mppi_robotarm_amd.chain import CHAIN7_SIGMA, CHAIN7_X0, ChainEngine, gravity_torque  # noqa: E402
ch = ChainEngine(131072, 128, 0.006, 100.0, 0.98, CHAIN7_SIGMA, [0.5, 0.5, 5, 5], [5, 5, 50, 50], 0.0, device=0)
run(ch, max(1, n // 10), CHAIN7_X0, np.tile(gravity_torque(CHAIN7_X0[:7]), (128, 1)), "c5 K=131072 T=128", chunk=200,
    reset=32)
ch.close()
# config 5's 8-way shard: a quad per sample
ch = ChainEngine(16384, 128, 0.006, 100.0, 0.98, CHAIN7_SIGMA, [0.5, 0.5, 5, 5], [5, 5, 50, 50], 0.0, device=0)
assert ch.lanes_per_sample == 4
run(ch, max(1, n // 10), CHAIN7_X0, np.tile(gravity_torque(CHAIN7_X0[:7]), (128, 1)), "c5 shard K=16384 T=128 (quad)",
    chunk=200, reset=32)
ch.close()
