"""A/B of the window search (diagnostic tool, not product): the candidate
table (MPPI_SEARCH=table) against the default full scan, in ONE process on the
same inputs, batches interleaved.  Two regimes: the nominal held at run.py's
[10, -2] (no update: the samples leave the window) and the fused device loop
(the nominal converges and the samples hover around the window, as in bench.py).

    python tools/ab_search.py [K T batches launches_per_batch]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from mppi_robotarm_amd.engine import RolloutEngine  # noqa: E402
from mppi_robotarm_amd.params import X0_RUNPY, ArmParams  # noqa: E402


def engine(K, T, full):
    if full:
        os.environ.pop("MPPI_SEARCH", None)
    else:
        os.environ["MPPI_SEARCH"] = "table"
    e = RolloutEngine(K, T, 0.006, 100.0, 0.98, np.eye(2) * 20.0, [0.5, 0.5, 5, 5], [5, 5, 50, 50], 0.0,
                      ArmParams(), device=0)
    os.environ.pop("MPPI_SEARCH", None)
    return e


def main():
    a = [int(x) for x in sys.argv[1:]]
    K, T, nb, nl = (a + [65536, 64, 20, 200][len(a):])[:4]
    path = np.load(os.path.join(ROOT, "tests", "golden", "paths.npz"))["xydq_circle"][:, :4]
    torch.cuda.set_device(0)
    for fused in (False, True):
        engs = {}
        for full in (False, True):
            e = engine(K, T, full)
            e.set_step_inputs(X0_RUNPY, path[:30], np.tile([10.0, -2.0], (T, 1)))
            noise = [e.philox_noise(99, i) for i in range(8)]
            engs["full" if full else "table"] = (e, noise)
        times = {k: [] for k in engs}
        st = torch.cuda.current_stream()
        for b in range(nb + 3):
            for k, (e, noise) in engs.items():
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                for i in range(nl):
                    e.rollout(noise[i % 8], fused_update=fused)
                e1.record(st)
                e1.synchronize()
                if b >= 3:
                    times[k].append(e0.elapsed_time(e1) * 1e3 / nl)
        for k in engs:
            engs[k][0].synchronize()
        base = np.median(times["full"])
        print(f"{'fused' if fused else 'fixed'} K={K} T={T}: " + ", ".join(
            f"{k} {np.median(v):.2f} us (min {np.min(v):.2f}, x{np.median(v) / base:.3f})" for k, v in times.items()),
            flush=True)
        for e, _ in engs.values():
            e.close()


if __name__ == "__main__":
    main()
