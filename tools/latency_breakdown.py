"""Where the drop-in's control-step latency goes (diagnostic tool, not product).

MPPIControllerForPathTracking.calc_control_input at the bench's K, T with device
noise, on the one-call tick (mppi_dropin_tick_launch / _wait: native waypoint update, inputs
staged as kernel arguments, fused launch, wait, host trajectory, next noise):

  * closed loop: run.py's driver (harness), plant work between ticks — the
    bench's control_step_latency_ms;
  * back to back: calls with nothing in between (the next step's Philox draw,
    queued behind each call, is then paid by the following call);
  * phases of one call: Python before the native call (checks, engine lookup,
    buffer binding check), the native call (waypoint update + stage + launch +
    queue the next noise + wait + host trajectory), Python after; the device work alone (one fused
    rollout launch, and one Philox draw, HIP-event timed on the stream).

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
from mppi_robotarm_amd.harness import run_closed_loop  # noqa: E402
from mppi_robotarm_amd.params import X0_RUNPY, runpy_config  # noqa: E402


def us(v):
    return f"{np.median(v) * 1e6:8.1f} us (p90 {np.percentile(v, 90) * 1e6:7.1f})"


def main():
    a = [int(x) for x in sys.argv[1:]]
    K, T, n = (a + [65536, 64, 200][len(a):])[:3]
    torch.cuda.set_device(0)
    path = np.load(os.path.join(ROOT, "tests", "golden", "paths.npz"))["xydq_circle"][:, :4]
    kw = runpy_config()
    kw.update(number_of_samples_K=K, horizon_step_T=T, visualze_sampled_trajs=False)

    run_closed_loop(path, ticks=100, noise="device", seed=0, verbose=False, device=0, **kw)["controller"].close()
    cl_phases = []
    ctl = {}

    def on_tick(k, state, u):   # the native phase ends of the tick just run (the controller's engine)
        eng_ = ctl["c"]._engine if "c" in ctl else None
        if eng_ is not None and k > 3:
            cl_phases.append(eng_.dropin_times() * 1e-6)

    from mppi_robotarm_amd.controller import MPPIControllerForPathTracking as _C
    ctl["c"] = _C(ref_path=path, noise="device", seed=0, verbose=False, device=0, **kw)
    rec = run_closed_loop(path, ticks=n, controller=ctl["c"], on_tick=on_tick)
    ctl["c"].close()
    closed = rec["latency_s"][3:]
    cl_phases = np.array(cl_phases)

    c = MPPIControllerForPathTracking(ref_path=path, noise="device", seed=0, verbose=False, device=0, **kw)
    x = X0_RUNPY.copy()
    for _ in range(5):
        c.calc_control_input(x)
        c.prev_waypoints_idx = 0
    eng = c._get_engine()
    stamps = {}
    launch, wait = eng.dropin_tick_launch, eng.dropin_tick_wait

    def t_launch(*args):
        stamps["l0"] = time.perf_counter()
        out = launch(*args)
        stamps["l1"] = time.perf_counter()
        return out

    def t_wait():
        stamps["w0"] = time.perf_counter()
        wait()
        stamps["w1"] = time.perf_counter()

    eng.dropin_tick_launch, eng.dropin_tick_wait = t_launch, t_wait
    whole, pre, nat, mid, wt, post = [], [], [], [], [], []
    for _ in range(n):
        c.prev_waypoints_idx = 0
        t0 = time.perf_counter()
        c.calc_control_input(x)
        t3 = time.perf_counter()
        whole.append(t3 - t0)
        pre.append(stamps["l0"] - t0)
        nat.append(stamps["l1"] - stamps["l0"])
        mid.append(stamps["w0"] - stamps["l1"])
        wt.append(stamps["w1"] - stamps["w0"])
        post.append(t3 - stamps["w1"])
    eng.dropin_tick_launch, eng.dropin_tick_wait = launch, wait
    phases = []
    for _ in range(n):
        c.prev_waypoints_idx = 0
        c.calc_control_input(x)
        phases.append(eng.dropin_times() * 1e-6)
    phases = np.array(phases)

    # device work alone, HIP events on the engine's stream
    s = torch.cuda.current_stream()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    kern, phil = [], []
    for _ in range(50):
        ev[0].record(s)
        eng.rollout(c._noise_dev, fused_update=True)
        ev[1].record(s)
        eng.philox_noise(0, 1, out=c._noise_dev)
        ev[2].record(s)
        torch.cuda.synchronize()
        kern.append(ev[0].elapsed_time(ev[1]) * 1e-3)
        phil.append(ev[1].elapsed_time(ev[2]) * 1e-3)
    c.close()

    print(f"K={K} T={T}, device noise, one-call drop-in tick (mppi_dropin_tick), {n} calls")
    print(f"  closed loop (run.py driver, plant between ticks) {us(closed)}")
    print(f"  back to back (no work between calls)             {us(whole)}")
    print(f"    Python before the native launch                {us(pre)}")
    print(f"    native launch (waypoint, stage, launch, noise) {us(nat)}")
    print(f"    Python between (sampled_traj_list zeros)       {us(mid)}")
    print(f"    native wait (+ fp64 optimal trajectory)        {us(wt)}")
    print(f"    Python after                                   {us(post)}")
    names = ["waypoint update + stage inputs (host keys)", "launch fused rollout", "queue next Philox draw",
             "wait for the rollout's outputs", "copy outputs + fp64 optimal trajectory"]
    prev = np.zeros(len(phases))
    for i, nm in enumerate(names):
        print(f"      native: {nm:43s}{us(phases[:, i] - prev)}")
        prev = phases[:, i]
    print("  closed loop, native phases of the same ticks:")
    prev = np.zeros(len(cl_phases))
    for i, nm in enumerate(names):
        print(f"      native: {nm:43s}{us(cl_phases[:, i] - prev)}")
        prev = cl_phases[:, i]
    print(f"  device: fused rollout launch                     {us(kern)}")
    print(f"  device: Philox draw of the next step's noise     {us(phil)}")


if __name__ == "__main__":
    main()
