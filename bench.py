#!/usr/bin/env python3
"""Benchmark of the MPPI rollout-and-reduce hot path (BASELINE.json metric).

One "step" = one full MPPI control step of the hot path on device over one
batch of synthetic noise: K x T rollouts + running / terminal cost + soft-min
weights + weighted noise sum (control.py:81-118) + median filter, u += w_eps
and shift (control.py:122-149), so consecutive steps chain on the updated
nominal control exactly like the reference's receding horizon.  N = 1: one
launch per step (fused last-workgroup update).  N > 1 (torchrun, one process
per GPU, RCCL): rollout launch -> one all_gather of the 130-double device
partials over xGMI -> merge + update launch.  Weak scaling: K per GPU is fixed
(default 65536 = BASELINE config 3 at N = 1, config 4's K = 524288 at N = 8).

Inputs: run.py constants (dt 0.006, lambda 100, alpha 0.98, Sigma 20 I,
weights [.5 .5 5 5] / [5 5 50 50]), start pose of run.py, the first window of
xydq_circle.txt, noise N(0, Sigma) from the device Philox generator, 10
distinct buffers rotated so their total (335 MB at K=65536 T=64) exceeds the
256 MiB Infinity Cache.  Everything is resident in HBM before timing starts.

``--workload c2``: BASELINE config 2's size on the same 2-DoF path (K=4096
T=32, 10 noise buffers of 1 MiB: they stay in the Infinity Cache, as a
controller's one redrawn buffer would).  ``c3`` remains the headline line.

``--workload c5``: BASELINE config 5 instead — the 7-DoF chain
(mppi_robotarm_amd/chain.py, build-defined model) at K=131072 T=128, strong
scaling (K fixed, split over the ranks), 28 B of noise per state-step, the
config-5 start pose on xydq_circle.txt and gravity-holding nominal torques.

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from mppi_robotarm_amd.distributed import attach_exchange, check_exchange, exchange_partials  # noqa: E402
from mppi_robotarm_amd.engine import RolloutEngine  # noqa: E402
from mppi_robotarm_amd.params import ArmParams, X0_RUNPY  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
BYTES_PER_STATE_STEP = 8  # fp32 eps[t][k][0:2] read once
C5_BYTES_PER_STATE_STEP = 28  # fp32 eps[t][0:7][k] read once ("C5 (du=7): 28 B/state-step")
# VALU issue roofline (SURVEY §8d asks for it beside the HBM one), priced against this chip's measured issue
# rates: tools/ubench_issue.hip (profiles/ubench_issue.json) times independent instruction streams of the c3
# horizon loop's mix with 1, 2 and 4 waves on every SIMD of the chip (the clock the chip picks under that load),
# in nanoseconds per wave-instruction.  One wave alone on its SIMD (the c3 launch: 1024 waves on 1024 SIMDs)
# issues the mix at one instruction per ~2.9 ns (~7 cycles at the 2.39 GHz s_memtime rate the same run reports);
# the SIMD saturates near one per ~1.8 ns with four.  The guide's 2- and 4-cycle figures are single-class
# streams; the mix (packed FMAs, transcendentals) is what the loop issues.
SIMDS = 1024
UBENCH_JSON = os.path.join(ROOT, "profiles", "ubench_issue.json")


def issue_ceilings(path=UBENCH_JSON):
    """(lone-wave, SIMD-saturated) ns per instruction per SIMD for the c3 mix, from the committed ubench run."""
    try:
        rows = json.load(open(path))["rows"]
        mix = {r["waves_per_simd"]: r["event_ns_per_inst_wave"] for r in rows if r["op"] == "c3_mix"}
        return mix[1], min(ns / w for w, ns in mix.items())
    except Exception:
        return None


def valu_roofline(tj, kern_ms):
    """VALU issue roofline of the rollout launch: the PMC count in the traffic json (SQ_INSTS_VALU, whole device,
    per launch; tools/traffic_summary.py) over this run's kernel time, per SIMD, against the measured issue rates
    of issue_ceilings() (profiles/ubench_issue.json)."""
    n = tj.get("valu_insts_per_launch") if tj else None
    waves = tj.get("waves_per_launch") if tj else None
    ceil = issue_ceilings()
    if not n or not waves or ceil is None:
        return None
    lone_ns, simd_ns = ceil
    # wave-instructions each busy SIMD issues (waves are spread evenly, <= 1 workgroup per CU; c2's 512 waves
    # leave half the SIMDs empty)
    per_simd = n / min(waves, SIMDS)
    achieved = per_simd / (kern_ms * 1e6)   # wave-instructions per SIMD per ns
    out = {"bound": "valu-issue", "achieved": achieved, "peak": 1.0 / simd_ns, "unit": "wave-instr/SIMD/ns",
           "frac": achieved * simd_ns, "waves_per_simd": waves / SIMDS, "busy_simds": min(waves, SIMDS), "valu_insts_per_launch": n,
           "source": "SQ_INSTS_VALU (" + str(tj.get("source", "")).split("; ")[-1] + "), live kernel time; peak and "
                     "lone-wave ceiling: the c3 mix in profiles/ubench_issue.json (tools/ubench_issue.hip)"}
    if waves / SIMDS <= 1.0:
        # one wave per SIMD cannot reach the SIMD's rate: its own measured ceiling
        out["lone_wave_ceiling"] = 1.0 / lone_ns
        out["frac_one_wave_ceiling"] = achieved * lone_ns
    for key in ("valu_active_frac_of_wave_time", "cycles_per_valu_inst"):
        if tj.get(key) is not None:
            out[key] = tj[key]   # SQ_ACTIVE_INST_VALU of the committed PMC pass (how busy the VALU is)
    return out


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=1000)
    p.add_argument("--warmup", type=int, default=100)
    p.add_argument("--settle-ms", type=float, default=200.0,
                   help="untimed steps for this long before the W warmup steps: the GPU clock takes ~0.1 s of "
                        "load to ramp (measured: 33.4 us/step after 20 warmup steps, 30.9 after 2000)")
    p.add_argument("--workload", choices=("c3", "c2", "c5"), default="c3",
                   help="c3: 2-DoF arm, K per GPU (BASELINE metric); c2: same path at config 2's K=4096 T=32; "
                        "c5: 7-DoF chain, K total (config 5)")
    p.add_argument("--K", type=int, default=None, help="c3: samples per GPU (65536); c2: 4096; c5: samples in total (131072)")
    p.add_argument("--T", type=int, default=None, help="horizon (c3: 64, c2: 32, c5: 128)")
    p.add_argument("--nbuf", type=int, default=None, help="rotated noise buffers (c3: 10, c5: 4)")
    p.add_argument("--lps", type=int, default=0, help="lanes per sample (0 = auto; c5: 1 or 4)")
    p.add_argument("--precision", choices=("f32", "f64"), default="f32",
                   help="c5: rollout arithmetic of the chain (f64: for spread weights, DESIGN §3b)")
    p.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline budget (0 = skip)")
    p.add_argument("--traffic-json", default=None,
                   help="measured HBM bytes per launch (default profiles/traffic.json, c2/c5: profiles/traffic_<workload>.json)")
    p.add_argument("--launch", choices=("eager", "graph"), default="eager",
                   help="N = 1: back-to-back launches from the host loop (default) or replay of a captured HIP graph")
    p.add_argument("--backend", default=None,
                   help="torch.distributed backend for N > 1: nccl (= RCCL; default when every rank has its own GPU) "
                        "or gloo (default when ranks share GPUs: a one-GPU rehearsal, RCCL refuses two ranks on one "
                        "GPU)")
    p.add_argument("--exchange", choices=("auto", "launch", "rccl"), default="auto",
                   help="N > 1: partial rows exchanged inside the rollout launch (IPC inboxes over xGMI; auto: "
                        "after a one-step check against RCCL, else RCCL) or by an RCCL all_gather + merge launch")
    return p.parse_args()


def host_cores() -> int:
    """CPUs this process may run on (its affinity mask / cgroup share): on the GPU box
    os.cpu_count() reports the whole host (256) while a one-GPU job is allotted 16."""
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        return os.cpu_count() or 1


def cpu_baseline(args, window, x0, u):
    """C oracle restatement (OpenMP over samples) on the host cores this job may use, rank 0, N = 1."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import coracle  # checker / baseline only
    arm = ArmParams()
    K, T = args.K, args.T
    rng = np.random.default_rng(7)
    eps = (rng.standard_normal((K, T, 2)) * np.sqrt(20.0)).astype(np.float32)
    lam = 100.0
    avail = host_cores()
    threads = min(avail, int(os.environ.get("OMP_NUM_THREADS") or avail))
    t0 = time.perf_counter()
    n = 0
    while True:
        S = coracle.rollout_costs(x0, u, eps, window, 0.006, lam, 0.98, np.eye(2) * 20.0,
                                  [0.5, 0.5, 5.0, 5.0], [5.0, 5.0, 50.0, 50.0], arm, nthreads=threads)
        coracle.weighted_noise(S, eps, lam)
        n += 1
        el = time.perf_counter() - t0
        if el >= args.cpu_seconds / 2:
            break
    out = {"value": K * T * n / el, "unit": "state-steps/s", "cores": threads,
           "kind": "port",
           "sample": f"{n} full steps of K={K} T={T} (rollout+cost+softmin+weighted noise), "
                     f"C fp64 restatement oracle/mppi_oracle.c, OpenMP on {threads} threads, {el:.1f} s",
           "cores_available": avail, "os_cpu_count": os.cpu_count(),
           "OMP_NUM_THREADS": os.environ.get("OMP_NUM_THREADS"),
           "cores_note": "threads = the CPUs in this job's affinity mask (the pool allots 16 host CPUs per GPU; "
                         "os_cpu_count is the whole host)"}
    out["numpy_fp64_1thread"] = numpy_baseline(eps, window, x0, u, lam, args.cpu_seconds / 2)
    return out


def numpy_baseline(eps, window, x0, u, lam, seconds):
    """the vectorised fp64 NumPy restatement (oracle/mppi_oracle.py), one thread, on the
    whole workload (whole steps: rollout + cost + weights + weighted noise; at least one)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import mppi_oracle as O  # checker / baseline only
    sub = eps
    Ks, T = sub.shape[0], sub.shape[1]
    t0 = time.perf_counter()
    n = 0
    while True:
        S = O.rollout_costs(x0, u, sub, window, 0, 0.006, lam, 0.98, np.eye(2) * 20.0,
                            np.array([0.5, 0.5, 5.0, 5.0]), np.array([5.0, 5.0, 50.0, 50.0]))
        O.weighted_noise(O.compute_weights(S, lam), sub)
        n += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    return {"value": Ks * T * n / el, "unit": "state-steps/s", "cores": 1,
            "sample": f"{n} full steps of K={Ks} T={T} (the whole workload), "
                      f"oracle/mppi_oracle.py NumPy fp64, {el:.1f} s"}


def cpu_baseline_c5(args, window, x0, u, K, T):
    """C chain oracle (OpenMP over samples) on the host cores, rank 0, N = 1."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import chain_oracle
    import coracle  # checker / baseline only
    from mppi_robotarm_amd.chain import CHAIN7_SIGMA
    rng = np.random.default_rng(7)
    eps = (rng.standard_normal((T, 7, K)) * np.sqrt(np.diag(CHAIN7_SIGMA))[None, :, None]).astype(np.float32)
    avail = host_cores()
    threads = min(avail, int(os.environ.get("OMP_NUM_THREADS") or avail))
    t0 = time.perf_counter()
    n = 0
    while True:
        S = coracle.chain_rollout_costs(x0, u, eps, window, 0.006, 100.0, 0.98, CHAIN7_SIGMA, [0.5, 0.5, 5.0, 5.0],
                                        [5.0, 5.0, 50.0, 50.0], chain_oracle.ChainParams(), layout="TNK",
                                        nthreads=threads)
        coracle.chain_weighted_noise(S, eps, 100.0, layout="TNK")
        n += 1
        el = time.perf_counter() - t0
        if el >= args.cpu_seconds:
            break
    return {"value": K * T * n / el, "unit": "state-steps/s", "cores": threads, "kind": "port",
            "sample": f"{n} full steps of K={K} T={T} (7-link rollout+cost+softmin+weighted noise), C fp64 "
                      f"restatement oracle/chain_oracle.c, OpenMP on {threads} threads, {el:.1f} s",
            "cores_available": avail, "os_cpu_count": os.cpu_count()}


def dropin_latency(K, T, device, ticks=200, warm=100):
    """SURVEY §8(d)'s control-step latency: the wall time of the drop-in's
    calc_control_input, median over a closed loop of run.py's driver
    (mppi_robotarm_amd.harness, the plant stepped on the host between ticks) at
    the bench's K and T, plus the same calls back to back (nothing between them,
    so each call also waits for the previous call's noise draw).  Steady state:
    a first closed loop of `warm` ticks and the first `warm` back-to-back calls
    are not counted (the first ~100 calls of a process run 10-20% slower:
    tools/lat_compare.py)."""
    from mppi_robotarm_amd.harness import run_closed_loop
    from mppi_robotarm_amd.controller import MPPIControllerForPathTracking
    from mppi_robotarm_amd.params import runpy_config
    path = np.load(os.path.join(ROOT, "tests", "golden", "paths.npz"))["xydq_circle"][:, :4]
    for n in (warm, ticks):
        rec = run_closed_loop(path, ticks=n, number_of_samples_K=K, horizon_step_T=T, noise="device", seed=0,
                              verbose=False, visualze_sampled_trajs=False, device=device)
        rec["controller"].close()
    lat = rec["latency_s"][3:] * 1e3
    kw = runpy_config()
    kw.update(number_of_samples_K=K, horizon_step_T=T, visualze_sampled_trajs=False)
    c = MPPIControllerForPathTracking(ref_path=path, noise="device", seed=0, verbose=False, device=device, **kw)
    x = X0_RUNPY.copy()
    b2b = []
    for i in range(warm + ticks):
        c.prev_waypoints_idx = 0
        t0 = time.perf_counter()
        c.calc_control_input(x)
        b2b.append(time.perf_counter() - t0)
    c.close()
    b2b = np.array(b2b[warm:]) * 1e3
    return float(np.median(lat)), float(np.percentile(lat, 90)), float(np.median(b2b))


def sampled_latency(K, T, device, calls=20, warm=5, noise="device"):
    """calc_control_input back to back (ms, median) with run.py's visualze_sampled_trajs=True: the K x T
    re-roll of control.py:135-145 on the device and its fp64 sampled_traj_list read back every call (fp32 DMA,
    widened on host threads: controller.SampledReadback).  noise="numpy": run.py's exact flags together (the
    drop-in's default noise, the reference's np.random stream drawn on the device, the next call's draw queued
    behind the re-roll).  Returns (median ms, detail dict)."""
    from mppi_robotarm_amd.controller import MPPIControllerForPathTracking
    from mppi_robotarm_amd.params import runpy_config
    path = np.load(os.path.join(ROOT, "tests", "golden", "paths.npz"))["xydq_circle"][:, :4]
    kw = runpy_config()
    kw.update(number_of_samples_K=K, horizon_step_T=T, visualze_sampled_trajs=True)
    c = MPPIControllerForPathTracking(ref_path=path, noise=noise, seed=0, verbose=False, device=device, **kw)
    np.random.seed(0)
    ts = []
    for i in range(warm + calls):
        c.prev_waypoints_idx = 0
        t0 = time.perf_counter()
        out = c.calc_control_input(X0_RUNPY)
        ts.append(time.perf_counter() - t0)
        del out
    detail = {"calls": calls, "warm": warm}
    if noise == "numpy":
        detail["queued_draws_used"] = c._npre_used
        detail["device_draws"] = c._npdev.draws if c._npdev else 0
        detail["device_draw_retries"] = c._npdev.retries if c._npdev else None
    rb = c._sampled_pool._rb
    if rb is not None:
        # the read-back alone on a tensor of the same shape: the floor under the sampled leg
        tr = torch.randn((K, T, 4), device=f"cuda:{device}", dtype=torch.float32)
        dst = np.empty((K, T, 4))
        rt = []
        for i in range(12):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            rb.run(tr, dst)
            rt.append(time.perf_counter() - t0)
        detail["readback_only_ms"] = float(np.median(rt[2:])) * 1e3
        detail["readback_workers"] = rb.workers
        detail["readback_bytes_over_link"] = int(tr.numel() * 4)
        # its floor: the same fp32 bytes in one DMA into page-locked memory, nothing widened
        pin = torch.empty((K, T, 4), dtype=torch.float32, pin_memory=True)
        ft = []
        for i in range(12):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            pin.copy_(tr)
            torch.cuda.synchronize()
            ft.append(time.perf_counter() - t0)
        detail["fp32_dma_floor_ms"] = float(np.median(ft[2:])) * 1e3
        del pin
    c.close()
    return float(np.median(ts[warm:])) * 1e3, detail


def numpy_noise_latency(K, T, device, calls=20, warm=5, sigma=None):
    """calc_control_input back to back (ms, median) with the drop-in's default noise="numpy": the reference's
    own draw, np.random.multivariate_normal on the legacy global RNG (control.py:154-164), NumPy's values and
    state, drawn on the device (mppi_np_*, engine.NpDeviceStream; the host draw, hostrng, for other Sigmas)."""
    from mppi_robotarm_amd.controller import MPPIControllerForPathTracking
    from mppi_robotarm_amd.params import runpy_config
    path = np.load(os.path.join(ROOT, "tests", "golden", "paths.npz"))["xydq_circle"][:, :4]
    kw = runpy_config()
    kw.update(number_of_samples_K=K, horizon_step_T=T, visualze_sampled_trajs=False)
    if sigma is not None:
        kw["sigma"] = sigma
    c = MPPIControllerForPathTracking(ref_path=path, noise="numpy", verbose=False, device=device, **kw)
    np.random.seed(0)
    ts = []
    for i in range(warm + calls):
        c.prev_waypoints_idx = 0
        t0 = time.perf_counter()
        c.calc_control_input(X0_RUNPY)
        ts.append(time.perf_counter() - t0)
    detail = {"calls": calls, "warm": warm, "queued_draws_used": c._npre_used,
              "device_draws": c._npdev.draws if c._npdev else 0,
              "device_draw_retries": c._npdev.retries if c._npdev else None}
    c.close()
    return float(np.median(ts[warm:])) * 1e3, detail


def numpy_noise_closed_loop(K, T, device, ticks=100, warm=30):
    """The drop-in with its default noise="numpy" in run.py's closed loop (mppi_robotarm_amd.harness, the plant
    stepped on the host between ticks): median calc_control_input wall time (ms) after a first loop of `warm`
    ticks; the next call's draw runs beside the step and under the plant step."""
    from mppi_robotarm_amd.harness import run_closed_loop
    path = np.load(os.path.join(ROOT, "tests", "golden", "paths.npz"))["xydq_circle"][:, :4]
    np.random.seed(0)
    for n in (warm, ticks):
        rec = run_closed_loop(path, ticks=n, number_of_samples_K=K, horizon_step_T=T, noise="numpy",
                              verbose=False, visualze_sampled_trajs=False, device=device)
        rec["controller"].close()
    return float(np.median(rec["latency_s"][3:] * 1e3))


def chain_dropin_latency(K, T, device, precision="f32", calls=40, warm=10, noise="device"):
    """The chain drop-in's calc_control_input back to back (ms, median) from the config-5 start state, the
    start nominal re-staged before each call (the bench loop's reset: no plant between calls).  noise="numpy":
    the drop-in's default, the reference's own np.random.multivariate_normal stream (drawn on the device)."""
    from mppi_robotarm_amd.chain import CHAIN7_X0, ChainMPPIController, gravity_torque
    path = np.load(os.path.join(ROOT, "tests", "golden", "paths.npz"))["xydq_circle"][:, :4]
    c = ChainMPPIController(0.006, path, T, K, u_init=gravity_torque(CHAIN7_X0[:7]), device=device, noise=noise,
                            precision=precision)
    np.random.seed(0)
    u0 = c.u_prev.copy()
    ts = []
    for i in range(warm + calls):
        c.u_prev[:] = u0
        c.prev_waypoints_idx = 0
        t0 = time.perf_counter()
        c.calc_control_input(CHAIN7_X0)
        ts.append(time.perf_counter() - t0)
    c.close()
    return float(np.median(ts[warm:])) * 1e3


def exchange_costs(eng, noise, partial, gathered, world, xmode, args, steps=200):
    """N > 1, after the timed region: the per-step cost of each way to finish a multi-GPU step on this node,
    timed the same way as the headline (barrier + synchronise on both sides, max over ranks): the rank's fused
    step without any exchange (its own shard's update: the floor), the in-launch exchange (when attached), and
    rollout + RCCL all-gather + merge launch.  The ranks' nominals diverge here, which nothing after reads."""
    import torch.distributed as dist

    def sync():
        if torch.cuda.is_available():   # (a CPU test drives this with a stand-in engine)
            torch.cuda.synchronize()

    def timed(fn):
        dist.barrier()
        sync()
        t0 = time.perf_counter()
        for i in range(steps):
            fn(i)
        sync()
        dist.barrier()
        el = time.perf_counter() - t0
        dev = eng.device if args.backend == "nccl" else "cpu"
        tt = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        return float(tt[0]) * 1e3 / steps

    nb = len(noise)

    def local(i):
        eng.rollout(noise[i % nb], fused_update=True)

    def launch(i):
        eng.rollout(noise[i % nb], fused_update=True, exchange=True)

    def rccl(i):
        eng.rollout(noise[i % nb], partial_out=partial)
        exchange_partials(partial, gathered)
        eng.merge(gathered, world, fused_update=True)

    out = {"steps": steps, "no_exchange_ms_per_step": timed(local),
           "rccl_allgather_merge_ms_per_step": timed(rccl),
           "in_launch_ms_per_step": timed(launch) if xmode == "launch" else None}
    eng.synchronize()
    return out


def launch_ranks(args) -> int:
    """`--gpus N` (N > 1) without a launcher: start N rank processes under
    torch.distributed.run on this node (127.0.0.1) and return their exit code.
    Runs before anything touches the GPU (device_count() does not initialise HIP
    on this image), and starts the ranks as children rather than exec-ing."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = launcher_cmd(args.gpus, port, sys.argv[1:])
    return subprocess.call(cmd, env=launcher_env())


def launcher_env() -> dict:
    """The ranks' environment: this one with HSA_ENABLE_IPC_MODE_LEGACY=0 (distributed.IPC_ENV: the host
    driver's HIP IPC is dmabuf only, which the in-launch exchange's inbox handles and RCCL's intra-node
    transport both need; an external torchrun inherits it from the driver's environment)."""
    from mppi_robotarm_amd.distributed import IPC_ENV
    return dict(os.environ, **{IPC_ENV: "0"})


def launcher_cmd(n: int, port: int, argv) -> list:
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)


def default_backend(world: int) -> str:
    """nccl (RCCL over xGMI) when every rank can own a GPU, else gloo."""
    return "nccl" if torch.cuda.device_count() >= world else "gloo"


def progress(msg: str) -> None:
    """A phase line on stderr (a long profiled run then shows it is alive); stdout keeps only the JSON line."""
    print(f"bench [rank {os.environ.get('RANK', '0')}]: {msg}", file=sys.stderr, flush=True)


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))
    c5 = args.workload == "c5"
    if args.K is None:
        args.K = {"c5": 131072, "c2": 4096}.get(args.workload, 65536)
    if args.T is None:
        args.T = {"c5": 128, "c2": 32}.get(args.workload, 64)
    if args.nbuf is None:
        args.nbuf = 4 if c5 else 10
    if args.traffic_json is None:
        name = "traffic.json" if args.workload == "c3" else f"traffic_{args.workload}.json"
        if args.K != {"c5": 131072, "c2": 4096}.get(args.workload, 65536):
            name = f"traffic_{args.workload}_k{args.K}.json"   # e.g. config 5's 8-way shard, K = 16384
        args.traffic_json = os.path.join(ROOT, "profiles", name)
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    local_rank = local_rank % max(1, torch.cuda.device_count())  # rehearsal: several ranks on one GPU
    torch.cuda.set_device(local_rank)
    if args.backend is None:
        args.backend = default_backend(world)
    if world > 1:
        import torch.distributed as dist
        # the process-group set-up may print to stdout (gloo's "Rank n is connected" lines); rank 0's stdout
        # carries only the JSON line, so the set-up's fd 1 goes to stderr
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)
        try:
            if args.backend == "nccl":
                dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
            else:
                dist.init_process_group(args.backend)
            dist.barrier()
        finally:
            os.dup2(saved, 1)
            os.close(saved)
    T = args.T
    path = np.load(os.path.join(ROOT, "tests", "golden", "paths.npz"))["xydq_circle"][:, :4]
    window = path[0:30]
    if c5:
        from mppi_robotarm_amd.chain import CHAIN7_SIGMA, CHAIN7_X0, ChainEngine, ChainParams, gravity_torque
        from mppi_robotarm_amd.distributed import shard_geometry
        K_total = args.K                                   # strong scaling: config 5 fixes K
        K, k_offset = shard_geometry(K_total, world, rank)
        eng = ChainEngine(K, T, 0.006, 100.0, 0.98, CHAIN7_SIGMA, [0.5, 0.5, 5.0, 5.0], [5.0, 5.0, 50.0, 50.0],
                          0.0, ChainParams(), K_total=K_total, k_offset=k_offset, device=local_rank,
                          precision=args.precision, lanes_per_sample=args.lps)
        x0 = CHAIN7_X0.copy()
        u = np.tile(gravity_torque(x0[:7]), (T, 1))
    else:
        K = args.K
        K_total, k_offset = K * world, K * rank
        eng = RolloutEngine(K, T, 0.006, 100.0, 0.98, np.eye(2) * 20.0, [0.5, 0.5, 5.0, 5.0],
                            [5.0, 5.0, 50.0, 50.0], 0.0, ArmParams(), K_total=K_total, k_offset=k_offset,
                            device=local_rank, lanes_per_sample=args.lps)
        x0 = X0_RUNPY.copy()
        u = np.array([[10.0, -2.0]] * T)
    progress(f"{args.workload} K={K} T={T}: engine ready")
    eng.set_step_inputs(x0, window, u)
    noise = [eng.philox_noise(1234, i) for i in range(args.nbuf)]
    partial = eng.new_partial()
    gathered = torch.empty(world * eng.partial_len, dtype=torch.float64, device=eng.device)
    stream = torch.cuda.current_stream()

    # N = 1: the device-resident loop has no host synchronisation.  Default:
    # the host loop launches step after step (a launch costs less host time than
    # a step takes on the GPU, so the queue never drains; measured 31 us/step
    # against 36 with graph replay, whose per-node cost is higher on ROCm 7.2).
    # --launch graph captures a chunk of steps (one per noise buffer, an even
    # count so the ping-pong parameter block returns to the same parity) once
    # and replays it.
    use_graph = world == 1 and args.launch == "graph" and args.nbuf % 2 == 0 and not c5
    chunk = args.nbuf if use_graph else 1
    steps = (args.steps + chunk - 1) // chunk * chunk

    xmode = "none" if world == 1 else "rccl"
    xreport = {}   # the step-1 self-check: which exchange, and why a fallback happened (distributed.py)
    if world > 1 and args.exchange != "rccl":
        ok = attach_exchange(eng, report=xreport) and check_exchange(eng, noise[0], partial, gathered,
                                                                     report=xreport)
        if not ok and args.exchange == "launch":
            raise RuntimeError(f"in-launch exchange unavailable: {xreport}")
        xmode = "launch" if ok else "rccl"
    xreport["picked"] = xmode

    # c5: the plant-less device loop (fixed start state, the nominal updated every step) drifts for the chain:
    # |u| grows ~1 N m per step and after ~250 steps most rollouts overflow (tools/loop_drift.py).  Every
    # C5_RESET steps the start nominal is staged again (a 27 KB host-to-device copy, inside the timed region),
    # so the timed steps stay in the regime of a controller near its path.  The 2-DoF loop is stationary.
    C5_RESET = 32

    def step(i, ev_pair=None):
        if c5 and i % C5_RESET == 0:
            eng.set_step_inputs(x0, window, u)
        if ev_pair is not None:
            ev_pair[0].record(stream)
        if world == 1:
            eng.rollout(noise[i % args.nbuf], fused_update=True)
        elif xmode == "launch":
            eng.rollout(noise[i % args.nbuf], fused_update=True, exchange=True)
        else:
            eng.rollout(noise[i % args.nbuf], partial_out=partial)
        if ev_pair is not None:
            ev_pair[1].record(stream)
        if xmode == "rccl":
            exchange_partials(partial, gathered)
            eng.merge(gathered, world, fused_update=True)

    # clock settle (untimed): a controller runs continuously, so the metric is
    # the steady-state rate; then the W warmup steps of the contract
    t_settle = time.perf_counter()
    i = 0
    while (time.perf_counter() - t_settle) * 1e3 < args.settle_ms:   # rank-local: no collectives
        for _ in range(16):
            if c5 and i % C5_RESET == 0:
                eng.set_step_inputs(x0, window, u)
            if world == 1:
                eng.rollout(noise[i % args.nbuf], fused_update=True)
            else:
                eng.rollout(noise[i % args.nbuf], partial_out=partial)
            i += 1
        torch.cuda.synchronize()
    for i in range(args.warmup):
        step(i)
    torch.cuda.synchronize()
    graph = None
    if use_graph:
        s_cap = torch.cuda.Stream()
        s_cap.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s_cap):
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph, stream=s_cap):
                for i in range(chunk):
                    step(i)
        torch.cuda.current_stream().wait_stream(s_cap)
        graph.replay()      # one untimed replay
        torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    progress(f"settled and warmed up (exchange: {xmode}); timing {steps} steps")
    nev = steps // chunk
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(nev)]
    whole = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
    t0 = time.perf_counter()
    if world == 1 or xmode == "launch":
        # one event pair around the whole timed region on the launch stream
        whole[0].record(stream)
        for c in range(nev):
            if graph is not None:
                graph.replay()
            else:
                step(c)
        whole[1].record(stream)
    else:
        for c in range(nev):
            step(c, ev[c])   # events bracket the rollout launch only (the exchange is timed by the wall clock)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    # average duration per launch of the rollout kernel (events on the launch
    # stream); at N = 1 the back-to-back launches' average, boundaries included
    if world == 1 or xmode == "launch":
        kern_ms = whole[0].elapsed_time(whole[1]) / steps
    else:
        kern_ms = sum(a.elapsed_time(b) for a, b in ev) / steps
    ranks_seen = 1
    n_dev = 1
    if world > 1:
        import socket
        where = [None] * world
        dist.all_gather_object(where, (socket.gethostname(), local_rank))
        n_dev = len(set(where))                        # distinct GPUs (a rehearsal puts ranks on one)
        dev = eng.device if args.backend == "nccl" else "cpu"
        tt = torch.tensor([elapsed, kern_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed, kern_ms = float(tt[0]), float(tt[1])
        one = torch.ones(1, dtype=torch.float64, device=dev)
        dist.all_reduce(one, op=dist.ReduceOp.SUM)      # every rank took part in the timed region
        ranks_seen = int(one.item())
    args.steps = steps
    eng.synchronize()   # raises if an in-launch hand-off timed out anywhere in the run (results invalid)
    u_final = eng.nominal()
    assert np.all(np.isfinite(u_final)), "non-finite nominal control"
    xcosts = exchange_costs(eng, noise, partial, gathered, world, xmode, args) if world > 1 and not c5 else None

    if rank == 0:
        ms_per_step = elapsed * 1e3 / args.steps
        value = K_total * T * args.steps / elapsed
        alg_bytes = (C5_BYTES_PER_STATE_STEP if c5 else BYTES_PER_STATE_STEP) * K * T
        achieved = alg_bytes / (kern_ms * 1e-3) / 1e9
        traffic = None
        valu = None
        if os.path.exists(args.traffic_json):
            try:
                tj = json.load(open(args.traffic_json))
                if tj.get("K") == K and tj.get("T") == T and tj.get("workload", "c3") == args.workload:
                    traffic = tj.get("hbm_bytes_per_launch")
                    valu = valu_roofline(tj, kern_ms)
            except Exception:
                traffic = None
        out = {
            "metric": (f"MPPI rollouts/sec (K×T state-steps/s), 7-DoF chain K={K_total} T={T} (BASELINE config 5)"
                       if c5 else f"MPPI rollouts/sec (K×T state-steps/s) + control-step latency, K={K} T={T}"),
            "value": value,
            "unit": "state-steps/s",
            "n_gpus": n_dev,
            "ranks": world,
            "ranks_per_gpu": world / n_dev,
            "ranks_seen": ranks_seen,
            "steps": args.steps,
            "warmup": args.warmup, "settle_ms": args.settle_ms,
            "ms_per_step": ms_per_step,
            "rollouts_per_s": K_total * args.steps / elapsed,
            "control_step_latency_ms": None,   # filled below (N = 1, c3): the drop-in's calc_control_input
            "device_step_ms": ms_per_step,
            "kernel_ms": kern_ms,
            "higher_is_better": True,
            "scaling": "strong" if c5 else "weak",
            "vs_baseline": None,
            "dtype": args.precision if c5 else "f32",
            "data": "synthetic",
            "config": {"workload": (f"7-DoF chain MPPI step (build-defined model, armature + damping), K={K_total} "
                                    f"(K/GPU={K}) T={T}, run.py constants, config-5 start pose, xydq_circle.txt "
                                    f"window, Philox N(0,Sigma7) noise x{args.nbuf} buffers" if c5 else
                                    f"2-DoF arm MPPI step, K={K_total} (K/GPU={K}) T={T}, run.py constants, "
                                    f"xydq_circle.txt window, Philox N(0,20I) noise x{args.nbuf} buffers"),
                       "K_total": K_total, "K_per_gpu": K, "T": T,
                       "lanes_per_sample": eng.lanes_per_sample,
                       "exchange": xmode, "backend": args.backend if world > 1 else None,
                       "parallelism": (f"samples sharded x{world} ranks on {n_dev} GPU(s), " + (
                           ("partial rows exchanged inside the rollout launch (IPC inboxes"
                            + (" over xGMI)" if n_dev == world else "; shared GPU: no xGMI link crossed)"))
                           if xmode == "launch" else "all_gather of partials + merge launch"
                           + (" (RCCL)" if args.backend == "nccl" else f" ({args.backend})"))) if world > 1
                       else "single device, fused update" + (f", HIP graph of {chunk} steps" if use_graph
                                                               else ", back-to-back launches")},
            "exchange_selfcheck": xreport if world > 1 else None,
            "exchange_costs": xcosts,
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic},
            "valu_roofline": valu,
        }
        if world == 1 and not c5:
            progress("device loop timed; drop-in latency legs")
            med, p90, b2b = dropin_latency(K, T, local_rank)
            out["control_step_latency_ms"] = med
            out["control_step_latency_p90_ms"] = p90
            out["control_step_latency_back_to_back_ms"] = b2b
            progress("sampled-trajectories leg")
            out["control_step_latency_sampled_trajs_ms"], out["sampled_trajs_detail"] = sampled_latency(
                K, T, local_rank)
            progress("run.py-flags leg (NumPy noise + sampled trajectories)")
            out["control_step_latency_runpy_flags_ms"], out["runpy_flags_detail"] = sampled_latency(
                K, T, local_rank, noise="numpy")
            progress("NumPy-noise leg")
            out["control_step_latency_numpy_noise_ms"], out["numpy_noise_detail"] = numpy_noise_latency(
                K, T, local_rank)
            out["control_step_latency_numpy_noise_general_sigma_ms"], out["numpy_noise_general_sigma_detail"] = (
                numpy_noise_latency(K, T, local_rank, sigma=np.array([[20.0, 6.0], [6.0, 12.0]])))
            out["control_step_latency_numpy_noise_closed_loop_ms"] = numpy_noise_closed_loop(K, T, local_rank)
            out["control_step_latency_def"] = (
                "median wall time of MPPIControllerForPathTracking.calc_control_input (drop-in, noise='device') "
                "in run.py's closed loop at this K, T: stage inputs, one fused launch (rollouts, soft-min, "
                "weighted noise, median filter, update, shift), wait on its host-mapped result, fp64 optimal "
                "trajectory on the host; the next tick's Philox draw is queued behind the launch and overlaps the "
                "plant step between ticks. back_to_back: the same calls with nothing between them (each then "
                "also waits for the previous draw). Steady state: 200 ticks each, after 100 uncounted. These "
                "two run with visualze_sampled_trajs=False; sampled_trajs: back to back with run.py's own "
                "visualze_sampled_trajs=True, i.e. also the (K, T, 4) fp64 sampled_traj_list (134 MB at K = "
                "65536) re-rolled on the device, its fp32 states DMA'd in chunks and widened to fp64 by host threads "
                "every call (sampled_trajs_detail.readback_only_ms: that read-back alone); runpy_flags: run.py's "
                "exact flags together, noise='numpy' (the default) and visualze_sampled_trajs=True; numpy_noise: back to back with the "
                "drop-in's default noise='numpy', the reference's own np.random.multivariate_normal stream "
                "(NumPy's values and RNG state) drawn on the device every call (mppi_np_*): each call queues the "
                "next call's draw beside its step, used when np.random is still where the call left it; "
                "numpy_noise_general_sigma: numpy_noise with Sigma = [[20, 6], [6, 12]] (a full 2 x 2 transform, np.dot's "
                "rounding pinned at run time, hostrng.dot2_model); "
                "numpy_noise_closed_loop: the same in run.py's closed loop (100 ticks after 30). "
                "ms_per_step is the device-resident loop")
        if world == 1 and c5:
            out["control_step_latency_back_to_back_ms"] = chain_dropin_latency(K, T, local_rank, args.precision)
            progress("NumPy-noise leg")
            out["control_step_latency_numpy_noise_ms"] = chain_dropin_latency(K, T, local_rank, args.precision,
                                                                              calls=10, warm=3, noise="numpy")
            out["control_step_latency_def"] = (
                "median wall time of ChainMPPIController.calc_control_input (noise='device') at this K, T, back "
                "to back from the config-5 start state (no plant model exists for the build-defined chain, so no "
                "closed loop): one fused launch (rollouts, soft-min, weighted noise, median filter, update, shift), "
                "one read-back, fp64 optimal trajectory on the host, the next step's Philox draw queued behind "
                "the launch (each call then also waits for the previous draw). 40 calls after 10 uncounted. "
                "numpy_noise: the same with the drop-in's default noise='numpy', the reference's own "
                "np.random.multivariate_normal stream (NumPy's values and RNG state) drawn on the device every "
                "call, the next call's beside the step (10 calls after 3). ms_per_step is the device-resident loop")
        if world == 1 and args.cpu_seconds > 0:
            progress("CPU baseline")
            out["cpu_baseline"] = (cpu_baseline_c5(args, window, x0, u, K, T) if c5
                                   else cpu_baseline(args, window, x0, u))
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
