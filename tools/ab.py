"""A/B timing of two builds of the C ABI in ONE process on the same inputs
(diagnostic tool, not product).  Batches of fused launches alternate between
the builds, so clock and thermal drift hit both alike.

    python tools/ab.py LIB_A.so LIB_B.so [LIB_C.so ...] [K T batches launches_per_batch]
    WORKLOAD=c5: the 7-link chain engine (default K 131072, T 128)
    WORKLOAD=philox: the arm's noise draw (mppi_noise_philox) instead of the rollout
    LPS=n: lanes per sample of every arm build; LPS_LIST=a,b,...: per build (the same .so may repeat)

Prints, per build, the median / min per-launch time (HIP events around each
batch on the launching stream) and each build's ratio to the first.
"""
import ctypes as C
import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from mppi_robotarm_amd import _native as N  # noqa: E402
from mppi_robotarm_amd.params import X0_RUNPY, ArmParams  # noqa: E402


def make_ctx(L, K, T, lam, stream, lps=0):
    a = ArmParams()
    cfg = N.ConfigC()
    cfg.K_local, cfg.T, cfg.K_total, cfg.k_offset = K, T, K, 0
    cfg.delta_t, cfg.param_lambda, cfg.param_alpha, cfg.param_exploration = 0.006, lam, 0.98, 0.0
    cfg.sigma = (C.c_double * 4)(20, 0, 0, 20)
    cfg.stage_cost_weight = (C.c_double * 4)(0.5, 0.5, 5, 5)
    cfg.terminal_cost_weight = (C.c_double * 4)(5, 5, 50, 50)
    cfg.arm = N.ArmParamsC(a.m1, a.m2, a.l1, a.l2, a.lc1, a.lc2, a.g, a.fk_l1, a.fk_l2)
    cfg.lanes_per_sample = lps
    ctx = C.c_void_p()
    rc = L.mppi_ctx_create(C.byref(cfg), 0, C.c_void_p(stream), C.byref(ctx))
    assert rc == 0, L.mppi_last_error()
    return ctx


def chain_runs(libs, K, T, lam):
    from mppi_robotarm_amd import chain as CH
    path = np.load(os.path.join(ROOT, "tests", "golden", "paths.npz"))["xydq_circle"][:, :4]
    runs = []
    for p in libs:
        L = N.open_library(p)
        orig = N.load
        N.load = lambda L=L: L
        try:
            eng = CH.ChainEngine(K, T, 0.006, lam, 0.98, CH.CHAIN7_SIGMA, [0.5, 0.5, 5, 5], [5, 5, 50, 50], 0.0,
                                 device=0)
        finally:
            N.load = orig
        eng.set_step_inputs(CH.CHAIN7_X0, path[:30], np.tile(CH.gravity_torque(CH.CHAIN7_X0[:7]), (T, 1)))
        noise = [eng.philox_noise(1234, i) for i in range(4)]

        u0 = np.tile(CH.gravity_torque(CH.CHAIN7_X0[:7]), (T, 1))

        def batch(n, eng=eng, noise=noise, u0=u0):
            for i in range(n):
                if i % 32 == 0:   # as bench.py: the plant-less chain loop drifts into overflow otherwise
                    eng.set_step_inputs(CH.CHAIN7_X0, path[:30], u0)
                eng.rollout(noise[i % len(noise)], fused_update=True)
        def close(eng=eng, p=p):   # same launch sequence in every build: the nominals must match
            u = eng.nominal()
            print(f"    {os.path.basename(p)}: nominal sha1 {hashlib.sha1(u.tobytes()).hexdigest()[:12]}")
            eng.close()
        runs.append((p, batch, close, []))
    return runs


def arm_runs(libs, K, T, lam, stream):
    path = np.load(os.path.join(ROOT, "tests", "golden", "paths.npz"))["xydq_circle"][:, :4]
    win = np.ascontiguousarray(path[:30])
    u = np.array([[10.0, -2.0]] * T)
    dp = lambda a: a.ctypes.data_as(C.POINTER(C.c_double))
    runs = []
    lps = [int(x) for x in os.environ.get("LPS_LIST", "").split(",") if x] or [int(os.environ.get("LPS", "0"))] * len(libs)
    for p, lp in zip(libs, lps):
        L = N.open_library(p)
        ctx = make_ctx(L, K, T, lam, stream, lp)
        x0 = np.asarray(X0_RUNPY, dtype=np.float64)
        assert L.mppi_set_step_inputs(ctx, dp(x0), dp(win), 30, dp(u)) == 0
        noise = [torch.empty(T * K * 2, dtype=torch.float32, device="cuda") for _ in range(8)]
        for i, nz in enumerate(noise):
            assert L.mppi_noise_philox(ctx, 1234, i, C.c_void_p(nz.data_ptr())) == 0

        def batch(n, L=L, ctx=ctx, noise=noise):
            for i in range(n):
                assert L.mppi_rollout(ctx, C.c_void_p(noise[i % len(noise)].data_ptr()), None, None, 1) == 0
        runs.append((f"{os.path.basename(p)} lps={lp}", batch, lambda L=L, ctx=ctx: L.mppi_ctx_destroy(ctx), []))
    return runs


def philox_runs(libs, K, T, stream):
    runs = []
    for p in libs:
        L = N.open_library(p)
        ctx = make_ctx(L, K, T, 100.0, stream, 0)
        out = torch.empty(T * K * 2, dtype=torch.float32, device="cuda")

        def batch(n, L=L, ctx=ctx, out=out):
            for i in range(n):
                assert L.mppi_noise_philox(ctx, 1234, i, C.c_void_p(out.data_ptr())) == 0

        def close(L=L, ctx=ctx, out=out, p=p):
            print(f"    {os.path.basename(p)}: last draw sum {float(out.double().sum()):.6e}")
            L.mppi_ctx_destroy(ctx)
        runs.append((os.path.basename(p), batch, close, []))
    return runs


def main():
    libs = [os.path.abspath(a) for a in sys.argv[1:] if a.endswith(".so")]
    nums = [a for a in sys.argv[1:] if not a.endswith(".so")]
    c5 = os.environ.get("WORKLOAD") == "c5"
    K = int(nums[0]) if len(nums) > 0 else (131072 if c5 else 65536)
    T = int(nums[1]) if len(nums) > 1 else (128 if c5 else 64)
    batches = int(nums[2]) if len(nums) > 2 else (16 if c5 else 40)
    per = int(nums[3]) if len(nums) > 3 else (20 if c5 else 50)
    lam = float(os.environ.get("LAMBDA", "100"))
    torch.cuda.set_device(0)
    stream = torch.cuda.current_stream().cuda_stream
    if os.environ.get("WORKLOAD") == "philox":
        runs = philox_runs(libs, K, T, stream)
    else:
        runs = chain_runs(libs, K, T, lam) if c5 else arm_runs(libs, K, T, lam, stream)
    torch.cuda.synchronize()
    for _, batch, _, _ in runs:   # warm-up
        batch(10)
    torch.cuda.synchronize()
    for b in range(batches):
        order = runs if b % 2 == 0 else runs[::-1]
        for _, batch, _, times in order:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            batch(per)
            e1.record()
            torch.cuda.synchronize()
            times.append(e0.elapsed_time(e1) * 1e3 / per)
    base = None
    for p, _, close, times in runs:
        t = np.array(times)
        base = np.median(t) if base is None else base
        print(f"{os.path.basename(p):36s} median {np.median(t):7.2f} us  min {t.min():7.2f}  max {t.max():7.2f}"
              f"  x{np.median(t) / base:.4f}")
        close()
    print(f"(K={K} T={T} lambda={lam} {'chain' if c5 else 'arm'}, {batches} x {per} launches each)")


if __name__ == "__main__":
    main()
